"""Lab (not shipped): a wider parity sweep than the test suite's: the -EIG
pipeline on the largest components of many generator seeds against the
oracle (Lanczos restatement: lambda within 1e-9 relative, split equal off the
median's 1e-8 band; KL() from the GPU split: swap log bit for bit), plus the
device split against the host's.  usage: python tools/parity_sweep.py"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import load_package  # noqa: E402

sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle  # noqa: E402  (test infrastructure: the checker)

ek = load_package()
ctx = ek.Context(0)
oracle.set_threads(16)
cases = [(0.1, s) for s in range(20, 45)] + [(0.3, s) for s in range(50, 56)] + [(1.0, s) for s in (61, 62)]
bad = 0
for mult, seed in cases:
    h, _ = ek.Hypergraph.generate(mult, seed).largest_component()
    L = h.laplacian()
    ctx.spmv_setup(h.nodes, 0, L.rowptr, L.col, L.val)
    lam, v, st = ctx.lanczos_fiedler()
    g = oracle.Graph.from_pins(h.nodes, *h.pins())
    lam_o, v_o, st_o = g.lanczos()
    v_o = v_o * np.sign(v_o @ v)
    med, bits = ek.median_split(v)
    med_o, bits_o = ek.median_split(v_o)
    mask = (np.abs(v - med) > 1e-8) & (np.abs(v_o - med_o) > 1e-8)
    ok_l = abs(lam - lam_o) <= 1e-9 * abs(lam_o) and st["converged"] and st_o["converged"]
    ok_s = bool(np.array_equal(bits[mask], bits_o[mask]))
    ctx.kl_graph_setup(h.kl_graph())
    ctx.kl_nets_setup(*h.pins())
    med_d, n0, n1 = ctx.kl_set_partition_fiedler()
    ok_d = med_d == med and n0 == int(np.count_nonzero(bits == 0))
    log_d, res_d = ctx.kl_run()
    idx = np.arange(h.nodes, dtype=np.int32)
    olog, ores = g.kl(idx[bits == 0], idx[bits == 1])
    ok_k = res_d["iterations"] == ores["iterations"] and len(log_d) == len(olog) and all(
        np.array_equal(log_d[f], olog[f]) for f in ("iter", "node_left", "node_right")) and all(
        np.array_equal(log_d[f].view(np.uint32), olog[f].view(np.uint32)) for f in ("max_gain", "min_gain", "gain", "cut"))
    ok = ok_l and ok_s and ok_d and ok_k
    bad += not ok
    print(f"{mult}x seed {seed}: n={h.nodes} lambda {lam:.12e} (oracle {lam_o:.12e}) matvecs {st['matvecs']}/{st_o['matvecs']} "
          f"split {'=' if ok_s else 'DIFF'} device-split {'=' if ok_d else 'DIFF'} KL swaps {res_d['iterations']} "
          f"{'=' if ok_k else 'DIFF'} -> {'ok' if ok else 'FAIL'}", flush=True)
print(f"{len(cases) - bad} of {len(cases)} cases equal", flush=True)
ctx.close()
