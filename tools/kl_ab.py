"""Lab (not shipped): KL swap-loop time on the 1x / 2x synthetic and the 1x
largest component from a fixed GPU split, several runs, with the loop variant
the environment selects (EK_KL_TWOBAR=1: two barriers per swap).  Prints ms,
us/swap and the swap log's md5 (must not depend on the variant).
usage: python tools/kl_ab.py [reps]"""
import hashlib
import importlib.util
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("eigkl_amd", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
ek = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ek)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
ctx = ek.Context(0)
h1 = ek.Hypergraph.generate(1.0, 1)
for name, h in (("syn1", h1), ("syn1_lcc", h1.largest_component()[0]), ("syn2", ek.Hypergraph.generate(2.0, 2))):
    L = h.laplacian()
    ctx.spmv_setup(h.nodes, 0, L.rowptr, L.col, L.val)
    lam, v, st = ctx.lanczos_fiedler()
    _, bits = ek.median_split(v)
    ctx.kl_graph_setup(h.kl_graph())
    ctx.kl_nets_setup(*h.pins())
    ms = []
    for _ in range(reps):
        ctx.kl_set_partition_bits(bits)
        log, res = ctx.kl_run()
        ms.append(res["loop_ms"])
    print(f"{name}: {res['iterations']} swaps, loop ms {' '.join(f'{x:.2f}' for x in ms)}, "
          f"us/swap {1e3 * min(ms) / res['iterations']:.3f}, net cut {res['net_cut_best']}, "
          f"log md5 {hashlib.md5(log.tobytes()).hexdigest()[:12]}, status {res.get('status')}", flush=True)
ctx.close()
