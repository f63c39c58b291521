#!/usr/bin/env python3
"""Lab (not shipped): KL swap-loop us/swap and swap-log md5 from a fixed GPU
split, on the headline workload (1.15x seed-1 largest component) and the 1x /
2x synthetics, REPS runs each; the md5 must not change with loop variants.
usage: python tools/kl_quick.py [REPS]"""
import hashlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import load_package  # noqa: E402

ek = load_package()
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
ctx = ek.Context(0)
for name, h in (("lcc1.15", ek.Hypergraph.generate(1.15, 1).largest_component()[0]),
                ("syn1", ek.Hypergraph.generate(1.0, 1)), ("syn2", ek.Hypergraph.generate(2.0, 2))):
    ctx.spmv_setup_pins(h)
    lam, v, st = ctx.lanczos_fiedler()
    _, bits = ek.median_split(v)
    ctx.kl_graph_setup(h.kl_graph())
    ctx.kl_nets_setup(*h.pins())
    ms = []
    for _ in range(reps):
        ctx.kl_set_partition_bits(bits)
        log, res = ctx.kl_run()
        ms.append(res["loop_ms"])
    print(f"{name}: {res['iterations']} swaps, loop ms min {min(ms):.3f} ({1e3 * min(ms) / res['iterations']:.3f} us/swap), "
          f"net cut {res['net_cut_best']}, md5 {hashlib.md5(log.tobytes()).hexdigest()[:12]}", flush=True)
ctx.close()
