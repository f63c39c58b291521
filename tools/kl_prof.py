#!/usr/bin/env python3
"""Lab (not shipped): the KL swap loop's phase stamps and per-wave timeline
(EK_KL_PROF=1 build of k_kl_swap_loop) on the bench's headline workload (the
1.15x seed-1 synthetic's largest component) from its GPU Fiedler split, plus
the plain loop's us/swap.  usage: python tools/kl_prof.py [MULT]"""
import importlib.util
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("eigkl_amd", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
ek = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ek)
mult = float(sys.argv[1]) if len(sys.argv) > 1 else 1.15
h, _ = ek.Hypergraph.generate(mult, 1).largest_component()
ctx = ek.Context(0)
ctx.spmv_setup_pins(h)
lam, v, st = ctx.lanczos_fiedler()
_, bits = ek.median_split(v)
ctx.kl_graph_setup(h.kl_graph())
ctx.kl_nets_setup(*h.pins())
for prof in (False, True, False):
    if prof:
        os.environ["EK_KL_PROF"] = "1"
    else:
        os.environ.pop("EK_KL_PROF", None)
    ctx.kl_set_partition_bits(bits)
    log, res = ctx.kl_run()
    print(f"prof={prof}: {res['iterations']} swaps, loop {res['loop_ms']:.3f} ms, "
          f"{1e3 * res['loop_ms'] / res['iterations']:.3f} us/swap", flush=True)
ctx.close()
