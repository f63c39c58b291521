"""Lab (not shipped): the KL swap loop's rate on graphs whose side / lock
bitmaps exceed the on-chip budget (the global-state loop) against the on-chip
loop: the -EIG pipeline on generator graphs of growing size, KL loop ms and
us per swap.  usage: python tools/kl_big.py"""
import importlib.util
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("eigkl_amd", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
ek = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ek)
ctx = ek.Context(0)
for mult, seed in ((1.15, 1), (2.0, 2), (3.0, 3), (5.0, 5), (10.0, 10)):
    h = ek.Hypergraph.generate(mult, seed)
    ctx.spmv_setup_pins(h)
    lam, v, st = ctx.lanczos_fiedler()
    ctx.kl_graph_setup(h.kl_graph())
    ctx.kl_nets_setup(*h.pins())
    ctx.kl_set_partition_fiedler()
    for rep in range(2):
        ctx.kl_set_partition_fiedler()
        log, res = ctx.kl_run()
    it = res["iterations"]
    print(f"{mult}x n={h.nodes} swaps={it} kl_loop_ms={res['loop_ms']:.2f} us_per_swap={1e3 * res['loop_ms'] / max(it, 1):.3f}",
          flush=True)
