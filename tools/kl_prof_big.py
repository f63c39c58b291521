"""Lab (not shipped): the KL swap loop's phase stamps (EK_KL_PROF=1, the
diagnostic instantiation) on the 1.15x graph (bitmaps in LDS) and on the 10x
graph (bitmaps off chip, k_kl_swap_loop<.., GB>), -EIG split.  The [kl] lines
on stderr give us per swap by phase.  usage: EK_KL_PROF=1 python tools/kl_prof_big.py"""
import importlib.util
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("eigkl_amd", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
ek = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ek)
ctx = ek.Context(0)
for mult, seed in ((1.15, 1), (10.0, 10)):
    h = ek.Hypergraph.generate(mult, seed)
    ctx.spmv_setup_pins(h)
    lam, v, st = ctx.lanczos_fiedler()
    ctx.kl_graph_setup(h.kl_graph())
    ctx.kl_nets_setup(*h.pins())
    for rep in range(2):
        ctx.kl_set_partition_fiedler()
        print(f"== {mult}x n={h.nodes} rep {rep}", file=sys.stderr, flush=True)
        log, res = ctx.kl_run()
    it = res["iterations"]
    print(f"{mult}x n={h.nodes} swaps={it} kl_loop_ms={res['loop_ms']:.2f} us_per_swap={1e3 * res['loop_ms'] / max(it, 1):.3f}",
          flush=True)
