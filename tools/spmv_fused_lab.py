"""Lab (not shipped): the headline SpMV back to back in its three forms
(ek_spmv_bench fused 0: plain y = L x; 1: + the Lanczos epilogue; 2: + the
solve's finalize prologue and ||w||^2 partials, as the step launches it) and the
gather-only ceiling; after a solve, so the matrix is the solve's own.
usage: python tools/spmv_fused_lab.py"""
import importlib.util
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("eigkl_amd", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
ek = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ek)
h, _ = ek.Hypergraph.generate(1.15, 1).largest_component()
ctx = ek.Context(0)
ctx.spmv_setup_pins(h)
ctx.lanczos_fiedler()
for rep in range(2):
    r = {f"fused{f}": round(ctx.spmv_bench(300, fused=f), 3) for f in (0, 1, 2)}
    r["gather_only"] = round(ctx.spmv_gather_bench(300), 3)
    print(r, flush=True)
