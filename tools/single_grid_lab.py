"""Lab (not shipped): VERDICT r5 next-4's single-grid question on the headline
matrix.  A skipped Lanczos step is the SpMV and then a launch that reduces the
SpMV's per-block partials and updates every row.  ek_spmv_gather_bench's
EK_GATHER_MODE prices, on the product SpMV's grid and access pattern
(kernels_spmv.hip k_lab_gather_step):
  0 the gather alone, 1 gather + update as two launches (a kernel boundary),
  2 one grid with an in-launch wait for every block's partial, 3 the update alone.
usage: python tools/single_grid_lab.py"""
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
for rep in range(3):
    r = {}
    for mode in (0, 1, 2, 3):
        os.environ["EK_GATHER_MODE"] = str(mode)
        r[f"mode{mode}"] = round(ctx.spmv_gather_bench(300), 3)
    r["boundary_form_minus_update"] = round(r["mode1"] - r["mode3"], 3)
    r["single_grid_minus_update"] = round(r["mode2"] - r["mode3"], 3)
    print(r, flush=True)
os.environ.pop("EK_GATHER_MODE")
