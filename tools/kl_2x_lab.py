"""Lab (not shipped): Lanczos + KL on the 2x synthetic (configs[3]); the swap
loop must stay on chip (LDS) at this size."""
import importlib.util, os, sys, time
REPO = os.environ.get("GRAFT_REPO_ROOT", ".")
spec = importlib.util.spec_from_file_location("eigkl_amd", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
ek = importlib.util.module_from_spec(spec); spec.loader.exec_module(ek)
h = ek.Hypergraph.generate(2.0, 2); L = h.laplacian(); ctx = ek.Context(0)
ctx.spmv_setup(h.nodes, 0, L.rowptr, L.col, L.val)
ctx.kl_graph_setup(h.kl_graph()); ctx.kl_nets_setup(*h.pins())
lam, v, st = ctx.lanczos_fiedler(); med, bits = ek.median_split(v)
for rep in range(2):
    ctx.kl_set_partition_bits(bits); _, res = ctx.kl_run(cap=0)
    print("2x: n", h.nodes, "lanczos_ms", round(st["total_ms"], 2), "swaps", res["iterations"], "loop_ms", round(res["loop_ms"], 2), "us/swap", round(res["loop_ms"] * 1e3 / max(1, res["iterations"]), 3), "net_cut", res["net_cut_best"])
