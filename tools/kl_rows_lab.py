"""Lab (not shipped): how many rows each swap of the ibm18-shape run updates
(tot = deg(node1) + deg(node2)), against the swap loop's rows per G1 pass."""
import importlib.util
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("eigkl_amd", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
ek = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ek)
h = ek.Hypergraph.generate(1.0, 1)
L = h.laplacian()
ctx = ek.Context(0)
ctx.spmv_setup(h.nodes, 0, L.rowptr, L.col, L.val)
G = h.kl_graph()
ctx.kl_graph_setup(G)
ctx.kl_nets_setup(*h.pins())
lam, v, st = ctx.lanczos_fiedler()
med, bits = ek.median_split(v)
ctx.kl_set_partition_bits(bits)
log, res = ctx.kl_run()
deg = np.diff(G.rowptr)
tot = deg[log["node_left"]] + deg[log["node_right"]]
print("swaps", len(tot), "mean tot", tot.mean(), "max", tot.max())
for cap in (8, 16, 24, 32, 48, 64, 88):
    print(f"tot > {cap}: {np.mean(tot > cap) * 100:.1f} %")
