"""Lab (not shipped): the median split of the GPU Fiedler vector on the 1x and 2x synthetics."""
import importlib.util, os
import numpy as np
REPO = os.environ.get("GRAFT_REPO_ROOT", ".")
spec = importlib.util.spec_from_file_location("eigkl_amd", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
ek = importlib.util.module_from_spec(spec); spec.loader.exec_module(ek)
import sys
for mult, seed in ((float(sys.argv[1]), int(sys.argv[2])),) if len(sys.argv) > 2 else ((2.0, 2),):
    h = ek.Hypergraph.generate(mult, seed); L = h.laplacian(); ctx = ek.Context(0)
    ctx.spmv_setup(h.nodes, 0, L.rowptr, L.col, L.val)
    lam, v, st = ctx.lanczos_fiedler(); med, bits = ek.median_split(v)
    vals, cnt = np.unique(v, return_counts=True)
    print(mult, st, "n", h.nodes, "lambda", lam, "median", med, "n1", int(bits.sum()), "distinct", len(vals), "top count", cnt.max(), "at", vals[cnt.argmax()])
    ctx.close()
