"""Lab (not shipped): wall time of the GPU Lanczos solve with and without the
per-SpMV timing events, to see how much of a step is host launch overhead."""
import importlib.util
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("eigkl_amd", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
ek = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ek)
h = ek.Hypergraph.generate(float(sys.argv[1]) if len(sys.argv) > 1 else 1.0, 1)
L = h.laplacian()
ctx = ek.Context(0)
ctx.spmv_setup(h.nodes, 0, L.rowptr, L.col, L.val)
for ts in (False, True, False, True):
    t0 = time.time()
    lam, v, st = ctx.lanczos_fiedler(time_spmv=ts)
    wall = time.time() - t0
    print(f"time_spmv={ts}: wall {wall*1e3:.2f} ms, total_ms {st['total_ms']:.2f}, matvecs {st['matvecs']}, "
          f"restarts {st['restarts']}, us/step {wall*1e6/st['matvecs']:.1f}", flush=True)
ctx.close()
