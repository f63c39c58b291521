"""Lab (not shipped): host-side wall of each call in one bench solve
(Lanczos, median split, partition upload, KL run) at ibm18 shape."""
import importlib.util
import os
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("eigkl_amd", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
ek = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ek)
h = ek.Hypergraph.generate(1.0, 1)
L = h.laplacian()
n = h.nodes
ctx = ek.Context(0)
ctx.spmv_setup(n, 0, L.rowptr, L.col, L.val)
ctx.kl_graph_setup(h.kl_graph())
ctx.kl_nets_setup(*h.pins())
for rep in range(3):
    t = [time.time()]
    lam, v, st = ctx.lanczos_fiedler()
    t.append(time.time())
    med, bits = ek.median_split(v)
    t.append(time.time())
    idx = np.arange(n, dtype=np.int32)
    o0, o1 = idx[bits == 0], idx[bits == 1]
    t.append(time.time())
    ctx.kl_set_partition(o0, o1)
    t.append(time.time())
    _, res = ctx.kl_run(cap=0)
    t.append(time.time())
    d = np.diff(t) * 1e3
    print(f"lanczos {d[0]:.2f}  median {d[1]:.2f}  idx {d[2]:.2f}  set_partition {d[3]:.2f}  kl_run {d[4]:.2f} "
          f"(loop {res['loop_ms']:.2f}, total {res['total_ms']:.2f})  sum {d.sum():.2f} ms", flush=True)
ctx.close()
