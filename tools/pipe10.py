"""Lab (not shipped): the phases of the -EIG file path on configs[4]'s 10x
graph (2.02M nodes) on one GPU, warm context.  usage: python tools/pipe10.py [mult seed]"""
import importlib.util
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("eigkl_amd", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
ek = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ek)
mult, seed = (float(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (10.0, 10)
d = tempfile.mkdtemp(prefix="ekp10_")
p = os.path.join(d, "h.hgr")
ek.Hypergraph.generate(mult, seed).write(p)
c = ek.Context(0)
keys = ("t_read", "t_laplacian", "t_lanczos", "t_split", "t_kl_graph_wait", "t_kl_setup", "t_kl", "t_write", "t_total")
for i in range(4):
    t = time.time()
    r, _ = c.solve_file(p, eig=1, out_dir=d)
    w = time.time() - t
    print(f"wall {w * 1e3:.1f} ms | " + " ".join(f"{k[2:]} {r[k] * 1e3:.1f}" for k in keys) +
          f" | swaps {r['kl']['iterations']} matvecs {r['lanczos']['matvecs']}", flush=True)
c.close()
