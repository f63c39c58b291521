"""Lab (not shipped): EK_TRACE phase marks of a few in-process solves of the
1x synthetic written to a .hgr (bench.py's step).  usage:
EK_TRACE=1 python tools/trace_solve.py [reps]"""
import importlib.util
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("eigkl_amd", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
ek = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ek)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
w = tempfile.mkdtemp()
p = os.path.join(w, "syn1.hgr")
ek.Hypergraph.generate(1.0, 1).write(p)
ctx = ek.Context(0)
for i in range(reps):
    print(f"=== step {i}", file=sys.stderr, flush=True)
    t = time.perf_counter()
    r, _ = ctx.solve_file(p, eig=1, out_dir=w, log_cap=110000)
    print(f"=== python wall {1e3 * (time.perf_counter() - t):.2f} ms", file=sys.stderr, flush=True)
    print("=== " + " ".join(f"{k} {1e3 * r[k]:.2f}" for k in r if k.startswith("t_")), file=sys.stderr, flush=True)
ctx.close()
