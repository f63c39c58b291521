"""Lab (not shipped): A/B of Lanczos kernel builds.  Runs the GPU Lanczos
solve on the 1x seed-1 synthetic (and its largest connected component) a few
times with the library named by EK_LIB_PATH (default: the in-tree build) and
prints the device time per solve, the matvec count and a hash of the result
bits, so builds that must be bit-identical can be compared run to run.
Usage: EK_LIB_PATH=... python tools/lanczos_ab.py [reps] [check_every]"""
import hashlib
import importlib.util
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("eigkl_amd", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
ek = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ek)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
check_every = int(sys.argv[2]) if len(sys.argv) > 2 else 8
print(f"lib {ek.LIB_PATH}", flush=True)
h1 = ek.Hypergraph.generate(1.0, 1)
hl, _ = h1.largest_component()
ctx = ek.Context(0)
for name, h in (("syn1", h1), ("syn1_lcc", hl)):
    L = h.laplacian()
    ctx.spmv_setup(h.nodes, 0, L.rowptr, L.col, L.val)
    ms = []
    for i in range(reps):
        t0 = time.time()
        lam, v, st = ctx.lanczos_fiedler(check_every=check_every)
        ms.append((time.time() - t0) * 1e3)
    dig = hashlib.md5(v.tobytes()).hexdigest()[:12]
    print(f"{name}: wall ms {' '.join(f'{x:.2f}' for x in ms)}; device {st['total_ms']:.2f} ms, "
          f"{st['matvecs']} matvecs, {st['restarts']} restarts, us/step {1e3 * min(ms[1:]) / st['matvecs']:.1f}, "
          f"lambda {lam.hex()}, v md5 {dig}", flush=True)
ctx.close()
