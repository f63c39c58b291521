"""Lab (not shipped): the device Laplacian build (ek_spmv_setup_pins) at the
1x and 10x synthetic sizes, repeated, for rocprofv3 --kernel-trace --stats."""
import importlib.util
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("eigkl_amd", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
ek = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ek)
ctx = ek.Context(0)
for mult in (1.0, 10.0):
    h = ek.Hypergraph.generate(mult, int(mult))
    for rep in range(4):
        t = time.time()
        dev = ctx.spmv_setup_pins(h)
        print(f"{mult}x device={dev} {1e3 * (time.time() - t):.2f} ms", flush=True)
