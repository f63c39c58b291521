#!/usr/bin/env python3
"""Lab: resident Lanczos solves in a loop (for rocprofv3 kernel traces).
usage: python tools/lanczos_loop.py [workload] [reps]   (lcc1.15 | ibm10 | ibm01 | syn0.25)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import circuit_path, load_package  # noqa: E402

w = sys.argv[1] if len(sys.argv) > 1 else "lcc1.15"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
ek = load_package()
c = ek.Context(0)
if w.startswith("lcc"):
    h = ek.Hypergraph.generate(float(w[3:]), 1).largest_component()[0]
elif w.startswith("syn"):
    h = ek.Hypergraph.generate(float(w[3:]), 3)
else:
    h = ek.Hypergraph.read(circuit_path(w))
c.spmv_setup_pins(h)
for _ in range(reps):
    lam, v, st = c.lanczos_fiedler()
print(w, lam, st["matvecs"], st["projected_steps"], flush=True)
c.close()
