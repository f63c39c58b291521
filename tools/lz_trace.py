#!/usr/bin/env python3
"""Lab: one resident Lanczos solve of a workload with EK_LANCZOS_TRACE=1
(restarts, kept vectors, and the restart's host / device time split on
stderr).  usage: python tools/lz_trace.py [MULT[lcc] SEED]  (default 1.15lcc 1)"""
import importlib.util
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("EK_LANCZOS_TRACE", "1")
spec = importlib.util.spec_from_file_location("eigkl_amd", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
ek = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ek)
a, sd = (sys.argv[1:3] + ["1.15lcc", "1"][len(sys.argv[1:3]):])[:2]
lcc = a.endswith("lcc")
h = ek.Hypergraph.generate(float(a[:-3] if lcc else a), int(sd))
if lcc:
    h, _ = h.largest_component()
c = ek.Context(0)
c.spmv_setup_pins(h)
for _ in range(2):
    lam, v, st = c.lanczos_fiedler()
    print({k: st[k] for k in ("matvecs", "restarts", "projected_steps", "total_ms")}, flush=True)
c.close()
