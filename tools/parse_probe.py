#!/usr/bin/env python3
"""Lab: ek_hgr_read time on the headline workload's .hgr (EK_TRACE=1: slurp / lines / parse split)."""
import sys, time, os, tempfile
sys.path.insert(0, "tests")
from conftest import load_package
ek = load_package()
h = ek.Hypergraph.generate(1.15, 1).largest_component()[0]
d = tempfile.mkdtemp()
p = os.path.join(d, "lcc.hgr")
h.write(p) if hasattr(h, "write") else None
print(os.path.getsize(p) if os.path.exists(p) else "no write")
ts = []
for _ in range(15):
    t = time.perf_counter(); g = ek.Hypergraph.read(p); ts.append(time.perf_counter() - t)
ts.sort(); print("read ms: min %.2f med %.2f" % (ts[0]*1e3, ts[len(ts)//2]*1e3))
