#!/usr/bin/env python3
"""Lab: EK_TRACE phase marks and the Python-side wall of ek_solve_file on the
headline workload's .hgr (5 calls), to place what lies outside t_total.
usage: EK_TRACE=1 python tools/solve_file_trace.py"""
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import load_package  # noqa: E402

ek = load_package()
h = ek.Hypergraph.generate(1.15, 1).largest_component()[0]
d = tempfile.mkdtemp()
p = os.path.join(d, "lcc.hgr")
h.write(p)
c = ek.Context(0)
for i in range(5):
    t = time.perf_counter()
    r, _ = c.solve_file(p, eig=1, out_dir=d)
    w = time.perf_counter() - t
    print(f"call {i}: wall {w * 1e3:.2f} ms, t_total {r['t_total'] * 1e3:.2f} ms, outside {(w - r['t_total']) * 1e3:.2f} ms",
          file=sys.stderr, flush=True)
c.close()
