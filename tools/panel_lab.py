#!/usr/bin/env python3
"""Lab: the column-panel SpMV against the CSR-adaptive one (EK_SPMV_PANEL=0/1)
on the synthetic at several sizes: back-to-back launches (ek_spmv_bench) and
inside a resident Lanczos solve (every 4th SpMV event-timed).
usage: python tools/panel_lab.py [mult ...]"""
import importlib.util
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("ek", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
ek = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ek)
mults = [float(a) for a in sys.argv[1:]] or [1.0, 2.0, 10.0]
ctx = ek.Context(0)
for mult in mults:
    h = ek.Hypergraph.generate(mult, {1.0: 1, 2.0: 2, 10.0: 10}.get(mult, 3))
    for panel in ("0", "1"):
        os.environ["EK_SPMV_PANEL"] = panel
        ctx.spmv_setup_pins(h)
        b = ctx.spmv_bytes(fused=False)
        us = ctx.spmv_bench(100, fused=False)
        usf = ctx.spmv_bench(100, fused=True)
        ctx.lanczos_fiedler()  # warm (first-solve allocations)
        lam, _, st = ctx.lanczos_fiedler(time_spmv=True)
        us_in = 1e3 * st["spmv_ms"] / max(1, st["spmv_timed"])
        print(f"{mult:5.1f}x panel={panel}: b2b {us:8.2f} us ({b / us / 1e3 / 8000:.3f} of 8 TB/s), fused {usf:8.2f} us; "
              f"in-solve {us_in:8.2f} us; Lanczos {st['total_ms']:8.2f} ms, {st['matvecs']} matvecs, lambda {lam:.3e}",
              flush=True)
ctx.close()
