#!/usr/bin/env python3
"""Lab (not shipped): Lanczos matvecs and solve time against the basis size
(ncv) and the restart floor, on the shipped circuits and the connected
synthetics.  usage: python tools/ncv_ab.py NCV[:KEEP],...   (KEEP -1 = ncv/5)"""
import importlib.util
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("eigkl_amd", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
ek = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ek)
variants = [(int(v.split(":")[0]), int(v.split(":")[1]) if ":" in v else -1) for v in sys.argv[1].split(",")]
ctx = ek.Context(0)
cases = [(c, ek.Hypergraph.read(os.path.join(REPO, "tests", "golden", "circuit", f"{c}.hgr")))
         for c in ("ibm01", "industry2", "ibm10")]
cases += [("syn1_lcc", ek.Hypergraph.generate(1.0, 1).largest_component()[0]),
          ("syn115_lcc", ek.Hypergraph.generate(1.15, 1).largest_component()[0]),
          ("syn2_lcc", ek.Hypergraph.generate(2.0, 2).largest_component()[0])]
for name, h in cases:
    ctx.spmv_setup_pins(h)
    for ncv, keep in variants:
        ctx.lanczos_fiedler(ncv=ncv, keep_min=keep)
        best = None
        for _ in range(2):
            lam, v, st = ctx.lanczos_fiedler(ncv=ncv, keep_min=keep)
            best = st if best is None or st["total_ms"] < best["total_ms"] else best
        print(f"{name:10s} n={v.size:8d} ncv {ncv:4d} keep {keep:3d}  matvecs {best['matvecs']:5d} restarts "
              f"{best['restarts']:3d}  {best['total_ms']:8.2f} ms  lambda {lam:.12e}", flush=True)
ctx.close()
