#!/usr/bin/env python3
"""Lab: Lanczos matvecs and time against ncv on the 10x synthetic (disconnected) and the 5x LCC."""
import importlib.util, os, sys
REPO = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
spec = importlib.util.spec_from_file_location("eigkl_amd", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
ek = importlib.util.module_from_spec(spec); spec.loader.exec_module(ek)
ctx = ek.Context(0)
for name, h in (("syn10", ek.Hypergraph.generate(10.0, 10)), ("syn5lcc", ek.Hypergraph.generate(5.0, 5).largest_component()[0])):
    ctx.spmv_setup_pins(h)
    for ncv in (80, 100, 120):
        ctx.lanczos_fiedler(ncv=ncv)
        best = None
        for _ in range(2):
            lam, v, st = ctx.lanczos_fiedler(ncv=ncv)
            best = st if best is None or st["total_ms"] < best["total_ms"] else best
        print(f"{name} n={v.size} ncv {ncv} matvecs {best['matvecs']} restarts {best['restarts']} {best['total_ms']:.2f} ms lambda {lam:.6e}", flush=True)
