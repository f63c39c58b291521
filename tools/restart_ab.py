#!/usr/bin/env python3
"""Lab (not shipped): Lanczos matvecs / restarts / solve time per restart
policy on the shipped circuits and the connected synthetics.
usage: python tools/restart_ab.py VAR=VAL[,VAR=VAL..] ...   ("-" = no overrides)"""
import importlib.util
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("eigkl_amd", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
ek = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ek)
variants = sys.argv[1:] or ["-"]
ctx = ek.Context(0)
cases = [(c, ek.Hypergraph.read(os.path.join(REPO, "tests", "golden", "circuit", f"{c}.hgr")))
         for c in ("ibm01", "industry2", "ibm10")]
cases += [("syn1_lcc", ek.Hypergraph.generate(1.0, 1).largest_component()[0]),
          ("syn115_lcc", ek.Hypergraph.generate(1.15, 1).largest_component()[0]),
          ("syn2_lcc", ek.Hypergraph.generate(2.0, 2).largest_component()[0])]
for name, h in cases:
    ctx.spmv_setup_pins(h)
    for var in variants:
        env = dict(kv.split("=", 1) for kv in var.split(",")) if var != "-" else {}
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        ctx.lanczos_fiedler()
        lam, v, st = ctx.lanczos_fiedler()
        for k, o in saved.items():
            if o is None:
                os.environ.pop(k)
            else:
                os.environ[k] = o
        print(f"{name:11s} n={h.nodes:7d} {var:22s} matvecs {st['matvecs']:5d} restarts {st['restarts']:3d} "
              f"{st['total_ms']:8.2f} ms  lambda {lam:.12e} residual {st['residual']:.2e}", flush=True)
ctx.close()
