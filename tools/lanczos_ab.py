#!/usr/bin/env python3
"""Lab (not shipped): resident Lanczos solves on the synthetic under
environment variants, one line per (size, variant): solve time, matvecs and
the first bits of lambda (variants that claim the same bits must agree).
usage: python tools/lanczos_ab.py MULT[,MULT..] VAR=VAL[,VAR=VAL..] [...]
       (each further argument is one variant; "-" = no overrides)"""
import importlib.util
import os
import struct
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("ek", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
ek = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ek)
mults = [float(m) for m in sys.argv[1].split(",")]
variants = sys.argv[2:] or ["-"]
ctx = ek.Context(0)
for mult in mults:
    h = ek.Hypergraph.generate(mult, {1.0: 1, 2.0: 2, 10.0: 10}.get(mult, 3))
    ctx.spmv_setup_pins(h)
    for rep in range(int(os.environ.get("REPS", "2"))):
        for var in variants:
            env = dict(kv.split("=", 1) for kv in var.split(",")) if var != "-" else {}
            saved = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            ctx.lanczos_fiedler()  # warm
            lam, v, st = ctx.lanczos_fiedler()
            for k, o in saved.items():
                if o is None:
                    os.environ.pop(k)
                else:
                    os.environ[k] = o
            bits = struct.pack("<d", lam).hex()
            print(f"{mult:5.1f}x {var:28s} Lanczos {st['total_ms']:9.3f} ms  {st['matvecs']} matvecs "
                  f"({1000 * st['total_ms'] / st['matvecs']:.2f} us/matvec, u32 {st.get('update32_steps')}/"
                  f"{st.get('update32_fallbacks')})  lambda {lam:.6e} "
                  f"[{bits}] v[0:2] {v[0]:.17g} {v[1]:.17g}", flush=True)
ctx.close()
