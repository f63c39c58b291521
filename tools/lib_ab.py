#!/usr/bin/env python3
"""Lab: the same resident Lanczos solves through two builds of the library
(EK_LIB_PATH), one child process per build: lambda, matvecs, projected steps,
median solve time and an md5 of the Fiedler vector's bits.

usage: python tools/lib_ab.py LIB_A LIB_B [workload ...]   (lcc1.15 ibm10 ibm01 syn0.25)
A side given as VAR=VALUE instead runs the built library with that variable
set (e.g. EK_PRO_MERGE=0 EK_PRO_MERGE=1); EK_AB_ROUNDS alternates the sides."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import hashlib, os, sys, time
import numpy as np
sys.path.insert(0, os.path.join(%r, "tests"))
from conftest import circuit_path, load_package
ek = load_package()
c = ek.Context(0)
for w in sys.argv[1:]:
    if w.startswith("lcc"):
        h = ek.Hypergraph.generate(float(w[3:]), 1).largest_component()[0]
    elif w.startswith("syn"):
        h = ek.Hypergraph.generate(float(w[3:]), 3)
    else:
        h = ek.Hypergraph.read(circuit_path(w))
    c.spmv_setup_pins(h)
    ts = []
    for r in range(6):
        t = time.time()
        lam, v, st = c.lanczos_fiedler()
        ts.append(time.time() - t)
    md5 = hashlib.md5(np.ascontiguousarray(v).tobytes()).hexdigest()[:12]
    print(f"  {w}: lambda {lam:.16e} matvecs {st['matvecs']} projected {st['projected_steps']} "
          f"median {np.median(ts[1:]) * 1e3:.2f} ms min {min(ts[1:]) * 1e3:.2f} ms v md5 {md5}", flush=True)
c.close()
""" % REPO


def main():
    sides, work = sys.argv[1:3], sys.argv[3:] or ["ibm01", "lcc1.15"]
    for _ in range(int(os.environ.get("EK_AB_ROUNDS", "1"))):
        for side in sides:
            print(side, flush=True)
            if "=" in side and not side.endswith(".so"):
                k, v = side.split("=", 1)
                env = dict(os.environ, **{k: v})
            else:
                env = dict(os.environ, EK_LIB_PATH=os.path.abspath(side))
            subprocess.run([sys.executable, "-c", CHILD] + work, check=True, timeout=600, env=env)


if __name__ == "__main__":
    main()
