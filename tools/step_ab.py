#!/usr/bin/env python3
"""Lab: the bench's warm step (ek_solve_file on the headline .hgr, context
kept) through two builds of the library (EK_LIB_PATH) or two settings of one
variable (VAR=VALUE), one child process per side, alternating: median step
wall and the phases (Lanczos, KL adjacency wait, KL).
usage: python tools/step_ab.py SIDE_A SIDE_B [rounds]"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import os, sys, tempfile, time
import numpy as np
sys.path.insert(0, os.path.join(%r, "tests"))
from conftest import load_package
ek = load_package()
d = tempfile.mkdtemp(prefix="ekstep_")
p = os.path.join(d, "h.hgr")
ek.Hypergraph.generate(1.15, 1).largest_component()[0].write(p)
c = ek.Context(0)
w, ph = [], []
for i in range(14):
    t = time.time()
    r, _ = c.solve_file(p, eig=1, out_dir=d)
    w.append(time.time() - t)
    ph.append((r["t_lanczos"], r["t_kl_graph_wait"], r["t_kl"], r["kl"]["loop_ms"] / r["kl"]["iterations"]))
ph = np.array(ph[2:])
print(f"  step median {np.median(w[2:]) * 1e3:.2f} ms mean {np.mean(w[2:]) * 1e3:.2f} | lanczos {np.median(ph[:, 0]) * 1e3:.2f} "
      f"graph_wait {np.median(ph[:, 1]) * 1e3:.2f} kl {np.median(ph[:, 2]) * 1e3:.2f} ms, {np.median(ph[:, 3]) * 1e3:.3f} us/swap",
      flush=True)
c.close()
""" % REPO


def main():
    sides = sys.argv[1:3]
    for _ in range(int(sys.argv[3]) if len(sys.argv) > 3 else 3):
        for side in sides:
            print(side, flush=True)
            if "=" in side and not side.endswith(".so"):
                k, v = side.split("=", 1)
                env = dict(os.environ, **{k: v})
            else:
                env = dict(os.environ, EK_LIB_PATH=os.path.abspath(side))
            subprocess.run([sys.executable, "-c", CHILD], check=True, timeout=600, env=env)


if __name__ == "__main__":
    main()
