"""Lab (not shipped): the headline LCC's Lanczos solve under two settings of
one environment switch (EK_AB_10X=1: the 10x synthetic instead), alternating processes; per process the median device
time of 6 solves after a warm one.  usage: python tools/env_ab.py VAR A B [reps]"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r"""
import sys, numpy as np; sys.path.insert(0, %r); from conftest import load_package
import os
ek = load_package()
h = ek.Hypergraph.generate(10.0, 10) if os.environ.get("EK_AB_10X") else ek.Hypergraph.generate(1.15, 1).largest_component()[0]
c = ek.Context(0); c.spmv_setup_pins(h)
t = []
for _ in range(7):
    lam, v, st = c.lanczos_fiedler(); t.append(st['total_ms'])
print(sys.argv[1], 'lanczos ms median %%.3f' %% float(np.median(t[1:])), 'min %%.3f' %% min(t[1:]),
      'matvecs', st['matvecs'], 'lambda %%.15g' %% lam, flush=True)
""" % os.path.join(REPO, "tests")
var, a, b = sys.argv[1], sys.argv[2], sys.argv[3]
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
for rep in range(reps):
    for v in (a, b):
        subprocess.run([sys.executable, "-c", CODE, f"{var}={v}"], check=True, timeout=300, env=dict(os.environ, **{var: v}))
