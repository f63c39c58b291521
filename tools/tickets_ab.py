"""Lab (not shipped): the partially reorthogonalised Lanczos solve of the
headline LCC with and without the in-launch jobs' tickets (EK_PRO_TICKETS),
alternating processes; median of the solve's device time over 6 solves each.
usage: python tools/tickets_ab.py"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r"""
import sys, numpy as np; sys.path.insert(0, %r); from conftest import load_package
ek = load_package(); h, _ = ek.Hypergraph.generate(1.15, 1).largest_component(); c = ek.Context(0); c.spmv_setup_pins(h)
t = []
for _ in range(7):
    lam, v, st = c.lanczos_fiedler(); t.append(st['total_ms'])
print(sys.argv[1], 'lanczos ms', ' '.join('%%.2f' %% x for x in t[1:]), 'median %%.3f' %% float(np.median(t[1:])),
      'matvecs', st['matvecs'], 'lambda %%.15g' %% lam, flush=True)
""" % os.path.join(REPO, "tests")
for rep in range(2):
    for v in ("1", "0"):
        subprocess.run([sys.executable, "-c", CODE, f"EK_PRO_TICKETS={v}"], check=True, timeout=300,
                       env=dict(os.environ, EK_PRO_TICKETS=v))
