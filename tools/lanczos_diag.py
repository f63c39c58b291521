#!/usr/bin/env python3
"""Where a resident Lanczos solve's wall time goes (lab): the default solve,
the same with check_every=0 (whole cycles enqueued at once: no mid-cycle host
checks between chunks) and with graphs off, each as ms per matvec, plus the
driver's EK_LANCZOS_TRACE summary (cycle vs restart host time) on stderr.
usage: python tools/lanczos_diag.py [lcc1.15|ibm10|...] [reps]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import load_package  # noqa: E402
from pro_ab import graph  # noqa: E402


def main():
    w = sys.argv[1] if len(sys.argv) > 1 else "lcc1.15"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    ek = load_package()
    h = graph(ek, w)
    c = ek.Context(0)
    c.spmv_setup_pins(h)
    for name, kw in [("default", {}), ("check_every=0", dict(check_every=0)), ("full reorth", dict(reorth=1)),
                     ("full, check_every=0", dict(reorth=1, check_every=0))]:
        ts = []
        for _ in range(reps + 1):
            t = time.time()
            lam, v, st = c.lanczos_fiedler(**kw)
            ts.append(time.time() - t)
        ms = float(np.median(ts[1:])) * 1e3
        print(f"{w} {name}: {ms:.2f} ms, {st['matvecs']} matvecs, {1e3 * ms / st['matvecs']:.1f} us/matvec, "
              f"{st['restarts']} restarts, projected {st['projected_steps']}", flush=True)
    os.environ["EK_LANCZOS_TRACE"] = "1"
    c.lanczos_fiedler()
    c.close()


if __name__ == "__main__":
    main()
