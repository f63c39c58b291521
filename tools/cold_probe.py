#!/usr/bin/env python3
"""Fresh-process wall of the drop-in tool, split by EK_COLD_TRACE stamps.

Runs `gKL2 <hgr> -EIG --quiet` REPS times from a fresh process each and
reports, per start-up event, the median offset (s) from the launch
(time.time() before the spawn; the library stamps CLOCK_REALTIME):
lib_loaded (exec + dynamic loading + static init), main, read_done,
hip_first_call / hip_device_count / hip_props / hip_set_device / hip_stream0 /
hip_streams (ek_init on its thread),
laplacian_start/done, lanczos_done, kl_start/done, solve_done,
ctx_destroy_start/done, atexit, and `exit` (the child reaped).

usage: python tools/cold_probe.py HGR [REPS] [extra env K=V ...]
"""
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def probe(hgr, reps=5, env_extra=None, cwd=None):
    # EK_COLD_BUILD: another build directory (an A/B library beside its own gKL2)
    tool = os.path.join(REPO, "eig-kl-algorithm_amd", os.environ.get("EK_COLD_BUILD", "build"), "bin", "gKL2")
    env = dict(os.environ, EK_COLD_TRACE="1", **(env_extra or {}))
    cwd = cwd or tempfile.mkdtemp(prefix="ekcold_")
    runs = []
    for _ in range(reps):
        t0 = time.time()
        r = subprocess.run([tool, hgr, "-EIG", "--quiet"], cwd=cwd, env=env, capture_output=True, text=True,
                           timeout=300)
        t1 = time.time()
        if r.returncode != 0:
            return {"error": f"rc {r.returncode}: {r.stderr[-300:]}"}
        ev = {}
        for ln in r.stderr.splitlines():
            if ln.startswith("[cold] "):
                _, name, t = ln.split()
                ev.setdefault(name, float(t) - t0)
        ev["exit"] = t1 - t0
        runs.append(ev)
    names = [k for k in runs[0] if all(k in x for x in runs)]
    med = {k: round(float(np.median([x[k] for x in runs])), 4) for k in names}
    return dict(sorted(med.items(), key=lambda kv: kv[1]))


if __name__ == "__main__":
    hgr = os.path.abspath(sys.argv[1])
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    extra = dict(a.split("=", 1) for a in sys.argv[3:])
    print(json.dumps(probe(hgr, reps, extra)))
