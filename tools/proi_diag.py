#!/usr/bin/env python3
"""Lab: determinism of the in-launch PRO decision.  One process per setting
(graphs / in-launch on or off), each running the Lanczos solve 3 times on
one workload; prints which runs give identical bits.

usage: python tools/proi_diag.py [workload]   (ibm01 | syn0.25)"""
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W = sys.argv[1] if len(sys.argv) > 1 else "ibm01"
GEN = {"ibm01": "ek.Hypergraph.read(circuit_path('ibm01'))", "syn0.25": "ek.Hypergraph.generate(0.25, 3)"}[W]
CODE = (
    "import sys, numpy as np; sys.path.insert(0, %r); from conftest import load_package, circuit_path\n"
    "ek = load_package(); h = %s; c = ek.Context(0); c.spmv_setup_pins(h); out = []\n"
    "for _ in range(3):\n"
    "    lam, v, st = c.lanczos_fiedler(); out.append(np.concatenate([[lam, st['matvecs'], st['residual'], "
    "st['projected_steps']], v]))\n"
    "np.save(sys.argv[1], np.stack(out))"
) % (os.path.join(REPO, "tests"), GEN)

runs = {}
for name, env in [("inl_graph", {}), ("inl_graph_b", {}), ("inl_eager", {"EK_LANCZOS_GRAPH": "0"}),
                  ("kpro_eager", {"EK_PRO_INLAUNCH": "0", "EK_LANCZOS_GRAPH": "0"}),
                  ("kpro_graph", {"EK_PRO_INLAUNCH": "0"}),
                  ("kpro_apart", {"EK_PRO_INLAUNCH": "0", "EK_LANCZOS_GRAPH": "0", "EK_PRO_APART": "1"})]:
    path = f"/tmp/proi_{name}.npy"
    e = dict(os.environ, EK_REORTH="3", **env)
    subprocess.run([sys.executable, "-c", CODE, path], check=True, timeout=120, env=e)
    runs[name] = np.load(path)
    x = runs[name]
    print(name, "lambda", [f"{r[0]:.15e}" for r in x], "mv", [int(r[1]) for r in x], "res",
          [f"{r[2]:.3e}" for r in x], "proj", [int(r[3]) for r in x], flush=True)
ref = runs["kpro_eager"][0].view(np.uint64)
for name, x in runs.items():
    print(name, "vs kpro_eager[0]:", [bool(np.array_equal(r.view(np.uint64), ref)) for r in x], flush=True)
