#!/usr/bin/env python3
"""A/B of where the partial reorthogonalisation's decision runs (resident
inputs, one GPU): the k_pro launch (EK_PRO_INLAUNCH=0) against the decider
workgroup inside the projection launch (EK_PRO_INLAUNCH=1, the default).
Modes alternate per round so box drift hits both; median Lanczos time per
mode, matvecs, projected steps, and whether the two give the same bits.

usage: python tools/proi_ab.py [ROUNDS] [workload ...]   (lcc1.15 ibm10 ibm01 lcc2 syn0.25)
EK_AB_VAR=NAME toggles that variable instead (0 / 1), e.g. EK_PRO_MERGE."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import circuit_path, load_package  # noqa: E402


def graph(ek, w):
    if w.startswith("lcc"):
        return ek.Hypergraph.generate(float(w[3:]), 1).largest_component()[0]
    if w.startswith("syn"):
        return ek.Hypergraph.generate(float(w[3:]), 3)
    return ek.Hypergraph.read(circuit_path(w))


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    var = os.environ.get("EK_AB_VAR", "EK_PRO_INLAUNCH")
    work = sys.argv[2:] or ["lcc1.15", "ibm10", "ibm01"]
    ek = load_package()
    c = ek.Context(0)
    for w in work:
        h = graph(ek, w)
        c.spmv_setup_pins(h)
        ts = {"0": [], "1": []}
        out = {}
        for r in range(rounds + 1):
            for mode in ("0", "1"):
                os.environ[var] = mode
                t = time.time()
                lam, v, st = c.lanczos_fiedler()
                dt = time.time() - t
                if r > 0:  # (round 0: first launches, graph captures)
                    ts[mode].append(dt)
                out[mode] = (lam, v, st)
        same = all(np.array_equal(np.asarray(out["0"][k]).view(np.uint64), np.asarray(out["1"][k]).view(np.uint64))
                   for k in (0, 1))
        st0, st1 = out["0"][2], out["1"][2]
        print(f"{w}: n={h.nodes} {var}=0 {np.median(ts['0']) * 1e3:.2f} ms | =1 "
              f"{np.median(ts['1']) * 1e3:.2f} ms | matvecs {st0['matvecs']}/{st1['matvecs']} projected "
              f"{st0['projected_steps']}/{st1['projected_steps']} | same bits {same} | "
              f"min {min(ts['0']) * 1e3:.2f} / {min(ts['1']) * 1e3:.2f} ms", flush=True)
    os.environ.pop(var, None)
    c.close()


if __name__ == "__main__":
    main()
