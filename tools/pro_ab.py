#!/usr/bin/env python3
"""A/B of the Lanczos reorthogonalisation rule on one GPU (resident inputs):
reorth=1 (full Gram-Schmidt every step) against reorth=3 (partial, k_pro),
median solve time over REPS runs per workload, matvecs and projected steps.

usage: python tools/pro_ab.py [REPS] [workload ...]   (workloads: lcc1.15 ibm10 ibm01 lcc2 syn10)"""
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
        return ek.Hypergraph.generate(float(w[3:]), 10)
    return ek.Hypergraph.read(circuit_path(w))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    work = sys.argv[2:] or ["lcc1.15", "ibm10", "ibm01", "lcc2"]
    ek = load_package()
    c = ek.Context(0)
    for w in work:
        h = graph(ek, w)
        c.spmv_setup_pins(h)
        res = {}
        for mode in (1, 3):
            ts, st = [], None
            for _ in range(reps + 1):
                t = time.time()
                lam, v, st = c.lanczos_fiedler(reorth=mode)
                ts.append(time.time() - t)
            res[mode] = (float(np.median(ts[1:])) * 1e3, lam, st)
        (tf, lf, sf), (tp, lp, sp) = res[1], res[3]
        print(f"{w}: n={h.nodes} full {tf:.2f} ms ({sf['matvecs']} mv) | partial {tp:.2f} ms ({sp['matvecs']} mv, "
              f"{sp['projected_steps']} projected, {sp['update32_fallbacks']} fp64 updates) | d_lambda "
              f"{lp - lf:.2e} | speedup {tf / tp:.2f}x", flush=True)
    c.close()


if __name__ == "__main__":
    main()
