#!/usr/bin/env python3
"""ORACLE — test/baseline infrastructure only: the CPU baseline leg of bench.py.

Runs the oracle restatement of the reference path (oracle/eko_eig.cpp: fp64
Lanczos for the Fiedler pair, the cEIG.cpp:194-207 solve; oracle/eko_kl.cpp:
cKL's KL() loop, cKL.cpp:288-406) on this host's cores, pinned to the first
T CPUs of the process's affinity mask (cKL forces its thread count to every
core, cKL.cpp:451-452, so the count is set through the mask, not the
environment).  Started by bench.py as a child process that never touches the
GPU; prints one JSON line.

  parse      .hgr read + cKL adjacency (eko_read, cKL.cpp:84-149)
  lanczos    Laplacian + Lanczos to convergence (eko_lanczos)
  kl         KL() from the GPU run's split (remain[] lists in node order, the
             -EIG branch cKL.cpp:155-174), compared swap by swap with the GPU
             swap log and net cuts bench.py saved

The Lanczos runs to convergence, capped at MAX_MATVEC matvecs (bench.py
passes 3x the GPU solve's count: on the disconnected synthetic the null space
is huge and the thick-restart restatement can take far longer than the GPU's
implicit-restart solve to settle on one null vector; a capped run is reported
as such, never extrapolated).

usage: cpu_baseline.py HGR SPLIT_NPZ THREADS [MAX_MATVEC]
"""
import json
import os
import sys
import time

import numpy as np


def main():
    hgr, split_npz, threads = sys.argv[1], sys.argv[2], int(sys.argv[3])
    max_matvec = int(sys.argv[4]) if len(sys.argv) > 4 else 0

    def note(msg):
        print(f"[cpu_baseline {threads}t] {msg}", file=sys.stderr, flush=True)

    cpus = sorted(os.sched_getaffinity(0))
    threads = max(1, min(threads, len(cpus)))
    os.sched_setaffinity(0, cpus[:threads])  # before libgomp starts its pool
    os.environ["EKO_THREADS"] = str(threads)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import oracle

    oracle.set_threads(threads)
    t0 = time.time()
    g = oracle.Graph.read(hgr)
    t_parse = time.time() - t0
    note(f"parsed in {t_parse:.2f} s; Lanczos (cap {max_matvec or 'none'} matvecs)")
    t1 = time.time()
    lam, _, st = g.lanczos(deflate=True, max_matvec=max_matvec)
    t_lanczos = time.time() - t1
    note(f"Lanczos {t_lanczos:.2f} s, {st['matvecs']} matvecs, converged {st['converged']}; KL")
    z = np.load(split_npz)
    bits, glog = z["bits"], z["log"]
    idx = np.arange(len(bits), dtype=np.int32)
    t2 = time.time()
    olog, ores = g.kl(idx[bits == 0], idx[bits == 1], cap=None)
    t_kl = time.time() - t2
    note(f"KL {t_kl:.2f} s, {ores['iterations']} swaps")
    n = min(len(olog), len(glog))
    fields_equal = len(olog) == len(glog) and all(
        np.array_equal(olog[f], glog[f]) for f in ("iter", "node_left", "node_right")) and all(
        np.array_equal(olog[f].view(np.uint32), glog[f].view(np.uint32)) for f in ("max_gain", "min_gain", "gain", "cut"))
    first_diff = None
    if not fields_equal:
        for i in range(n):
            if olog[i].tobytes() != glog[i].tobytes():
                first_diff = i
                break
    out = {"threads": threads, "cpus": cpus[:threads], "parse_s": round(t_parse, 3), "lanczos_s": round(t_lanczos, 3),
           "lanczos_matvecs": st["matvecs"], "lanczos_converged": bool(st["converged"]), "lambda1": lam,
           "kl_s": round(t_kl, 3), "kl_iterations": int(ores["iterations"]),
           "total_s": round(t_parse + t_lanczos + t_kl, 3),
           "swap_log_match": bool(fields_equal), "first_mismatch": first_diff,
           "net_cut_best": int(ores["net_cut_best"]), "net_cut_final": int(ores["net_cut_final"]),
           "best_iter": int(ores["best_iter"])}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
