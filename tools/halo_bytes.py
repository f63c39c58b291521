#!/usr/bin/env python3
"""Bytes a rank receives per sharded Lanczos step: the all-gather of whole
slots (ctx.cpp exchange_f) against the halo exchange (halo_build: only the
rows of other ranks its columns read, + one ||f||^2 partial per peer), from
the nnz-balanced shard map and the Laplacian rows (host only, no GPU).

usage: python tools/halo_bytes.py [MULT[lcc] SEED ...]   (default: 10 10, 1.15lcc 1)
"""
import importlib.util
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    spec = importlib.util.spec_from_file_location("eigkl_amd", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
    ek = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ek)
    args = sys.argv[1:] or ["10", "10", "1.15lcc", "1"]
    for a, sd in zip(args[0::2], args[1::2]):
        lcc = a.endswith("lcc")
        h = ek.Hypergraph.generate(float(a[:-3] if lcc else a), int(sd))
        if lcc:
            h, _ = h.largest_component()
        for R in (2, 4, 8):
            off = ek.shard_map(h, R)
            ldv = -(-int(np.diff(off).max()) // 1024) * 1024
            S = ldv + 64
            recv, own_frac = [], []
            for r in range(R):
                rows = h.laplacian_rows(int(off[r]), int(off[r + 1]))
                c = rows.col
                mine = (c >= off[r]) & (c < off[r + 1])
                own_frac.append(float(mine.mean()))
                recv.append(len(np.unique(c[~mine])) + (R - 1))
            full = (R - 1) * S
            tot_h, tot_f = sum(recv), R * full
            print(json.dumps({"workload": a, "ranks": R, "nodes": h.nodes, "full_recv_doubles_per_rank": full,
                              "halo_recv_doubles_max_rank": max(recv), "halo_recv_doubles_mean": round(tot_h / R),
                              "halo_over_full": round(tot_h / tot_f, 3),
                              "halo_taken": tot_h <= 0.75 * tot_f,
                              "MB_per_step_full_per_rank": round(8 * full / 1e6, 2),
                              "MB_per_step_halo_max_rank": round(8 * max(recv) / 1e6, 2),
                              "own_fraction_mean": round(float(np.mean(own_frac)), 3)}), flush=True)


if __name__ == "__main__":
    main()
