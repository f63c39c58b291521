#!/usr/bin/env python3
"""Sharded Lanczos step, full vs partial reorthogonalisation, on ONE GPU:
the forced 1-rank RCCL path (EK_COMM_FORCE=1: ncclAllGather / ncclAllReduce
issued exactly as with N ranks) against the single-context step.
Per workload and form: median of 3 resident solves (ms), matvecs, projected
steps, collectives, and ms per matvec.

usage: python tools/mr_pro_lab.py [MULT[lcc] SEED ...]   (default: 1.15lcc 1, 10 10)
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
    args = sys.argv[1:] or ["1.15lcc", "1", "10", "10"]
    for a, sd in zip(args[0::2], args[1::2]):
        lcc = a.endswith("lcc")
        h = ek.Hypergraph.generate(float(a[:-3] if lcc else a), int(sd))
        if lcc:
            h, _ = h.largest_component()
        out = {}
        for form in ("single", "rccl1"):
            if form == "rccl1":
                os.environ["EK_COMM_FORCE"] = "1"
            c = ek.Context(0)
            try:
                if form == "rccl1":
                    c.comm_init(1, 0, ek.comm_unique_id())
                c.spmv_setup_pins(h)
                for reorth in (3, 1):
                    ts, st = [], None
                    for _ in range(4):
                        _, _, st = c.lanczos_fiedler(reorth=reorth)
                        ts.append(st["total_ms"])
                    out[f"{form}/reorth{reorth}"] = {
                        "ms": round(float(np.median(ts[1:])), 3), "matvecs": st["matvecs"],
                        "projected": st["projected_steps"], "allgathers": st["allgathers"],
                        "allreduces": st["allreduces"], "restarts": st["restarts"],
                        "us_per_matvec": round(1e3 * float(np.median(ts[1:])) / st["matvecs"], 2)}
                    print(f"[mr_pro_lab] {a} {form} reorth {reorth}: {out[f'{form}/reorth{reorth}']}", flush=True)
            finally:
                c.close()
                os.environ.pop("EK_COMM_FORCE", None)
        print(json.dumps({"workload": a, "seed": int(sd), "nodes": h.nodes, "forms": out}), flush=True)


if __name__ == "__main__":
    main()
