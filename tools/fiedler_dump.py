"""Dump the GPU Fiedler vector of the headline LCC (1.15x seed 1) under a few
Lanczos settings to gpurun_out/fiedler/*.npy, for the near-median analysis
of the headline split.  GPU run:
    python tools/fiedler_dump.py [out_dir]"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import load_package  # noqa: E402


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "gpurun_out", "fiedler")
    os.makedirs(out, exist_ok=True)
    ek = load_package()
    h, _ = ek.Hypergraph.generate(1.15, 1).largest_component()
    L = h.laplacian()
    c = ek.Context(0)
    c.spmv_setup(h.nodes, 0, L.rowptr, L.col, L.val)
    info = {}
    for name, kw in [("default", {}), ("spectra", dict(keep_min=0, basis32=False)),
                     ("tol14", dict(tol=1e-14)), ("tol14_spectra", dict(tol=1e-14, keep_min=0, basis32=False))]:
        lam, v, st = c.lanczos_fiedler(**kw)
        v = v * np.sign(v[np.argmax(np.abs(v))])
        np.save(os.path.join(out, f"{name}.npy"), v)
        info[name] = dict(lam=lam, **{k: st[k] for k in ("matvecs", "residual", "converged")})
        print(name, info[name], flush=True)
    json.dump(info, open(os.path.join(out, "info.json"), "w"), indent=1)
    c.close()


if __name__ == "__main__":
    main()
