#!/usr/bin/env python3
"""One resident Lanczos solve of a bench workload, for rocprofv3 counter passes
(bench.py runs it under `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` as a
child process before it touches the GPU itself).  The SpMV dispatches then sit
exactly where they sit in the timed solve: between the basis passes.

usage: python tools/spmv_probe.py MULT SEED
"""
import importlib.util
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    mult, seed = float(sys.argv[1]), int(sys.argv[2])
    spec = importlib.util.spec_from_file_location("eigkl_amd", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
    ek = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ek)
    h = ek.Hypergraph.generate(mult, seed)
    L = h.laplacian()
    ctx = ek.Context(0)
    ctx.spmv_setup(h.nodes, 0, L.rowptr, L.col, L.val)
    lam, _, st = ctx.lanczos_fiedler()
    print(f"probe: {h.nodes} nodes, {st['matvecs']} matvecs, lambda1 {lam:.3e}", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
