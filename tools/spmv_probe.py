#!/usr/bin/env python3
"""Child workload for bench.py's rocprofv3 passes (run BEFORE bench.py touches
the GPU itself, each pass a process of its own):

  resident MULT SEED       one resident Lanczos solve (rows built on the
                           device): the PMC FETCH_SIZE / WRITE_SIZE passes and
                           the 10x kernel trace.  The SpMV dispatches sit
                           where they sit in the timed solve, between the
                           basis passes.
  file MULT SEED W K       W untimed + K ek_solve_file steps on the generated
                           .hgr: the bench's timed step, for the kernel-trace
                           pass whose average SpMV duration the line's
                           roofline uses.

  b2b MULT SEED [fused]    200 back-to-back launches on resident buffers
                           (ek_spmv_bench; fused: the Lanczos epilogue)
  shard MULT SEED N        rank 0's rows of the N-rank nnz-balanced shard map
                           (ek_spmv_setup_pins computes it without a
                           collective), 200 back-to-back fused SpMV launches
                           over the padded all-gather layout (ek_spmv_bench):
                           bench.py's per-GPU SpMV leg at N > 1, one process.

usage: python tools/spmv_probe.py MODE MULT SEED [W K | N]
       python tools/spmv_probe.py MULT SEED          (= resident)
MULT with the suffix "lcc" (e.g. 1.15lcc): the largest connected component of
that synthetic (bench.py's headline workload).
"""
import importlib.util
import os
import shutil
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    args = sys.argv[1:]
    mode = args.pop(0) if args and args[0] in ("resident", "file", "shard", "b2b") else "resident"
    lcc = args[0].endswith("lcc")
    mult, seed = float(args[0][:-3] if lcc else args[0]), int(args[1])
    spec = importlib.util.spec_from_file_location("eigkl_amd", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
    ek = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ek)
    h = ek.Hypergraph.generate(mult, seed)
    if lcc:
        h, _ = h.largest_component()
    ctx = ek.Context(0)
    if mode == "shard":
        nranks = int(args[2])

        def no_collective(*_):
            raise RuntimeError("the shard probe runs no collective")

        # (the slot layout: the halo layout's setup all-gathers the other
        # ranks' requests, which this one-process probe cannot answer)
        os.environ["EK_MR_HALO"] = "0"
        ctx.comm_init_host(nranks, 0, no_collective, no_collective)
        ctx.spmv_setup_pins(h)
        us = ctx.spmv_bench(200, fused=True)
        _, r0, nr = ctx.spmv_dims()
        print(f"probe: rank 0 of {nranks}: rows {r0}..{r0 + nr}, {us:.2f} us per SpMV", flush=True)
    elif mode == "b2b":  # 200 back-to-back SpMV launches (fused: the Lanczos epilogue), resident matrix and x
        ctx.spmv_setup_pins(h)
        fused = {"fused": 1, "solve": 2}.get(args[2] if len(args) > 2 else "", 0)
        us = ctx.spmv_bench(200, fused=fused)
        print(f"probe: back to back (fused={fused}) {us:.2f} us per SpMV", flush=True)
    elif mode == "resident":
        ctx.spmv_setup_pins(h)
        for _ in range(int(args[2]) if len(args) > 2 else 1):  # (optional: solves in a row)
            lam, _, st = ctx.lanczos_fiedler()
        print(f"probe: {h.nodes} nodes, {st['matvecs']} matvecs, lambda1 {lam:.3e}", flush=True)
    else:
        warm, steps = int(args[2]), int(args[3])
        work = tempfile.mkdtemp(prefix="ekprobe_")
        path = os.path.join(work, "w.hgr")
        h.write(path)
        for i in range(warm + steps):
            r, _ = ctx.solve_file(path, eig=1, out_dir=work)
        print(f"probe: {steps} timed file steps, last {r['t_total'] * 1e3:.1f} ms", flush=True)
        shutil.rmtree(work, ignore_errors=True)
    ctx.close()


if __name__ == "__main__":
    main()
