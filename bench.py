#!/usr/bin/env python3
"""bench.py — wall-clock to the final cut on MI355X (BASELINE.json metric).

One step = one in-process run of the whole hot path on a .hgr file, the body
of `gKL2 <file> -EIG` (ek_solve_file): parse -> clique Laplacian -> GPU
Lanczos Fiedler vector (rows sharded over the ranks, RCCL all-gather /
all-reduce over xGMI when N > 1) -> median split -> KL adjacency (host, built
while the GPU solves) -> GPU KL swap loop to termination (rank 0: the loop is a
sequential dependency chain) -> results/<base>_KL_CutSize_EIG_output.txt.

N = 1 workload: configs[2] "ibm18.hgr EIG+KL on 1 MI355X".  ibm18.hgr is not
shipped.  Real ibm18 is ONE connected circuit of 210,613 cells; the seeded
ISPD98-shaped generator leaves ~7 % of its nodes in no net, and on such a
disconnected graph lambda1 = 0 has a large eigenspace, so the Lanczos length
there is set by rounding noise (the 1.0x seed-1 synthetic took 503, 1071 and
1085 matvecs in three builds differing in last bits).  The stand-in is
therefore the largest connected component of the generator's 1.15x seed-1
output: 211,813 nodes (>= ibm18's cells and >= the 1.0x synthetic's 201,920),
240,591 nets, 597,707 pins, written to a file in the untimed setup
(`--workload full --mult 1.0` gives the whole 1.0x synthetic, which is also
timed as configs.syn1).  `value` = seconds per step (lower is better), the GPU
context staying up across steps like a service (a fresh process also pays HIP
start-up: `e2e_fresh_process_s`).
N > 1: the same file; the Lanczos rows are sharded (strong scaling of the
sharded phase), the KL loop stays on rank 0.  `--gpus N` without WORLD_SIZE
starts the N ranks itself (torch.distributed.run, before any GPU call).

Also reported: `roofline` of the Lanczos SpMV (HIP kernel timestamps of the
SpMVs of the timed steps; SURVEY §8d algorithmic bytes; PMC traffic from
rocprofv3 passes over a resident solve run as child processes before the
GPU is touched here), `cpu_baseline` (the oracle restatement on this host's
cores, 1 core and all cores, whole solve of the headline workload to
convergence, swap log compared), per-config sub-results (ibm01, ibm10, the
whole 1.0x and 2.0x synthetics), the resident-input solve time and the syn10
sharded Lanczos phase.
"""
import argparse
import csv
import glob
import json
import os
import re
import shutil
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
GOLD = os.path.join(REPO, "tests", "golden", "circuit")


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def load_pkg():
    import importlib.util
    spec = importlib.util.spec_from_file_location("eigkl_amd", os.path.join(REPO, "eig-kl-algorithm_amd", "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    sys.modules["eigkl_amd"] = mod
    return mod


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def rocprof_pass(what, probe_args, work, tag):
    """One rocprofv3 pass over tools/spmv_probe.py (a child process started
    BEFORE this process touches the GPU).  what = "trace": --kernel-trace
    --stats, returns {kernel name: (calls, average ns)}; otherwise a PMC
    counter (FETCH_SIZE / WRITE_SIZE), returns the SpMV dispatches' average in
    bytes (kB -> bytes) and their count.  None on failure."""
    if not shutil.which("rocprofv3"):
        return None
    d = os.path.join(work, f"rp_{tag}_{what}")
    mode = ["--kernel-trace", "--stats"] if what == "trace" else ["--pmc", what]
    cmd = (["timeout", "-s", "KILL", "150", "rocprofv3"] + mode + ["--output-format", "csv", "-d", d, "-o", "p", "--",
           sys.executable, os.path.join(REPO, "tools", "spmv_probe.py")] + [str(a) for a in probe_args])
    env = dict(os.environ, TMPDIR="/tmp")
    r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=180)
    pat = "*kernel_stats.csv" if what == "trace" else "*counter_collection.csv"
    files = glob.glob(os.path.join(d, "**", pat), recursive=True)
    if r.returncode != 0 or not files:
        log(f"rocprofv3 {what} pass ({tag}) failed (rc {r.returncode}): {r.stderr[-300:]}")
        return {"error": f"rc {r.returncode}, {len(files)} output files"}
    if what == "trace":
        return {row["Name"]: (int(row["Calls"]), float(row["AverageNs"])) for row in csv.DictReader(open(files[0]))}
    # every SpMV form: k_spmv_adaptive (CSR segments) and k_spmv_panel (the
    # column-panel form of a large x: the 10x synthetic)
    rows = list(csv.DictReader(open(files[0])))
    vals = [float(row["Counter_Value"]) for row in rows
            if "k_spmv_adaptive" in row["Kernel_Name"] or "k_spmv_panel" in row["Kernel_Name"]]
    kernels = sorted({re.search(r"k_spmv\w*(<[^>]*>)?", row["Kernel_Name"]).group(0) for row in rows
                      if "k_spmv" in row["Kernel_Name"]})
    if not vals:
        names = sorted({row["Kernel_Name"].split("(")[0][:50] for row in rows})
        log(f"rocprofv3 {what} pass ({tag}): NO SpMV dispatch among {len(rows)} rows (kernels: {names[:12]})")
        return {"error": f"no k_spmv dispatch in {len(rows)} counter rows"}
    return {"bytes": sum(vals) / len(vals) * 1024.0, "dispatches": len(vals), "kernels": kernels}


def kernel_avg_us(stats, needle):
    """(calls, average us) of the kernels whose name holds `needle` (calls-weighted)."""
    if not stats or "error" in stats:
        return 0, None
    rows = [v for k, v in stats.items() if needle in k]
    calls = sum(c for c, _ in rows)
    return (calls, sum(c * a for c, a in rows) / calls / 1e3) if calls else (0, None)


def traffic_of(fetch, write):
    """PMC traffic per SpMV launch, or {"error": ...} naming the pass that failed (never a silent None)."""
    if not fetch or not write:
        return {"error": "PMC passes not run"}
    bad = {k: v["error"] for k, v in (("FETCH_SIZE", fetch), ("WRITE_SIZE", write)) if "error" in v}
    if bad:
        return {"error": bad}
    return {"traffic": round(2 * fetch["bytes"] + write["bytes"]), "fetch_raw_bytes": round(fetch["bytes"]),
            "write_bytes": round(write["bytes"]), "dispatches": fetch["dispatches"], "kernels": fetch["kernels"]}


def compare_results(mine, ref):
    """cKL results rows 'iter\\tcut\\tgain' (cKL.cpp:315,380): iteration and gain
    columns as printed, the cut within max(0.05, 3e-5 |cut0|) (the reference's
    initial cut is a racy OpenMP fp32 sum, cKL.cpp:203).  Returns (ok, detail)."""
    a = [ln.split("\t") for ln in mine.strip().splitlines()]
    b = [ln.split("\t") for ln in ref.strip().splitlines()]
    if len(a) != len(b):
        return False, f"{len(a)} rows vs {len(b)}"
    tol = max(0.05, 3e-5 * abs(float(b[0][1])))
    worst = 0.0
    for i, (x, y) in enumerate(zip(a, b)):
        if x[0] != y[0] or x[2] != y[2]:
            return False, f"row {i}: {x} vs {y}"
        worst = max(worst, abs(float(x[1]) - float(y[1])))
        if worst > tol:
            return False, f"row {i}: cut {x[1]} vs {y[1]}"
    return True, f"{len(a)} rows equal (iteration, gain as printed; cut within {worst:.3g} <= {tol:.3g})"


def headline_parity(ctx, path, out_dir, n, last, is_headline):
    """The timed step's own output against the committed REFERENCE fixture
    (tests/golden/syn115_lcc: the real cKL's results file on the split of the
    converged Fiedler vector; data, not the oracle): its device split on every
    node, and its results file row by row (cKL.cpp:436-444, cEIG.cpp:204-209)."""
    import gzip
    gold = os.path.join(REPO, "tests", "golden", "syn115_lcc")
    if not is_headline or not os.path.exists(os.path.join(gold, "ref_results.txt.gz")):
        return {"headline_vs_reference": None, "why": "no reference fixture for this workload"}
    meta = json.load(open(os.path.join(gold, "meta.json")))
    bits_ref = np.unpackbits(np.load(os.path.join(gold, "split_bits.npy")))[:n]
    sides = ctx.kl_sides(0)  # the initial partition the last timed step's device split left
    ndiff = int(np.count_nonzero(sides != bits_ref))
    near = np.zeros(n, bool)
    near[meta["near_median_nodes"]] = True
    mine = open(os.path.join(out_dir, "results", os.path.basename(path) + "_KL_CutSize_EIG_output.txt")).read()
    ok, detail = compare_results(mine, gzip.open(os.path.join(gold, "ref_results.txt.gz"), "rt").read())
    iters_ok = last["kl"]["iterations"] == meta["reference_run"]["iterations"]
    return {"headline_vs_reference": bool(ok and ndiff == 0 and iters_ok),
            "split_nodes_differing": ndiff, "near_median_nodes_differing": int(np.count_nonzero((sides != bits_ref) & near)),
            "near_median_nodes": int(near.sum()), "results_file": detail,
            "iterations": [last["kl"]["iterations"], meta["reference_run"]["iterations"]],
            "reference": "tests/golden/syn115_lcc: real cKL (built from cKL.cpp) run on the converged Fiedler split"}


def cpu_baseline(hgr, split_npz, threads, max_matvec):
    """oracle/cpu_baseline.py in a child process (CPU only), pinned to `threads` cores;
    its progress lines go straight to this process's stderr."""
    cmd = [sys.executable, os.path.join(REPO, "oracle", "cpu_baseline.py"), hgr, split_npz, str(threads),
           str(max_matvec)]
    env = dict(os.environ, OMP_NUM_THREADS=str(threads), OMP_PROC_BIND="true")
    r = subprocess.run(cmd, stdout=subprocess.PIPE, text=True, timeout=600, env=env)
    if r.returncode != 0:
        return {"error": f"rc {r.returncode}"}
    return json.loads(r.stdout.strip().splitlines()[-1])


def become_subreaper():
    """Orphans of this bench's children (a profiler's helper, a tool's child)
    are re-parented to this process instead of init, so reap_strays() sees and
    ends exactly the processes this run left behind (procs_at_end 1)."""
    import ctypes
    try:
        ctypes.CDLL(None, use_errno=True).prctl(36, 1, 0, 0, 0)  # PR_SET_CHILD_SUBREAPER
    except (OSError, AttributeError):
        pass


def reap_strays():
    """Descendants still alive at the end: logged by command line, then ended (by PID)."""
    try:
        import psutil
    except ImportError:
        return None
    left = []
    for p in psutil.Process().children(recursive=True):
        try:
            left.append({"pid": p.pid, "cmd": " ".join(p.cmdline())[:160]})
            p.terminate()
        except psutil.Error:
            pass
    # the whole child tree at exit, logged even when empty (the
    # driver's procs_at_end 1 with no stray of ours listed)
    log(f"child tree at exit: {left if left else 'none'}")
    if left:
        log(f"processes this bench left behind (terminated): {left}")
        _, alive = psutil.wait_procs([psutil.Process(x["pid"]) for x in left if psutil.pid_exists(x["pid"])], timeout=5)
        for p in alive:
            p.kill()
    return left


def main():
    become_subreaper()
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mult", type=float, default=1.15)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--workload", choices=["lcc", "full"], default="lcc",
                    help="lcc: the synthetic's largest connected component (default); full: the whole synthetic")
    ap.add_argument("--comm", choices=["auto", "rccl", "host"], default="auto",
                    help="multi-rank exchange: RCCL over xGMI, or host-staged (several ranks per GPU)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip sub-configs, sweep, PMC and syn10 legs")
    ap.add_argument("--no-pmc", action="store_true")
    ap.add_argument("--prof-dir", default=None,
                    help="keep the rocprofv3 passes' CSVs here (default: a temporary directory)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU, started before any GPU call or package import
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"WORLD_SIZE {world} != --gpus {args.gpus}: reporting the {world} ranks that run")
    work = tempfile.mkdtemp(prefix=f"ekbench_r{rank}_")
    if args.prof_dir:
        work = os.path.join(os.path.abspath(args.prof_dir), f"rank{rank}")
        os.makedirs(work, exist_ok=True)
    extras = not args.no_extras and world == 1

    # rocprofv3 passes first: child processes, before this process touches the GPU
    #  * kernel trace of the bench's own step (1 untimed + 3 solve_file steps):
    #    the SpMV's average duration the line's roofline is computed from;
    #  * PMC FETCH_SIZE / WRITE_SIZE of the SpMV over a resident solve (1x, 10x);
    #  * kernel trace of the 10x resident solve (syn10's roofline).
    prof = {}
    lcc = args.workload == "lcc"
    wl = f"{args.mult:g}lcc" if lcc else f"{args.mult:g}"  # tools/spmv_probe.py's workload argument
    if world > 1 and rank == 0 and not args.no_extras and not args.no_pmc:
        # the sharded SpMV (syn10 at this N): rank 0's rows, one process with
        # no collective, while the other ranks wait in the rendezvous below
        t = time.time()
        shard = ["shard", 10.0, 10, world]
        prof["trace10"] = rocprof_pass("trace", shard, work, f"10x_shard{world}")
        prof["fetch10"] = rocprof_pass("FETCH_SIZE", shard, work, f"10x_shard{world}")
        prof["write10"] = rocprof_pass("WRITE_SIZE", shard, work, f"10x_shard{world}")
        log(f"rocprofv3 shard passes {time.time() - t:.1f} s")
    if extras and not args.no_pmc:
        t = time.time()
        prof["trace"] = rocprof_pass("trace", ["file", wl, args.seed, 1, 3], work, "1x")
        prof["fetch"] = rocprof_pass("FETCH_SIZE", ["resident", wl, args.seed], work, "1x")
        prof["write"] = rocprof_pass("WRITE_SIZE", ["resident", wl, args.seed], work, "1x")
        prof["trace10"] = rocprof_pass("trace", ["resident", 10.0, 10], work, "10x")
        prof["fetch10"] = rocprof_pass("FETCH_SIZE", ["resident", 10.0, 10], work, "10x")
        prof["write10"] = rocprof_pass("WRITE_SIZE", ["resident", 10.0, 10], work, "10x")
        log(f"rocprofv3 passes {time.time() - t:.1f} s: " + json.dumps(
            {k: (v if not k.startswith("trace") else {n[:40]: c for n, c in list((v or {}).items())[:6]})
             for k, v in prof.items()}))

    import torch.distributed as dist
    if world > 1:
        # gloo prints its peer connections on fd 1: rank 0's stdout must carry
        # the JSON line alone, so fd 1 points at stderr while it connects
        sys.stdout.flush()
        fd1 = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo")
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(fd1, 1)
            os.close(fd1)

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(x):
        if world == 1:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    ek = load_pkg()
    ndev = ek.device_count()
    comm = args.comm
    if world > 1 and comm == "auto":
        comm = "rccl" if ndev >= world else "host"
    ctx = ek.Context(local_rank % max(ndev, 1))
    if world > 1:
        if comm == "rccl":
            uid = [ek.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            ctx.comm_init(world, rank, uid[0])
        else:
            import torch

            def allgather(x):
                parts = [torch.empty(len(x), dtype=torch.float64) for _ in range(world)]
                dist.all_gather(parts, torch.from_numpy(x))
                return torch.cat(parts).numpy()

            def allreduce(x):
                t = torch.from_numpy(x)  # shares memory: in place
                dist.all_reduce(t)

            ctx.comm_init_host(world, rank, allgather, allreduce)

    # ---------------- untimed setup: the workload file
    h = ek.Hypergraph.generate(args.mult, args.seed)
    if lcc:
        h, _ = h.largest_component()
    nets, n, npins = h.dims()
    path = os.path.join(work, f"syn{args.mult:g}x_seed{args.seed}{'_lcc' if lcc else ''}.hgr")
    h.write(path)
    out_dir = os.path.join(work, "out")
    os.makedirs(out_dir, exist_ok=True)

    def step(time_spmv=False):
        return ctx.solve_file(path, eig=1, out_dir=out_dir, write_results=(rank == 0), time_spmv=time_spmv,
                              log_cap=(n // 2 if rank == 0 else 0))

    for _ in range(args.warmup):
        step()
    barrier()
    ctx.synchronize()
    t0 = time.time()
    results, step_walls = [], []
    for _ in range(args.steps):
        ts = time.time()
        results.append(step())
        step_walls.append(time.time() - ts)
    ctx.synchronize()
    barrier()
    elapsed = max_over_ranks(time.time() - t0)
    sec_per_step = elapsed / args.steps
    last, swap_log = results[-1]
    # the SpMV's kernel timestamps come from one more step, untimed: the timed
    # steps launch without timing events (a launch with events costs the host
    # ~7 us more, tools/lanczos_wall.py).  (The timed steps replay the
    # Lanczos chunks' HIP graphs on one context; a step with events launches
    # eagerly.)
    ev_step = step(time_spmv=True)
    barrier()
    log(f"timed: {args.steps} steps, {sec_per_step * 1e3:.2f} ms/step; last step {last['t_total']:.4f} s "
        f"(lanczos {last['t_lanczos']:.4f}, kl {last['t_kl']:.4f}, {last['lanczos']['matvecs']} matvecs, "
        f"{last['kl']['iterations']} swaps)")
    parity = None
    if rank == 0:
        parity = headline_parity(ctx, path, out_dir, n, last, lcc and args.mult == 1.15 and args.seed == 1)
        log(f"parity: {parity}")
    # the gather-only ceiling of the step's own SpMV (same grid, matrix stream
    # and x gathers, nothing else; ek_spmv_gather_bench), and the product
    # kernel back to back on the same matrix, for the roofline's reading
    ceil_us = ctx.spmv_gather_bench(200)
    prod_bb_us = ctx.spmv_bench(200, fused=False)
    lz = [r[0]["lanczos"] for r in results]
    spmv_timed = ev_step[0]["lanczos"]["spmv_timed"]
    spmv_us = 1e3 * ev_step[0]["lanczos"]["spmv_ms"] / max(1, spmv_timed)
    comm_ms = sum(x["comm_ms"] for x in lz) / len(lz)
    phases = {k: round(float(np.median([r[0][k] for r in results])), 4) for k in
              ("t_read", "t_laplacian", "t_spmv_setup", "t_lanczos", "t_split", "t_kl_graph_wait", "t_kl_setup",
               "t_kl", "t_write", "t_total")}
    phases["lanczos_device_ms"] = round(float(np.median([x["total_ms"] for x in lz])), 3)
    # the slowest step's phases (an outlier step shows which phase it lost time in)
    worst = max(results, key=lambda r: r[0]["t_total"])[0]
    phases_worst = {k: round(float(worst[k]), 4) for k in phases if k.startswith("t_")}
    off = ek.shard_map(h, world)  # the nnz-balanced map ek_solve_file's device build used
    row0, nrows = int(off[rank]), int(off[rank + 1] - off[rank])
    alg_bytes = ctx.spmv_bytes(fused=False)  # 12 nnz + 4(nrows+1) + 8n (x) + 8 nrows (y)
    fused_bytes = ctx.spmv_bytes(fused=True)  # + the fused epilogue's f read and basis-column write
    packed, stored = ctx.spmv_format(fused=True)
    # the same for every rank: every rank's SpMV is timed; report rank 0's and the max
    spmv_us_max = max_over_ranks(spmv_us)
    nnz_local = int((alg_bytes - 4 * (nrows + 1) - 8 * n - 8 * nrows) // 12)

    # ---------------- resident-input solve (inputs already in HBM): the solve alone
    L_rows = None
    resident = None
    res_bits = res_log = None
    if rank == 0 or world > 1:
        Lr = h.laplacian()
        rp = Lr.rowptr[row0: row0 + nrows + 1].astype(np.int64)
        ctx.spmv_setup(n, row0, (rp - rp[0]).astype(np.int32), Lr.col[rp[0]: rp[-1]], Lr.val[rp[0]: rp[-1]])
        L_rows = Lr
        if rank == 0:
            ctx.kl_graph_setup(h.kl_graph())
            ctx.kl_nets_setup(*h.pins())
        times, kres, klog, bits_r = [], None, None, None
        for i in range(4):
            barrier()
            t = time.time()
            lam_r, v_r, st_r = ctx.lanczos_fiedler()
            if rank == 0:
                _, bits_r = ek.median_split(v_r)
                ctx.kl_set_partition_bits(bits_r)
                klog, kres = ctx.kl_run()
            ctx.synchronize()
            barrier()
            if i:
                times.append(max_over_ranks(time.time() - t))
        resident = {"solve_s": round(float(np.median(times)), 5), "lanczos_ms": round(st_r["total_ms"], 3),
                    "lanczos_matvecs": st_r["matvecs"]}
        if rank == 0:
            res_bits, res_log = bits_r, klog
            resident.update({"kl_loop_ms": round(kres["loop_ms"], 3), "kl_iterations": kres["iterations"],
                             "us_per_swap": round(1e3 * kres["loop_ms"] / max(1, kres["iterations"]), 3),
                             "swap_log_equals_timed_steps": bool(world == 1 and len(klog) == len(swap_log) and
                                                                 klog.tobytes() == swap_log.tobytes())})

    # ---------------- syn10 (configs[4]): the sharded Lanczos phase at this N
    syn10 = None
    if not args.no_extras:
        h10 = ek.Hypergraph.generate(10.0, 10)
        n10 = h10.nodes
        c10 = ctx
        c10.spmv_setup_pins(h10)  # this rank's nnz-balanced rows, built on the device
        _, r0, nr = c10.spmv_dims()
        hl10, rv10, sd10 = c10.spmv_exchange()
        st10 = None
        tt = []
        for i in range(2):
            barrier()
            t = time.time()
            _, _, st10 = c10.lanczos_fiedler(time_spmv=(i == 1))
            c10.synchronize()
            barrier()
            tt.append(max_over_ranks(time.time() - t))
        cs10 = c10.comm_stats()  # the timed solve's collectives (time_spmv on the last one)
        ceil10_us = c10.spmv_gather_bench(100)
        # (every collective on every rank, in the same order: the max is taken
        # here once, not inside rank-0-only blocks below)
        ceil10_max = max_over_ranks(ceil10_us)
        b10 = c10.spmv_bytes(fused=False)
        us10 = 1e3 * st10["spmv_ms"] / max(1, st10["spmv_timed"])
        us10_max = max_over_ranks(us10)
        syn10 = {"workload": "synthetic 10x seed 10", "nodes": n10, "ranks": world, "lanczos_s": round(tt[-1], 4),
                 "matvecs": st10["matvecs"], "spmv_us_per_launch_max_rank": round(us10_max, 3),
                 "spmv_bytes_per_rank": int(b10),
                 "spmv_GBps_per_gpu": round(b10 / us10_max / 1e3, 1),
                 "spmv_frac_per_gpu": round(b10 / us10_max / 1e3 / HBM_PEAK_GBS, 4),
                 "spmv_GBps_aggregate": round(world * b10 / us10_max / 1e3, 1),
                 "spmv_timing": "HIP kernel start/end events of every 4th SpMV (this process)",
                 "collectives_per_solve": {"allgather": st10["allgathers"], "allreduce": st10["allreduces"]},
                 "comm_ms_per_solve": round(max_over_ranks(st10["comm_ms"]), 3), "comm": comm if world > 1 else None,
                 "exchange": {"form": ("halo (rows each rank reads, RCCL send/recv)" if hl10 else
                                       "all-gather of whole slots") if world > 1 else None,
                              "recv_MB_per_step_rank0": round(8 * rv10 / 1e6, 3),
                              "send_MB_per_step_rank0": round(8 * sd10 / 1e6, 3)},
                 "projected_steps": st10["projected_steps"],
                 "ceiling": {"gather_only_us_max_rank": round(ceil10_max, 3),
                             "ceiling_frac_per_gpu": round(b10 / ceil10_max / 1e3 / HBM_PEAK_GBS, 4),
                             "what": "ek_spmv_gather_bench: the SpMV's grid, matrix stream and x / value gathers "
                                     "with nothing else, back to back"}}
        if world > 1:
            # per rank, the timed solve's exchange of f and its all-reduces
            # separately (RCCL: HIP events around each on its stream, waits for
            # the peers included), the max over ranks; messages per exchange
            xs = 1e3 * cs10["exchange_ms"] / max(1, cs10["exchanges_timed"])
            ars = 1e3 * cs10["allreduce_ms"] / max(1, cs10["allreduces_timed"])
            syn10["collectives"] = {
                "exchange_us_avg_max_rank": round(max_over_ranks(xs), 2),
                "allreduce_us_avg_max_rank": round(max_over_ranks(ars), 2),
                "exchange_ms_per_solve_max_rank": round(max_over_ranks(cs10["exchange_ms"]), 3),
                "allreduce_ms_per_solve_max_rank": round(max_over_ranks(cs10["allreduce_ms"]), 3),
                "exchanges_timed": cs10["exchanges_timed"], "allreduces_timed": cs10["allreduces_timed"],
                "messages_per_exchange_rank0": {
                    "sends": round(cs10["sends"] / max(1, cs10["exchanges"]), 3),
                    "recvs": round(cs10["recvs"] / max(1, cs10["exchanges"]), 3)},
                "timing": ("HIP events around each RCCL collective on its stream" if comm == "rccl" else
                           "host clock around each host-staged collective")}
        calls10, us10_rp = kernel_avg_us(prof.get("trace10"), "k_spmv")
        if us10_rp:  # the rocprofv3 kernel trace (a child pass before this process touched the GPU)
            syn10["rocprof"] = {"spmv_avg_us": round(us10_rp, 3), "spmv_calls": calls10,
                                "achieved_GBps": round(b10 / us10_rp / 1e3, 1),
                                "frac": round(b10 / us10_rp / 1e3 / HBM_PEAK_GBS, 4),
                                "frac_of_ceiling": round(ceil10_max / us10_rp, 4),
                                "what": ("the resident 1-rank solve" if world == 1 else
                                         f"rank 0's shard of the {world}-rank map, 200 back-to-back fused launches "
                                         "(tools/spmv_probe.py shard)")}
        if world > 1:  # every rank's shard back to back (events), the max over ranks
            us_bb = max_over_ranks(c10.spmv_bench(200, fused=True))
            syn10["spmv_back_to_back_us_max_rank"] = round(us_bb, 3)
            syn10["spmv_back_to_back_frac_per_gpu"] = round(b10 / us_bb / 1e3 / HBM_PEAK_GBS, 4)
        if (extras or world > 1) and not args.no_pmc and rank == 0:
            t10 = traffic_of(prof.get("fetch10"), prof.get("write10"))
            if "error" not in t10:
                t10["per_algorithmic_byte"] = round(t10["traffic"] / b10, 3)
                t10["stored_bytes_per_rank"] = int(c10.spmv_format(fused=False)[1])
                t10["per_stored_byte"] = round(t10["traffic"] / t10["stored_bytes_per_rank"], 3)
            else:
                log(f"syn10 traffic: {t10['error']}")
            syn10["traffic"] = t10
        if extras and rank == 0:  # the whole -EIG pipeline on it below (sub-config syn10_pipeline)
            h10.write(os.path.join(work, "syn10.hgr"))
        del h10

    if rank != 0:
        ctx.close()
        if world > 1:
            dist.destroy_process_group()
        return

    # ---------------- sub-configs (N = 1): the file path on other inputs
    subs = {}
    if extras:
        inputs = [("ibm01", os.path.join(GOLD, "ibm01.hgr"), "configs[1] ibm01.hgr (shipped)"),
                  ("ibm10", os.path.join(GOLD, "ibm10.hgr"), "ibm10.hgr: the largest shipped ISPD98 circuit, connected"),
                  ("syn1", (1.0, 1), "the whole 1.0x seed-1 synthetic (SURVEY §8d's first stand-in; disconnected: "
                                     "lambda1 = 0, its Lanczos length set by rounding noise)"),
                  ("syn2", (2.0, 2), "configs[3] circuit_generator 2.0x shape, seed 2 (disconnected)")]
        if os.path.exists(os.path.join(work, "syn10.hgr")):
            inputs.append(("syn10_pipeline", os.path.join(work, "syn10.hgr"),
                           "configs[4]'s graph (10x seed 10, 2.02M nodes) through the whole -EIG file path on ONE "
                           "GPU: Lanczos, device split, KL (the on-chip loop with its bitmaps off chip)"))
        for name, p, what in inputs:
            if isinstance(p, tuple):
                hp = ek.Hypergraph.generate(*p)
                p = os.path.join(work, f"{name}.hgr")
                hp.write(p)
                del hp
            walls, rr = [], None
            # the previous rounds' headline workload (syn1) keeps the
            # headline's treatment: 2 untimed + 10 timed steps; the others a
            # median of 2 warm runs
            nrun, nwarm = (12, 2) if name == "syn1" else (3, 1)
            for i in range(nrun):
                t = time.time()
                rr, _ = ctx.solve_file(p, eig=1, out_dir=out_dir)
                walls.append(time.time() - t)
            subs[name] = {"what": what, "nodes": rr["nodes"], "wall_s": round(float(np.median(walls[nwarm:])), 4),
                          "ms_per_step": round(1e3 * float(np.mean(walls[nwarm:])), 3),
                          "steps_timed": nrun - nwarm,
                          "lambda1": rr["lambda"], "matvecs": rr["lanczos"]["matvecs"],
                          "restarts": rr["lanczos"]["restarts"], "lanczos_s": round(rr["t_lanczos"], 4),
                          "kl_iterations": rr["kl"]["iterations"], "kl_s": round(rr["t_kl"], 4),
                          "best_cut": rr["kl"]["best_cut"], "net_cut_best": rr["kl"]["net_cut_best"],
                          "best_iter": rr["kl"]["best_iter"]}
            log(f"sub-config {name}: {subs[name]}")

    # ---------------- SpMV size sweep (informational, back-to-back launches)
    sweep = []
    if extras:
        for mult, seed in ((args.mult, args.seed), (2.0, 2)):
            hs = h if mult == args.mult else ek.Hypergraph.generate(mult, seed)
            Ls = L_rows if mult == args.mult else hs.laplacian()
            c2 = ek.Context(0)
            c2.spmv_setup(hs.nodes, 0, Ls.rowptr, Ls.col, Ls.val)
            us = c2.spmv_bench(200, fused=False)
            b2 = c2.spmv_bytes(fused=False)
            sweep.append({"mult": mult, "bytes_per_launch": int(b2), "avg_launch_us": round(us, 3),
                          "GB/s": round(b2 / us / 1e3, 1), "frac": round(b2 / us / 1e3 / HBM_PEAK_GBS, 4)})
            c2.close()

    # ---------------- fresh-process wall of the drop-in tool (HIP start-up included),
    # split by the library's EK_COLD_TRACE stamps (tools/cold_probe.py)
    fresh = fresh_breakdown = None
    if extras:
        sys.path.insert(0, os.path.join(REPO, "tools"))
        import cold_probe
        fb = cold_probe.probe(path, 5, cwd=out_dir)
        if "error" in fb:
            fresh = fb["error"]
        else:
            fresh = fb["exit"]
            fresh_breakdown = {"offsets_s": fb, "what": (
                "median offsets from the spawn of `gKL2 <headline .hgr> -EIG --quiet` (5 runs): lib_loaded = exec + "
                "dynamic loading; hip_first_call..hip_streams = ek_init on its thread (beside the parse); "
                "laplacian/lanczos/kl = the solve's phases incl. first-launch costs; exit = the child reaped "
                "(the executables leave the context to the process exit: EK_CLI_NO_TEARDOWN)")}

    # ---------------- CPU baseline: oracle restatement on this host's cores,
    # the whole solve of the headline workload itself to convergence, all
    # cores (`value`) and 1 core; its KL() runs from the GPU run's split and
    # its swap log is compared with the GPU's
    cpu = None
    if extras and not args.no_cpu_baseline:
        split_npz = os.path.join(work, "split.npz")
        np.savez(split_npz, bits=res_bits, log=res_log)
        ncpu = len(os.sched_getaffinity(0))
        all_cores = min(16, ncpu)  # the GPU box grants each job a 16-CPU share
        cap = 0 if lcc else 3 * last["lanczos"]["matvecs"]  # a disconnected workload: capped (a lower bound)
        legs = {}
        for key, th in (("all", all_cores), ("one", 1)):
            t = time.time()
            legs[key] = cpu_baseline(path, split_npz, th, cap)
            log(f"cpu baseline, {th} thread(s): {time.time() - t:.1f} s: {legs[key]}")
        best = legs["all"]
        if "error" not in best:
            cpu = {"value": round(best["total_s"], 3), "unit": "s", "cores": best["threads"], "kind": "port",
                   "sample": ("the headline workload itself (" + f"{n:,} nodes), "
                              + "whole solve on the oracle restatement of cEIG+cKL (oracle/eko_eig.cpp, eko_kl.cpp), "
                              f"OpenMP on {best['threads']} pinned host cores: parse, Laplacian + Lanczos "
                              + (f"to convergence ({best['lanczos_matvecs']} matvecs)" if best["lanczos_converged"]
                                 else f"capped at {best['lanczos_matvecs']} matvecs, not converged (a lower bound)")
                              + f", KL() from the GPU run's split ({best['kl_iterations']} swaps, swap log "
                                "compared with the GPU's)"),
                   "gpu_same_sample_s": round(sec_per_step, 4),
                   "gpu_speedup_same_sample": round(best["total_s"] / sec_per_step, 1),
                   "lanczos_converged": best["lanczos_converged"], "lanczos_matvecs": best["lanczos_matvecs"],
                   "parse_s": best["parse_s"], "lanczos_s": best["lanczos_s"], "kl_s": best["kl_s"],
                   "swap_log_match": best["swap_log_match"], "first_mismatch": best["first_mismatch"],
                   "one_core": legs.get("one"),
                   "reference_cKL_note": "real cKL (oracle/_ref, built from /root/reference) is O(n^2) in setup and "
                                         "per swap (cKL.cpp:53-72, 225-251): tests/golden/ref_runs.json and "
                                         "tests/golden/syn115_lcc/meta.json hold its measured times on the "
                                         "1.0x LCC (2,440 s) and on this workload"}
        else:
            cpu = {"error": best["error"]}

    # the roofline's duration: the rocprofv3 kernel trace of the bench's own step
    # (a child pass before this process touched the GPU; profiles/ holds the
    # same summary from the round's runs); the event-timed figure of the timed
    # steps is kept beside it
    calls_rp, us_rp = kernel_avg_us(prof.get("trace"), "k_spmv")
    us_line = us_rp if us_rp else spmv_us
    trace = prof.get("trace") or {}
    spmv_names = sorted((k for k in trace if "k_spmv" in k), key=lambda k: -trace[k][0]) \
        if "error" not in trace else []
    kname = spmv_names[0].replace("ek::dev::", "") if spmv_names else \
        f"k_spmv_adaptive<{'coded' if packed else 'plain'}>"
    roof = {"bound": "hbm", "kernel": f"{kname} (Lanczos CSR SpMV, fp64)",
            "achieved": round(alg_bytes / us_line / 1e3, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(alg_bytes / us_line / 1e3 / HBM_PEAK_GBS, 4), "traffic": None,
            "bytes_per_launch": int(alg_bytes),
            "bytes_rule": "SURVEY §8d: 12 nnz + 4 (n+1) + 8 n (x) + 8 n (y)",
            "avg_launch_us": round(us_line, 3),
            "timing": ("rocprofv3 --kernel-trace --stats over tools/spmv_probe.py file (1 untimed + 3 solve_file "
                       f"steps of this workload, {calls_rp} SpMV dispatches), run by this bench before it touched the "
                       "GPU: achieved = bytes_per_launch / its AverageNs" if us_rp else
                       "HIP kernel start/end events (no rocprofv3 on this host)"),
            "events": {"avg_launch_us": round(spmv_us, 3), "launches_timed": spmv_timed,
                       "frac": round(alg_bytes / spmv_us / 1e3 / HBM_PEAK_GBS, 4),
                       "what": "HIP kernel start/end timestamps of every 4th SpMV of each Lanczos cycle of one "
                               "untimed step after the timed ones (eager launches: events are not graph nodes); the "
                               "start marker precedes the dispatch, so this also holds the ~1.5 us kernel boundary"},
            "ceiling_frac": round(alg_bytes / ceil_us / 1e3 / HBM_PEAK_GBS, 4),
            "frac_of_ceiling": round(ceil_us / us_line, 4),
            "ceiling": {"gather_only_us": round(ceil_us, 3), "product_back_to_back_us": round(prod_bb_us, 3),
                        "back_to_back_frac": round(alg_bytes / prod_bb_us / 1e3 / HBM_PEAK_GBS, 4),
                        "what": ("ceiling_frac = bytes_per_launch / the gather-only kernel's time / peak: "
                                 "ek_spmv_gather_bench runs this SpMV's grid over the same matrix words and makes the "
                                 "same x and value-table gathers, summing in registers (no row reduction, no y, no "
                                 "epilogue), 200 launches back to back; frac_of_ceiling = frac / ceiling_frac")},
            "fused_bytes_per_launch": int(fused_bytes),
            "fused_frac": round(fused_bytes / us_line / 1e3 / HBM_PEAK_GBS, 4),
            "stored_bytes_per_launch": int(stored),
            "storage": ("dictionary-coded CSR: 32-bit (code<<colbits | col) words + exact fp64 value table"
                        if packed else "CSR: int32 col + fp64 val"),
            "sweep_back_to_back": sweep}
    if us_rp:
        roof["kernel_trace_top"] = {
            name.split("(")[0].replace("void ", "")[:60]: {"calls": c, "avg_us": round(a / 1e3, 3)}
            for name, (c, a) in sorted(prof["trace"].items(), key=lambda kv: -kv[1][0] * kv[1][1])[:8]}
    t1 = traffic_of(prof.get("fetch"), prof.get("write")) if extras and not args.no_pmc else None
    if t1 and "error" in t1:
        log(f"headline traffic: {t1['error']}")
        roof["traffic_error"] = t1["error"]
    elif t1:
        roof["traffic"] = t1.pop("traffic")
        roof["traffic_detail"] = dict(t1, per_algorithmic_byte=round(roof["traffic"] / alg_bytes, 3),
            correction="traffic = 2 x FETCH_SIZE + WRITE_SIZE (gfx950: FETCH_SIZE counts half of wide reads, "
                       "MI355X_MICROARCH.md HBM; this kernel's widths: profiles/r02/pmc_calib_*); L2 memory-side "
                       "requests, Infinity-Cache hits included",
            source="rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE passes over tools/spmv_probe.py resident in this run")

    strays = reap_strays()
    out = {
        "metric": "wall-clock to final cut (s) + cut size, ibm18.hgr; SpMV GB/s vs HBM peak",
        "value": round(sec_per_step, 6),
        "unit": "s",
        "value_is": ("the warm-context step: one in-process .hgr file -> results file solve (ek_solve_file) with the "
                     "GPU context up, as a service runs it; e2e_s is the metric as SURVEY §8d states it"),
        "e2e_s": fresh,
        "e2e_is": ("process start -> results written: `gKL2 <headline .hgr> -EIG` spawned fresh (HIP start-up, library "
                   "load, parse, solve, write), median of 5 (e2e_fresh_breakdown)"),
        "cut": last["kl"]["net_cut_best"],
        "cut_is": ("integer net cut of the best KL prefix (nets with pins on both sides), cKL.cpp:392-403's split; "
                   "the fp32 running cut is result.best_cut"),
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(sec_per_step * 1e3, 4),
        "higher_is_better": False,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64 (Lanczos) + f32 (KL gains, bit-exact with cKL)",
        "data": "synthetic (seeded ISPD98-shaped generator written to .hgr; ibm18.hgr not shipped)",
        "config": {"workload": (f"ibm18-size connected synthetic: largest component of the {args.mult:g}x seed-"
                                f"{args.seed} generator output, .hgr file -> results file" if lcc else
                                f"ibm18-shape synthetic {args.mult:g}x seed {args.seed}: .hgr file -> results file"),
                   "nodes": n, "nets": nets, "pins": npins, "laplacian_nnz": nnz_local if world == 1 else None,
                   "parallelism": f"lanczos row-shard x{world} ({comm if world > 1 else 'single'}), KL 1 GPU"},
        "roofline": roof,
        "cpu_baseline": cpu,
        "parity": parity,
        "result": {"lambda1": last["lambda"], "lanczos_matvecs": last["lanczos"]["matvecs"],
                   "lanczos_restarts": last["lanczos"]["restarts"], "residual": last["lanczos"]["residual"],
                   "kl_iterations": last["kl"]["iterations"], "kl_loop_ms": round(last["kl"]["loop_ms"], 3),
                   "initial_cut": last["kl"]["initial_cut"], "best_cut": last["kl"]["best_cut"],
                   "net_cut_best": last["kl"]["net_cut_best"], "net_cut_final": last["kl"]["net_cut_final"],
                   "best_iter": last["kl"]["best_iter"], "phases_median_s": phases, "phases_slowest_step_s": phases_worst,
                   "step_walls_s": [round(w, 4) for w in step_walls],
                   "step_totals_s": [round(r[0]["t_total"], 4) for r in results],
                   "comm_ms_per_step": round(comm_ms, 3), "spmv_us_max_rank": round(spmv_us_max, 3),
                   "resident_solve": resident},
        "e2e_fresh_process_s": fresh,
        "e2e_fresh_breakdown": fresh_breakdown,
        "configs": subs,
        "syn10_sharded_lanczos": syn10,
        "stray_processes_reaped": strays,
    }
    print(json.dumps(out), flush=True)
    ctx.close()
    if not args.prof_dir:
        shutil.rmtree(work, ignore_errors=True)
    if world > 1:
        dist.destroy_process_group()
    try:  # last word on descendants, after the context and the process group are gone
        import psutil
        kids = [(p.pid, " ".join(p.cmdline())[:120]) for p in psutil.Process().children(recursive=True)]
        log(f"descendants at return: {kids if kids else 'none'}")
    except Exception as e:  # noqa: BLE001 (diagnostic only)
        log(f"descendants at return: unknown ({e})")


if __name__ == "__main__":
    main()
