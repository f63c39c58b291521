"""The library's own sharded Lanczos with 2 ranks, on one GPU.

Two processes each open a context on GPU 0 and join a 2-rank exchange through
ek_comm_init_host: every collective of the sharded path (the all-gather of f
before each SpMV, the all-reduces of alpha, of the Gram-Schmidt coefficients
and of ||f||^2, the final all-gather and the residual) goes through the
library's comm seam, staged through host memory and carried by
torch.distributed gloo.  RCCL, the production backend, refuses two ranks on
one device; the device code, the shard map (row0 > 0, padded slices), the
unfused step sequence and the global-index restart vectors are the same.

Checks: the 2-rank Fiedler pair against the reference's pre_saved_EIG files
(ibm01, industry2; the SURVEY §8c tolerances), the 2-rank SpMV against the
1-rank one per row, the sharded solve_file (parse -> results file) against the
reference cKL results, and a disconnected synthetic whose solve goes through
breakdowns and injected restart vectors on both ranks."""
import os
import socket

import numpy as np
import pytest

from conftest import circuit_path, compare_results_text, eig_path, ref_results_path

pytestmark = pytest.mark.gpu
WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _fiedler_ok(ek, name, lam, v):
    lam_ref, med_ref, bits_ref, v_ref, _, _ = ek.eig_read(eig_path(name), len(v))
    v = v * np.sign(v @ v_ref)
    _, bits = ek.median_split(v)
    mask = np.abs(v_ref - med_ref) > 1e-8
    return {"dlam": abs(lam - lam_ref), "dv": float(np.abs(v - v_ref).max()),
            "bits_equal": bool(np.array_equal(bits[mask], bits_ref[mask]))}


def _worker(rank, port, tmp, out):
    import datetime
    import faulthandler
    import sys
    import torch
    import torch.distributed as dist
    faulthandler.enable()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD, timeout=datetime.timedelta(seconds=90))
    from conftest import load_package
    ek = load_package()
    res = {}
    try:
        ctx = ek.Context(0)

        def allgather(x):
            parts = [torch.empty(len(x), dtype=torch.float64) for _ in range(WORLD)]
            dist.all_gather(parts, torch.from_numpy(x))
            return torch.cat(parts).numpy()

        def allreduce(x):
            dist.all_reduce(torch.from_numpy(x))  # in place (shared memory)

        ctx.comm_init_host(WORLD, rank, allgather, allreduce)
        one = ek.Context(0)  # an unsharded context for the 1-rank comparison
        for name in ("ibm01", "industry2"):
            h = ek.Hypergraph.read(circuit_path(name))
            n = h.nodes
            row0, nrows, nloc = ek.shard_rows(n, WORLD, rank)
            S = h.laplacian_rows(row0, row0 + nrows)
            ctx.spmv_setup(n, row0, S.rowptr, S.col, S.val)
            lam, v, st = ctx.lanczos_fiedler()
            r = _fiedler_ok(ek, name, lam, v)
            r.update(converged=bool(st["converged"]), residual=st["residual"], matvecs=st["matvecs"],
                     row0=row0, nrows=nrows, comm_ms=st["comm_ms"])
            # SpMV: this rank's rows vs the same rows of a 1-rank SpMV
            x = np.random.default_rng(7).standard_normal(n)
            y = ctx.spmv_host(x)
            L = h.laplacian()
            one.spmv_setup(n, 0, L.rowptr, L.col, L.val)
            y1 = one.spmv_host(x)[row0: row0 + nrows]
            absrow = np.add.reduceat(np.abs(S.val * x[S.col]), S.rowptr[:-1])
            r["spmv_rows_ok"] = bool(np.all(np.abs(y - y1) <= 1e-14 * absrow + 1e-300))
            r["spmv_max_abs_diff"] = float(np.abs(y - y1).max())
            res[name] = r
        # the whole file path, sharded: rank 0 writes the results file
        rr, _ = ctx.solve_file(circuit_path("ibm01"), eig=1, out_dir=os.path.join(tmp, f"r{rank}"))
        res["solve_file"] = {"iterations": rr["kl"]["iterations"], "net_cut_best": rr["kl"]["net_cut_best"]}
        # disconnected synthetic: breakdowns, injected vectors over global indices on both ranks
        h = ek.Hypergraph.generate(0.25, 3)
        n = h.nodes
        row0, nrows, _ = ek.shard_rows(n, WORLD, rank)
        S = h.laplacian_rows(row0, row0 + nrows)
        ctx.spmv_setup(n, row0, S.rowptr, S.col, S.val)
        lam, v, st = ctx.lanczos_fiedler()
        res["syn0.25"] = {"lam": lam, "residual": st["residual"], "converged": bool(st["converged"]),
                          "finite": bool(np.all(np.isfinite(v))), "norm": float(np.linalg.norm(v)),
                          "v_head": v[:64].tolist()}
        one.close()
        ctx.close()
    except Exception:  # reported to the parent; the peer's next collective then fails too
        import traceback
        res["error"] = traceback.format_exc()
        print(f"[rank {rank}] {res['error']}", file=sys.stderr, flush=True)
    finally:
        out[rank] = res
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_sharded_lanczos_through_comm_seam(tmp_path):
    import torch.multiprocessing as mp
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(_free_port(), str(tmp_path), out), nprocs=WORLD, join=True)
    r0, r1 = out[0], out[1]
    errors = {k: out[k]["error"] for k in (0, 1) if "error" in out[k]}
    assert not errors, errors
    for r in (r0, r1):
        for name in ("ibm01", "industry2"):
            x = r[name]
            assert x["converged"] and x["residual"] < 1e-9, x
            assert x["dlam"] <= 1e-10 and x["dv"] <= 1e-8 and x["bits_equal"], x
            assert x["spmv_rows_ok"], x
    assert r1["ibm01"]["row0"] > 0 and r0["ibm01"]["nrows"] + r1["ibm01"]["nrows"] == 12752
    # every rank holds the same full vector: identical Ritz pairs
    assert r0["ibm01"]["dv"] == r1["ibm01"]["dv"]
    s0, s1 = r0["syn0.25"], r1["syn0.25"]
    for s in (s0, s1):
        assert s["converged"] and s["finite"] and abs(s["norm"] - 1) < 1e-10 and s["residual"] < 1e-8, s
        assert abs(s["lam"]) < 1e-8
    assert s0["v_head"] == s1["v_head"]
    # sharded file path == the reference cKL results (ibm01: even n, sign-independent)
    res = tmp_path / "r0" / "results" / "ibm01.hgr_KL_CutSize_EIG_output.txt"
    compare_results_text(res.read_text(), open(ref_results_path("ibm01")).read())
    assert r0["solve_file"]["net_cut_best"] == 367
