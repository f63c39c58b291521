"""The N>1 data path on CPU (gloo, world_size 2): the row-sharded Lanczos
exchange pattern the HIP path runs over RCCL (ctx.cpp Lanczos):
rows split by ek_shard_rows, x replicated by an all-gather of the rank-major
padded slices, every dot product / norm all-reduced.  Each rank runs the
product's host pieces (generator, Laplacian, shard map) and a numpy restatement
of the per-rank arithmetic; the sharded recurrence must reproduce the
single-process one."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import load_package

WORLD = 2
STEPS = 12


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _local_spmv(rp, col, val, x):
    y = np.zeros(len(rp) - 1)
    nz = np.diff(rp) > 0
    y[nz] = np.add.reduceat(val * x[col], rp[:-1][nz])
    return y


def _lanczos_steps(matvec, dot, n_local, mask, n, x0, steps):
    """Deflated three-term Lanczos + one CGS pass (the default reorth=1 path)."""
    u0 = mask / np.sqrt(n)
    f = x0 - dot(u0, x0) * u0
    V, alpha, beta = [], [], []
    b = np.sqrt(dot(f, f))
    for i in range(steps):
        v = f / b
        V.append(v)
        w = matvec(v)
        a = dot(v, w)
        f = w - a * v - (beta[-1] * V[-2] if i > 0 else 0.0)
        h = np.array([dot(q, f) for q in V] + [dot(u0, f)])
        f = f - sum(hj * q for hj, q in zip(h[:-1], V)) - h[-1] * u0
        alpha.append(a + h[i])
        b = np.sqrt(dot(f, f))
        beta.append(b)
    return np.array(alpha), np.array(beta)


def _worker(rank, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        ek = load_package()
        h = ek.Hypergraph.generate(0.05, 3)
        n = h.nodes
        L = h.laplacian()
        row0, nrows, nloc = ek.shard_rows(n, WORLD, rank)
        rp = L.rowptr[row0: row0 + nrows + 1].astype(np.int64)
        lrp, lcol, lval = rp - rp[0], L.col[rp[0]: rp[-1]], L.val[rp[0]: rp[-1]]
        mask = np.zeros(nloc)
        mask[:nrows] = 1.0

        def allgather(xloc):
            parts = [torch.zeros(nloc, dtype=torch.float64) for _ in range(WORLD)]
            dist.all_gather(parts, torch.from_numpy(np.ascontiguousarray(xloc)))
            return torch.cat(parts).numpy()[:n]

        def matvec(xloc):
            y = np.zeros(nloc)
            y[:nrows] = _local_spmv(lrp, lcol, lval, allgather(xloc))
            return y

        def dot(a, b):
            t = torch.tensor([float(a @ b)], dtype=torch.float64)
            dist.all_reduce(t)
            return float(t.item())

        x0 = np.random.default_rng(1).uniform(-0.5, 0.5, n)
        xl = np.zeros(nloc)
        xl[:nrows] = x0[row0: row0 + nrows]
        # sharded SpMV == full SpMV
        y_full = allgather(matvec(xl))
        y_ref = _local_spmv(L.rowptr.astype(np.int64), L.col, L.val, x0)
        spmv_err = float(np.abs(y_full - y_ref).max())
        a_sh, b_sh = _lanczos_steps(matvec, dot, nloc, mask, n, xl, STEPS)
        a_1, b_1 = _lanczos_steps(lambda v: _local_spmv(L.rowptr.astype(np.int64), L.col, L.val, v),
                                  lambda a, b: float(a @ b), n, np.ones(n), n, x0, STEPS)
        out[rank] = (spmv_err, float(np.abs(a_sh - a_1).max()), float(np.abs(b_sh - b_1).max()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_sharded_lanczos_matches_single_process():
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(_free_port(), out), nprocs=WORLD, join=True)
    for r in range(WORLD):
        spmv_err, da, db = out[r]
        assert spmv_err <= 1e-13
        assert da <= 1e-10 and db <= 1e-10, (da, db)


def test_shard_map_is_what_the_library_enforces():
    ek = load_package()
    n = 201920
    for world in (2, 4, 8):
        slices = [ek.shard_rows(n, world, r) for r in range(world)]
        nloc = slices[0][2]
        assert all(s[2] == nloc for s in slices)
        assert nloc * world >= n and nloc * (world - 1) < n
        assert sum(s[1] for s in slices) == n
