"""The N>1 data path on CPU (gloo, world_size 2): the row-sharded Lanczos
exchange the HIP path runs over RCCL (ctx.cpp
Lanczos::factorize_mr), restated in numpy on each rank with the product's host
pieces (generator, Laplacian rows, the nnz-balanced shard map):

* rank r owns rows [off[r], off[r+1]) of ek_shard_map (unequal slices);
* ONE all-gather per step: every rank's f slice padded to a slot of S
  doubles, with the rank's ||f||^2 partial in the slot's tail, so the matrix
  reads x through columns remapped to r*S + (c - off[r]) and every rank sums
  the ranks' partials in rank order (the same bits everywhere);
* the SpMV split around that all-gather: the owned slot's entries summed from
  the rank's own f while the gather is in flight, the halo's after it;
* ONE all-reduce per step: [V^T w | V^T v_i | V^T v_{i-1}], from which
  alpha = (V^T w)_i and the projection of f' = w - alpha v_i - beta v_{i-1}
  come by linearity.

The sharded recurrence must reproduce the single-process three-term + CGS one
(the single-GPU step) within fp64 round-off, with exactly two collectives per
step."""
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


def _lanczos_single(matvec, n, x0, steps):
    """Deflated three-term Lanczos + one CGS pass of f' (the single-GPU reorth=1 step)."""
    u0 = np.ones(n) / np.sqrt(n)
    f = x0 - (u0 @ x0) * u0
    V, alpha, beta = [], [], []
    b = np.sqrt(f @ f)
    for i in range(steps):
        v = f / b
        V.append(v)
        w = matvec(v)
        a = v @ w
        f = w - a * v - (beta[-1] * V[-2] if i > 0 else 0.0)
        h = np.array([q @ f for q in V] + [u0 @ f])
        f = f - sum(hj * q for hj, q in zip(h[:-1], V)) - h[-1] * u0
        alpha.append(a + h[i])
        b = np.sqrt(f @ f)
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
        off = ek.shard_map(h, WORLD)
        row0, nrows = int(off[rank]), int(off[rank + 1] - off[rank])
        M = int(np.diff(off).max())
        ldv = -(-M // 1024) * 1024
        S = ldv + 64  # the library's slot: Lanczos rows + 64, ||f||^2 partial at [ldv]
        S_rows = h.laplacian_rows(row0, row0 + nrows)
        owner = np.searchsorted(off[1:-1], S_rows.col, side="right")
        colx = owner * S + (S_rows.col - off[owner])  # k_remap_cols
        own = owner == rank  # the owned slot's entries (k_own_count)
        real = np.zeros(ldv)
        real[:nrows] = 1.0
        u0 = real / np.sqrt(n)
        calls = {"allgather": 0, "allreduce": 0}

        def allgather(slot):
            calls["allgather"] += 1
            parts = [torch.zeros(S, dtype=torch.float64) for _ in range(WORLD)]
            dist.all_gather(parts, torch.from_numpy(np.ascontiguousarray(slot)))
            return torch.cat(parts).numpy()

        def allreduce(buf):
            calls["allreduce"] += 1
            t = torch.from_numpy(buf)
            dist.all_reduce(t)
            return t.numpy()

        # start vector (deflated), distributed; its setup collectives are not steps
        x0 = np.random.default_rng(1).uniform(-0.5, 0.5, n)
        f = np.zeros(ldv)
        f[:nrows] = x0[row0: row0 + nrows]
        f -= (allreduce(np.array([u0 @ f]))[0]) * u0
        V, alpha, beta = [], [], []
        base = dict(calls)
        for i in range(STEPS):
            slot = np.zeros(S)
            slot[:ldv] = f
            slot[ldv] = f @ f                          # this rank's ||f||^2 partial
            x = allgather(slot)                        # collective 1
            fn2 = sum(x[r * S + ldv] for r in range(WORLD))  # rank order: same bits on every rank
            b_prev = np.sqrt(fn2)
            v = f / b_prev
            # the overlapped SpMV (ctx.cpp factorize_mr): the owned slot's
            # entries summed from f itself (while the all-gather is in flight),
            # the halo's from the gathered x, the row sum starting from the
            # owned part, then scaled by 1/||f||
            rp64 = S_rows.rowptr.astype(np.int64)
            y_own = _local_spmv(rp64, np.where(own, colx - rank * S, 0), np.where(own, S_rows.val, 0.0), f)
            y_halo = _local_spmv(rp64, colx, np.where(own, 0.0, S_rows.val), x)
            w = np.zeros(ldv)
            w[:nrows] = (y_own + y_halo) / b_prev
            V.append(v)
            if i > 0:
                beta.append(b_prev)
            vim1 = V[-2] if i > 0 else v
            P = np.concatenate([[q @ y for q in V] + [u0 @ y] for y in (w, v, vim1)])
            P = allreduce(P)                           # collective 2
            tot = i + 2
            Pw, Pv, Pm = P[:tot], P[tot:2 * tot], P[2 * tot:]
            a = Pw[i]
            bb = b_prev if i > 0 else 0.0
            hcoef = Pw - a * Pv - bb * Pm
            fp = w - a * v - (bb * vim1 if i > 0 else 0.0)
            f = fp - sum(hj * q for hj, q in zip(hcoef[:-1], V)) - hcoef[-1] * u0
            alpha.append(a + hcoef[i])
        steps_calls = {k: calls[k] - base[k] for k in calls}
        fn2_last = allreduce(np.array([f @ f]))[0]
        beta.append(np.sqrt(fn2_last))
        a1, b1 = _lanczos_single(lambda y: _local_spmv(L.rowptr.astype(np.int64), L.col, L.val, y), n, x0, STEPS)
        # the sharded SpMV through the padded layout == the full SpMV's rows
        xs = np.zeros(WORLD * S)
        for r in range(WORLD):
            xs[r * S: r * S + off[r + 1] - off[r]] = x0[off[r]: off[r + 1]]
        y_sh = _local_spmv(S_rows.rowptr.astype(np.int64), colx, S_rows.val, xs)
        y_ref = _local_spmv(L.rowptr.astype(np.int64), L.col, L.val, x0)[row0: row0 + nrows]
        out[rank] = {"spmv_err": float(np.abs(y_sh - y_ref).max()), "da": float(np.abs(np.array(alpha) - a1).max()),
                     "db": float(np.abs(np.array(beta) - b1).max()), "calls": steps_calls, "nrows": nrows,
                     "alpha": np.array(alpha).tobytes()}
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_sharded_lanczos_two_collectives_per_step():
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(_free_port(), out), nprocs=WORLD, join=True)
    for r in range(WORLD):
        o = out[r]
        assert o["spmv_err"] <= 1e-13
        assert o["da"] <= 1e-10 and o["db"] <= 1e-10, (o["da"], o["db"])
        assert o["calls"] == {"allgather": STEPS, "allreduce": STEPS}  # one of each per step
    assert out[0]["alpha"] == out[1]["alpha"]  # the same projected matrix on every rank
    assert out[0]["nrows"] != out[1]["nrows"]  # nnz-balanced slices are unequal


def test_shard_map_is_what_the_library_enforces():
    ek = load_package()
    h = ek.Hypergraph.generate(0.25, 3)
    for world in (2, 4, 8):
        off = ek.shard_map(h, world)
        assert off[0] == 0 and off[-1] == h.nodes and np.all(np.diff(off) > 0)
    n = 201920
    for world in (2, 4, 8):  # the equal map stays available (ek_spmv_setup accepts any tiling)
        slices = [ek.shard_rows(n, world, r) for r in range(world)]
        nloc = slices[0][2]
        assert all(s[2] == nloc for s in slices)
        assert nloc * world >= n and nloc * (world - 1) < n
        assert sum(s[1] for s in slices) == n


def _halo_worker(rank, world, port, out):
    """ctx.cpp halo_build / halo_exchange restated: the request lists from the
    slot-layout columns, one all-gather of the counts and one of the lists
    (setup), then per step ONE exchange of packed messages (here the
    host-staged form: an all-gather of every rank's padded messages, of which
    each rank copies its one piece per peer) into the compact x whose block q
    is q's message as sent: the rows of q this rank reads, then q's ||f||^2
    partial at the block end (RCCL: one ncclSend / ncclRecv per peer)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ek = load_package()
        h = ek.Hypergraph.generate(0.05, 3)
        n = h.nodes
        L = h.laplacian()
        off = ek.shard_map(h, world)
        row0, nrows = int(off[rank]), int(off[rank + 1] - off[rank])
        ldv = -(-int(np.diff(off).max()) // 1024) * 1024
        S = ldv + 64
        Sr = h.laplacian_rows(row0, row0 + nrows)
        owner = np.searchsorted(off[1:-1], Sr.col, side="right")
        colx = owner * S + (Sr.col - off[owner])

        def ag(a):
            parts = [torch.zeros(len(a), dtype=torch.float64) for _ in range(world)]
            dist.all_gather(parts, torch.from_numpy(np.ascontiguousarray(a, np.float64)))
            return np.stack([p.numpy() for p in parts])

        req = [np.unique(Sr.col[owner == q]) - off[q] if q != rank else np.zeros(0, np.int64) for q in range(world)]
        C = ag(np.array([len(r) for r in req], np.float64)).astype(np.int64)  # C[r, q]
        lmax = max(1, max(sum(C[r, q] for q in range(world) if q != r) for r in range(world)))
        mine = np.zeros(lmax)
        cat = np.concatenate([req[q] for q in range(world)]) if world > 1 else np.zeros(0)
        mine[:len(cat)] = cat
        lall = ag(mine).astype(np.int64)
        # send lists: rank r's request from this rank inside r's list
        sidx = []
        for r in range(world):
            if r == rank:
                continue
            o = sum(C[r, q] for q in range(rank) if q != r)
            sidx += list(lall[r, o:o + C[r, rank]]) + [ldv]
        sidx = np.array(sidx, np.int64)
        rcnt = [nrows if q == rank else C[rank, q] for q in range(world)]
        base = np.concatenate([[0], np.cumsum(np.array(rcnt) + 1)])  # each block: rows, then the partial
        pidx = base[:-1] + np.array(rcnt)
        src = []
        smax = 1
        for q in range(world):
            o = 0
            for r in range(world):
                if r == q:
                    continue
                if r == rank:
                    src.append(o)
                o += C[r, q] + 1
            if q == rank:
                src.append(0)
            smax = max(smax, o)
        # the compact column map (monotone)
        pos = [dict((int(l), k) for k, l in enumerate(req[q])) for q in range(world)]
        colh = np.array([base[q] + (c - q * S if q == rank else pos[q][c - q * S])
                         for q, c in zip(colx // S, colx)], np.int64)
        rp = Sr.rowptr.astype(np.int64)
        for r_ in range(nrows):  # rows stay sorted
            seg = colh[rp[r_]:rp[r_ + 1]]
            assert np.all(np.diff(seg) > 0)
        # one step's exchange of a vector f (its partial at f[ldv])
        x0 = np.random.default_rng(5).standard_normal(n)
        f = np.zeros(S)
        f[:nrows] = x0[row0: row0 + nrows]
        f[ldv] = f[:nrows] @ f[:nrows]
        sbuf = np.zeros(smax)
        sbuf[:len(sidx)] = f[sidx]                        # k_halo_pack (messages)
        X = np.zeros(base[-1])
        X[base[rank]: base[rank] + nrows] = f[:nrows]      # ... the own block and partial
        X[pidx[rank]] = f[ldv]
        g = ag(sbuf)                                       # the step's one exchange
        pieces = 0
        for q in range(world):
            if q != rank:                                  # one piece per peer: rows + partial
                X[base[q]: base[q + 1]] = g[q, src[q]: src[q] + rcnt[q] + 1]
                pieces += 1
        P = X[pidx]                                        # the SpMV prologue reads them at the block ends
        # the same products in the same order: y bit-equal to the slot layout's
        xs = np.zeros(world * S)
        for q in range(world):
            xs[q * S: q * S + off[q + 1] - off[q]] = x0[off[q]: off[q + 1]]
        y_slot = _local_spmv(rp, colx, Sr.val, xs)
        y_halo = _local_spmv(rp, colh, Sr.val, X)
        parts = list(P)
        out[rank] = {"same_bits": y_slot.tobytes() == y_halo.tobytes(),
                     "partials": [float(p) for p in parts], "pieces": pieces,
                     "own_partial": float(f[ldv]),
                     "recv": int(sum(rcnt[q] + 1 for q in range(world) if q != rank)),
                     "recv_full": int((world - 1) * S)}
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_halo_exchange_layout(world):
    """The compact halo layout gives the slot layout's SpMV bit for bit, and
    every rank reads every rank's ||f||^2 partial (the same values, rank
    order) out of the blocks it received."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_halo_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        assert out[r]["same_bits"], out[r]
        assert out[r]["partials"] == out[0]["partials"]
        assert out[r]["partials"][r] == out[r]["own_partial"]
        assert out[r]["pieces"] == world - 1  # one message from every peer
        assert out[r]["recv"] <= out[r]["recv_full"]


def test_bench_collectives_on_every_rank():
    """bench.py at N > 1: every collective (max_over_ranks, barrier, dist.*)
    must run on every rank in the same order, so none may sit under a
    condition that differs between ranks.  A static check of the script: a
    collective's enclosing ifs may test only rank-independent names (world,
    args, extras, the loop index, comm), or `... or world > 1` (every rank
    enters at N > 1).  Round 6 had one under `if us10_rp:` (rank 0's rocprof
    result), and the N = 2 run died with its ranks' all-reduces paired wrongly."""
    import ast
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")
    tree = ast.parse(open(path).read())
    parents = {ch: node for node in ast.walk(tree) for ch in ast.iter_child_nodes(node)}
    allowed = {"world", "args", "extras", "i", "comm"}

    def all_ranks_enter(test):  # `x or world > 1`
        return isinstance(test, ast.BoolOp) and isinstance(test.op, ast.Or) and any(
            isinstance(v, ast.Compare) and isinstance(v.left, ast.Name) and v.left.id == "world" for v in test.values)

    bad = []
    for node in ast.walk(tree):
        if not isinstance(node, ast.Call):
            continue
        f = node.func
        is_dist = isinstance(f, ast.Attribute) and isinstance(f.value, ast.Name) and f.value.id == "dist"
        if not (isinstance(f, ast.Name) and f.id in ("max_over_ranks", "barrier")) and not is_dist:
            continue
        if is_dist and f.attr in ("destroy_process_group", "init_process_group"):
            continue  # (setup and teardown: outside the measured sequence)
        p = parents.get(node)
        while p is not None and not isinstance(p, ast.FunctionDef):
            if isinstance(p, ast.If) and not all_ranks_enter(p.test):
                extra = {n.id for n in ast.walk(p.test) if isinstance(n, ast.Name)} - allowed
                if extra:
                    bad.append((node.lineno, sorted(extra)))
            p = parents.get(p)
    assert not bad, f"collectives under rank-dependent conditions (line, names): {bad}"
