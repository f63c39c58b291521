"""The Laplacian assembled on the GPU from the pins (ek_spmv_setup_pins,
kernels_build.hip) against the host build (ek_laplacian_build +
ek_spmv_setup, itself pinned to the oracle's std::map build of cEIG.cpp:86-133
in test_host_logic): the same values in the same row blocks, so every SpMV
and the whole Lanczos run must be bit-identical, on every circuit shape —
short rows (per-thread sort), industry2's long rows (the workgroup LDS sort),
a net too large for it (host fallback), repeated pins, and a shard's rows."""
import numpy as np
import pytest

from conftest import circuit_path

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctxs(ek):
    a, b = ek.Context(0), ek.Context(0)
    yield a, b
    a.close()
    b.close()


def _host_rows(ek, ctx, h):
    L = h.laplacian()
    ctx.spmv_setup(h.nodes, 0, L.rowptr, L.col, L.val)
    return L


@pytest.mark.parametrize("which", ["fract", "ibm01", "industry2", "ibm10", "syn0.25", "syn1"])
def test_device_build_bit_identical(ek, ctxs, which):
    dev_ctx, host_ctx = ctxs
    h = ek.Hypergraph.generate(float(which[3:]), 7) if which.startswith("syn") else ek.Hypergraph.read(circuit_path(which))
    _host_rows(ek, host_ctx, h)
    assert dev_ctx.spmv_setup_pins(h) is True
    assert dev_ctx.spmv_format() == host_ctx.spmv_format()  # same coding decision, same stored bytes
    assert dev_ctx.spmv_bytes() == host_ctx.spmv_bytes()
    x = np.random.default_rng(5).standard_normal(h.nodes)
    y_dev, y_host = dev_ctx.spmv_host(x), host_ctx.spmv_host(x)
    assert np.array_equal(y_dev.view(np.uint64), y_host.view(np.uint64))
    if which in ("ibm01", "industry2", "syn0.25"):
        a, b = dev_ctx.lanczos_fiedler(), host_ctx.lanczos_fiedler()
        assert a[0] == b[0] and a[2]["matvecs"] == b[2]["matvecs"]
        assert np.array_equal(a[1], b[1])


def test_device_build_plain_form_and_fallbacks(ek, ctxs, monkeypatch):
    dev_ctx, host_ctx = ctxs
    h = ek.Hypergraph.read(circuit_path("ibm01"))
    x = np.random.default_rng(9).standard_normal(h.nodes)
    _host_rows(ek, host_ctx, h)
    y_ref = host_ctx.spmv_host(x)
    monkeypatch.setenv("EK_SPMV_PLAIN", "1")  # plain CSR read straight from the device-built arrays
    assert dev_ctx.spmv_setup_pins(h) is True and dev_ctx.spmv_format()[0] is False
    _host_rows(ek, host_ctx, h)
    assert np.array_equal(dev_ctx.spmv_host(x).view(np.uint64), host_ctx.spmv_host(x).view(np.uint64))
    monkeypatch.delenv("EK_SPMV_PLAIN")
    monkeypatch.setenv("EK_HOST_LAPLACIAN", "1")
    assert dev_ctx.spmv_setup_pins(h) is False
    assert np.array_equal(dev_ctx.spmv_host(x).view(np.uint64), y_ref.view(np.uint64))
    monkeypatch.delenv("EK_HOST_LAPLACIAN")
    # a 9,000-pin net: its rows exceed the LDS sort -> host build, same result
    rng = np.random.default_rng(3)
    n = 20000
    nets = [np.sort(rng.choice(n, 9000, replace=False))] + [np.sort(rng.choice(n, 3, replace=False)) for _ in range(30000)]
    net_ptr = np.concatenate([[0], np.cumsum([len(e) for e in nets])]).astype(np.int64)
    big = ek.Hypergraph.from_pins(n, net_ptr, np.concatenate(nets).astype(np.int32))
    assert dev_ctx.spmv_setup_pins(big) is False
    _host_rows(ek, host_ctx, big)
    x = rng.standard_normal(n)
    assert np.array_equal(dev_ctx.spmv_host(x).view(np.uint64), host_ctx.spmv_host(x).view(np.uint64))


def test_device_build_repeated_pins_and_edge_nets(ek, ctxs):
    dev_ctx, host_ctx = ctxs
    net_ptr = np.array([0, 3, 4, 4, 6, 9, 11], np.int64)
    pins = np.array([0, 1, 1, 2, 3, 4, 5, 6, 0, 6, 7], np.int32)
    h = ek.Hypergraph.from_pins(9, net_ptr, pins)
    _host_rows(ek, host_ctx, h)
    assert dev_ctx.spmv_setup_pins(h) is True
    x = np.random.default_rng(1).standard_normal(9)
    assert np.array_equal(dev_ctx.spmv_host(x).view(np.uint64), host_ctx.spmv_host(x).view(np.uint64))


@pytest.mark.parametrize("ranks", [2, 3])
def test_device_build_shard_rows(ek, ctxs, ranks, monkeypatch):
    """A rank's shard built on the device equals the same rows of the full
    matrix (host build); the collectives are never reached by a plain SpMV.
    (EK_MR_HALO=0: the halo layout's setup all-gathers the ranks' requests,
    which one process playing every rank in turn cannot answer.)"""
    monkeypatch.setenv("EK_MR_HALO", "0")
    dev_ctx, host_ctx = ctxs
    h = ek.Hypergraph.read(circuit_path("industry2"))
    n = h.nodes
    _host_rows(ek, host_ctx, h)
    x = np.random.default_rng(2).standard_normal(n)
    y_full = host_ctx.spmv_host(x)

    def never(*_):
        raise AssertionError("no collective expected")

    try:
        off = ek.shard_map(h, ranks)  # the nnz-balanced map the device build uses
        for r in range(ranks):
            dev_ctx.comm_init_host(ranks, r, never, never)
            assert dev_ctx.spmv_setup_pins(h) is True
            row0, nrows = int(off[r]), int(off[r + 1] - off[r])
            assert dev_ctx.spmv_dims() == (n, row0, nrows)
            y = dev_ctx.spmv_host(x)
            S = h.laplacian_rows(row0, row0 + nrows)
            absrow = np.add.reduceat(np.abs(S.val * x[S.col]), S.rowptr[:-1])
            assert np.all(np.abs(y - y_full[row0: row0 + nrows]) <= 1e-14 * absrow + 1e-300)
    finally:
        dev_ctx.comm_init_host(1, 0, never, never)


def test_device_build_rejects_bad_pins(ek, ctxs):
    """ek_spmv_setup_pins validates its input before any upload: a pin outside
    [0, n) (reported with the first offender's value) or a decreasing net_ptr
    is EK_EINVAL, and the context then still builds a valid matrix."""
    import ctypes
    lib = ek._lib
    ctx, _ = ctxs
    dev = ctypes.c_int32(0)

    def setup(n, net_ptr, pins):
        net_ptr = np.ascontiguousarray(net_ptr, np.int64)
        pins = np.ascontiguousarray(pins, np.int32)
        rc = lib.ek_spmv_setup_pins(ctx._c, n, len(net_ptr) - 1, ek._p(net_ptr), ek._p(pins), ctypes.byref(dev))
        return rc, lib.ek_last_error().decode(errors="replace")

    rc, msg = setup(4, [0, 2, 4], [0, 1, 2, 7])
    assert rc == ek.EK_EINVAL and "pin 7 out of range" in msg
    rc, msg = setup(4, [0, 2, 4], [0, -3, 2, 9])
    assert rc == ek.EK_EINVAL and "pin -3 out of range" in msg
    rc, msg = setup(4, [0, 3, 2, 4], [0, 1, 2, 3])
    assert rc == ek.EK_EINVAL and "not monotone" in msg
    h = ek.Hypergraph.read(circuit_path("fract"))
    assert ctx.spmv_setup_pins(h) is True
