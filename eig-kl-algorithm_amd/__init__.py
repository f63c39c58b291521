"""eig-kl-algorithm_amd — Python mirror of the MI355X EIG+KL bipartitioner.

A thin ctypes layer over ``build/libeigkl_hip.so`` (C-ABI: include/eigkl.h).
It mirrors the reference's surface (yhinai/EIG-KL-Algorithm):

* ``cEIG(path)``, ``cKL(path, EIG=False)``, ``gKL(...)``, ``gKL2(...)`` run the
  drop-in tools in-process with the reference's argv/CWD semantics
  (cEIG.cpp:138-237, cKL.cpp:424-468, gKL.cu:672-713, gKL2.cu:989-1033);
* ``Hypergraph`` (read / generate / clique expansions), ``Context`` (SpMV seam,
  Lanczos Fiedler solver, KL swap loop) expose the hot path piecewise.

There is no CPU fallback: importing fails loudly when the HIP library has not
been built, and GPU calls raise ``EKError`` when no gfx950 device is usable.
The directory name is not a Python identifier; load it with
``importlib`` (see ``load()`` in tests/conftest.py or __graft_entry__.py).
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# EK_LIB_PATH: a design lab's A/B build of the same library (profiles/r03/scripts/ab_lab.sh)
LIB_PATH = os.environ.get("EK_LIB_PATH") or os.path.join(HERE, "build", "libeigkl_hip.so")
BIN_DIR = os.path.join(HERE, "build", "bin")

if not os.path.exists(LIB_PATH):
    raise ImportError(f"{LIB_PATH} is not built: run `make -C {HERE}` "
                      "(the HIP path has no CPU fallback)")

_lib = ctypes.CDLL(LIB_PATH)
_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int32

EK_OK, EK_EINVAL, EK_EIO, EK_EHIP, EK_ENOMEM, EK_ENOCONV, EK_ESTATE, EK_ECOMM = 0, -1, -2, -3, -4, -5, -6, -7

SWAP_DTYPE = np.dtype([("iter", "<u4"), ("node_left", "<u4"), ("node_right", "<u4"),
                       ("max_gain", "<f4"), ("min_gain", "<f4"), ("gain", "<f4"),
                       ("cut", "<f4"), ("pad", "<u4")])


class _AbiStruct(ctypes.Structure):
    """A mirror of an eigkl.h struct (layout ABI_VERSION): refused against a
    library that cannot state its ABI (an older EK_LIB_PATH lab build)."""

    def __init__(self, *a, **k):
        if not _ABI_CHECKED:
            raise RuntimeError(f"{type(self).__name__}: {_lib._name} has no ek_abi_version, its layout is unknown")
        super().__init__(*a, **k)


class LanczosOpts(_AbiStruct):
    _fields_ = [("ncv", _I32), ("maxit", _I32), ("tol", ctypes.c_double), ("deflate", _I32),
                ("time_spmv", _I32), ("reorth", _I32), ("check_every", _I32), ("basis32", _I32),
                ("alpha_last", _I32), ("keep_min", _I32), ("reorth_thresh", ctypes.c_double)]


class LanczosStats(_AbiStruct):
    _fields_ = [("restarts", _I32), ("matvecs", _I32), ("converged", _I32), ("residual", ctypes.c_double),
                ("total_ms", ctypes.c_double), ("spmv_ms", ctypes.c_double), ("spmv_timed", _I32),
                ("comm_ms", ctypes.c_double), ("allgathers", _I32), ("allreduces", _I32),
                ("update32_steps", _I32), ("update32_fallbacks", _I32), ("projected_steps", _I32),
                ("reprojected", _I32), ("ortho_max", ctypes.c_double)]


class KLResult(_AbiStruct):
    _fields_ = [("iterations", _I64), ("initial_cut", ctypes.c_float), ("best_cut", ctypes.c_float),
                ("final_cut", ctypes.c_float), ("best_iter", _I64), ("net_cut_initial", _I64),
                ("net_cut_best", _I64), ("net_cut_final", _I64), ("loop_ms", ctypes.c_double),
                ("total_ms", ctypes.c_double)]


class SolveOpts(_AbiStruct):
    _fields_ = [("eig", _I32), ("seed", ctypes.c_uint32), ("write_results", _I32), ("limit", _I32),
                ("out_dir", ctypes.c_char_p), ("sign_ref", ctypes.c_char_p), ("lanczos", LanczosOpts)]


_SOLVE_TIMES = ("t_read", "t_laplacian", "t_lanczos", "t_split", "t_kl_graph_wait", "t_kl_setup", "t_kl",
                "t_write", "t_total", "t_spmv_setup")


class SolveResult(_AbiStruct):
    _fields_ = ([("nets", _I64), ("nodes", _I64), ("pins", _I64), ("lambda_", ctypes.c_double),
                 ("median", ctypes.c_double), ("lanczos", LanczosStats), ("kl", KLResult)]
                + [(k, ctypes.c_double) for k in _SOLVE_TIMES])


ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), _I64,
                                ctypes.POINTER(ctypes.c_double))
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), _I64)


def _sig(name, res, *args):
    try:
        fn = getattr(_lib, name)
    except AttributeError:
        if os.environ.get("EK_LIB_PATH"):  # (a lab's older A/B build: the entry is simply absent)
            return None
        raise
    fn.restype = res
    fn.argtypes = list(args)
    return fn


_sig("ek_last_error", ctypes.c_char_p)
_sig("ek_version", ctypes.c_char_p)
ABI_VERSION = 4  # eigkl.h EIGKL_ABI_VERSION: the ctypes struct mirrors below follow that layout
if _sig("ek_abi_version", ctypes.c_int) is not None:
    if _lib.ek_abi_version() != ABI_VERSION:
        raise ImportError(f"libeigkl_hip ABI {_lib.ek_abi_version()} != the {ABI_VERSION} these bindings mirror: rebuild")
    _ABI_CHECKED = True
else:
    # an EK_LIB_PATH lab build older than the ABI query: its struct layouts are
    # unknown, so every entry that takes one of the mirrors below refuses
    import warnings
    warnings.warn(f"{_lib._name} has no ek_abi_version: calls passing ABI-{ABI_VERSION} structs are refused")
    _ABI_CHECKED = False
_sig("ek_hgr_read", ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(_P))
_sig("ek_hgr_generate", ctypes.c_int, ctypes.c_double, ctypes.c_uint64, ctypes.POINTER(_P))
_sig("ek_hgr_from_pins", ctypes.c_int, _I64, _I64, _P, _P, ctypes.POINTER(_P))
_sig("ek_hgr_write", ctypes.c_int, _P, ctypes.c_char_p)
_sig("ek_hgr_dims", ctypes.c_int, _P, ctypes.POINTER(_I64), ctypes.POINTER(_I64), ctypes.POINTER(_I64))
_sig("ek_hgr_copy_pins", ctypes.c_int, _P, _P, _P)
_sig("ek_hgr_free", None, _P)
_sig("ek_laplacian_build", ctypes.c_int, _P, ctypes.POINTER(_P))
_sig("ek_kl_graph_build", ctypes.c_int, _P, ctypes.POINTER(_P))
_sig("ek_laplacian_build_rows", ctypes.c_int, _P, _I64, _I64, ctypes.POINTER(_P))
_sig("ek_synchronize", ctypes.c_int, _P)
_sig("ek_csr_dims", ctypes.c_int, _P, ctypes.POINTER(_I64), ctypes.POINTER(_I64), ctypes.POINTER(_I32))
_sig("ek_csr_copy", ctypes.c_int, _P, _P, _P, _P, _P)
_sig("ek_csr_free", None, _P)
_sig("ek_shard_rows", ctypes.c_int, _I64, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_I64),
     ctypes.POINTER(_I64), ctypes.POINTER(_I64))
_sig("ek_shard_map", ctypes.c_int, _I64, _I64, _P, _P, ctypes.c_int, _P)
_sig("ek_device_count", ctypes.c_int, ctypes.POINTER(ctypes.c_int))
_sig("ek_init", ctypes.c_int, ctypes.c_int, ctypes.POINTER(_P))
_sig("ek_destroy", None, _P)
_sig("ek_get_stream", ctypes.c_int, _P, ctypes.POINTER(_P))
_sig("ek_comm_unique_id", ctypes.c_int, _P)
_sig("ek_comm_init", ctypes.c_int, _P, ctypes.c_int, ctypes.c_int, _P)
_sig("ek_comm_init_host", ctypes.c_int, _P, ctypes.c_int, ctypes.c_int, ALLGATHER_FN, ALLREDUCE_FN, _P)
_sig("ek_hgr_largest_component", ctypes.c_int, _P, ctypes.POINTER(_P), _P)
_sig("ek_random_split", ctypes.c_int, _I64, ctypes.c_uint32, _P, _P)
_sig("ek_solve_default_opts", None, ctypes.POINTER(SolveOpts))
_sig("ek_solve_file", ctypes.c_int, _P, ctypes.c_char_p, ctypes.POINTER(SolveOpts), _P, _I64,
     ctypes.POINTER(SolveResult))
_sig("ek_spmv_setup", ctypes.c_int, _P, _I64, _I64, _I64, _P, _P, _P)
_sig("ek_spmv", ctypes.c_int, _P, _P, _P, _P)
_sig("ek_spmv_setup_pins", ctypes.c_int, _P, _I64, _I64, _P, _P, ctypes.POINTER(ctypes.c_int32))
_sig("ek_spmv_host", ctypes.c_int, _P, _P, _P)
_sig("ek_spmv_bytes", _I64, _P)
_sig("ek_spmv_dims", ctypes.c_int, _P, ctypes.POINTER(_I64), ctypes.POINTER(_I64), ctypes.POINTER(_I64))
_sig("ek_spmv_format", ctypes.c_int, _P, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(_I64))
_sig("ek_spmv_exchange", ctypes.c_int, _P, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(_I64), ctypes.POINTER(_I64))
_sig("ek_comm_stats", ctypes.c_int, _P, ctypes.POINTER(_I64), ctypes.POINTER(_I64), ctypes.POINTER(_I64),
     ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_I64), ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_I64))
_sig("ek_spmv_gather_bench", ctypes.c_int, _P, ctypes.c_int, ctypes.POINTER(ctypes.c_double))
_sig("ek_spmv_bench", ctypes.c_int, _P, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double))
_sig("ek_lanczos_default_opts", None, ctypes.POINTER(LanczosOpts))
_sig("ek_lanczos_fiedler", ctypes.c_int, _P, ctypes.POINTER(LanczosOpts), ctypes.POINTER(ctypes.c_double), _P,
     ctypes.POINTER(LanczosStats))
_sig("ek_median_split", ctypes.c_int, _I64, _P, ctypes.POINTER(ctypes.c_double), _P)
_sig("ek_align_sign", ctypes.c_int, _I64, _P, _P)
_sig("ek_eig_write", ctypes.c_int, ctypes.c_char_p, _I64, ctypes.c_double, ctypes.c_double, _P, _P)
_sig("ek_eig_read", ctypes.c_int, ctypes.c_char_p, _I64, ctypes.POINTER(ctypes.c_double),
     ctypes.POINTER(ctypes.c_double), _P, _P, _P, ctypes.POINTER(_I64), _P, ctypes.POINTER(_I64))
_sig("ek_kl_graph_setup", ctypes.c_int, _P, _I64, _P, _P, _P)
_sig("ek_kl_nets_setup", ctypes.c_int, _P, _I64, _P, _P)
_sig("ek_kl_set_partition", ctypes.c_int, _P, _P, _I64, _P, _I64)
_sig("ek_kl_set_partition_bits", ctypes.c_int, _P, _I64, _P)
_sig("ek_kl_set_partition_fiedler", ctypes.c_int, _P, _P, _P, _P)
_sig("ek_kl_run", ctypes.c_int, _P, _I32, _P, _I64, ctypes.POINTER(KLResult))
_sig("ek_kl_sides", ctypes.c_int, _P, _I32, _P)
_sig("ek_cli_main", ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p))

lib = _lib


class EKError(RuntimeError):
    def __init__(self, code, what):
        super().__init__(f"{what}: {_lib.ek_last_error().decode(errors='replace')} (status {code})")
        self.code = code


def _chk(rc, what):
    if rc != EK_OK:
        raise EKError(rc, what)


def _p(a):
    return a.ctypes.data_as(_P) if a is not None else None


def version():
    return _lib.ek_version().decode()


# ---------------------------------------------------------------------------
# host side
class CSR:
    def __init__(self, rowptr, col, val, nfwd=None):
        self.rowptr, self.col, self.val, self.nfwd = rowptr, col, val, nfwd

    @property
    def nrows(self):
        return len(self.rowptr) - 1

    @property
    def nnz(self):
        return len(self.col)


def _take_csr(handle):
    nr, nnz, vb = _I64(), _I64(), _I32()
    _lib.ek_csr_dims(handle, ctypes.byref(nr), ctypes.byref(nnz), ctypes.byref(vb))
    rowptr = np.empty(nr.value + 1, np.int32)
    col = np.empty(nnz.value, np.int32)
    val = np.empty(nnz.value, np.float64 if vb.value == 8 else np.float32)
    nfwd = np.empty(nr.value, np.int32) if vb.value == 4 else None
    _lib.ek_csr_copy(handle, _p(rowptr), _p(col), _p(val), _p(nfwd))
    _lib.ek_csr_free(handle)
    return CSR(rowptr, col, val, nfwd)


class Hypergraph:
    """A .hgr circuit (cKL.cpp:84-116 / cEIG.cpp:177-182 readers)."""

    def __init__(self, handle):
        self._h = handle

    @classmethod
    def read(cls, path):
        h = _P()
        _chk(_lib.ek_hgr_read(os.fsencode(path), ctypes.byref(h)), f"read {path}")
        return cls(h)

    @classmethod
    def generate(cls, multiplier=1.0, seed=1):
        """Seeded ISPD98-shaped synthetic circuit (circuit_generator.py:41-59)."""
        h = _P()
        _chk(_lib.ek_hgr_generate(float(multiplier), int(seed), ctypes.byref(h)), "generate")
        return cls(h)

    @classmethod
    def from_pins(cls, nodes, net_ptr, pins):
        net_ptr = np.ascontiguousarray(net_ptr, np.int64)
        pins = np.ascontiguousarray(pins, np.int32)
        h = _P()
        _chk(_lib.ek_hgr_from_pins(len(net_ptr) - 1, int(nodes), _p(net_ptr), _p(pins), ctypes.byref(h)),
             "from_pins")
        return cls(h)

    def __del__(self):
        if getattr(self, "_h", None):
            _lib.ek_hgr_free(self._h)
            self._h = None

    def dims(self):
        a, b, c = _I64(), _I64(), _I64()
        _lib.ek_hgr_dims(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
        return a.value, b.value, c.value

    @property
    def nets(self):
        return self.dims()[0]

    @property
    def nodes(self):
        return self.dims()[1]

    def pins(self):
        nets, _, npins = self.dims()
        net_ptr = np.empty(nets + 1, np.int64)
        pins = np.empty(npins, np.int32)
        _lib.ek_hgr_copy_pins(self._h, _p(net_ptr), _p(pins))
        return net_ptr, pins

    def write(self, path):
        _chk(_lib.ek_hgr_write(self._h, os.fsencode(path)), f"write {path}")

    def largest_component(self):
        """(Hypergraph of the largest connected component, node map old -> new or -1)."""
        c = _P()
        m = np.empty(self.nodes, np.int32)
        _chk(_lib.ek_hgr_largest_component(self._h, ctypes.byref(c), _p(m)), "largest_component")
        return Hypergraph(c), m

    def laplacian(self):
        """fp64 clique Laplacian (cEIG.cpp:86-133)."""
        c = _P()
        _chk(_lib.ek_laplacian_build(self._h, ctypes.byref(c)), "laplacian")
        return _take_csr(c)

    def laplacian_rows(self, row0, row1):
        """Rows [row0, row1) of the Laplacian (global columns, rowptr from 0): one rank's shard."""
        c = _P()
        _chk(_lib.ek_laplacian_build_rows(self._h, int(row0), int(row1 - row0), ctypes.byref(c)), "laplacian_rows")
        return _take_csr(c)

    def kl_graph(self):
        """fp32 KL adjacency in cKL summation order (cKL.cpp:84-149, 225-251)."""
        c = _P()
        _chk(_lib.ek_kl_graph_build(self._h, ctypes.byref(c)), "kl_graph")
        return _take_csr(c)


def shard_rows(n, nranks, rank):
    a, b, c = _I64(), _I64(), _I64()
    _chk(_lib.ek_shard_rows(int(n), int(nranks), int(rank), ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)),
         "shard_rows")
    return a.value, b.value, c.value


def shard_map(hgr, nranks):
    """nnz-balanced row offsets (nranks + 1) of the sharded Lanczos (ek_shard_map): rank r owns
    [off[r], off[r+1]); the map ek_spmv_setup_pins uses."""
    net_ptr, pins = hgr.pins()
    off = np.empty(int(nranks) + 1, np.int64)
    _chk(_lib.ek_shard_map(int(hgr.nodes), len(net_ptr) - 1, _p(net_ptr), _p(pins), int(nranks), _p(off)),
         "shard_map")
    return off


def median_split(v):
    """cEIG.cpp:55-65, 218: median and bits = (median > v)."""
    v = np.ascontiguousarray(v, np.float64)
    med = ctypes.c_double()
    bits = np.empty(len(v), np.uint8)
    _chk(_lib.ek_median_split(len(v), _p(v), ctypes.byref(med), _p(bits)), "median_split")
    return med.value, bits


def eig_write(path, lam, median, bits, v):
    bits = np.ascontiguousarray(bits, np.uint8)
    v = np.ascontiguousarray(v, np.float64)
    _chk(_lib.ek_eig_write(os.fsencode(path), len(v), float(lam), float(median), _p(bits), _p(v)), "eig_write")


def eig_read(path, n):
    """pre_saved_EIG file as cKL reads it (cKL.cpp:155-174)."""
    lam, med = ctypes.c_double(), ctypes.c_double()
    bits = np.zeros(n, np.uint8)
    v = np.zeros(n, np.float64)
    o0 = np.empty(n, np.int32)
    o1 = np.empty(n, np.int32)
    n0, n1 = _I64(), _I64()
    _chk(_lib.ek_eig_read(os.fsencode(path), n, ctypes.byref(lam), ctypes.byref(med), _p(bits), _p(v), _p(o0),
                          ctypes.byref(n0), _p(o1), ctypes.byref(n1)), f"eig_read {path}")
    return lam.value, med.value, bits, v, o0[: n0.value].copy(), o1[: n1.value].copy()


def random_split(n, seed):
    """cKL.cpp:176-192 with std::mt19937(seed): (remain[0], remain[1])."""
    o0 = np.empty(n // 2, np.int32)
    o1 = np.empty(n - n // 2, np.int32)
    _chk(_lib.ek_random_split(int(n), int(seed) & 0xFFFFFFFF, _p(o0), _p(o1)), "random_split")
    return o0, o1


def device_count():
    c = ctypes.c_int()
    _lib.ek_device_count(ctypes.byref(c))
    return c.value


def comm_unique_id():
    buf = ctypes.create_string_buffer(128)
    _chk(_lib.ek_comm_unique_id(buf), "comm_unique_id")
    return bytes(buf.raw)


# ---------------------------------------------------------------------------
# GPU side
class Context:
    """One MI355X (gfx950) device: SpMV seam, Lanczos Fiedler solver, KL loop."""

    def __init__(self, device=0):
        self._c = _P()
        _chk(_lib.ek_init(int(device), ctypes.byref(self._c)), "ek_init")
        self.n = 0
        self.nrows = 0

    def close(self):
        if getattr(self, "_c", None):
            _lib.ek_destroy(self._c)
            self._c = None

    def __del__(self):
        self.close()

    def synchronize(self):
        _chk(_lib.ek_synchronize(self._c), "synchronize")

    @property
    def stream(self):
        s = _P()
        _chk(_lib.ek_get_stream(self._c, ctypes.byref(s)), "stream")
        return s.value

    def comm_init(self, nranks, rank, uid):
        """RCCL over xGMI (one process per GPU)."""
        buf = ctypes.create_string_buffer(bytes(uid), 128)
        _chk(_lib.ek_comm_init(self._c, int(nranks), int(rank), buf), "comm_init")

    def comm_init_host(self, nranks, rank, allgather, allreduce):
        """Host-staged exchange (ek_comm_init_host): allgather(send: ndarray) -> ndarray of nranks*len(send),
        allreduce(buf: ndarray) -> None (in-place sum), e.g. over torch.distributed gloo."""
        def ag(_user, send, count, recv):
            try:
                src = np.ctypeslib.as_array(send, shape=(count,))
                dst = np.ctypeslib.as_array(recv, shape=(count * nranks,))
                dst[:] = allgather(src.copy())
                return 0
            except Exception:  # a failed collective must not unwind through C
                import traceback
                traceback.print_exc()
                return 1

        def ar(_user, buf, count):
            try:
                allreduce(np.ctypeslib.as_array(buf, shape=(count,)))
                return 0
            except Exception:
                import traceback
                traceback.print_exc()
                return 1

        self._comm_cbs = (ALLGATHER_FN(ag), ALLREDUCE_FN(ar))  # kept alive with the context
        _chk(_lib.ek_comm_init_host(self._c, int(nranks), int(rank), self._comm_cbs[0], self._comm_cbs[1], None),
             "comm_init_host")

    # SpMV seam (SparseSymMatProd::perform_op, cEIG.cpp:194)
    def spmv_setup(self, n, row0, rowptr, col, val):
        rowptr = np.ascontiguousarray(rowptr, np.int32)
        col = np.ascontiguousarray(col, np.int32)
        val = np.ascontiguousarray(val, np.float64)
        nrows = len(rowptr) - 1
        _chk(_lib.ek_spmv_setup(self._c, int(n), int(row0), nrows, _p(rowptr), _p(col), _p(val)), "spmv_setup")
        self.n, self.nrows = int(n), nrows

    def spmv_setup_pins(self, hgr):
        """This context's Laplacian rows assembled on the GPU from the pins (ek_spmv_setup_pins);
        returns True when the device build ran (False: the host fallback)."""
        net_ptr, pins = hgr.pins()
        dev = ctypes.c_int32(0)
        _chk(_lib.ek_spmv_setup_pins(self._c, hgr.nodes, len(net_ptr) - 1, _p(net_ptr), _p(pins), ctypes.byref(dev)),
             "spmv_setup_pins")
        self.n, _, self.nrows = self.spmv_dims()
        return bool(dev.value)

    def spmv_host(self, x):
        x = np.ascontiguousarray(x, np.float64)
        y = np.empty(self.nrows, np.float64)
        _chk(_lib.ek_spmv_host(self._c, _p(x), _p(y)), "spmv")
        return y

    def spmv_device(self, x_ptr, y_ptr, stream=None):
        _chk(_lib.ek_spmv(self._c, x_ptr, y_ptr, stream), "spmv")

    def spmv_dims(self):
        """(n, row0, nrows) of the rows the context owns (ek_spmv_dims)."""
        n, r0, nr = _I64(), _I64(), _I64()
        _chk(_lib.ek_spmv_dims(self._c, ctypes.byref(n), ctypes.byref(r0), ctypes.byref(nr)), "spmv_dims")
        return n.value, r0.value, nr.value

    def spmv_bytes(self, fused=False):
        """Algorithmic bytes of one SpMV; fused: the Lanczos form (+ f read, basis column write)."""
        return _lib.ek_spmv_bytes(self._c) + (16 * self.spmv_dims()[2] if fused else 0)

    def spmv_format(self, fused=False):
        """(packed, stored bytes per launch): the storage the SpMV reads (ek_spmv_format)."""
        pk, b = ctypes.c_int32(0), _I64(0)
        _chk(_lib.ek_spmv_format(self._c, ctypes.byref(pk), ctypes.byref(b)), "ek_spmv_format")
        return bool(pk.value), int(b.value) + (16 * self.spmv_dims()[2] if fused else 0)

    def spmv_exchange(self):
        """(halo, doubles received, doubles sent) per sharded Lanczos step (ek_spmv_exchange)."""
        hl, rv, sd = ctypes.c_int32(0), _I64(0), _I64(0)
        _chk(_lib.ek_spmv_exchange(self._c, ctypes.byref(hl), ctypes.byref(rv), ctypes.byref(sd)), "ek_spmv_exchange")
        return bool(hl.value), int(rv.value), int(sd.value)

    def comm_stats(self):
        """The sharded solves' exchange accounting since the last setup (ek_comm_stats):
        exchanges of f, point-to-point messages sent / received, and the last timed
        (time_spmv) solve's exchange and all-reduce milliseconds with their counts."""
        e, sd, rv, xt, at = _I64(0), _I64(0), _I64(0), _I64(0), _I64(0)
        xm, am = ctypes.c_double(0.0), ctypes.c_double(0.0)
        _chk(_lib.ek_comm_stats(self._c, ctypes.byref(e), ctypes.byref(sd), ctypes.byref(rv), ctypes.byref(xm),
                                ctypes.byref(xt), ctypes.byref(am), ctypes.byref(at)), "ek_comm_stats")
        return {"exchanges": int(e.value), "sends": int(sd.value), "recvs": int(rv.value),
                "exchange_ms": xm.value, "exchanges_timed": int(xt.value), "allreduce_ms": am.value,
                "allreduces_timed": int(at.value)}

    def spmv_gather_bench(self, iters=200):
        """Average microseconds per launch of the SpMV's gather-only ceiling kernel (ek_spmv_gather_bench)."""
        us = ctypes.c_double()
        _chk(_lib.ek_spmv_gather_bench(self._c, int(iters), ctypes.byref(us)), "spmv_gather_bench")
        return us.value

    def spmv_bench(self, iters=200, fused=True):
        """Average microseconds per back-to-back SpMV launch on resident buffers."""
        us = ctypes.c_double()
        _chk(_lib.ek_spmv_bench(self._c, int(iters), int(fused), ctypes.byref(us)), "spmv_bench")
        return us.value

    def lanczos_fiedler(self, ncv=0, tol=1e-10, maxit=1000, deflate=True, time_spmv=False, reorth=3, check_every=8,
                        basis32=True, alpha_last=False, keep_min=-1, reorth_thresh=0.0):
        """Fiedler pair (Spectra SymEigsSolver(nev=2, ncv=min(100,n/2)), cEIG.cpp:194-207).  check_every: steps
        between mid-cycle convergence tests after the first cycle (0: at cycle ends only, Spectra's schedule).
        basis32: the update reads the basis's fp32 shadow when that is exact to fp64 rounding (ek_lanczos_opts).
        alpha_last: the SpMV's last workgroup reduces alpha (default: every projection workgroup does).
        keep_min: floor on the vectors an implicit restart keeps (-1: ncv/5, 0: Spectra's nev_adjusted alone).
        reorth: 3 partial reorthogonalisation (Simon's omega recurrence, threshold reorth_thresh, <= 0:
        1e-10), 1 full (every step), 2 CGS2."""
        o = LanczosOpts(int(ncv), int(maxit), float(tol), 1 if deflate else 0, 1 if time_spmv else 0, int(reorth),
                        int(check_every), 1 if basis32 else 0, 1 if alpha_last else 0, int(keep_min),
                        float(reorth_thresh))
        st = LanczosStats()
        lam = ctypes.c_double()
        v = np.empty(self.n, np.float64)
        _chk(_lib.ek_lanczos_fiedler(self._c, ctypes.byref(o), ctypes.byref(lam), _p(v), ctypes.byref(st)),
             "lanczos_fiedler")
        return lam.value, v, {k: getattr(st, k) for k, _ in LanczosStats._fields_}

    # KL (cKL.cpp:288-406)
    def kl_graph_setup(self, csr):
        self.kl_n = csr.nrows
        _chk(_lib.ek_kl_graph_setup(self._c, csr.nrows, _p(np.ascontiguousarray(csr.rowptr, np.int32)),
                                    _p(np.ascontiguousarray(csr.col, np.int32)),
                                    _p(np.ascontiguousarray(csr.val, np.float32))), "kl_graph_setup")

    def kl_nets_setup(self, net_ptr, pins):
        net_ptr = np.ascontiguousarray(net_ptr, np.int64)
        pins = np.ascontiguousarray(pins, np.int32)
        _chk(_lib.ek_kl_nets_setup(self._c, len(net_ptr) - 1, _p(net_ptr), _p(pins)), "kl_nets_setup")

    def kl_set_partition(self, order0, order1):
        o0 = np.ascontiguousarray(order0, np.int32)
        o1 = np.ascontiguousarray(order1, np.int32)
        _chk(_lib.ek_kl_set_partition(self._c, _p(o0), len(o0), _p(o1), len(o1)), "kl_set_partition")
        self._n01 = (len(o0), len(o1))

    def kl_set_partition_bits(self, bits):
        """cKL.cpp:155-174 (-EIG): node i to split[bits[i]], ascending node order."""
        bits = np.ascontiguousarray(bits, np.uint8)
        _chk(_lib.ek_kl_set_partition_bits(self._c, len(bits), _p(bits)), "kl_set_partition_bits")
        n1 = int(np.count_nonzero(bits))
        self._n01 = (len(bits) - n1, n1)

    def kl_set_partition_fiedler(self):
        """The -EIG split on the device from the Fiedler vector the last lanczos_fiedler left on this context:
        median and the remain[] lists of median_split + kl_set_partition_bits.  Returns (median, n0, n1)."""
        med = ctypes.c_double()
        n0, n1 = ctypes.c_int64(), ctypes.c_int64()
        _chk(_lib.ek_kl_set_partition_fiedler(self._c, ctypes.byref(med), ctypes.byref(n0), ctypes.byref(n1)),
             "kl_set_partition_fiedler")
        self._n01 = (n0.value, n1.value)
        return med.value, n0.value, n1.value

    def kl_run(self, limit=-1, cap=None):
        cap = min(self._n01) if cap is None else cap
        log = np.zeros(max(cap, 1), SWAP_DTYPE)
        r = KLResult()
        _chk(_lib.ek_kl_run(self._c, int(limit), _p(log), cap, ctypes.byref(r)), "kl_run")
        res = {k: getattr(r, k) for k, _ in KLResult._fields_}
        return log[: min(r.iterations, cap)], res

    def solve_file(self, path, eig=1, seed=0, write_results=True, out_dir=None, limit=-1, sign_ref=None, ncv=0,
                   tol=1e-10, deflate=True, time_spmv=False, log_cap=0, check_every=8, basis32=True, alpha_last=False,
                   keep_min=-1, reorth=3, reorth_thresh=0.0):
        """The whole path, .hgr -> results/ (ek_solve_file).  eig: 1 GPU Fiedler split (gKL2 -EIG), 2 the
        pre_saved_EIG file (cKL -EIG), 0 random split with std::mt19937(seed).  Returns (result dict, swap log)."""
        o = SolveOpts()
        _lib.ek_solve_default_opts(ctypes.byref(o))
        o.eig, o.seed, o.write_results, o.limit = int(eig), int(seed) & 0xFFFFFFFF, 1 if write_results else 0, int(limit)
        o.out_dir = os.fsencode(out_dir) if out_dir else None
        o.sign_ref = os.fsencode(sign_ref) if sign_ref else None
        o.lanczos = LanczosOpts(int(ncv), 1000, float(tol), 1 if deflate else 0, 1 if time_spmv else 0, int(reorth),
                                int(check_every), 1 if basis32 else 0, 1 if alpha_last else 0, int(keep_min),
                                float(reorth_thresh))
        log = np.empty(max(int(log_cap), 1), SWAP_DTYPE)  # the library writes the first `iterations` records
        r = SolveResult()
        _chk(_lib.ek_solve_file(self._c, os.fsencode(path), ctypes.byref(o), _p(log), int(log_cap), ctypes.byref(r)),
             f"solve_file {path}")
        out = {k: getattr(r, k) for k in ("nets", "nodes", "pins", "median") + _SOLVE_TIMES}
        out["lambda"] = r.lambda_
        out["lanczos"] = {k: getattr(r.lanczos, k) for k, _ in LanczosStats._fields_}
        out["kl"] = {k: getattr(r.kl, k) for k, _ in KLResult._fields_}
        self.kl_n = r.nodes  # (kl_sides: the partition this solve left on the context)
        return out, log[: min(int(log_cap), r.kl.iterations)]

    def kl_sides(self, which):
        out = np.empty(self.kl_n, np.uint8)
        _chk(_lib.ek_kl_sides(self._c, int(which), _p(out)), "kl_sides")
        return out


# ---------------------------------------------------------------------------
# drop-in tools, in-process (same argv / CWD semantics as the executables)
def _cli(tool, *args):
    argv = [tool.encode()] + [os.fsencode(str(a)) for a in args]
    arr = (ctypes.c_char_p * len(argv))(*argv)
    return _lib.ek_cli_main(tool.encode(), len(argv), arr)


def cEIG(path, *flags):
    return _cli("cEIG", path, *flags)


def cKL(path, EIG=False, *flags):
    return _cli("cKL", path, *(["-EIG"] if EIG else []), *flags)


def gKL(path, EIG=False, *flags):
    return _cli("gKL", path, *(["-EIG"] if EIG else []), *flags)


def gKL2(path, EIG=False, *flags):
    return _cli("gKL2", path, *(["-EIG"] if EIG else []), *flags)
