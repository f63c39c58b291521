"""ORACLE — test infrastructure only.

ctypes wrapper over oracle/build/libekoracle.so (the CPU restatement of the
reference's cEIG/cKL path, see oracle/eko_kl.cpp and oracle/eko_eig.cpp).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module; the product never does.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libekoracle.so")

SWAP_DTYPE = np.dtype([("iter", "<u4"), ("node_left", "<u4"), ("node_right", "<u4"),
                       ("max_gain", "<f4"), ("min_gain", "<f4"), ("gain", "<f4"),
                       ("cut", "<f4"), ("pad", "<u4")])


class _KLResult(ctypes.Structure):
    _fields_ = [("iterations", ctypes.c_int64), ("initial_cut", ctypes.c_float),
                ("best_cut", ctypes.c_float), ("final_cut", ctypes.c_float),
                ("best_iter", ctypes.c_int64), ("net_cut_initial", ctypes.c_int64),
                ("net_cut_best", ctypes.c_int64), ("net_cut_final", ctypes.c_int64)]


class _LzOpts(ctypes.Structure):
    _fields_ = [("ncv", ctypes.c_int32), ("maxit", ctypes.c_int32), ("tol", ctypes.c_double),
                ("deflate", ctypes.c_int32), ("max_matvec", ctypes.c_int32)]


class _LzStats(ctypes.Structure):
    _fields_ = [("restarts", ctypes.c_int32), ("matvecs", ctypes.c_int32),
                ("converged", ctypes.c_int32), ("residual", ctypes.c_double)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.check_call(["make", "-s", "-C", HERE])
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        L.eko_read.argtypes = [ctypes.c_char_p, ctypes.POINTER(P)]
        L.eko_from_pins.argtypes = [ctypes.c_int64, ctypes.c_int64, P, P, ctypes.POINTER(P)]
        L.eko_free.argtypes = [P]
        L.eko_nodes.argtypes = [P]
        L.eko_nodes.restype = ctypes.c_int64
        L.eko_nets.argtypes = [P]
        L.eko_nets.restype = ctypes.c_int64
        L.eko_kl_csr.argtypes = [P, P, P, P, P]
        L.eko_kl_csr.restype = ctypes.c_int64
        L.eko_kl.argtypes = [P, P, ctypes.c_int64, P, ctypes.c_int64, ctypes.c_int32, P,
                             ctypes.c_int64, ctypes.POINTER(_KLResult)]
        L.eko_net_cut.argtypes = [P, P]
        L.eko_net_cut.restype = ctypes.c_int64
        L.eko_laplacian.argtypes = [P, P, P, P]
        L.eko_laplacian.restype = ctypes.c_int64
        L.eko_spmv.argtypes = [P, P, P]
        L.eko_lanczos.argtypes = [P, ctypes.POINTER(_LzOpts), P, P, ctypes.POINTER(_LzStats)]
        L.eko_bucket_growth.argtypes = [ctypes.c_int64, P]
        L.eko_random_split.argtypes = [ctypes.c_int64, ctypes.c_uint32, P, P]
        L.eko_set_threads.argtypes = [ctypes.c_int]
        L.eko_get_threads.restype = ctypes.c_int
        # one thread unless asked: the checker's results do not depend on it,
        # and an oversubscribed host makes OpenMP barriers crawl
        L.eko_set_threads(int(os.environ.get("EKO_THREADS", "1")))
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class Graph:
    """cKL's in-memory graph (cKL.cpp:35-149) plus the hypergraph pins."""

    def __init__(self, handle):
        self._h = handle

    @classmethod
    def read(cls, path):
        h = ctypes.c_void_p()
        rc = lib().eko_read(os.fsencode(path), ctypes.byref(h))
        if rc != 0:
            raise IOError(f"oracle: cannot read {path} ({rc})")
        return cls(h)

    @classmethod
    def from_pins(cls, nodes, net_ptr, pins):
        net_ptr = np.ascontiguousarray(net_ptr, dtype=np.int64)
        pins = np.ascontiguousarray(pins, dtype=np.int32)
        h = ctypes.c_void_p()
        lib().eko_from_pins(len(net_ptr) - 1, nodes, _p(net_ptr), _p(pins), ctypes.byref(h))
        return cls(h)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().eko_free(self._h)
            self._h = None

    @property
    def nodes(self):
        return lib().eko_nodes(self._h)

    @property
    def nets(self):
        return lib().eko_nets(self._h)

    def kl_csr(self):
        n = self.nodes
        nnz = lib().eko_kl_csr(self._h, None, None, None, None)
        rowptr = np.empty(n + 1, np.int32)
        col = np.empty(nnz, np.int32)
        w = np.empty(nnz, np.float32)
        nfwd = np.empty(n, np.int32)
        lib().eko_kl_csr(self._h, _p(rowptr), _p(col), _p(w), _p(nfwd))
        return rowptr, col, w, nfwd

    def laplacian(self):
        n = self.nodes
        nnz = lib().eko_laplacian(self._h, None, None, None)
        rowptr = np.empty(n + 1, np.int32)
        col = np.empty(nnz, np.int32)
        val = np.empty(nnz, np.float64)
        lib().eko_laplacian(self._h, _p(rowptr), _p(col), _p(val))
        return rowptr, col, val

    def spmv(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.empty_like(x)
        lib().eko_spmv(self._h, _p(x), _p(y))
        return y

    def net_cut(self, side):
        side = np.ascontiguousarray(side, dtype=np.uint8)
        return lib().eko_net_cut(self._h, _p(side))

    def kl(self, order0, order1, limit=-1, cap=None):
        """KL() (cKL.cpp:288-406) from the given remain[] lists. Returns (log, result dict)."""
        order0 = np.ascontiguousarray(order0, dtype=np.int32)
        order1 = np.ascontiguousarray(order1, dtype=np.int32)
        cap = cap if cap is not None else min(len(order0), len(order1))
        log = np.zeros(cap, SWAP_DTYPE)
        res = _KLResult()
        lib().eko_kl(self._h, _p(order0), len(order0), _p(order1), len(order1), limit,
                     _p(log), cap, ctypes.byref(res))
        out = {k: getattr(res, k) for k, _ in _KLResult._fields_}
        return log[: min(res.iterations, cap)], out

    def lanczos(self, ncv=0, tol=1e-10, maxit=1000, deflate=True, max_matvec=0):
        o = _LzOpts(ncv, maxit, tol, 1 if deflate else 0, max_matvec)
        st = _LzStats()
        lam = ctypes.c_double()
        v = np.empty(self.nodes, np.float64)
        rc = lib().eko_lanczos(self._h, ctypes.byref(o), ctypes.byref(lam), _p(v), ctypes.byref(st))
        return lam.value, v, {"restarts": st.restarts, "matvecs": st.matvecs,
                              "converged": bool(st.converged), "residual": st.residual, "rc": rc}


def set_threads(t):
    """OpenMP threads of the restatement (CPU baseline); results do not depend on it."""
    lib().eko_set_threads(int(t))


def random_split(n, seed):
    """cKL.cpp:176-192 with std::mt19937(seed) in place of random_device: (remain[0], remain[1])."""
    o0 = np.empty(n // 2, np.int32)
    o1 = np.empty(n - n // 2, np.int32)
    lib().eko_random_split(int(n), int(seed) & 0xFFFFFFFF, _p(o0), _p(o1))
    return o0, o1


def bucket_growth(nkeys):
    out = np.empty(nkeys, np.int64)
    lib().eko_bucket_growth(nkeys, _p(out))
    return out


def read_eig_file(path):
    """cEIG output (cEIG.cpp:213-220) read back the way cKL does (cKL.cpp:162-173).

    Returns lambda, median, bits (uint8, file order = node id), v (fp64 as printed),
    and the remain[] lists in file order."""
    with open(path) as f:
        lam = float(f.readline())
        med = float(f.readline())
        rows = [ln.split() for ln in f if ln.strip()]
    node = np.array([int(r[0]) for r in rows], np.int64)
    bits = np.array([int(r[1]) for r in rows], np.uint8)
    v = np.array([float(r[2]) for r in rows], np.float64)
    order0 = node[bits == 0].astype(np.int32)
    order1 = node[bits == 1].astype(np.int32)
    return lam, med, bits, v, order0, order1


def format_results(log, initial_cut):
    """results/<base>_KL_CutSize*_output.txt rows (cKL.cpp:315,380): ostream default = %g."""
    lines = [f"0\t{initial_cut:g}\t0"]
    lines += [f"{int(r['iter'])}\t{float(r['cut']):g}\t{float(r['gain']):g}" for r in log]
    return "\n".join(lines) + "\n"


_libc = None


def c_hexfloat(x):
    """glibc printf("%a", (double)x) — the format the SURVEY §8c swap-log md5s use."""
    global _libc
    if _libc is None:
        _libc = ctypes.CDLL(None)
        _libc.snprintf.restype = ctypes.c_int
    buf = ctypes.create_string_buffer(64)
    _libc.snprintf(buf, 64, b"%a", ctypes.c_double(float(x)))
    return buf.value.decode()


def swap_log_text(log):
    """SURVEY §8c swap-log format: '%u %u %u %a %a %a' = iteration node1 node2 maxG minG gain."""
    return "".join(f"{int(r['iter'])} {int(r['node_left'])} {int(r['node_right'])} "
                   f"{c_hexfloat(r['max_gain'])} {c_hexfloat(r['min_gain'])} "
                   f"{c_hexfloat(r['gain'])}\n" for r in log)
