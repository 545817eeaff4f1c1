"""ctypes binding of libias.so (include/ias.h) — the host-side view used by
the tests, bench.py and __graft_entry__.

The product is the C-ABI library; this module only moves numpy arrays across
it.  Loading fails loudly when libias.so is missing: there is no Python or
CPU fallback for any compute entry point.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
LIB_PATH = os.environ.get("IAS_LIB", os.path.join(PKG_ROOT, "libias.so"))

MEMORY_HOST, MEMORY_DEVICE = 0, 1
ORDER_REFERENCE, ORDER_SORTED = 0, 1

STATUS = {
    0: "IAS_SUCCESS", 1: "IAS_ERROR_INVALID_ARGUMENT", 2: "IAS_ERROR_DIMENSION_MISMATCH",
    3: "IAS_ERROR_OUT_OF_MEMORY", 4: "IAS_ERROR_DEVICE", 5: "IAS_ERROR_IO",
    6: "IAS_ERROR_FORMAT", 7: "IAS_ERROR_UNSUPPORTED", 8: "IAS_ERROR_INFEASIBLE",
    9: "IAS_ERROR_OVERFLOW", 10: "IAS_ERROR_UNAVAILABLE", 11: "IAS_ERROR_INSUFFICIENT_CAPACITY",
}


class IasError(RuntimeError):
    def __init__(self, status: int, where: str, detail: str = ""):
        self.status = status
        super().__init__(f"{where}: {STATUS.get(status, status)} {detail}".strip())


i64p = C.POINTER(C.c_int64)
i32p = C.POINTER(C.c_int32)
f64p = C.POINTER(C.c_double)


class Csr(C.Structure):
    _fields_ = [("rows", C.c_int64), ("cols", C.c_int64), ("nnz", C.c_int64),
                ("row_ptr", i64p), ("col", i32p), ("val", f64p),
                ("memory", C.c_int32), ("device", C.c_int32)]


class Coo(C.Structure):
    _fields_ = [("rows", C.c_int64), ("cols", C.c_int64), ("nnz", C.c_int64),
                ("row_offset", i64p), ("row", i32p), ("col", i32p), ("val", f64p),
                ("memory", C.c_int32), ("device", C.c_int32), ("choice", C.c_int32),
                ("reserved", C.c_int32)]


class Ell(C.Structure):
    _fields_ = [("rows", C.c_int64), ("cols", C.c_int64), ("nnz", C.c_int64),
                ("max_nnz_per_row", C.c_int32), ("choice", C.c_int32),
                ("nnz_row", i32p), ("col", i32p), ("val", f64p),
                ("memory", C.c_int32), ("device", C.c_int32)]


class Dia(C.Structure):
    _fields_ = [("rows", C.c_int64), ("cols", C.c_int64),
                ("num_diagonals", C.c_int32), ("choice", C.c_int32),
                ("diagonal_offsets", i32p), ("diagonal_ind", i32p), ("val", f64p),
                ("memory", C.c_int32), ("device", C.c_int32)]


class Opts(C.Structure):
    _fields_ = [("order", C.c_int32), ("output_memory", C.c_int32), ("device", C.c_int32),
                ("reserved0", C.c_int32), ("stream", C.c_void_p), ("plan", C.c_void_p)]


class Report(C.Structure):
    _fields_ = [("ms_total", C.c_double), ("ms_analysis", C.c_double),
                ("ms_symbolic", C.c_double), ("ms_numeric", C.c_double),
                ("ms_upload", C.c_double), ("ms_download", C.c_double),
                ("flops", C.c_int64), ("nnz_c", C.c_int64),
                ("max_row_products", C.c_int64), ("max_row_nnz", C.c_int64),
                ("ms_stream", C.c_double), ("stream_products", C.c_int64), ("stream_nnz", C.c_int64),
                ("stream_launches", C.c_int32), ("kernel", C.c_int32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class MtxInfo(C.Structure):
    _fields_ = [("is_pattern", C.c_int32), ("is_real", C.c_int32), ("is_integer", C.c_int32),
                ("is_symmetric", C.c_int32), ("rows", C.c_int64), ("cols", C.c_int64),
                ("nnz_file", C.c_int64)]


# every symbol include/ias.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "ias_abi_version", "ias_status_string", "ias_last_diag", "ias_device_count", "ias_opts_default",
    "ias_plan_create", "ias_plan_destroy",
    "ias_csr_alloc", "ias_csr_copy", "ias_csr_free", "ias_coo_free", "ias_ell_free", "ias_dia_free",
    "ias_coo_copy", "ias_ell_copy", "ias_dia_copy",
    "ias_mtx_read", "ias_mtx_read_pair", "ias_mtx_write",
    "ias_csr_to_coo", "ias_csr_to_ell", "ias_csr_to_dia", "ias_coo_to_csr", "ias_ell_to_csr",
    "ias_dia_to_csr", "ias_csr_transpose",
    "ias_sizeof_csr", "ias_sizeof_coo", "ias_sizeof_ell", "ias_sizeof_dia",
    "ias_csr_mul_csr", "ias_coo_mul_coo", "ias_ell_mul_ell", "ias_dia_mul_dia",
    "ias_dia_mul_dia_into", "ias_dia_mul_dia_ndiag", "ias_device_release", "ias_device_cached_bytes",
    "ias_csr_mul_csr_nnz", "ias_csr_mul_csr_compute", "ias_csr_mul_csr_into",
    "ias_flops", "ias_sum_csr", "ias_sum_coo", "ias_sum_ell", "ias_sum_dia",
    "ias_csr_row_view", "ias_partition_rows", "ias_row_ptr_shift",
    "ias_csr_mul_csr_multi", "ias_dist_unique_id", "ias_dist_create", "ias_dist_create_loopback", "ias_dist_destroy",
    "ias_dist_allgatherv_csr", "ias_dist_csr_mul_csr",
    "ias_gen_rmat", "ias_gen_band", "ias_gen_ell",
    "ias_mkl_available", "ias_mkl_sp2m",
    "ias_features", "ias_density_image", "ias_matnet_load", "ias_matnet_free", "ias_matnet_shape",
    "ias_matnet_predict",
]


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libias.so not found at {LIB_PATH}: run `make -C ia-spgemm_amd` "
                          "(or __graft_entry__.build()); there is no fallback path")
    lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    P = C.POINTER
    sig = {
        "ias_abi_version": (C.c_int, []),
        "ias_status_string": (C.c_char_p, [C.c_int]),
        "ias_last_error": (C.c_char_p, []),
        "ias_last_diag": (C.c_uint32, []),
        "ias_device_count": (C.c_int, [i32p]),
        "ias_opts_default": (None, [P(Opts)]),
        "ias_plan_create": (C.c_int, [P(C.c_void_p), C.c_int32, C.c_void_p]),
        "ias_plan_destroy": (C.c_int, [C.c_void_p]),
        "ias_csr_alloc": (C.c_int, [P(Csr), C.c_int64, C.c_int64, C.c_int64, C.c_int32, C.c_int32]),
        "ias_csr_copy": (C.c_int, [P(Csr), P(Csr), C.c_int32, C.c_int32]),
        "ias_csr_free": (C.c_int, [P(Csr)]),
        "ias_coo_free": (C.c_int, [P(Coo)]),
        "ias_ell_free": (C.c_int, [P(Ell)]),
        "ias_dia_free": (C.c_int, [P(Dia)]),
        "ias_coo_copy": (C.c_int, [P(Coo), P(Coo), C.c_int32, C.c_int32]),
        "ias_ell_copy": (C.c_int, [P(Ell), P(Ell), C.c_int32, C.c_int32]),
        "ias_dia_copy": (C.c_int, [P(Dia), P(Dia), C.c_int32, C.c_int32]),
        "ias_mtx_read": (C.c_int, [C.c_char_p, P(Csr), P(MtxInfo)]),
        "ias_mtx_read_pair": (C.c_int, [C.c_char_p, C.c_char_p, P(Csr), P(Csr), P(MtxInfo), P(MtxInfo)]),
        "ias_mtx_write": (C.c_int, [C.c_char_p, P(Csr)]),
        "ias_csr_to_coo": (C.c_int, [P(Csr), P(Coo), C.c_double]),
        "ias_csr_to_ell": (C.c_int, [P(Csr), P(Ell), C.c_double]),
        "ias_csr_to_dia": (C.c_int, [P(Csr), P(Dia), C.c_double]),
        "ias_coo_to_csr": (C.c_int, [P(Coo), P(Csr)]),
        "ias_ell_to_csr": (C.c_int, [P(Ell), P(Csr)]),
        "ias_dia_to_csr": (C.c_int, [P(Dia), P(Csr)]),
        "ias_csr_transpose": (C.c_int, [P(Csr), P(Csr)]),
        "ias_sizeof_csr": (C.c_double, [P(Csr)]),
        "ias_sizeof_coo": (C.c_double, [P(Coo)]),
        "ias_sizeof_ell": (C.c_double, [P(Ell)]),
        "ias_sizeof_dia": (C.c_double, [P(Dia)]),
        "ias_csr_mul_csr": (C.c_int, [P(Csr), P(Csr), P(Csr), P(Opts), P(Report)]),
        "ias_coo_mul_coo": (C.c_int, [P(Coo), P(Coo), P(Coo), P(Opts), P(Report)]),
        "ias_ell_mul_ell": (C.c_int, [P(Ell), P(Ell), P(Ell), P(Opts), P(Report)]),
        "ias_dia_mul_dia": (C.c_int, [P(Dia), P(Dia), P(Dia), P(Opts), P(Report)]),
        "ias_dia_mul_dia_into": (C.c_int, [P(Dia), P(Dia), P(Dia), P(Opts), P(Report)]),
        "ias_dia_mul_dia_ndiag": (C.c_int, [P(Dia), P(Dia), i32p]),
        "ias_device_release": (C.c_int, [C.c_int32, i64p]),
        "ias_device_cached_bytes": (C.c_int, [C.c_int32, i64p]),
        "ias_csr_mul_csr_nnz": (C.c_int, [C.c_void_p, P(Csr), P(Csr), i64p, i64p, P(Report)]),
        "ias_csr_mul_csr_compute": (C.c_int, [C.c_void_p, P(Csr), P(Csr), P(Csr), C.c_int32, P(Report)]),
        "ias_csr_mul_csr_into": (C.c_int, [C.c_void_p, P(Csr), P(Csr), P(Csr), C.c_int32, P(Report)]),
        "ias_flops": (C.c_int, [P(Csr), P(Csr), i64p]),
        "ias_sum_csr": (C.c_int, [P(Csr), f64p]),
        "ias_sum_coo": (C.c_int, [P(Coo), f64p]),
        "ias_sum_ell": (C.c_int, [P(Ell), f64p]),
        "ias_sum_dia": (C.c_int, [P(Dia), f64p]),
        "ias_csr_row_view": (C.c_int, [P(Csr), C.c_int64, C.c_int64, P(Csr)]),
        "ias_partition_rows": (C.c_int, [P(Csr), P(Csr), C.c_int32, i64p]),
        "ias_row_ptr_shift": (C.c_int, [i64p, C.c_int64, C.c_int64, C.c_int32, C.c_void_p]),
        "ias_csr_mul_csr_multi": (C.c_int, [P(Csr), P(Csr), P(Csr), C.c_int32, i32p, P(Opts), P(Report)]),
        "ias_dist_unique_id": (C.c_int, [C.c_char_p, C.c_int32]),
        "ias_dist_create": (C.c_int, [P(C.c_void_p), C.c_char_p, C.c_int32, C.c_int32, C.c_int32]),
        "ias_dist_create_loopback": (C.c_int, [P(C.c_void_p), C.c_char_p, C.c_int32, C.c_int32, C.c_int32]),
        "ias_dist_destroy": (C.c_int, [C.c_void_p]),
        "ias_dist_allgatherv_csr": (C.c_int, [C.c_void_p, P(Csr), P(Csr), C.c_void_p]),
        "ias_dist_csr_mul_csr": (C.c_int, [C.c_void_p, P(Csr), P(Csr), P(Csr), C.c_int32, C.c_int32,
                                           P(Report)]),
        "ias_gen_rmat": (C.c_int, [C.c_int32, C.c_double, C.c_double, C.c_double, C.c_double,
                                   C.c_uint64, C.c_int32, P(Csr)]),
        "ias_gen_band": (C.c_int, [C.c_int64, C.c_int32, C.c_uint64, C.c_int32, P(Csr)]),
        "ias_gen_ell": (C.c_int, [C.c_int64, C.c_int32, C.c_uint64, C.c_int32, P(Csr)]),
        "ias_mkl_available": (C.c_int, [i32p, C.c_char_p, C.c_int32]),
        "ias_mkl_sp2m": (C.c_int, [P(Csr), P(Csr), P(Csr), C.c_int32, f64p]),
        "ias_features": (C.c_int, [P(Csr), P(Csr), C.c_int32, f64p]),
        "ias_density_image": (C.c_int, [P(Csr), i64p]),
        "ias_matnet_load": (C.c_int, [C.c_char_p, P(C.c_void_p)]),
        "ias_matnet_free": (C.c_int, [C.c_void_p]),
        "ias_matnet_shape": (C.c_int, [C.c_void_p, i32p, i32p]),
        "ias_matnet_predict": (C.c_int, [C.c_void_p, i64p, i64p, f64p, C.POINTER(C.c_float), i32p]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


lib = _load()


def check(status: int, where: str):
    if status != 0:
        detail = lib.ias_last_error().decode(errors="replace")
        raise IasError(status, where, detail)


# ---------------------------------------------------------------- numpy <-> structs
def _ptr(a: Optional[np.ndarray], ct):
    if a is None or a.size == 0:
        return C.cast(C.c_void_p(0 if a is None else a.ctypes.data), C.POINTER(ct))
    return a.ctypes.data_as(C.POINTER(ct))


@dataclass
class HostCsr:
    """A CSR matrix in numpy arrays (int64 row_ptr, int32 col, float64 val)."""
    rows: int
    cols: int
    row_ptr: np.ndarray
    col: np.ndarray
    val: np.ndarray

    @property
    def nnz(self) -> int:
        return int(self.row_ptr[-1] - self.row_ptr[0]) if self.rows else 0

    def struct(self) -> Csr:
        self.row_ptr = np.ascontiguousarray(self.row_ptr, dtype=np.int64)
        self.col = np.ascontiguousarray(self.col, dtype=np.int32)
        self.val = np.ascontiguousarray(self.val, dtype=np.float64)
        return Csr(self.rows, self.cols, self.nnz, _ptr(self.row_ptr, C.c_int64),
                   _ptr(self.col, C.c_int32), _ptr(self.val, C.c_double), MEMORY_HOST, 0)

    @staticmethod
    def from_scipy(m) -> "HostCsr":
        m = m.tocsr()
        return HostCsr(m.shape[0], m.shape[1], m.indptr.astype(np.int64),
                       m.indices.astype(np.int32), m.data.astype(np.float64))

    def rows_sorted(self):
        """Per-row (col, val) sorted by column: the canonical form for set parity."""
        out = []
        for i in range(self.rows):
            s, e = self.row_ptr[i], self.row_ptr[i + 1]
            o = np.argsort(self.col[s:e], kind="stable")
            out.append((self.col[s:e][o], self.val[s:e][o]))
        return out


def _np(ptr, n, dtype):
    if n == 0:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dtype, copy=True)


def csr_to_numpy(m: Csr, free: bool = True) -> HostCsr:
    """Copy a library-owned host CSR into numpy and free it."""
    if m.memory != MEMORY_HOST:
        h = Csr()
        check(lib.ias_csr_copy(C.byref(m), C.byref(h), MEMORY_HOST, 0), "ias_csr_copy")
        if free:
            lib.ias_csr_free(C.byref(m))
        m, free = h, True
    rp = _np(m.row_ptr, m.rows + 1, np.int64)
    nnz = int(rp[-1] - rp[0]) if m.rows else 0
    out = HostCsr(int(m.rows), int(m.cols), rp - rp[0] if m.rows else rp,
                  _np(m.col, nnz, np.int32), _np(m.val, nnz, np.float64))
    if free:
        lib.ias_csr_free(C.byref(m))
    return out


# ---------------------------------------------------------------- convenience API
def device_count() -> int:
    n = C.c_int32(0)
    st = lib.ias_device_count(C.byref(n))
    return int(n.value) if st == 0 else 0


def mtx_read(path: str):
    m, info = Csr(), MtxInfo()
    check(lib.ias_mtx_read(path.encode(), C.byref(m), C.byref(info)), f"ias_mtx_read({path})")
    return csr_to_numpy(m), info


def mtx_write(path: str, A: HostCsr) -> None:
    sa = A.struct()
    check(lib.ias_mtx_write(path.encode(), C.byref(sa)), f"ias_mtx_write({path})")


def mtx_read_pair(path_a: str, path_b: str):
    a, b, ia, ib = Csr(), Csr(), MtxInfo(), MtxInfo()
    check(lib.ias_mtx_read_pair(path_a.encode(), path_b.encode(), C.byref(a), C.byref(b),
                                C.byref(ia), C.byref(ib)), "ias_mtx_read_pair")
    return csr_to_numpy(a), csr_to_numpy(b), ia, ib


def gen_rmat(scale, edge_factor, a=0.45, b=0.15, c=0.15, seed=1, value_mode=0) -> HostCsr:
    m = Csr()
    check(lib.ias_gen_rmat(scale, edge_factor, a, b, c, seed, value_mode, C.byref(m)), "ias_gen_rmat")
    return csr_to_numpy(m)


def gen_band(n, half_width, seed=7, value_mode=0) -> HostCsr:
    m = Csr()
    check(lib.ias_gen_band(n, half_width, seed, value_mode, C.byref(m)), "ias_gen_band")
    return csr_to_numpy(m)


def gen_ell(n, per_row, seed=7, value_mode=0) -> HostCsr:
    m = Csr()
    check(lib.ias_gen_ell(n, per_row, seed, value_mode, C.byref(m)), "ias_gen_ell")
    return csr_to_numpy(m)


def flops(A: HostCsr, B: HostCsr) -> int:
    out = C.c_int64(0)
    sa, sb = A.struct(), B.struct()
    check(lib.ias_flops(C.byref(sa), C.byref(sb), C.byref(out)), "ias_flops")
    return int(out.value)


def opts(order=ORDER_REFERENCE, output_memory=MEMORY_HOST, device=-1, plan=None) -> Opts:
    o = Opts()
    lib.ias_opts_default(C.byref(o))
    o.order, o.output_memory, o.device = order, output_memory, device
    o.plan = plan
    return o


def spgemm(A: HostCsr, B: Optional[HostCsr] = None, order=ORDER_REFERENCE, device=0):
    """C = A*B through ias_csr_mul_csr with host operands; returns (HostCsr, Report)."""
    sa = A.struct()
    sb = sa if B is None else B.struct()
    c, rep = Csr(), Report()
    o = opts(order=order, output_memory=MEMORY_HOST, device=device)
    check(lib.ias_csr_mul_csr(C.byref(sa), C.byref(sb) if B is not None else C.byref(sa),
                              C.byref(c), C.byref(o), C.byref(rep)), "ias_csr_mul_csr")
    return csr_to_numpy(c), rep


def mkl_available():
    a = C.c_int32(0)
    buf = C.create_string_buffer(256)
    lib.ias_mkl_available(C.byref(a), buf, 256)
    return bool(a.value), buf.value.decode(errors="replace")


def mkl_sp2m(A: HostCsr, B: HostCsr, threads=0):
    sa, sb, c = A.struct(), B.struct(), Csr()
    ms = C.c_double(0)
    check(lib.ias_mkl_sp2m(C.byref(sa), C.byref(sb), C.byref(c), threads, C.byref(ms)), "ias_mkl_sp2m")
    return csr_to_numpy(c), float(ms.value)


# ---------------------------------------------------------------- input-aware selector
def features(A: HostCsr, B: HostCsr, n: int = 26) -> np.ndarray:
    sa, sb = A.struct(), B.struct()
    out = np.zeros(n, np.float64)
    check(lib.ias_features(C.byref(sa), C.byref(sb), n, _ptr(out, C.c_double)), "ias_features")
    return out


def density_image(A: HostCsr) -> np.ndarray:
    sa = A.struct()
    out = np.zeros(128 * 128, np.int64)
    check(lib.ias_density_image(C.byref(sa), _ptr(out, C.c_int64)), "ias_density_image")
    return out.reshape(128, 128)


def matnet_predict(weights: str, img_a: np.ndarray, img_b: np.ndarray, feats: np.ndarray):
    """(chosen, probs) of MatNet with the named weight set (or blob path)."""
    net = C.c_void_p()
    check(lib.ias_matnet_load(weights.encode(), C.byref(net)), "ias_matnet_load")
    try:
        nf, nc = C.c_int32(0), C.c_int32(0)
        check(lib.ias_matnet_shape(net, C.byref(nf), C.byref(nc)), "ias_matnet_shape")
        a = np.ascontiguousarray(img_a, np.int64).ravel()
        b = np.ascontiguousarray(img_b, np.int64).ravel()
        f = np.ascontiguousarray(feats, np.float64)
        assert f.size == nf.value, (f.size, nf.value)
        probs = (C.c_float * nc.value)()
        ch = C.c_int32(0)
        check(lib.ias_matnet_predict(net, _ptr(a, C.c_int64), _ptr(b, C.c_int64), _ptr(f, C.c_double), probs,
                                     C.byref(ch)), "ias_matnet_predict")
        return int(ch.value), np.array(probs[:], np.float64)
    finally:
        lib.ias_matnet_free(net)
