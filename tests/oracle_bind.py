"""ctypes binding of oracle/libias_oracle.so — the CPU restatement of the
reference path (oracle/ias_oracle.c).  TEST INFRASTRUCTURE: imported only by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB = os.path.join(ORACLE_DIR, "libias_oracle.so")

i64p, i32p, f64p = C.POINTER(C.c_int64), C.POINTER(C.c_int32), C.POINTER(C.c_double)


class OCsr(C.Structure):
    _fields_ = [("rows", C.c_int64), ("cols", C.c_int64), ("nnz", C.c_int64),
                ("row_ptr", i64p), ("col", i32p), ("val", f64p),
                ("memory", C.c_int32), ("device", C.c_int32)]


class OCoo(C.Structure):
    _fields_ = [("rows", C.c_int64), ("cols", C.c_int64), ("nnz", C.c_int64),
                ("row_offset", i64p), ("row", i32p), ("col", i32p), ("val", f64p),
                ("memory", C.c_int32), ("device", C.c_int32), ("choice", C.c_int32),
                ("reserved", C.c_int32)]


class OEll(C.Structure):
    _fields_ = [("rows", C.c_int64), ("cols", C.c_int64), ("nnz", C.c_int64),
                ("max_nnz_per_row", C.c_int32), ("choice", C.c_int32),
                ("nnz_row", i32p), ("col", i32p), ("val", f64p),
                ("memory", C.c_int32), ("device", C.c_int32)]


class ODia(C.Structure):
    _fields_ = [("rows", C.c_int64), ("cols", C.c_int64),
                ("num_diagonals", C.c_int32), ("choice", C.c_int32),
                ("diagonal_offsets", i32p), ("diagonal_ind", i32p), ("val", f64p),
                ("memory", C.c_int32), ("device", C.c_int32)]


def _build():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", ORACLE_DIR], check=True, capture_output=True)


_build()
lib = C.CDLL(LIB)
P = C.POINTER
for name, res, args in [
    ("ora_mtx_read", C.c_int, [C.c_char_p, P(OCsr), i32p]),
    ("ora_flops", C.c_int64, [P(OCsr), P(OCsr)]),
    ("ora_csr_mul_csr", None, [P(OCsr), P(OCsr), P(OCsr)]),
    ("ora_csr_mul_csr_digest", None, [P(OCsr), P(OCsr), i64p, C.POINTER(C.c_uint64)]),
    ("ora_csr_mul_csr_digest_sorted", None, [P(OCsr), P(OCsr), i64p, C.POINTER(C.c_uint64)]),
    ("ora_csr_to_coo", C.c_int, [P(OCsr), P(OCoo), C.c_double]),
    ("ora_coo_mul_coo", None, [P(OCoo), P(OCoo), P(OCoo)]),
    ("ora_csr_to_ell", C.c_int, [P(OCsr), P(OEll), C.c_double]),
    ("ora_ell_mul_ell", None, [P(OEll), P(OEll), P(OEll)]),
    ("ora_csr_to_dia", C.c_int, [P(OCsr), P(ODia), C.c_double]),
    ("ora_dia_mul_dia", None, [P(ODia), P(ODia), P(ODia)]),
    ("ora_sizeof_csr", C.c_double, [P(OCsr)]),
    ("ora_sizeof_coo", C.c_double, [P(OCoo)]),
    ("ora_sizeof_ell", C.c_double, [P(OEll)]),
    ("ora_sizeof_dia", C.c_double, [P(ODia)]),
    ("ora_features", None, [P(OCsr), P(OCsr), C.c_int32, f64p]),
    ("ora_density_image", None, [P(OCsr), i64p]),
    ("ora_free_csr", None, [P(OCsr)]),
    ("ora_free_coo", None, [P(OCoo)]),
    ("ora_free_ell", None, [P(OEll)]),
    ("ora_free_dia", None, [P(ODia)]),
]:
    f = getattr(lib, name)
    f.restype, f.argtypes = res, args


def _arr(p, n, dt):
    if n == 0:
        return np.zeros(0, dt)
    return np.ctypeslib.as_array(p, shape=(n,)).astype(dt, copy=True)


class Mat:
    """numpy CSR (int64 row_ptr, int32 col, float64 val)."""

    def __init__(self, rows, cols, row_ptr, col, val):
        self.rows, self.cols = int(rows), int(cols)
        self.row_ptr = np.ascontiguousarray(row_ptr, np.int64)
        self.col = np.ascontiguousarray(col, np.int32)
        self.val = np.ascontiguousarray(val, np.float64)

    @property
    def nnz(self):
        return int(self.row_ptr[-1] - self.row_ptr[0]) if self.rows else 0

    def struct(self):
        return OCsr(self.rows, self.cols, self.nnz,
                    self.row_ptr.ctypes.data_as(i64p), self.col.ctypes.data_as(i32p),
                    self.val.ctypes.data_as(f64p), 0, 0)

    @staticmethod
    def of(m):
        """from any object with rows/cols/row_ptr/col/val (e.g. ias.HostCsr)."""
        return Mat(m.rows, m.cols, m.row_ptr, m.col, m.val)


def _take_csr(c: OCsr) -> Mat:
    m = Mat(c.rows, c.cols, _arr(c.row_ptr, c.rows + 1, np.int64), _arr(c.col, c.nnz, np.int32),
            _arr(c.val, c.nnz, np.float64))
    lib.ora_free_csr(C.byref(c))
    return m


def mtx_read(path):
    c = OCsr()
    flags = (C.c_int32 * 4)()
    rc = lib.ora_mtx_read(path.encode(), C.byref(c), flags)
    if rc != 0:
        raise RuntimeError(f"ora_mtx_read({path}) = {rc}")
    return _take_csr(c), list(flags)


def flops(A: Mat, B: Mat) -> int:
    a, b = A.struct(), B.struct()
    return int(lib.ora_flops(C.byref(a), C.byref(b)))


def csr_mul_csr(A: Mat, B: Mat) -> Mat:
    a, b, c = A.struct(), B.struct(), OCsr()
    lib.ora_csr_mul_csr(C.byref(a), C.byref(b), C.byref(c))
    return _take_csr(c)


def csr_mul_csr_digest(A: Mat, B: Mat, sorted_rows: bool = False):
    """(row_ptr of C, digest) of CSR_MUL_CSR without storing C (see tests/fulldigest.py);
    sorted_rows: the digest of C with every row sorted by column (IAS_ORDER_SORTED)."""
    a, b = A.struct(), B.struct()
    nnz = np.zeros(A.rows, np.int64)
    d = C.c_uint64(0)
    f = lib.ora_csr_mul_csr_digest_sorted if sorted_rows else lib.ora_csr_mul_csr_digest
    f(C.byref(a), C.byref(b), nnz.ctypes.data_as(i64p), C.byref(d))
    rp = np.zeros(A.rows + 1, np.int64)
    np.cumsum(nnz, out=rp[1:])
    return rp, int(d.value)


def coo_mul_coo(A: Mat, B: Mat):
    """returns (Mat in forward first-touch order, row index array)."""
    a, b = A.struct(), B.struct()
    ca, cb, cc = OCoo(), OCoo(), OCoo()
    lib.ora_csr_to_coo(C.byref(a), C.byref(ca), 0.0)
    lib.ora_csr_to_coo(C.byref(b), C.byref(cb), 0.0)
    lib.ora_coo_mul_coo(C.byref(ca), C.byref(cb), C.byref(cc))
    m = Mat(cc.rows, cc.cols, _arr(cc.row_offset, cc.rows + 1, np.int64),
            _arr(cc.col, cc.nnz, np.int32), _arr(cc.val, cc.nnz, np.float64))
    rows = _arr(cc.row, cc.nnz, np.int32)
    for x in (ca, cb, cc):
        lib.ora_free_coo(C.byref(x))
    return m, rows


def ell_mul_ell(A: Mat, B: Mat):
    """returns dict(K, nnz_row, col[rows,K], val[rows,K], nnz)."""
    a, b = A.struct(), B.struct()
    ea, eb, ec = OEll(), OEll(), OEll()
    lib.ora_csr_to_ell(C.byref(a), C.byref(ea), 0.0)
    lib.ora_csr_to_ell(C.byref(b), C.byref(eb), 0.0)
    lib.ora_ell_mul_ell(C.byref(ea), C.byref(eb), C.byref(ec))
    K = ec.max_nnz_per_row
    out = dict(K=K, nnz=int(ec.nnz), nnz_row=_arr(ec.nnz_row, ec.rows, np.int32),
               col=_arr(ec.col, ec.rows * K, np.int32).reshape(ec.rows, K),
               val=_arr(ec.val, ec.rows * K, np.float64).reshape(ec.rows, K))
    for x in (ea, eb, ec):
        lib.ora_free_ell(C.byref(x))
    return out


def csr_to_dia(A: Mat, gate=0.0):
    a, d = A.struct(), ODia()
    lib.ora_csr_to_dia(C.byref(a), C.byref(d), gate)
    out = dict(choice=d.choice, nd=d.num_diagonals,
               offsets=_arr(d.diagonal_offsets, d.num_diagonals, np.int32),
               ind=_arr(d.diagonal_ind, max(d.rows + d.cols - 1, 0), np.int32),
               val=_arr(d.val, d.rows * d.num_diagonals, np.float64).reshape(d.rows, d.num_diagonals))
    lib.ora_free_dia(C.byref(d))
    return out


def dia_mul_dia(A: Mat, B: Mat):
    a, b = A.struct(), B.struct()
    da, db, dc = ODia(), ODia(), ODia()
    lib.ora_csr_to_dia(C.byref(a), C.byref(da), 0.0)
    lib.ora_csr_to_dia(C.byref(b), C.byref(db), 0.0)
    lib.ora_dia_mul_dia(C.byref(da), C.byref(db), C.byref(dc))
    out = dict(nd=dc.num_diagonals, offsets=_arr(dc.diagonal_offsets, dc.num_diagonals, np.int32),
               ind=_arr(dc.diagonal_ind, max(dc.rows + dc.cols - 1, 0), np.int32),
               val=_arr(dc.val, dc.rows * dc.num_diagonals, np.float64).reshape(dc.rows, dc.num_diagonals))
    for x in (da, db, dc):
        lib.ora_free_dia(C.byref(x))
    return out


def gate_choices(A: Mat, gate=50.0):
    """(coo, ell, dia) feasibility under the reference size gates."""
    a = A.struct()
    co, el, di = OCoo(), OEll(), ODia()
    r = (lib.ora_csr_to_coo(C.byref(a), C.byref(co), gate) == 0,
         lib.ora_csr_to_ell(C.byref(a), C.byref(el), gate) == 0,
         lib.ora_csr_to_dia(C.byref(a), C.byref(di), gate) == 0)
    lib.ora_free_coo(C.byref(co)); lib.ora_free_ell(C.byref(el)); lib.ora_free_dia(C.byref(di))
    return r


def features(A: Mat, B: Mat, n: int = 26):
    a, b = A.struct(), B.struct()
    out = np.zeros(n, np.float64)
    lib.ora_features(C.byref(a), C.byref(b), n, out.ctypes.data_as(f64p))
    return out


def density_image(A: Mat):
    a = A.struct()
    out = np.zeros(128 * 128, np.int64)
    lib.ora_density_image(C.byref(a), out.ctypes.data_as(i64p))
    return out.reshape(128, 128)
