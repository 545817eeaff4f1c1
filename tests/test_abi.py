"""The C-ABI library loads without a GPU and exports every symbol include/ias.h
declares; host-only entry points behave (no compute calls here)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np

import ias

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ias.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ias_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    names = header_functions()
    assert len(names) > 40
    out = subprocess.run(["nm", "-D", "--defined-only", ias.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (ias_\w+)", out))
    missing = [n for n in names if n not in exported]
    assert not missing, f"declared in include/ias.h but not exported: {missing}"
    for n in names:
        assert hasattr(ias.lib, n)
    assert set(ias.EXPORTS) <= set(names) | {"ias_last_error"}


def test_only_c_symbols_exported():
    out = subprocess.run(["nm", "-D", "--defined-only", ias.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    ours = re.findall(r" T (ias_\w+)", out)
    assert all(not n.startswith("_Z") for n in ours)


def test_version_and_status_strings():
    assert ias.lib.ias_abi_version() == 6
    # the header the library was built from says the same (build() checks it)
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "ias.h")).read()
    assert int(re.search(r"#define IAS_ABI_VERSION (\d+)", hdr).group(1)) == ias.lib.ias_abi_version()
    for s in range(12):
        assert ias.lib.ias_status_string(s)
    assert ias.lib.ias_status_string(99) == b"unknown status"


def test_opts_default():
    o = ias.Opts()
    ias.lib.ias_opts_default(C.byref(o))
    assert o.order == 0 and o.output_memory == -1 and o.device == -1 and not o.plan


def test_struct_layouts_match_header(tmp_path):
    # the ctypes mirrors against the C compiler's own layout of include/ias.h
    src = tmp_path / "layout.c"
    src.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "ias.h"\n'
        'int main(void){printf("%zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(ias_csr), '
        'offsetof(ias_csr, memory), sizeof(ias_opts), sizeof(ias_report), '
        'offsetof(ias_report, ms_stream), sizeof(ias_coo), sizeof(ias_ell), sizeof(ias_dia));return 0;}\n')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()]
    assert got == [C.sizeof(ias.Csr), ias.Csr.memory.offset, C.sizeof(ias.Opts), C.sizeof(ias.Report),
                   ias.Report.ms_stream.offset, C.sizeof(ias.Coo), C.sizeof(ias.Ell), C.sizeof(ias.Dia)]


def test_host_alloc_copy_free():
    m = ias.Csr()
    ias.check(ias.lib.ias_csr_alloc(C.byref(m), 3, 4, 5, ias.MEMORY_HOST, 0), "alloc")
    assert m.rows == 3 and m.nnz == 5 and m.memory == 0
    ias.check(ias.lib.ias_csr_free(C.byref(m)), "free")
    assert m.rows == 0 and not m.row_ptr


def test_row_view_copy_rebases():
    A = ias.gen_band(64, 2, seed=3)
    s = A.struct()
    v, cp = ias.Csr(), ias.Csr()
    ias.check(ias.lib.ias_csr_row_view(C.byref(s), 10, 20, C.byref(v)), "view")
    assert v.rows == 10 and v.nnz == A.row_ptr[20] - A.row_ptr[10]
    ias.check(ias.lib.ias_csr_copy(C.byref(v), C.byref(cp), ias.MEMORY_HOST, 0), "copy")
    got = ias.csr_to_numpy(cp)
    np.testing.assert_array_equal(got.row_ptr, A.row_ptr[10:21] - A.row_ptr[10])
    np.testing.assert_array_equal(got.col, A.col[A.row_ptr[10]:A.row_ptr[20]])


def test_invalid_arguments():
    assert ias.lib.ias_csr_mul_csr(None, None, None, None, None) == 1
    assert ias.lib.ias_mtx_read(b"/nonexistent.mtx", C.byref(ias.Csr()), None) == 5


def test_no_device_reports_error_not_crash():
    if ias.device_count() > 0:
        return
    A = ias.gen_band(16, 1)
    try:
        ias.spgemm(A)
    except ias.IasError as e:
        assert e.status == 4  # IAS_ERROR_DEVICE: no silent CPU fallback
    else:
        raise AssertionError("spgemm must fail without a HIP device (no CPU fallback)")
