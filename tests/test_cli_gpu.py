"""The two CLIs end to end on the GPU: report
lines, verified sums against the oracle, the timeout verdict, the selector
line.  The binaries are started as child processes."""
import os
import re
import subprocess

import numpy as np
import pytest

import ias
import oracle_bind as ob

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "ia-spgemm_amd", "bin")


def run(*args):
    p = subprocess.run(list(args), capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    return p.stdout


def blocks(out):
    """{alg: {field: value}} of the report (main.cpp:968-1000 layout)."""
    res = {}
    for m in re.finditer(r"Algorithm (\d+):\n((?:[a-z_A-Z]+: [-0-9.e+]+\n)+)", out):
        res[int(m.group(1))] = {k: float(v) for k, v in re.findall(r"(\w+): ([-0-9.e+]+)", m.group(2))}
    return res


def test_spgemm_cpu_report(inputs_dir):
    path = os.path.join(inputs_dir, "dia.mtx")
    out = run(os.path.join(BIN, "spgemm-cpu"), path, "--time-scale", "0")
    b = blocks(out)
    assert sorted(b) == [1, 2, 3, 4, 5], out
    A = ias.mtx_read(path)[0]
    want = float(np.sum(ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(A)).val))
    for alg in (2, 3, 4, 5):
        assert b[alg]["verified_sum"] == pytest.approx(want, abs=1e-6), (alg, out)
        assert b[alg]["run_time"] > 0
    for alg in (3, 4, 5):
        assert "trans_time" in b[alg]
    assert re.search(r"The Chosen One = Algorithm [1-5]", out)
    assert re.search(r"MAX SPEED IS [0-9.]+ for ALGORITHM [1-5]", out)


def test_spgemm_cpu_timeout_verdict(inputs_dir):
    """An algorithm slower than time_scale x MKL reports zeros (main.cpp:770-800)."""
    out = run(os.path.join(BIN, "spgemm-cpu"), os.path.join(inputs_dir, "dia.mtx"), "--time-scale", "1e-12")
    b = blocks(out)
    if b[1]["run_time"] == 0.0:
        pytest.skip("MKL unavailable on this box: no deadline to apply")
    for alg in (2, 3, 4, 5):
        assert b[alg]["run_time"] == 0.0 and b[alg]["verified_sum"] == 0.0 and b[alg]["memory_size"] == 0.0


def test_spgemm_gpu_aat(inputs_dir):
    """spgemm-gpu --aat: A^T built on the device; both orders give the oracle's sum."""
    path = os.path.join(inputs_dir, "LFAT5.mtx")
    out = run(os.path.join(BIN, "spgemm-gpu"), path, "--aat")
    b = blocks(out)
    A = ias.mtx_read(path)[0]
    At = ias.HostCsr.from_scipy(__import__("scipy.sparse", fromlist=["csr_matrix"]).csr_matrix(
        (A.val, A.col, A.row_ptr), shape=(A.rows, A.cols)).T.tocsr())
    want = float(np.sum(ob.csr_mul_csr(ob.Mat.of(A), ob.Mat.of(At)).val))
    assert sorted(b) == [1, 2]
    for alg in (1, 2):
        assert b[alg]["verified_sum"] == pytest.approx(want, rel=1e-12, abs=2e-6)
    assert re.search(r"MatNet predicts Algorithm (CUSP|cuSPARSE|NSPARSE) is optimal", out)
