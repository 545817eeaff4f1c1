"""Deterministic synthetic inputs: the generators reproduce the recorded
statistics and bytes (tests/golden/generator_stats.json, written by
tests/golden/make_generator_stats.py), independent of thread count."""
import json
import os
import subprocess
import sys

import pytest

import ias

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
import make_generator_stats as mg  # noqa: E402


@pytest.fixture(scope="module")
def stats(golden_dir):
    with open(os.path.join(golden_dir, "generator_stats.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name", [k for k in mg.CASES if not k.startswith(("k3", "k4"))])
def test_small_generators(stats, name):
    kind, args = mg.CASES[name]
    A = mg.make(kind, args)
    rec = stats[name]
    assert (A.rows, A.nnz, ias.flops(A, A)) == (rec["rows"], rec["nnz"], rec["flops"])
    assert mg.digest(A) == rec["sha256"]


@pytest.mark.parametrize("name", ["k3p_rmat20_ef20_s2", "k3_rmat20_ef32_s1", "k4_rmat23_ef24_s3"])
def test_headline_matrix(stats, name):
    """K3' (north-star headline, 2^20 rows, ~20 nnz/row), K3 (avg 32/row,
    nnz(C) > 2^31) and K4 (2^23 rows, avg 24/row, the 8-GPU configuration):
    same bytes every run."""
    kind, args = mg.CASES[name]
    A = mg.make(kind, args)
    rec = stats[name]
    assert (A.rows, A.nnz, ias.flops(A, A)) == (rec["rows"], rec["nnz"], rec["flops"])
    assert mg.digest(A) == rec["sha256"]


def test_thread_count_independent(stats):
    code = ("import sys; sys.path.insert(0, %r); sys.path.insert(0, %r); import make_generator_stats as mg;"
            "print(mg.digest(mg.make(*mg.CASES['rmat14_ef20_s2_int'])))"
            % (os.path.join(os.path.dirname(__file__), "golden"),
               os.path.join(os.path.dirname(os.path.dirname(__file__)), "ia-spgemm_amd")))
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True)
    assert out.stdout.strip() == stats["rmat14_ef20_s2_int"]["sha256"]


def test_value_modes():
    A = ias.gen_rmat(10, 8, seed=3, value_mode=1)
    assert set(A.val.tolist()) <= set(float(v) for v in range(1, 10))
    B = ias.gen_rmat(10, 8, seed=3, value_mode=0)
    assert (B.val > -1).all() and (B.val < 1).all()
    assert (A.col == B.col).all()
