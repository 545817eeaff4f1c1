"""bench.py's series labels (VERDICT r5 'weak-scaling line mixes families'):
the N = 1 `auto` line is the north-star K3' and names the K4 family's N = 1
point as its weak_anchor; N > 1 `auto` lines are the K4 family (weak); a
named --config is the same matrix at every N (strong).  CPU only."""
import math
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
import bench  # noqa: E402


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_auto_series(world):
    kind, prm, desc = bench.workload("auto", world)
    ser = bench.series("auto", world)
    assert ser["scaling"] == "weak"
    if world == 1:
        assert (prm["scale"], prm["ef"], prm["seed"]) == (20, 20, 2)
        assert ser["family"] == "K3'" and "weak_anchor" in ser["series"] and "K3'" in desc
    else:
        assert (prm["scale"], prm["ef"], prm["seed"]) == (20 + int(math.log2(world)), 24, 3)
        assert ser["family"] == "K4" and "K4 family" in desc and f"2^{prm['scale']}" in ser["series"]


@pytest.mark.parametrize("cfg,fam", [("k3p", "K3'"), ("k4", "K4"), ("k2", "K2")])
@pytest.mark.parametrize("world", [1, 8])
def test_named_config_is_strong(cfg, fam, world):
    kind, prm, desc = bench.workload(cfg, world)
    assert (kind, prm) == bench.CONFIGS[cfg][:2]   # the same matrix at every N
    ser = bench.series(cfg, world)
    assert ser["scaling"] == "strong" and ser["family"] == fam and fam in ser["series"]


def test_weak_anchor_is_the_k4_family_at_2_20():
    """weak_anchor's matrix = the K4 family's generator at scale 20 (what the
    N = 2 line doubles)"""
    kind, prm, _ = bench.workload("auto", 2)
    assert kind == "rmat" and prm["ef"] == 24 and prm["seed"] == 3 and prm["scale"] == 21
