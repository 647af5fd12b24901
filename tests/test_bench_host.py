"""Host-side pieces of bench.py (no GPU): the CPU-baseline leg for the
non-causal and causal workloads, its extrapolation above the dense-table limit,
and the config table the driver's JSON line is built from."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_configs_cover_baseline_rows():
    # BASELINE.json configs 2-5 (config 1 is the 5x5 main.py run, timed by tools/diag/config1_timing.py)
    assert set(bench.CONFIGS) == {"c2", "c3", "c4", "c5"}
    size, per_gpu, _, causal = bench.CONFIGS["c3"]
    assert (size, per_gpu, causal) == (128, 64, False)
    assert bench.CONFIGS["c5"][3] is True and bench.CONFIGS["c5"][0] == 128


@pytest.mark.parametrize("causal", [False, True])
def test_cpu_baseline_small(causal):
    out = bench.cpu_baseline(12, 0.2, 288, 500.0, 2, causal=causal)
    assert out["value"] > 0 and out["unit"] == "instance-steps/s" and out["kind"] == "port"
    assert out["cores"] >= 1 and out["host_cpu_count"] == os.cpu_count()
    assert (":329-338 (soft VI" in out["sample"]) == causal
    assert "K_b=288, K_f=500" in out["sample"]


def test_cpu_baseline_extrapolates_above_dense_limit(monkeypatch):
    monkeypatch.setattr(bench, "CPU_DENSE_MAX", 8)
    base = bench.cpu_baseline(8, 0.2, 128, 100.0, 1)
    big = bench.cpu_baseline(16, 0.2, 128, 100.0, 1)
    assert big["sample"].startswith("extrapolated") and "(S ratio)^2 = 16" in big["sample"]
    # (S ratio)^2 = 16: the same statements timed again, divided by 16
    assert 0 < big["value"] < base["value"]
