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
    # BASELINE.json configs 2-5 (config 1, the 5x5 main.py run, is timed by bench.config1_timings)
    # (c2s: config 2's |A| = 5 variant, the four moves + stay)
    assert set(bench.CONFIGS) == {"c2", "c2s", "c3", "c4", "c5"}
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


def test_cpu_baseline_stay_variant():
    t = bench.cpu_sweep_times(8, 0.2, 1, stay=True)
    assert t["n_actions"] == 5
    assert "A=5" in bench.cpu_baseline_from(t, 128, 100.0)["sample"]


def test_cpu_baseline_extrapolates_above_dense_limit(monkeypatch):
    monkeypatch.setattr(bench, "CPU_DENSE_MAX", 8)
    base = bench.cpu_baseline(8, 0.2, 128, 100.0, 1)
    big = bench.cpu_baseline(16, 0.2, 128, 100.0, 1)
    assert big["sample"].startswith("extrapolated") and "(S ratio)^2 = 16" in big["sample"]
    # (S ratio)^2 = 16: the same statements timed again, divided by 16
    assert 0 < big["value"] < base["value"]


def test_cpu_baseline_uses_mean_sweeps():
    t = bench.cpu_sweep_times(6, 0.2, 1)
    a = bench.cpu_baseline_from(t, 72, 100.0)
    b = bench.cpu_baseline_from(t, 72, 300.0)
    assert a["value"] > b["value"] > 0
    assert abs(1.0 / b["value"] - 1.0 / a["value"] - 200.0 * t["t_f"]) < 1e-12
    assert "means over instances" in a["sample"]


def test_config1_cpu_leg():
    out = bench.config1_timings(device_runs=False)
    # the reference's step counts for src/main.py's problem (tests/golden/config1.npz)
    assert out["irl"]["cpu_port_steps"] == 375 and out["irl_causal"]["cpu_port_steps"] == 419
    assert out["irl"]["cpu_port_steps_per_s"] > 0


def test_timed_steps_brackets_exactly_k_steps():
    calls, log = [], []
    clock_t = [0.0]

    def clock():
        return clock_t[0]

    def step(i, timed):
        calls.append((i, timed))
        clock_t[0] += 1.0 + i

    elapsed, per_step = bench.timed_steps(step, 3, 2, lambda: log.append("barrier"), lambda: log.append("sync"),
                                          clock=clock)
    assert calls == [(0, False), (1, False), (2, True), (3, True), (4, True)]
    assert elapsed == 3.0 + 4.0 + 5.0 and per_step == [1.0, 2.0, 3.0, 4.0, 5.0]
    assert log.count("barrier") == 2
    v, ms = bench.headline(elapsed, 64, 2, 3)
    assert v == 64 * 2 * 3 / 12.0 and ms == 4000.0


def test_full_run_default():
    """The default bench line (config 3) also runs irl to convergence (full_run);
    the long configs and overridden workloads only on request."""
    import bench
    assert bench.parse([]).full_run is True
    assert bench.parse(["--no-full-run"]).full_run is False
    assert bench.parse(["--config", "c4"]).full_run is False
    assert bench.parse(["--config", "c5", "--full-run"]).full_run is True
    assert bench.parse(["--size", "64"]).full_run is False
