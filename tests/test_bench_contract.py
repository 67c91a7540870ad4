"""The parts of bench.py's one-line contract that need no GPU: the metric and its
BASELINE.json spelling, argument defaults, the roofline object (fields, arithmetic,
the PMC traffic lookup) and the algorithmic bytes of a launch (SURVEY.md 8(d):
BigBridge 5,281,084 B per frame)."""
from __future__ import annotations

import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_metric_is_baselines(bench):
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        assert bench.METRIC == json.load(f)["metric"]
    assert bench.HBM_PEAK_GBS == 8000.0


def test_default_arguments(bench):
    a = bench.parse_args([])
    assert (a.gpus, a.workload, a.frames, a.batch) == (1, "frame", 128, 64)  # two cold batch launches
    assert a.steps > 0 and a.warmup >= 0 and not a.no_graph
    a = bench.parse_args(["--gpus", "8", "--steps", "20", "--warmup", "5"])
    assert (a.gpus, a.steps, a.warmup) == (8, 20, 5)


def test_roofline_fields_and_arithmetic(bench):
    bench.ACHIEVABLE.clear()
    bench.ACHIEVABLE.update({"mix_2r3w_GBps": 5800.0, "read_GBps": 7000.0})
    try:
        r = bench.roofline(5_281_084, region_ms=0.116, steps=20, eager_ms=[0.011, 0.012], workload="frame",
                           read_bytes=2_135_356, kernel_ms=0.00579)
    finally:
        bench.ACHIEVABLE.clear()
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel_us_avg", "graph_us_per_launch",
              "algorithmic_bytes_per_launch", "frac_of_achievable", "read_frac"):
        assert k in r, k
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    # the timed region's own events / K, not the 200-launch graph
    assert r["kernel_us_avg"] == pytest.approx(5.8, abs=1e-3)
    assert r["region_us_per_launch"] == pytest.approx(5.8, abs=1e-3)
    # with the steady-state figure (the region after its first launch) that one is used
    r2 = bench.roofline(5_281_084, region_ms=0.116, steps=20, steady_ms=0.0055, steady_unit=1)
    assert r2["kernel_us_avg"] == pytest.approx(5.5, abs=1e-3) and r2["kernel_us_steady_unit"] == 1
    assert r2["region_us_per_launch"] == pytest.approx(5.8, abs=1e-3)
    assert r["achieved"] == pytest.approx(5_281_084 / 5.8e-6 / 1e9, rel=1e-3)
    assert r["frac"] == pytest.approx(r["achieved"] / 8000.0, abs=1e-4)
    assert r["frac_of_achievable"] == pytest.approx(r["achieved"] / 5800.0, abs=1e-4)
    assert r["graph_us_per_launch"] == pytest.approx(5.79, abs=1e-3)
    assert r["read_frac"] == pytest.approx(2_135_356 / 5.8e-6 / 1e9 / 8000.0, abs=1e-4)
    # the committed PMC profile backs the traffic figure of every workload
    for wl in ("frame", "batch", "tile8192", "tile8192_random"):
        t = bench.measured_traffic(wl)
        assert t is not None and t > 0, wl


def test_algorithmic_bytes_of_bigbridge(bench):
    """codes 1,923,388 + offsets 196,608 + raster 3,145,728 + T1 512 +
    T2 14,848 = 5,281,084 B for one BigBridge frame."""
    import metalhuffman_amd as mh
    from metalhuffman_amd import frames as F
    ef = mh.encode_frame(F.bigbridge())
    t1, t2 = ef.tables()
    used_t2 = 14_848
    assert bench.algo_bytes([ef], used_t2) == 5_281_084
    assert bench.algo_read_bytes([ef], used_t2) == 5_281_084 - 3_145_728
