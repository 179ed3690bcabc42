"""CPU: the committed bench lines (latest profiles/rNN_bench_*.json, written by
bench.py on the MI355X) keep the driver's JSON contract: the required keys,
whole-job value = steps / elapsed, roofline and cpu_baseline objects, and the
parity flags the run checked."""
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
            "scaling", "vs_baseline", "dtype", "data", "config")


def _line(name):
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r[0-9][0-9]_bench_{name}.json")))
    if not paths:
        pytest.skip(f"no profiles/rNN_bench_{name}.json collected")
    with open(paths[-1]) as f:
        return json.loads(f.read().strip().splitlines()[-1])


@pytest.mark.parametrize("name", ["rt", "rast", "c4", "c5"])
def test_bench_line_contract(name):
    d = _line(name)
    for k in REQUIRED:
        assert k in d, k
    assert d["n_gpus"] >= 1 and d["steps"] > 0 and d["value"] > 0
    assert d["higher_is_better"] is True and d["data"] == "synthetic" and d["dtype"] == "f32"
    assert abs(d["value"] * d["ms_per_step"] / 1e3 - 1.0) < 1e-6          # value = steps / elapsed
    assert "workload" in d["config"]
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    if r["frac"] is not None:
        assert 0.0 <= r["frac"] <= 1.0, "a roofline fraction is bounded by the peak"
        assert r["frac"] == pytest.approx(r["achieved"] / r["peak"])
    cb = d["cpu_baseline"]
    assert cb["cores"] >= 1 and cb["kind"] in ("port", "reference") and cb["value"] > 0


def test_headline_line_checks_parity_and_roofline():
    d = _line("rt")
    assert d["metric"].startswith("frames/sec") and d["unit"] == "frames/s"
    assert d["frame_sha256_matches_golden"] is True and d["cpu_baseline"]["frame_matches_gpu"] is True
    r = d["roofline"]
    assert r["bound"] == "valu" and r["peak"] == pytest.approx(78.6432)       # no-FMA wave64 issue peak
    assert 0 < r["frac"] <= 1 and r["frac"] == pytest.approx(r["achieved"] / r["peak"])
    assert 0 < r["hbm_frac"] <= 1
    assert r["traffic"] > r["hbm_algorithmic_bytes_per_launch"] * 0.9     # PMC bytes >= the output written
    assert r["effective_vs_bruteforce"]["algorithmic_ops_per_launch"] > 0
    # the default line also pins C3 (the rasteriser) with its own roofline and CPU baseline
    c3 = d["rast"]
    assert c3["value"] > 0 and c3["single_frame_ms"] > 0 and 0 < c3["roofline"]["frac"] <= 1
    assert c3["cpu_baseline"]["frame_matches_gpu"] is True
