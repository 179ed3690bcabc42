"""CPU: the committed bench lines (latest profiles/rNN_bench_*.json, written by
bench.py on the MI355X) keep the driver's JSON contract: the required keys,
whole-job value = steps / elapsed, roofline and cpu_baseline objects, and the
parity flags the run checked."""
import json
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
            "scaling", "vs_baseline", "dtype", "data", "config")


def _line(name):
    """The latest committed driver-shaped default line (profiles/rNN_bench_default.json): the C2
    metric line itself for "rt", its C3/C4/C5 sub-record otherwise (the
    contract is pinned on the current line, not on an old per-workload file)."""
    _, d = _default()
    return d if name == "rt" else d[name]


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


def _default():
    """The latest committed driver-shaped default line (profiles/rNN_bench_default.json)."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_bench_default.json")))
    if not paths:
        pytest.skip("no profiles/rNN_bench_default.json collected")
    with open(paths[-1]) as f:
        return os.path.basename(paths[-1])[:3], json.loads(f.read().strip().splitlines()[-1])


def test_default_line_pins_every_config():
    """The default line (what the driver runs) carries C2 and the C3/C4/C5 sub-records, each
    with its roofline, its CPU baseline compared with the GPU's pixels, and its parity flags."""
    rnd, d = _default()
    for k in REQUIRED:
        assert k in d, k
    assert d["frame_sha256_matches_golden"] is True and d["frames_identical_in_call"] is True
    assert d["cpu_baseline"]["frame_matches_gpu"] is True
    for name in ("c4", "c5"):
        s = d[name]
        assert s["value"] > 0 and s["frames_identical_in_call"] is True
        assert s["cpu_baseline"]["sample_matches_gpu"] is True and s["cpu_baseline"]["value"] > 0
        assert "frac" in s["roofline"]
    assert d["rast"]["cpu_baseline"]["frame_matches_gpu"] is True and d["rast"]["frames_identical_in_batch"] is True


def test_default_line_roofline_is_the_kernels_own():
    """each workload's dominant-kernel fraction is its SQ lane-ops over that
    kernel's own live HIP-event time (frac), beside the call-span figure (frac_call) and the whole
    frame's (frac_frame); C5's CPU baseline is SURVEY 8d's 1,024-pixel stratified sample."""
    rnd, d = _default()
    if rnd < "r04":
        pytest.skip("the kernel-own fractions start with round 4's bench")
    for r, kern in ((d, "rt_lattice_kernel"), (d["c4"], "rt_lattice_lights_kernel"), (d["c5"], "rt_big_primary_kernel")):
        ro = r["roofline"]
        assert ro["kernel"] == kern and ro["kernel_ms"] > 0 and ro["kernel_launches"] >= 1
        assert ro["frac"] is not None and 0 < ro["frac"] <= 1
        assert ro["frac"] == pytest.approx(ro["achieved"] / ro["peak"])
        assert ro["frac_frame"] is not None and 0 < ro["frac_frame"] <= 1
        if ro.get("frac_call") is not None:
            assert ro["frac_call"] <= ro["frac"] * 1.001      # the call's span includes the kernel's
        live = r["kernel_ms_live"][kern]
        assert live["busy_ms"] / live["launches"] == pytest.approx(ro["kernel_ms"])
        assert live["busy_ms"] <= live["total_ms"] * (1 + 1e-9)
    if rnd >= "r05":   # every fraction also on the committed rocprofv3 mean
        for r in (d, d["c4"], d["c5"]):
            fp = r["roofline"]["frac_profile_mean"]
            assert fp is not None and 0 < fp <= 1 and "kernel_stats.csv" in r["roofline"]["frac_profile_mean_note"]
        assert d["c5"]["roofline"]["frac_profile_mean"] >= 0.30   # the C5 walk
    assert d["c5"]["cpu_baseline"]["sampled_pixels"] >= 1024
    assert d["c5"]["cpu_baseline"]["threads"] >= 1 and d["c5"]["cpu_baseline"]["cores"] == 1


def test_default_line_measures_the_boundary():
    """the host-buffer Draw (cg_rt_render / cg_rt_render_frames), pageable and
    pinned, single frame and pipelined, every frame golden."""
    rnd, d = _default()
    if rnd < "r04":
        pytest.skip("the draw record starts with round 4's bench")
    dr = d["draw"]
    assert dr["all_frames_golden"] is True
    assert dr["single_frame_ms"] > 0 and dr["fps_pageable"] > 0 and dr["fps_pinned"] > 0
    assert dr["fps_pinned"] < d["value"]          # the PCIe copy is never free


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


def _bench():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_roofline_frac_is_tied_to_the_profiled_machine_code(monkeypatch):
    """the executed-work fraction scales SQ counters of one build of a
    kernel; a profile whose code_sha256 differs from this build's kernel code nulls it."""
    import cgamd
    import codeobj
    if not os.path.exists(cgamd.LIB_PATH):
        pytest.skip("libcgamd.so not built")
    b = _bench()
    have = codeobj.kernel_sha256("rt_lattice_kernel", cgamd.LIB_PATH)
    assert have and len(have) == 64
    prof = {"valu_lane_ops_per_launch": 5.7e10, "frames_per_launch": 32, "wave_state_frac": {}}
    monkeypatch.setattr(b, "load_sq", lambda kernel, section="rt": dict(prof, code_sha256="0" * 64))
    r = b.valu_roofline("rt_lattice_kernel", "rt", 32, 1.0, 1.5)
    assert r["frac"] is None and r["achieved"] is None and "re-profile" in r["frac_null_reason"]
    monkeypatch.setattr(b, "load_sq", lambda kernel, section="rt": dict(prof))          # no hash recorded
    assert b.valu_roofline("rt_lattice_kernel", "rt", 32, 1.0, 1.5)["frac"] is None
    monkeypatch.setattr(b, "load_sq", lambda kernel, section="rt": dict(prof, code_sha256=have))
    r = b.valu_roofline("rt_lattice_kernel", "rt", 32, 1.0, 1.5)
    assert r["frac"] == pytest.approx(5.7e10 / 1.5e-3 / 1e12 / r["peak"])


def test_kernel_hash_tracks_machine_code():
    """Template instances are hashed together, unknown kernels have no hash, and different
    kernels hash differently."""
    import cgamd
    import codeobj
    if not os.path.exists(cgamd.LIB_PATH):
        pytest.skip("libcgamd.so not built")
    hs = {k: codeobj.kernel_sha256(k, cgamd.LIB_PATH)
          for k in ("rt_lattice_kernel", "rt_lattice_lights_kernel", "rt_big_primary_kernel", "rast_fill_kernel")}
    assert all(hs.values()) and len(set(hs.values())) == len(hs)
    assert codeobj.kernel_sha256("no_such_kernel", cgamd.LIB_PATH) is None


def test_kernel_hash_ignores_descriptor_layout(monkeypatch):
    """The descriptor's code-entry offset (bytes 16-23: where the code sits, which moves when
    another kernel of the code object changes size) does not change the hash; the code bytes
    and the rest of the descriptor (registers, LDS, scratch) do."""
    import codeobj
    kd = bytes(range(64))
    base = {"_Z9my_kernelv": b"\x01\x02\x03\x04", "_Z9my_kernelv.kd": kd}

    def h(syms):
        monkeypatch.setattr(codeobj, "kernel_symbols", lambda lib_path=None: syms)
        return codeobj.kernel_sha256("my_kernel")
    moved = dict(base, **{"_Z9my_kernelv.kd": kd[:16] + b"\xff" * 8 + kd[24:]})
    regs = dict(base, **{"_Z9my_kernelv.kd": kd[:48] + b"\xff" + kd[49:]})
    code = dict(base, **{"_Z9my_kernelv": b"\x01\x02\x03\x05"})
    assert h(base) == h(moved)
    assert h(base) != h(regs) and h(base) != h(code)


def test_stratified_sample_covers_the_whole_frame():
    """C4/C5 CPU baselines: a fixed stratified sample -- one pixel
    per cell of an n x n grid over the whole frame, C5's 1,024 pixels -- every cell once, inside
    the frame, reaching both borders' cells."""
    b = _bench()
    for W, H, n in ((1920, 1080, 32), (3840, 2160, 128)):
        xy = b.stratified_pixels(W, H, n)
        assert len(xy) == n * n and len({(x, y) for x, y in xy}) == n * n
        assert xy[:, 0].min() >= 0 and xy[:, 0].max() < W and xy[:, 1].min() >= 0 and xy[:, 1].max() < H
        cells = {(x * n // W, y * n // H) for x, y in xy}
        assert cells == {(i, j) for i in range(n) for j in range(n)}
    assert b.CPU_STRATA["c5"] ** 2 == 1024


def test_cpu_info_reports_physical_cores():
    b = _bench()
    ci = b.cpu_info()
    assert 1 <= ci["usable_cores"] <= ci["physical_cores"] <= ci["logical_cpus"]


def test_default_line_useful_fraction_matches_counts():
    """C2's, C4's and C5's dominant-kernel rooflines carry useful_frac, the
    reference's own per-ray arithmetic the kernel performs over its time; its op count per frame is
    the committed counts file's (profiles/rNN_work_counts.json, scripts/work_counts.py) recomputed
    with SURVEY 8d's weights."""
    import glob
    rnd, d = _default()
    if rnd < "r06":
        pytest.skip("useful_frac starts with round 6's bench")
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_work_counts.json")))
    assert paths, "no committed work counts"
    with open(paths[-1]) as f:
        wc = json.load(f)
    weights = wc["weights"]
    for name, r in (("rt", d), ("c4", d["c4"]), ("c5", d["c5"])):
        ro, w = r["roofline"], wc["workloads"][name]
        assert w["dominant_kernel"] == ro["kernel"]
        ops = sum(weights[k] * w["counts_per_frame"][k] for k in w["dominant_kinds"])
        assert ops == pytest.approx(w["useful_ops_per_frame"])
        assert ro["useful_ops_per_frame"] == pytest.approx(ops)
        assert ro["useful_counts_file"] == "profiles/" + os.path.basename(paths[-1])
        assert 0 < ro["useful_frac"] <= 1
        assert ro["useful_frac"] == pytest.approx(ro["useful_achieved"] / ro["peak"])
