"""Benchmark: frames/sec + Mray/s of the 1080p Cornell-box raytracer
(BASELINE.json metric, config C2: 1920x1080, focal 1080, camera (0,0,-3),
one light, 3x3 supersampling) on N MI355X.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload rt|rast|c4|c5]
                  [--no-cpu-baseline]

--workload rt (default) is the metric's config C2; rast is C3; c4 (3840x2160,
8x8 area light = 64 lights) and c5 (1080p over 1M random triangles) are the
build-defined SURVEY.md 8d workloads, measured the same way.

A step is one whole frame, inputs resident in HBM.  N = 1: frames rendered 32
per cg_rt_render_frames_device call.  N > 1 (default layout `bands`): every
rank renders one balanced contiguous band of rows through the library's
cg_rt_render_frames_dist (csrc/cg_dist.hip); ranks > 0 send their bands in the
RGB24 wire format to rank 0 over RCCL point-to-point (xGMI), and rank 0
assembles the frames in place.  `--layout stripes` (the gloo rehearsal's
default) is the older round-robin stripes + gather + unstripe path.

N > 1 either comes from a launcher (torchrun: WORLD_SIZE/RANK/LOCAL_RANK/
MASTER_* in the environment; WORLD_SIZE must equal --gpus) or, when WORLD_SIZE
is unset, from bench.py itself: the parent starts N fresh rank processes
before anything touches the GPU (launch_ranks), each with RANK = LOCAL_RANK =
r, WORLD_SIZE = N and MASTER_ADDR/PORT = 127.0.0.1:<free port>, relays rank 0's
single JSON line and exits non-zero if any rank fails or outlives
--rank-timeout.  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes
import datetime
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))


# ---- N > 1 without an external launcher -----------------------------------
# Everything here runs before torch / the library are imported: the parent never touches the GPU,
# and its children are fresh processes (never an exec of an initialised one).

def argv_gpus(argv):
    """--gpus N / --gpus=N from a command line (1 when absent)."""
    for i, a in enumerate(argv):
        if a == "--gpus" and i + 1 < len(argv):
            return int(argv[i + 1])
        if a.startswith("--gpus="):
            return int(a.split("=", 1)[1])
    return 1


def free_port(host="127.0.0.1"):
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind((host, 0))
        return sk.getsockname()[1]


def launch_plan(n, argv, base_env, port, addr="127.0.0.1", python=None):
    """(argv, env) of each of the n rank processes: the same bench.py command line, with the
    torch.distributed rendezvous of one node in the environment."""
    python = python or sys.executable
    plan = []
    for r in range(n):
        env = dict(base_env)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR=addr, MASTER_PORT=str(port))
        plan.append(([python, "-u"] + list(argv), env))
    return plan


def _die_with_parent():
    """Child side of Popen: SIGKILL this rank if the launching parent dies (Linux prctl)."""
    try:
        import ctypes as _c
        import signal as _s
        _c.CDLL("libc.so.6", use_errno=True).prctl(1, int(_s.SIGKILL))   # PR_SET_PDEATHSIG
    except (OSError, AttributeError):
        pass


def run_ranks(plan, timeout_s=None, poll_s=0.05, out=None, err=None):
    """Start every rank of `plan` as a child process, rank 0's stdout to `out` (the parent's
    stdout: its one JSON line), the other ranks' stdout to `err`; return 0 when every rank exits
    0, else the first failing rank's exit code (a signal -s as 128 + s), after terminating the
    others.  A rank still running after timeout_s seconds fails the job with 124."""
    import signal
    import subprocess
    out = out if out is not None else sys.stdout
    err = err if err is not None else sys.stderr
    out.flush()
    err.flush()
    procs = []
    try:
        for r, (cmd, env) in enumerate(plan):
            procs.append(subprocess.Popen(cmd, env=env, cwd=ROOT, stdout=out if r == 0 else err, stderr=err,
                                          preexec_fn=_die_with_parent))
        t0 = time.monotonic()
        failed = None
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                r, c = bad[0]
                failed = 128 - c if c < 0 else c
                print(f"bench.py launcher: rank {r} exited with {c}; stopping the other ranks",
                      file=err, flush=True)
                break
            if all(c == 0 for c in codes):
                return 0
            if timeout_s and time.monotonic() - t0 > timeout_s:
                print(f"bench.py launcher: ranks still running after {timeout_s} s; stopping them",
                      file=err, flush=True)
                failed = 124
                break
            time.sleep(poll_s)
        return failed
    finally:
        for p in procs:                     # exactly the PIDs started here
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        end = time.monotonic() + 10.0
        for p in procs:
            try:
                p.wait(timeout=max(0.1, end - time.monotonic()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()


def launch_if_needed(argv):
    """None when this process is a rank (a launcher set WORLD_SIZE, or N = 1); otherwise the
    exit code of the N-rank job started here.  WORLD_SIZE set and != --gpus fails loudly."""
    n = argv_gpus(argv)
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        given = any(a == "--gpus" or a.startswith("--gpus=") for a in argv)
        if given and int(ws) != n:
            raise SystemExit(f"bench.py: WORLD_SIZE={ws} from the launcher but --gpus {n}")
        return None
    if n <= 1:
        return None
    timeout = 0.0
    for i, a in enumerate(argv):
        if a == "--rank-timeout" and i + 1 < len(argv):
            timeout = float(argv[i + 1])
        elif a.startswith("--rank-timeout="):
            timeout = float(a.split("=", 1)[1])
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")     # dmabuf IPC only on this host driver
    plan = launch_plan(n, [os.path.abspath(__file__)] + list(argv), env, free_port())
    return run_ranks(plan, timeout_s=timeout or None)


if __name__ == "__main__":
    _rc = launch_if_needed(sys.argv[1:])
    if _rc is not None:
        sys.exit(_rc)
sys.path[:0] = [os.path.join(ROOT, "computer-graphics_amd"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tests", "golden")]

import numpy as np  # noqa: E402
import torch  # noqa: E402  (import before libcgamd: one HIP runtime in the process)
import torch.distributed as dist  # noqa: E402

import cgamd  # noqa: E402
import cgdist  # noqa: E402
import codeobj  # noqa: E402

PEAK_FP32_TFLOPS = 157.3    # MI355X_MICROARCH.md, Peak FP32 (vector), spec: counts an FMA as 2
# What a kernel without FMA (parity forbids contraction) can issue: a wave64 VALU
# instruction takes 2 cycles on a SIMD (MI355X_MICROARCH.md), so 256 CU x 4 SIMD x
# 32 lanes x 2.4 GHz = 78.6 T lane-ops/s.
PEAK_VALU_LANE_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
PEAK_HBM_GBS = 8000.0       # MI355X_MICROARCH.md, HBM3E peak, spec

RT_W, RT_H, RT_F = 1920, 1080, 1080.0
RAST_W, RAST_H, RAST_F = 1920, 1080, 768.0

# RT workloads: (width, height, focal, light set, scene, default stripe rows)
RT_WORKLOADS = {
    "rt": dict(W=1920, H=1080, F=1080.0, area=None, random=None, stripe=cgdist.LATTICE_STRIPE,
               name="rt_cornell_1920x1080_f1080_ss3x3"),
    "c4": dict(W=3840, H=2160, F=2160.0, area=(0.1, 8), random=None, stripe=cgdist.DEFAULT_STRIPE,
               name="rt_cornell_3840x2160_f2160_ss3x3_soft8x8"),
    "c5": dict(W=1920, H=1080, F=1080.0, area=None, random=1_000_000, stripe=32,
               name="rt_random1M_1920x1080_f1080_ss3x3"),
    # C2 after the reference's LEFT key (yaw 0.1745 rad, skeleton.cpp:233-244): the
    # yawed camera takes the lattice kernel with per-pixel columns (rows shared)
    "yaw": dict(W=1920, H=1080, F=1080.0, area=None, random=None, stripe=cgdist.LATTICE_STRIPE, yaw=0.1745,
                name="rt_cornell_1920x1080_f1080_ss3x3_yaw0.1745"),
    # C5 after the yaw key: the large-scene lattice with per-pixel columns
    "c5yaw": dict(W=1920, H=1080, F=1080.0, area=None, random=1_000_000, stripe=32, yaw=0.1745,
                  name="rt_random1M_1920x1080_f1080_ss3x3_yaw0.1745"),
    # SURVEY.md 8d's C2 variant: the reference's literal focal length 256 at 1080p
    # (most rays leave the box through the open front and hit nothing)
    "f256": dict(W=1920, H=1080, F=256.0, area=None, random=None, stripe=cgdist.LATTICE_STRIPE,
                 name="rt_cornell_1920x1080_f256_ss3x3"),
}


def rt_ops(counters):
    """SURVEY.md 8d algorithmic FP32 op count of a frame (or rows subset)."""
    return (33 * counters["n_t"] + 37 * counters["n_uv"] + 29 * counters["n_sph"]
            + 11 * counters["n_ray"] + 40 * counters["n_dl"])


def load_row_counters():
    """Per-row work counters of C2, generated by tests/golden/make_golden.py."""
    path = os.path.join(ROOT, "tests", "golden", "rt_1080p_row_counters.npz")
    if not os.path.exists(path):
        return None
    z = np.load(path)
    return {k: z[k].astype(np.int64) for k in ("n_ray", "n_t", "n_uv", "n_sph", "n_dl")}


def load_traffic(workload):
    """HBM bytes per frame of the dominant kernel(s) from the committed rocprofv3
    PMC summary (profiles/pmc_summary.json: bytes per launch / frames per launch),
    corrected per MI355X_MICROARCH.md (FETCH_SIZE x2 for wide streaming reads);
    None when absent."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(path) as f:
            sec = json.load(f).get(workload, {})
    except (OSError, ValueError):
        return None
    b = sec.get("hbm_bytes_per_launch")
    return None if b is None else b / sec.get("frames_per_launch", 1)


def load_sq(kernel, section="rt"):
    """Executed-work figures of a kernel (rocprofv3 SQ PMC counters per launch,
    scripts/sq_summary.py -> profiles/pmc_summary.json), with the frames per launch
    they were collected at; None when absent."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_summary.json")) as f:
            sec = json.load(f).get(section, {})
    except (OSError, ValueError):
        return None
    sq = sec.get("sq_kernels", {}).get(kernel)
    if sq is None:
        return None
    return dict(sq, frames_per_launch=sq.get("frames_per_launch", sec.get("frames_per_launch", 1)))


def profile_matches_binary(sq, kernel):
    """(ok, reason): the committed SQ profile was collected on the machine code of `kernel`
    that this libcgamd.so carries (codeobj.kernel_sha256: the kernel's gfx950 code + descriptor)."""
    want = sq.get("code_sha256")
    try:
        have = codeobj.kernel_sha256(kernel, cgamd.LIB_PATH)
    except (OSError, ValueError) as e:
        return False, f"cannot read the kernel's code object: {e}"
    if want is None:
        return False, "the committed SQ profile records no code_sha256 (collected before code identity was tracked)"
    if have != want:
        return False, (f"the committed SQ profile was collected on other machine code of {kernel} "
                       f"(profile {want[:12]}, this build {str(have)[:12]}): re-profile before quoting a fraction")
    return True, "profile code_sha256 == this build's"


def valu_roofline(kernel, section, frames, share, launch_ms):
    """The executed-work VALU roofline of one launch: SQ_INSTS_VALU x 64 lane-ops per
    frame (from the committed profile of this kernel on this workload) x frames x the
    share of the frame this launch renders, over the live launch time, against the
    no-FMA issue peak.  None when the kernel has no committed SQ profile; frac None
    (with the reason) when that profile describes other machine code than this build's."""
    sq = load_sq(kernel, section)
    if not sq or not launch_ms:
        return None
    ok, why = profile_matches_binary(sq, kernel)
    if not ok:
        return {"bound": "valu", "achieved": None, "peak": PEAK_VALU_LANE_TOPS, "unit": "T lane-ops/s",
                "frac": None, "frac_null_reason": why, "kernel": kernel}
    ops = sq["valu_lane_ops_per_launch"] / sq["frames_per_launch"] * frames * share
    achieved = ops / (launch_ms * 1e-3) / 1e12
    return {"bound": "valu", "achieved": achieved, "peak": PEAK_VALU_LANE_TOPS, "unit": "T lane-ops/s",
            "frac": achieved / PEAK_VALU_LANE_TOPS, "kernel": kernel, "executed_lane_ops_per_launch": ops,
            "basis": "executed VALU lane-ops (rocprofv3 SQ_INSTS_VALU x 64 per frame of this kernel, "
                     "profiles/pmc_summary.json) / live HIP-event launch time; peak = no-FMA wave64 issue "
                     "rate (2 cycles per VALU instruction)",
            "profile_wave_state": sq.get("wave_state_frac"), "profile_code": why}


def frame_valu(section, frames, share, frame_ms):
    """Every library kernel of the frame (profiles/pmc_summary.json frame_sq: each kernel's
    executed SQ lane-ops per frame) over the frames' whole device time: the fraction of the
    no-FMA issue peak the frame as a whole runs at (prepare, certificates, lists, walks,
    shading), beside the dominant kernel's own `frac`.  None fields with the reason when the
    profile is missing or any of its kernels' machine code differs from this build's."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_summary.json")) as f:
            fs = json.load(f).get(section, {}).get("frame_sq")
    except (OSError, ValueError):
        fs = None
    if not fs or not frame_ms:
        return {"frac_frame": None, "frac_frame_null_reason": "no committed whole-frame SQ profile"}
    stale = []
    for k, r in fs["kernels"].items():
        try:
            have = codeobj.kernel_sha256(k, cgamd.LIB_PATH)
        except (OSError, ValueError):
            have = None
        if have != r.get("code_sha256"):
            stale.append(k)
    if stale:
        return {"frac_frame": None, "frac_frame_null_reason": "profiled on other machine code of " + ", ".join(stale)}
    ops = fs["valu_lane_ops_per_frame"] * frames * share
    t = ops / (frame_ms * 1e-3) / 1e12
    return {"frac_frame": t / PEAK_VALU_LANE_TOPS, "frame_achieved": t, "frame_lane_ops": ops,
            "frame_ms": frame_ms, "frame_kernels": sorted(fs["kernels"]),
            "frame_basis": "sum over every kernel of the frame of its executed SQ lane-ops (profiles/pmc_summary.json "
                           "frame_sq) / the frames' device time (HIP events around each call)"}


def profile_mean_ms(kernel, section):
    """(mean ms per launch, file) of a kernel in the latest committed rocprofv3 --stats summary of
    this workload (profiles/rNN_<section>_kernel_stats.csv); (None, None) when absent."""
    import csv
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r[0-9][0-9]_{section}_kernel_stats.csv")))
    if not paths:
        return None, None
    with open(paths[-1]) as f:
        for r in csv.DictReader(f):
            if f"cg::{kernel}" in r["Name"].split("(")[0]:
                return float(r["AverageNs"]) / 1e6, os.path.basename(paths[-1])
    return None, os.path.basename(paths[-1])


def kernel_roofline(kern, section, steps, share, kt, call_launch_ms, fpl_call):
    """The dominant kernel's executed-work VALU roofline on ITS OWN time: lane-ops per launch
    (committed SQ profile) over the live HIP-event launch duration from the library's kernel
    timing over the timed region.  `frac_call` beside it: the same lane-ops over the call's span
    per launch (certificates, prepare and launch gaps included)."""
    kms, kn = live_kernel_ms(kt, kern)
    fpl = steps / kn if kn else fpl_call            # frames per launch in the timed region
    roof = (valu_roofline(kern, section, fpl, share, kms) if kms else None) or \
        {"bound": "valu", "achieved": None, "peak": PEAK_VALU_LANE_TOPS, "unit": "T lane-ops/s", "frac": None,
         "kernel": kern, "note": "no committed SQ profile of this kernel on this workload, or no live kernel time"}
    call = valu_roofline(kern, section, fpl_call, share, call_launch_ms)
    # the same lane-ops over the committed rocprofv3 mean launch duration of this kernel (VERDICT r04
    # item 6: the fraction reproducible from profiles/); the profile's launches carry the SQ
    # profile's frames per launch
    pm_ms, pm_file = profile_mean_ms(kern, section)
    sq = load_sq(kern, section)
    pm = valu_roofline(kern, section, sq["frames_per_launch"], share, pm_ms) if (sq and pm_ms) else None
    roof.update({"frac_profile_mean": pm.get("frac") if pm else None,
                 "frac_profile_mean_note": (f"lane-ops per launch over the mean launch duration in profiles/{pm_file} "
                                            "(rocprofv3 --kernel-trace --stats)") if pm_file else
                                           "no committed rocprofv3 summary of this workload"})
    roof.update(useful_roofline(section, kern, fpl, share, kms))
    roof.update({"kernel": kern, "kernel_ms": kms, "kernel_launches": kn, "frames_per_launch": fpl,
                 "kernel_ms_note": "HIP events recorded by the library around each launch of this kernel, on the "
                                   "stream it runs on, over the timed region (cg_kernel_timing): its busy time (the "
                                   "union of its launches' spans) per launch",
                 "frac_call": call.get("frac") if call else None,
                 "frac_call_note": "the same lane-ops over the call's HIP-event span per launch (the call's other "
                                   "kernels and gaps included)"})
    return roof


def load_work_counts():
    """The committed counts of the reference's own per-ray work the kernels perform
    (scripts/work_counts.py on the counting build -> the latest profiles/rNN_work_counts.json);
    None when absent."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_work_counts.json")))
    if not paths:
        return None, None
    with open(paths[-1]) as f:
        return json.load(f), os.path.basename(paths[-1])


def useful_roofline(workload, kernel, frames, share, launch_ms):
    """the dominant kernel's USEFUL fraction -- the reference's own arithmetic
    it performs (SURVEY 8d op weights times the counted t stages, u/v stages, sphere tests, rays and
    DirectLights, profiles/rNN_work_counts.json) over its live launch time, against the same no-FMA
    issue peak as `frac`.  Certificate FP64, masks, index math and packing count as overhead here,
    so frac - useful_frac is what the kernel spends beyond the reference's arithmetic."""
    wc, fname = load_work_counts()
    w = (wc or {}).get("workloads", {}).get(workload)
    if not w or not launch_ms or w.get("dominant_kernel") != kernel:
        return {"useful_frac": None, "useful_note": "no committed work counts for this kernel"}
    ops = w["useful_ops_per_frame"] * frames * share
    t = ops / (launch_ms * 1e-3) / 1e12
    return {"useful_frac": t / PEAK_VALU_LANE_TOPS, "useful_achieved": t, "useful_ops_per_launch": ops,
            "useful_ops_per_frame": w["useful_ops_per_frame"], "useful_counts_per_frame": w["counts_per_frame"],
            "useful_kinds": w["dominant_kinds"], "useful_counts_file": f"profiles/{fname}",
            "useful_note": "the reference's own FP32/FP64 per-ray operations this kernel performs (SURVEY 8d weights: "
                           "t stage 33, u/v stage 37, sphere 29, ray 11, DirectLight 40; counted on the "
                           "CG_WORK_COUNT build) / its live launch time / the no-FMA issue peak"}


def live_kernel_ms(kt, kernel):
    """(ms per launch, launches) of a kernel timed with HIP events inside the library over the
    timed region (cg_kernel_timing: events around each launch, on the stream it runs on): its
    busy time (the union of its launches' spans -- two large-scene frames in flight overlap
    their launches) over its launches."""
    ms, busy, n = (kt or {}).get(kernel, (0.0, 0.0, 0))
    return (busy / n if n else None), n


def read_kernel_times():
    names = ("rt_prepare_kernel", "rt_tile_cert_kernel", "rt_lattice_units_kernel", "rt_lattice_kernel",
             "rt_lattice_lights_kernel", "rt_pixel_kernel", "rt_big_primary_kernel", "rt_shadow_hints_kernel",
             "rt_big_frame", "rast_fill_kernel", "rast_post_kernel")
    return {k: cgamd.kernel_time(k) for k in names}


def cpu_info():
    """The host's CPUs: model, logical CPUs, physical cores (unique (package, core) pairs of
    /proc/cpuinfo), the CPUs this process may run on, and the cgroup CPU quota."""
    model, cores, logical = platform.processor() or platform.machine(), set(), 0
    try:
        pkg = core = None
        with open("/proc/cpuinfo") as f:
            for line in f:
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if k == "processor":
                    logical += 1
                elif k == "model name":
                    model = v
                elif k == "physical id":
                    pkg = v
                elif k == "core id":
                    core = v
                elif not k and pkg is not None:
                    cores.add((pkg, core))
                    pkg = core = None
        if pkg is not None:
            cores.add((pkg, core))
    except OSError:
        pass
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        quota = None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        pass
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    physical = len(cores) or logical or 1
    usable = min(physical, affinity, int(quota) if quota else physical)
    return {"model": model, "logical_cpus": logical or os.cpu_count(), "physical_cores": physical,
            "affinity_cpus": affinity, "cgroup_quota_cpus": quota, "usable_cores": max(1, usable)}


# the restatement's speed against the reference's own -O3 build.  The task's
# rules make the reference unbuildable here (it needs SDL2, absent, and building it against
# stand-in headers is not allowed), so the ratio is stated as a band, not certified:
# profiles/r04_cpu_restatement_timing.json.
REFERENCE_TIMING = {
    "certified": False,
    "reason": "the reference needs SDL2 (absent); builds against stand-in headers are outside the task's rules",
    "reference_c1_ms_survey": 268.0,
    "reference_c1_note": "SURVEY.md 6: the reference's -O3 build timed by the survey in its container (C1, 320x256)",
    "restatement_c1_ms_band": "profiles/r04_cpu_restatement_timing.json (same op sequence per ray; timed here)",
    "note": "the restatement performs the reference's FP32/FP64 operations per ray in the same order, -O3, no "
            "-march; its absolute speed relative to the reference build is known only to the band stated there",
}


def reference_timing():
    rec = dict(REFERENCE_TIMING)
    try:
        with open(os.path.join(ROOT, "profiles", "r04_cpu_restatement_timing.json")) as f:
            t = json.load(f)
        rec["restatement_c1_ms"] = t["restatement_ms"]
        rec["ratio_band"] = t["ratio_restatement_over_reference"]
    except (OSError, ValueError, KeyError):
        pass
    return rec


def cpu_baseline_rt(gpu_frame):
    """The oracle (this repo's bit-exact CPU restatement of the reference,
    single thread, -O3, no -march) on one full C2 frame; plus the SURVEY.md 8d
    aggregate on the box's physical cores (as many as this process may use)."""
    import oracle
    oracle.build()
    p = oracle.rt_params(RT_W, RT_H, RT_F)
    ci = cpu_info()
    t0 = time.perf_counter()
    ref = oracle.rt_draw(p)
    dt = time.perf_counter() - t0
    rec = {"value": 1.0 / dt, "unit": "frames/s", "cores": 1, "kind": "port",
           "sample": f"1 full {RT_W}x{RT_H} f{int(RT_F)} frame, 1 thread, {dt:.2f} s; CPU {ci['model']}",
           "frame_matches_gpu": bool(np.array_equal(ref, gpu_frame)), "host": ci,
           "vs_reference": reference_timing()}
    n = int(os.environ.get("CG_CPU_BASELINE_THREADS", "0")) or ci["usable_cores"]
    if n > 1:
        t0 = time.perf_counter()
        ref_mt = oracle.rt_draw(p, threads=n)
        dmt = time.perf_counter() - t0
        rec["aggregate"] = {"value": 1.0 / dmt, "unit": "frames/s", "cores": n,
                            "sample": f"1 full frame, {n} threads (rows interleaved) = min(physical cores "
                                      f"{ci['physical_cores']}, CPUs usable by this process "
                                      f"{ci['affinity_cpus']}, cgroup quota {ci['cgroup_quota_cpus']}), {dmt:.2f} s",
                            "frame_matches_gpu": bool(np.array_equal(ref_mt, gpu_frame))}
    return rec


def stratified_pixels(W, H, n_side):
    """SURVEY.md 8d's fixed stratified sample: the centre pixel of every cell of an n_side x n_side
    grid over the whole W x H frame (row-major cells)."""
    xs = ((np.arange(n_side) + 0.5) * W / n_side).astype(np.int64)
    ys = ((np.arange(n_side) + 0.5) * H / n_side).astype(np.int64)
    return np.stack(np.meshgrid(xs, ys), -1).reshape(-1, 2)


# C4 / C5 CPU samples: strata per side (C5: SURVEY 8d's 1,024 pixels; C4's pixels are ~6,000x
# cheaper, so a 128 x 128 grid costs about the same CPU time)
CPU_STRATA = {"c4": 128, "c5": 32, "c5yaw": 32, "yaw": 64, "f256": 64}


def cpu_threads(ci):
    """Threads for the CPU sample: the usable physical cores, capped by the job's CPU share
    (OMP_NUM_THREADS, 16 on the GPU box: its CPUs are shared between jobs)."""
    cap = 0
    for var, default in (("CG_CPU_BASELINE_THREADS", "0"), ("OMP_NUM_THREADS", "16")):
        try:
            cap = cap or int(os.environ.get(var, default) or 0)
        except ValueError:
            pass
    return max(1, min(ci["usable_cores"], cap or 16))


def cpu_baseline_rt_sampled(wl, gpu_frame, workload):
    """C4/C5 (and the C2 variants): the oracle on a fixed stratified pixel sample of the whole
    frame, pixels spread over the usable cores; the per-core rate comes from the
    workers' own CPU time (per-thread clocks, summed), extrapolated to the frame by pixel count,
    and the sampled pixels are compared with the GPU frame."""
    import oracle
    import make_golden as mg
    oracle.build()
    W, H = wl["W"], wl["H"]
    cfg = dict(width=W, height=H, focal=wl["F"], cam=[0, 0, -3.0, 1],
               R=list(cgamd.yaw_matrix(wl["yaw"])) if wl.get("yaw") else None,
               lights=[[[0.0, -0.5, -0.7, 1.0], [14.0, 14.0, 14.0]]])
    if wl["area"]:
        cfg["area"] = dict(side=wl["area"][0], n=wl["area"][1])
    if wl["random"]:
        cfg["scene"] = dict(random=wl["random"], seed=0x5EED)
    p, scene = mg.rt_params_of(cfg), mg.rt_oracle_scene(cfg)
    frame = gpu_frame.reshape(H, W)
    side = CPU_STRATA.get(workload, 32)
    xy = stratified_pixels(W, H, side)
    ci = cpu_info()
    nt = cpu_threads(ci)
    # per-core rate from the oracle workers' own CPU time (CLOCK_THREAD_CPUTIME_ID per worker;
    # the process's CPU time also counts the HIP runtime's and torch's threads)
    c0, t0 = time.process_time(), time.perf_counter()
    ref, cpu_s = oracle.rt_draw_pixels(p, xy, scene=scene, threads=nt, worker_cpu=True)
    proc_s, wall = time.process_time() - c0, time.perf_counter() - t0
    eq = ref == frame[xy[:, 1], xy[:, 0]]
    n = len(xy)
    return {"value": n / cpu_s / (W * H), "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": f"{n} pixels: the centre of each cell of a {side}x{side} grid over the whole {W}x{H} frame "
                      f"(fixed stratified sample, SURVEY.md 8d), on {nt} threads, {wall:.1f} s wall / {cpu_s:.1f} s of the "
                      f"workers' own CPU time; per-core rate = pixels / worker CPU seconds, extrapolated to the frame by "
                      f"pixel count; CPU {ci['model']}",
            "sampled_pixels": n, "threads": nt, "cpu_seconds": cpu_s, "process_cpu_seconds": proc_s,
            "wall_seconds": wall,
            "sample_matches_gpu": bool(eq.all()), "sample_mismatches": int((~eq).sum()),
            "aggregate": {"value": n / wall / (W * H), "unit": "frames/s", "cores": nt,
                          "sample": f"the same {n} pixels on {nt} threads, wall clock"},
            "host": ci}


def cpu_baseline_rast(gpu_frame, budget_s=10.0):
    import oracle
    oracle.build()
    p = oracle.rast_params(RAST_W, RAST_H, RAST_F)
    n, t0 = 0, time.perf_counter()
    while True:
        ref = oracle.rast_draw(p)[0]
        n += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": f"{n} full {RAST_W}x{RAST_H} f{int(RAST_F)} frames, 1 thread, {dt:.2f} s",
            "frame_matches_gpu": bool(np.array_equal(ref, gpu_frame))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed frames (default: rt/rast/f256 800 = 25 RT calls of 32, c4 64, c5 20, yaw 320)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed frames (default: rt/rast 32, c4/c5 3)")
    ap.add_argument("--workload", choices=["rt", "rast", "c4", "c5", "c5yaw", "yaw", "f256"], default="rt")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-steady", dest="steady", action="store_false",
                    help="rt, N = 1: omit the informational settled-clock figure measured after the timed region")
    ap.add_argument("--no-rast", action="store_true", help="rt: omit the C3 `rast` sub-record")
    ap.add_argument("--camera-path", choices=["fixed", "dolly"], default="fixed",
                    help="fixed: the workload's camera every frame (the metric); dolly: cameraPos.z steps 0.005 "
                         "per frame of a call (no repeated camera)")
    ap.add_argument("--no-draw", dest="draw", action="store_false",
                    help="rt, N = 1: omit the `draw` record (the host-buffer boundary: cg_rt_render / cg_rt_render_frames)")
    ap.add_argument("--no-sub", action="store_true",
                    help="rt: omit the C3/C4/C5 sub-records (only the C2 metric line)")
    ap.add_argument("--sub-frames", default="c4:32:3,c5:20:3",
                    help="rt: the build-defined sub-records as workload:steps:warmup (comma separated); "
                         "'' for none")
    ap.add_argument("--rast-batch", type=int, default=64,
                    help="rast: frames per cg_rast_draw_frames_device call (overlapped on the context's "
                         "internal streams); 1 = cg_rast_draw_device per frame")
    ap.add_argument("--stripe", type=int, default=None, help="stripe rows (default: per workload)")
    ap.add_argument("--batch", "--gather-batch", dest="batch", type=int, default=32,
                    help="RT frames per render call (launches of <= 32 frames, their certificates pipelined) "
                         "and, for N > 1, per transfer to rank 0 (halves the per-frame host cost of the "
                         "exchange vs 16); every frame is rendered and gathered")
    ap.add_argument("--layout", choices=["bands", "stripes"], default=None,
                    help="N > 1 RT sharding: balanced contiguous bands received in place (default with nccl), or "
                         "round-robin stripes + gather + unstripe (default with gloo: the rehearsal of N ranks on "
                         "fewer GPUs, through host memory)")
    ap.add_argument("--chunk", type=int, default=4,
                    help="N > 1 bands: frames per chunk of the library's render/transfer pipeline")
    ap.add_argument("--balance-rounds", type=int, default=3,
                    help="warm-up rounds that re-estimate band boundaries from per-rank timings")
    ap.add_argument("--dist-timeout-ms", type=int, default=int(os.environ.get("CG_DIST_TIMEOUT_MS", "120000")),
                    help="N > 1: deadline of every host wait on the library's RCCL communicator (init included); "
                         "past it the communicator is aborted and the run fails instead of hanging")
    ap.add_argument("--backend", default=os.environ.get("CG_DIST_BACKEND", "nccl"),
                    help="nccl (= RCCL over xGMI); gloo only to rehearse N>1 ranks on one GPU")
    ap.add_argument("--rank-timeout", type=float, default=0.0,
                    help="N > 1 started by bench.py itself: fail the job (exit 124) if a rank runs longer (s; 0 = none)")
    args = ap.parse_args()
    if args.layout is None:
        args.layout = "bands" if args.backend == "nccl" else "stripes"
    if args.steps is None:
        args.steps = {"rt": 800, "rast": 800, "c4": 64, "c5": 20, "c5yaw": 20, "yaw": 320, "f256": 800}[args.workload]
    if args.warmup is None:
        args.warmup = 32 if args.workload in ("rt", "rast", "yaw", "f256") else 3

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.backend != "nccl":
        # gloo rehearsal of N ranks on fewer GPUs: ranks share devices (RCCL
        # refuses that: "Duplicate GPU detected", measured on one MI355X)
        local %= max(1, torch.cuda.device_count())
    # CG_BENCH_FORCE_DIST=1 runs the multi-rank code path even with one rank
    # (a one-rank RCCL gather): a rehearsal of the N > 1 loop on one GPU.
    distributed = world > 1 or os.environ.get("CG_BENCH_FORCE_DIST") == "1"
    if distributed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        # torch's own collectives (barriers, the max-over-ranks reduction) get a deadline too
        pg_timeout = datetime.timedelta(milliseconds=max(args.dist_timeout_ms, 10000))
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=pg_timeout)
        else:
            dist.init_process_group(args.backend, timeout=pg_timeout)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local)
    # A dedicated (non-null) stream: our kernels, the HIP timing events and the
    # RCCL gather are all ordered on it.
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    assert sp, "need a non-null HIP stream handle"
    if args.workload == "rast":
        ctx = cgamd.Context(local)
        rec = measure_rast(args, ctx, dev, stream, sp, world, rank, args.steps, args.warmup,
                           cpu=world == 1 and not args.no_cpu_baseline)
        if rank == 0:
            print(json.dumps(rec), flush=True)
        if world > 1:
            dist.destroy_process_group()
        ctx.close()
        return
    rec = measure_rt(args, local, dev, stream, world, rank, distributed)
    finish_rt(args, local, dev, stream, world, rank, distributed, rec)
    if distributed:
        dist.destroy_process_group()


def camera_path(args, wl, cam, K):
    """The cameras of a call's K frames: the workload's camera for every frame (fixed, the
    metric's), or a dolly -- cameraPos.z = -3 + 0.005 k for frame k of the call (the reference's
    UP key, skeleton.cpp:216-218, at a twentieth of its stride) -- so that no rate can depend on
    a repeated camera."""
    if getattr(args, "camera_path", "fixed") != "dolly":
        return [cam] * K
    return [cgamd.rt_camera(wl["W"], wl["H"], wl["F"], (0.0, 0.0, float(np.float32(-3.0 + 0.005 * k)), 1.0),
                            R=cgamd.yaw_matrix(wl["yaw"]) if wl.get("yaw") else None) for k in range(K)]


def measure_draw(ctx, cam, lights, n_single=40, n_pipe=64, chunk=8):
    """The drop-in boundary itself (SURVEY 7 hard part 6): C2 frames delivered into HOST memory, as
    the reference's Draw(screen*) leaves them in screen->buffer (raytracer/Source/skeleton.cpp:91-94,
    104-169; SDLauxiliary.h:149-161).  single: one cg_rt_render per frame into a pageable buffer
    (render, D2H, synchronise -- the reference's own use, one Draw at a time); pipelined:
    cg_rt_render_frames, the D2H of a chunk overlapped with the render of the next, into pageable
    (numpy) and pinned (page-locked) memory.  Every frame is checked against the golden."""
    import hashlib
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        want = json.load(f)["rt"]["rt_1920x1080_f1080"]["argb_sha256"]
    npx = cam.width * cam.height
    buf = np.zeros(npx, np.uint32)
    lat, ok = [], True
    for i in range(n_single + 5):
        t0 = time.perf_counter()
        rc = ctx.lib.cg_rt_render(ctx.h, lights, len(lights), ctypes.byref(cam), buf.ctypes.data_as(ctypes.c_void_p),
                                  None)
        dt = time.perf_counter() - t0
        if rc:
            raise RuntimeError(f"cg_rt_render: {rc}")
        if i >= 5:
            lat.append(dt)
            ok &= hashlib.sha256(buf.tobytes()).hexdigest() == want
    cams = [cam] * n_pipe
    pageable = np.ones(n_pipe * npx, np.uint32)       # written once: its pages are mapped, as a reused screen buffer's
    pinned = torch.empty(n_pipe * npx, dtype=torch.int32, pin_memory=True)
    rec = {"single_frame_ms": 1e3 * float(np.median(lat)), "fps_single": 1.0 / float(np.mean(lat)),
           "single_note": f"median / mean-derived rate of {n_single} cg_rt_render calls (one Draw: render, D2H into a "
                          "pageable buffer, synchronise), wall clock"}
    for name, out in (("pageable", pageable), ("pinned", pinned)):
        ctx.rt_render_frames(cams[:chunk], out, chunk=chunk)          # warm: slots, copy stream
        t0 = time.perf_counter()
        _, st = ctx.rt_render_frames(cams, out, chunk=chunk)
        dt = time.perf_counter() - t0
        frames = (out if isinstance(out, np.ndarray) else out.numpy().view(np.uint32)).reshape(n_pipe, npx)
        ok &= all(hashlib.sha256(fr.tobytes()).hexdigest() == want for fr in frames)
        rec[f"fps_{name}"] = n_pipe / dt
        rec[f"{name}_render_ms_per_frame"] = st.kernel_ms / n_pipe
        rec[f"{name}_d2h_gbs"] = n_pipe * npx * 4 / dt / 1e9
    rec.update({"frames_pipelined": n_pipe, "chunk": chunk, "all_frames_golden": bool(ok),
                "note": "host-visible Draw rates (PCIe D2H of 8.3 MB per frame included); never the metric, whose "
                        "frames stay resident in HBM"})
    del pinned
    return rec


def measure_rt(args, local, dev, stream, world, rank, distributed):
    """One RT workload (args.workload, args.steps, args.warmup) on a fresh context;
    rank 0's JSON record (None on other ranks)."""
    sp = stream.cuda_stream
    ctx = cgamd.Context(local)
    wl = RT_WORKLOADS[args.workload]
    RT_W, RT_H, RT_F = wl["W"], wl["H"], wl["F"]
    if wl["random"]:
        n, n_sph = wl["random"], 0
        ctx.rt_set_scene(cgamd.random_scene(n, 0x5EED), n, None, 0)
    else:
        tris, n, sph = cgamd.rt_scene()
        n_sph = 1
        ctx.rt_set_scene(tris, n, sph, 1)
    cam = cgamd.rt_camera(RT_W, RT_H, RT_F, R=cgamd.yaw_matrix(wl["yaw"]) if wl.get("yaw") else None)
    lights = cgamd.area_lights(None, *wl["area"]) if wl["area"] else cgamd.default_lights()
    n_lights = len(lights)
    if distributed and args.layout == "bands":
        if args.backend != "nccl":
            raise SystemExit("--layout bands runs the library's RCCL path: use --backend nccl (one GPU per rank)")
        res = rt_bands_loop(args, ctx, dev, stream, world, rank, wl, cam, lights)
        ctx.close()
        return rt_report(args, wl, world, rank, n, n_sph, n_lights, res)
    S = args.stripe or wl["stripe"]
    rows = cgdist.shard_rows(RT_H, world, S)
    shard = cgamd.RtShard(rank, world, S)
    # Frames are rendered K per call (cg_rt_render_frames_device: one prepare +
    # one lattice launch for up to 32 frames, so even a 1/8 shard fills the
    # GPU) and, for N > 1, go to rank 0 K per RCCL gather (the per-collective
    # latency and host overhead would otherwise cap N-GPU throughput).  Two
    # batch buffers: the gather of batch j (on the process group's stream)
    # overlaps the renders of batch j+1 (on `stream`).  Every frame is
    # rendered, gathered and reassembled; only launches and transfers are batched.
    host_gather = distributed and args.backend != "nccl"     # gloo rehearsal: via host memory, per frame
    K = max(1, min(64, args.batch))
    NB = 2 if distributed else 1
    shard_px = rows * RT_W
    bufs = [torch.zeros(K * shard_px, dtype=torch.int32, device=dev) for _ in range(NB)]
    frames = torch.zeros(K * RT_H * RT_W, dtype=torch.int32, device=dev) if (rank == 0 and distributed) else None
    gathered = [torch.empty(world * K * shard_px, dtype=torch.int32, device=dev) for _ in range(NB)] \
        if (rank == 0 and distributed) else None
    if host_gather:
        buf_h = torch.empty(shard_px, dtype=torch.int32)
        gl_h = [torch.empty_like(buf_h) for _ in range(world)] if rank == 0 else None
    n_batches = -(-args.steps // K)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(n_batches)]
    lib, h, sh_p = ctx.lib, ctx.h, ctypes.byref(shard)
    cams = (cgamd.RtCamera * K)(*camera_path(args, wl, cam, K))   # the camera of every frame of a batch
    sp_v = ctypes.c_void_p(sp)
    pending = [None] * NB          # (work, frames in the batch, issue order) per batch buffer
    state = {"batch": 0, "last": None, "seq": 0}   # batches issued; (buffer, frames) of the latest batch

    def render(b, nf, i):
        if i is not None:
            ev[i][0].record(stream)
        rc = lib.cg_rt_render_frames_device(h, lights, n_lights, cams, nf, sh_p, ctypes.c_void_p(bufs[b].data_ptr()),
                                            shard_px, cgamd.PIX_ARGB8888, sp_v)
        if i is not None:
            ev[i][1].record(stream)
        if rc:
            raise RuntimeError(f"cg_rt_render_frames_device: {rc}")

    def issue(b, nf):
        """Gather nf frames' shards of buffer b to rank 0 (async)."""
        src = bufs[b][:nf * shard_px]
        dst = list(gathered[b][:world * nf * shard_px].view(world, nf * shard_px).unbind(0)) if rank == 0 else None
        pending[b] = (dist.gather(src, dst, dst=0, async_op=True), nf, state["seq"])
        state["seq"] += 1

    def finish(b):
        """Make `stream` wait for batch b's gather, then reassemble its frames on rank 0."""
        if pending[b] is None:
            return
        w, nf, _ = pending[b]
        w.wait()
        pending[b] = None
        if rank == 0:
            ctx.rt_unstripe_batch_device(gathered[b].data_ptr(), RT_W, RT_H, world, S, nf, frames.data_ptr(), sp)
            state["last"] = (b, nf)

    def batch(nf, i=None):
        """Render (and for N > 1 gather + reassemble) nf <= K frames."""
        b = state["batch"] % NB
        state["batch"] += 1
        finish(b)                                   # buffer b free again (batch j-2 reassembled)
        render(b, nf, i)
        if not distributed:
            state["last"] = (b, nf)
            return
        if host_gather:
            for k in range(nf):
                buf_h.copy_(bufs[b][k * shard_px:(k + 1) * shard_px])
                dist.gather(buf_h, gl_h, dst=0)
                if rank == 0:
                    gathered[b][:world * shard_px].copy_(torch.cat(gl_h))
                    ctx.rt_unstripe_device(gathered[b].data_ptr(), RT_W, RT_H, world, S,
                                           frames.data_ptr() + 4 * k * RT_H * RT_W, sp)
            state["last"] = (b, nf)
            return
        issue(b, nf)

    def drain():
        for b in sorted(range(NB), key=lambda q: pending[q][2] if pending[q] else -1):   # issue order
            finish(b)

    def run(n_frames, timed):
        for j in range(-(-n_frames // K)):
            batch(min(K, n_frames - j * K), j if timed else None)
        drain()

    run(args.warmup, False)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    # HIP events around the hot kernels, inside the library (CG_BENCH_NO_KTIME=1: off, for A/B
    # runs of the events' own cost; the roofline then has no live kernel time)
    cgamd.kernel_timing(os.environ.get("CG_BENCH_NO_KTIME") != "1")
    t0 = time.perf_counter()
    run(args.steps, True)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0   # before the closing barrier: its own latency is no step's
    if distributed:
        dist.barrier()
    kt = read_kernel_times()
    cgamd.kernel_timing(False)
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # device time of one render call (K frames); full batches only
    full = [a.elapsed_time(b) for j, (a, b) in enumerate(ev) if (j + 1) * K <= args.steps] or \
        [a.elapsed_time(b) for a, b in ev]
    launch_ms = float(np.mean(full))
    kernel_ms = launch_ms / K if (args.steps >= K) else launch_ms / args.steps

    outs = None
    if rank == 0:
        b_last, nf_last = state["last"]
        src = frames if distributed else bufs[b_last]
        step_px = RT_H * RT_W if distributed else shard_px
        outs = [src[k * step_px:k * step_px + RT_H * RT_W].cpu().numpy().view(np.uint32).copy()
                for k in range(nf_last)]
    # informational, after the timed region and its outputs: the same calls back to back once
    # the GPU's clocks have settled (the timed call follows W frames after host-side setup, when
    # the GPU is still at post-idle clocks); never the metric
    steady = None
    if not distributed and args.workload == "rt" and args.steady:
        run(4 * K, False)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        run(4 * K, False)
        torch.cuda.synchronize(dev)
        steady = 4 * K / (time.perf_counter() - t0)
    my_rows = cgdist.shard_row_map(RT_H, 0, world, S)
    scratch = ctx.rt_scratch_info() if n > 64 else None
    if scratch is not None:
        scratch["per_pool"] = ctx.rt_pool_demand()
    draw = measure_draw(ctx, cam, lights) if (not distributed and args.workload == "rt" and args.draw) else None
    res = dict(elapsed=elapsed, launch_ms=launch_ms, kernel_ms=kernel_ms, K=K, outs=outs, scratch=scratch, steady=steady,
               kt=kt, draw=draw,
               my_rows=my_rows[my_rows < RT_H],
               parallelism=(f"stripe{S}x{world}, {K} frames per launch and per gather" if world > 1
                            else f"single, {K} frames per call" +
                            (" (launches of <= 32)" if args.workload in ("rt", "c4", "yaw", "f256") else " (one launch per frame)")))
    ctx.close()
    return rt_report(args, wl, world, rank, n, n_sph, n_lights, res)


def finish_rt(args, local, dev, stream, world, rank, distributed, rec):
    """The default (metric) line also carries the other BASELINE GPU configs as
    sub-records, so one driver run pins every one of them: C3 (the rasteriser at
    1080p, `rast`), C4 (4K, 8x8 area light, `c4`) and C5 (1080p over 1M random
    triangles, `c5`), each with its own fps, roofline, CPU baseline and parity flag.
    Each runs on a fresh context after the C2 loop.  For N > 1 the RT sub-records
    go through the same band path as C2 (BASELINE: C4 and C5 are 8-GPU configs)
    and the rasteriser runs one replica per rank."""
    if args.workload == "rt" and not args.no_sub:
        if not args.no_rast:
            # C3 runs on a fresh context: the rasteriser overlaps frames on two
            # lane streams, and HIP deals a process's streams onto 4 hardware
            # queues, so lanes created beside the RT context's two streams can
            # share a queue and serialise (12.6k instead of 19.8k fps).
            ctx_r = cgamd.Context(dev.index)
            r = measure_rast(args, ctx_r, dev, stream, stream.cuda_stream, world, rank, 800, 64,
                             cpu=world == 1 and not args.no_cpu_baseline, cpu_budget_s=5.0)
            ctx_r.close()
            if rank == 0:
                rec["rast"] = r
        for item in filter(None, args.sub_frames.split(",")):
            name, steps, warm = item.split(":")
            sub = argparse.Namespace(**vars(args))
            sub.workload, sub.steps, sub.warmup, sub.stripe = name, int(steps), int(warm), None
            r = measure_rt(sub, local, dev, stream, world, rank, distributed)
            if rank == 0:
                rec[name] = r
    if rank == 0:
        print(json.dumps(rec), flush=True)


def rt_bands_loop(args, ctx, dev, stream, world, rank, wl, cam, lights):
    """N > 1 RT through the library's own multi-GPU path, cg_rt_render_frames_dist
    (csrc/cg_dist.hip): every rank renders one contiguous band of
    rows; ranks > 0 render theirs in the RGB24 wire format, cropped to the
    columns the camera can see anything in, and send it to rank 0 over the
    library's RCCL communicator (p2p over xGMI); rank 0 renders its band straight
    into the frames and assembles the received bands in place.  Inside a call the
    frames go in chunks (--chunk): the transfer of one chunk overlaps the render
    of the next.  During warm-up the library re-estimates the band boundaries from
    every rank's measured render time (cg_dist_rebalance; rank 0 also pays the
    assembly), so the bands take equal time."""
    W, H = wl["W"], wl["H"]
    K = max(1, min(64, args.batch))
    d = cgdist.join(ctx, chunk=args.chunk, timeout_ms=args.dist_timeout_ms)
    sp = stream.cuda_stream
    cams = (cgamd.RtCamera * K)(*camera_path(args, wl, cam, K))
    frames = torch.zeros(K * H * W, dtype=torch.int32, device=dev) if rank == 0 else None
    st = {"last": 0}

    def run(n_frames):
        for j in range(-(-n_frames // K)):
            nf = min(K, n_frames - j * K)
            d.render_frames(cams[:nf], frames.data_ptr() if rank == 0 else None, stream=sp, lights=lights)
            st["last"] = nf

    # Every host wait on the library's communicator is bounded (d.wait: cg_dist_wait polls the
    # streams and the communicator's async error, aborting it at the deadline), so a missing or
    # failed peer ends the run with an error instead of a hang.
    run(args.warmup)
    for _ in range(max(0, args.balance_rounds)):
        run(max(2 * K, args.warmup))
        d.wait(sp)
        d.rebalance()
    d.wait(sp)
    dist.barrier()
    torch.cuda.synchronize(dev)
    cgamd.kernel_timing(True)
    t0 = time.perf_counter()
    run(args.steps)
    d.wait(sp)
    torch.cuda.synchronize(dev)
    # the clock stops before the closing barrier (an RCCL all-reduce whose own latency is no
    # step's): rank 0's wait covers every band's arrival and assembly, and the max over ranks
    # below is the job's time
    elapsed = time.perf_counter() - t0
    dist.barrier()
    kt = read_kernel_times()
    cgamd.kernel_timing(False)
    rend, asm = d.last_times()
    tt = torch.tensor([elapsed, rend, asm], dtype=torch.float64, device=dev)
    allt = [torch.zeros_like(tt) for _ in range(world)]
    dist.all_gather(allt, tt)
    allt = torch.stack(allt).cpu().numpy()
    elapsed = float(allt[:, 0].max())
    bands = d.bands()
    outs = None
    if rank == 0:
        outs = [frames[k * H * W:(k + 1) * H * W].cpu().numpy().view(np.uint32).copy() for k in range(st["last"])]
    r0, nr = bands[rank]
    d.close()
    return dict(elapsed=elapsed, launch_ms=float(allt[rank, 1]) * min(K, 32), kernel_ms=float(allt[rank, 1]), K=K,
                outs=outs, my_rows=np.arange(r0, r0 + nr), kt=kt,
                parallelism=f"bands{world} via cg_rt_render_frames_dist (balanced, {args.balance_rounds} rounds), "
                            f"rgb24 wire, {K} frames per call in chunks of {args.chunk}",
                bands=[list(b) for b in bands], band_render_ms_per_frame=allt[:, 1].tolist(),
                assemble_ms_per_frame=float(allt[0, 2]))


def rt_report(args, wl, world, rank, n, n_sph, n_lights, res):
    """Rank 0's JSON record of an RT workload (None on other ranks)."""
    if rank != 0:
        return None
    RT_W, RT_H, RT_F = wl["W"], wl["H"], wl["F"]
    elapsed, launch_ms, kernel_ms, K, outs = res["elapsed"], res["launch_ms"], res["kernel_ms"], res["K"], res["outs"]
    out = outs[-1] if args.camera_path == "fixed" else outs[0]      # dolly: frame 0 has the workload's camera
    fps = args.steps / elapsed
    rc = load_row_counters() if args.workload == "rt" else None
    rec = {"metric": "frames/sec + Mray/s, 1080p Cornell-box raytracer" if args.workload == "rt" else
           f"frames/sec + Mray/s, build-defined workload {args.workload.upper()} (SURVEY.md 8d)",
           "value": fps,
           "unit": "frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": 1e3 * elapsed / args.steps, "higher_is_better": True,
           "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
           "config": {"workload": wl["name"], "width": RT_W, "height": RT_H,
                      "focal": RT_F, "camera": [0, 0, -3, 1], "yaw": wl.get("yaw", 0.0), "lights": n_lights,
                      "triangles": n,
                      "spheres": n_sph,
                      "parallelism": res["parallelism"]},
           "mrays_per_s": 9 * RT_W * RT_H * fps / 1e6, "mrays_counted": "primary sub-rays (9 per pixel)"}
    rec["kernel_ms_live"] = {k: {"total_ms": v[0], "busy_ms": v[1], "launches": v[2]}
                             for k, v in (res.get("kt") or {}).items() if v[2]}
    if res.get("draw"):
        rec["draw"] = res["draw"]
    if res.get("steady"):
        rec["steady_fps_info"] = {"value": res["steady"], "frames": 4 * K,
                                  "note": "not the metric: the same calls back to back after the timed region, "
                                          "GPU clocks settled (the timed call runs at post-idle clocks)"}
    if rc is not None:
        total = {k: int(v.sum()) for k, v in rc.items()}
        rec["mrays_per_s"] = total["n_ray"] * fps / 1e6
        rec["mrays_counted"] = "every ClosestIntersection call (primary + shadow, SURVEY.md 8d N_ray)"
        my_rows = res["my_rows"]
        launch = {k: int(v[my_rows].sum()) for k, v in rc.items()}
        # one lattice launch renders fpl <= 32 frames (a call of K frames is K/32
        # launches); the roofline is per launch, as rocprofv3 reports the kernel
        share = len(my_rows) / RT_H
        roof = kernel_roofline("rt_lattice_kernel", "rt", args.steps, share, res.get("kt"), kernel_ms * min(K, 32),
                               min(K, 32))
        fpl = roof["frames_per_launch"]
        launch_ms = roof["kernel_ms"] or kernel_ms * fpl
        ops = rt_ops(launch) * fpl
        achieved = ops / (launch_ms * 1e-3) / 1e12
        bytes_alg = 4.0 * len(my_rows) * RT_W * fpl
        traffic = load_traffic("rt")
        roof.update(frame_valu("rt", args.steps, share, kernel_ms * args.steps))
        roof.update({
            "traffic": (traffic * fpl * share) if traffic else None,
            "traffic_note": "HBM bytes per launch from PMC FETCH_SIZE x2 + WRITE_SIZE (MI355X_MICROARCH.md)",
            "kernel_note": "unrotated camera, one light: each 16x15-pixel tile traces its 33x31 distinct "
                           "sub-rays once (neighbouring pixels' sub-rays coincide bit for bit) and every "
                           "pixel sums its nine contributions in the reference's order",
            "frames_per_call": K, "call_ms_per_frame": kernel_ms,
            "call_ms_note": "HIP events around each call on the stream the kernels run on, per frame",
            "hbm_algorithmic_bytes_per_launch": bytes_alg,
            "hbm_achieved_gbs": bytes_alg / (launch_ms * 1e-3) / 1e9, "hbm_peak_gbs": PEAK_HBM_GBS,
            "hbm_frac": bytes_alg / (launch_ms * 1e-3) / 1e9 / PEAK_HBM_GBS,
            "effective_vs_bruteforce": {
                "algorithmic_ops_per_launch": ops, "tops": achieved,
                "vs_valu_peak": achieved / PEAK_VALU_LANE_TOPS,
                "note": "the reference's own FP32 work (SURVEY 8d op count) / time: not a roofline fraction -- "
                        "the lattice and the exact certificates skip most of that work"}})
        rec["roofline"] = roof
        rec["rays"] = {"reference_equivalent_mrays_per_s": total["n_ray"] * fps / 1e6,
                       "reference_equivalent_note": "ClosestIntersection calls the reference makes per frame "
                                                    "(primary + shadow, SURVEY 8d N_ray = 29,159,999)",
                       "lattice_primary_rays_per_frame": (RT_W // 16) * -(-RT_H // 15) * 33 * 31,
                       "lattice_primary_mrays_per_s": (RT_W // 16) * -(-RT_H // 15) * 33 * 31 * fps / 1e6,
                       "lattice_note": "distinct sub-rays the lattice kernel traces (33 x 31 per 16 x 15 tile, "
                                       "tiles with no candidate triangle exit without tracing)"}
    if args.workload != "rt":
        bytes_alg = 4.0 * RT_W * RT_H   # per frame
        kern = res.get("dominant_kernel", {"c4": "rt_lattice_lights_kernel", "c5": "rt_big_primary_kernel", "c5yaw": "rt_big_primary_kernel",
                                           "yaw": "rt_lattice_kernel", "f256": "rt_lattice_kernel"}[args.workload])
        fpl_call = min(K, 32) if args.workload in ("c4", "yaw", "f256") else 1   # batched lattice launches
        share = len(res["my_rows"]) / RT_H
        roof = kernel_roofline(kern, args.workload, args.steps, share, res.get("kt"), kernel_ms * fpl_call, fpl_call)
        fpl = roof["frames_per_launch"]
        roof.update(frame_valu(args.workload, args.steps, share, kernel_ms * args.steps))
        tpf = load_traffic(args.workload)   # HBM bytes per frame (PMC), dominant kernel(s)
        roof.update({"traffic": None if tpf is None else tpf * fpl,
                     "traffic_note": ("HBM bytes per launch from PMC FETCH_SIZE x2 + WRITE_SIZE (MI355X_MICROARCH.md); "
                                      + ("every rt_* kernel of the frame" if wl["random"] else
                                         "the light-set sweep + its unit-certificate kernel" if n_lights > 1
                                         else "the lattice kernel")),
                     "frames_per_call": K, "call_ms_per_frame": kernel_ms,
                     "call_ms_note": "HIP events around the whole frame (all kernels of the call)",
                     "hbm_algorithmic_bytes_per_frame": bytes_alg,
                     "hbm_achieved_gbs": bytes_alg / (kernel_ms * 1e-3) / 1e9, "hbm_peak_gbs": PEAK_HBM_GBS,
                     "hbm_frac": bytes_alg / (kernel_ms * 1e-3) / 1e9 / PEAK_HBM_GBS,
                     "hbm_note": "the frame's output bytes over the whole frame's time (all kernels)"})

        rec["roofline"] = roof
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline_rt_sampled(wl, out, args.workload)
    else:
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline_rt(out)
        golden = os.path.join(ROOT, "tests", "golden", "golden.json")
        with open(golden) as f:
            want = json.load(f)["rt"]["rt_1920x1080_f1080"]["argb_sha256"]
        import hashlib
        check = outs if args.camera_path == "fixed" else outs[:1]     # dolly: frame 0 has the golden camera
        rec["frame_sha256_matches_golden"] = all(hashlib.sha256(o.tobytes()).hexdigest() == want for o in check)
        rec["frames_checked"] = len(check)
    if args.camera_path == "fixed":
        # every frame of a call has the same camera: the call's frames must be identical
        rec["frames_identical_in_call"] = bool(all(np.array_equal(o, out) for o in outs))
    else:
        rec["config"]["camera_path"] = "dolly: cameraPos.z = -3 + 0.005 k for frame k of each call"
        rec["frames_distinct_in_call"] = bool(all(not np.array_equal(outs[k], outs[k + 1]) for k in range(len(outs) - 1)))
    if res.get("scratch"):
        sc = res["scratch"]
        rec["scratch"] = {"device_bytes": sc["bytes"], "listed_entries": sc["listed"],
                          "pool_capacity_entries": sc["capacity"], "capacity_per_listed": sc["capacity"] / max(1, sc["listed"]),
                          "overflowed_frames": sc["overflows"], "listed_per_pool": sc.get("per_pool"),
                          "note": "large-scene list pools sized from the frames' own demand (cg_rt_scratch_info)"}
    if "bands" in res:
        rec["config"]["bands"] = res["bands"]
        rec["distributed"] = {"band_render_ms_per_frame": res["band_render_ms_per_frame"],
                              "assemble_ms_per_frame": res["assemble_ms_per_frame"]}
    return rec


def measure_rast(args, ctx, dev, stream, sp, world, rank, steps, warmup, cpu, cpu_budget_s=10.0):
    """C3: rasteriser 1920x1080, focal 768 (replicas only across ranks).  A step
    is one frame: the whole Draw on the device -- geometry (shadow volumes +
    clip), span setup, ordered fill, post-pass.  Throughput: frames issued
    --rast-batch per cg_rast_draw_frames_device call, which overlaps them on
    the context's internal streams (each frame complete, into its own buffers).
    Latency: single frames, cg_rast_draw_device one at a time, each timed with
    HIP events on the stream it runs on.  Returns rank 0's record."""
    p = cgamd.rast_params(RAST_W, RAST_H, RAST_F)
    ctx.rast_set_scene()
    npx = RAST_W * RAST_H
    B = max(1, args.rast_batch)
    # outputs: colour (screen->buffer) and the depth buffer; the shadow buffer
    # stays internal, as in the reference (skeleton.cpp:41)
    argb = torch.zeros(B * npx, dtype=torch.int32, device=dev)
    depth = torch.zeros(B * npx, dtype=torch.float32, device=dev)
    _, n, _ = cgamd.rast_prepare(p)
    calls = []                      # frames per call over the timed steps
    left = steps
    while left > 0:
        calls.append(min(B, left))
        left -= calls[-1]
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in calls]

    def step(nf, i=None):
        if i is not None:
            ev[i][0].record(stream)
        if B == 1:
            ctx.rast_draw_device(p, argb.data_ptr(), depth.data_ptr(), None, sp)
        else:
            ctx.rast_draw_frames_device([p] * nf, argb.data_ptr(), depth.data_ptr(), None, npx, sp)
        if i is not None:
            ev[i][1].record(stream)

    for _ in range(max(1, -(-warmup // B))):
        step(B)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i, nf in enumerate(calls):
        step(nf, i)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0   # before the closing barrier: its own latency is no step's
    if world > 1:
        dist.barrier()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kernel_ms = float(sum(a.elapsed_time(b) for a, b in ev) / steps)   # device ms per frame
    # single-frame latency: one Draw at a time (the reference's own use)
    lat = []
    for _ in range(50):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        ctx.rast_draw_device(p, argb.data_ptr(), depth.data_ptr(), None, sp)
        b.record(stream)
        b.synchronize()
        lat.append(a.elapsed_time(b))
    lat_ms = float(np.median(lat[5:]))
    # the fill and post kernels' own times, in a separate loop (the timing events would
    # lengthen the single Draw measured above)
    cgamd.kernel_timing(True)
    for _ in range(20):
        ctx.rast_draw_device(p, argb.data_ptr(), depth.data_ptr(), None, sp)
    torch.cuda.synchronize(dev)
    kt = read_kernel_times()
    cgamd.kernel_timing(False)
    kt_single = {k: live_kernel_ms(kt, k)[0] for k in ("rast_fill_kernel", "rast_post_kernel")}
    if rank != 0:
        return None
    frames = argb.cpu().numpy().view(np.uint32).reshape(B, npx)
    out = frames[0].copy()
    same = bool((frames[:calls[-1]] == out).all())
    fps = world * steps / elapsed
    bytes_alg = 8.0 * npx          # colour + depth out
    traffic = load_traffic("rast")
    rec = {"metric": "frames/sec, 1080p Cornell-box rasteriser", "value": fps, "unit": "frames/s",
           "n_gpus": world, "steps": steps, "warmup": warmup,
           "ms_per_step": 1e3 * elapsed / steps, "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
           "config": {"workload": "rast_cornell_1920x1080_f768", "width": RAST_W, "height": RAST_H,
                      "focal": RAST_F, "triangles_after_clip": n,
                      "parallelism": (f"replicas{world}" if world > 1 else "single") +
                      (f", {B} frames per call overlapped on streams" if B > 1 else "")},
           "single_frame_ms": lat_ms,
           "single_frame_note": "device time of one cg_rast_draw_device (the whole Draw), frames issued one at "
                                "a time; median of 45",
           "single_frame_kernel_ms": kt_single,
           "single_frame_kernel_note": "mean live HIP-event time per launch of the fill and post kernels over 20 "
                                       "single Draws of a separate loop (cg_kernel_timing)",
           "roofline": {"bound": "hbm", "achieved": bytes_alg / (kernel_ms * 1e-3) / 1e9,
                        "peak": PEAK_HBM_GBS, "unit": "GB/s",
                        "frac": bytes_alg / (kernel_ms * 1e-3) / 1e9 / PEAK_HBM_GBS,
                        "traffic": traffic, "traffic_per_algorithmic": (traffic / bytes_alg) if traffic else None,
                        "algorithmic_bytes_per_frame": bytes_alg, "kernel_ms": kernel_ms,
                        "kernel": "rast_* (geometry .. fill/post), one frame",
                        "kernel_note": "device time per frame: each call's HIP-event span / its frames"},
           "frames_identical_in_batch": same}
    if cpu:
        rec["cpu_baseline"] = cpu_baseline_rast(out, cpu_budget_s)
    return rec


if __name__ == "__main__":
    main()
