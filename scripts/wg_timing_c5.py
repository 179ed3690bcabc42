"""Per-wave timing of C5's walk (rt_big_primary_kernel, kind 3) and shadow hints
(rt_shadow_hints_kernel, kind 4) in the diagnostic build (CGAMD_LIB=
computer-graphics_amd/_build_wgt/libcgamd.so, `make OUT=_build_wgt EXTRA=-DCG_WG_TIMING`): one
frame at a time (CG_BIG_SLOTS=1), warm-up frames, then one recorded frame; the records go to
gpurun_out/wgt_c5/c5.npy (cg_rt.hip's record layout, one per wave) and a summary is printed:
each kernel's span, the waves' durations, peak concurrency, the time after the last wave started,
and list-scheduling makespans (observed start order / longest first) on the peak concurrency."""
import ctypes
import heapq
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "computer-graphics_amd"))
import cgamd  # noqa: E402

W, H, F, N = 1920, 1080, 1080.0, 1_000_000
OUT = os.path.join(ROOT, "gpurun_out", "wgt_c5")
os.makedirs(OUT, exist_ok=True)
CAP = 400_000
US = 0.01


def makespan(d, slots):
    h = [0.0] * slots
    for x in d:
        heapq.heappush(h, heapq.heappop(h) + x)
    return max(h)


def peak(t0, t1):
    ev = sorted([(a, 1) for a in t0] + [(b, -1) for b in t1])
    c = m = 0
    for _, s in ev:
        c += s
        m = max(m, c)
    return m


dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
stream = torch.cuda.Stream(dev)
with cgamd.Context(0) as ctx:
    lib = ctx.lib
    assert hasattr(lib, "cg_diag_wg_timing_big"), "needs the CG_WG_TIMING build (CGAMD_LIB)"
    lib.cg_diag_wg_timing_big.argtypes = [ctypes.c_void_p, ctypes.c_uint]
    ctx.rt_set_scene(cgamd.random_scene(N, 0x5EED), N, None, 0)
    cams = [cgamd.rt_camera(W, H, F)]
    buf = torch.zeros(H * W, dtype=torch.int32, device=dev)
    rec = torch.zeros(CAP * 6, dtype=torch.int64, device=dev)
    for _ in range(4):
        ctx.rt_render_frames_device(cams, buf.data_ptr(), None, stream.cuda_stream)
    torch.cuda.synchronize(dev)
    assert lib.cg_diag_wg_timing_big(ctypes.c_void_p(rec.data_ptr()), CAP) == 0
    ctx.rt_render_frames_device(cams, buf.data_ptr(), None, stream.cuda_stream)
    torch.cuda.synchronize(dev)
    assert lib.cg_diag_wg_timing_big(None, 0) == 0
    r = rec.view(CAP, 6).cpu().numpy().view(np.uint64)
    r = r[r[:, 1] != 0].astype(np.int64)
    np.save(os.path.join(OUT, "c5.npy"), r)
    kind = (r[:, 0] >> 56) & 0xFF
    res = {}
    for k, name in ((3, "walk"), (4, "hints")):
        q = r[kind == k]
        if not len(q):
            continue
        d = (q[:, 2] - q[:, 1]) * US
        order = np.argsort(q[:, 1], kind="stable")
        slots = peak(q[:, 1].tolist(), q[:, 2].tolist())
        res[name] = {"waves": int(len(q)), "span_us": float((q[:, 2].max() - q[:, 1].min()) * US),
                     "wave_us_median": float(np.median(d)), "wave_us_p90": float(np.percentile(d, 90)),
                     "wave_us_max": float(d.max()), "peak_concurrency": int(slots),
                     "packed_us": float(d.sum() / slots),
                     "tail_after_last_start_us": float((q[:, 2].max() - q[:, 1].max()) * US),
                     "sim_observed_order_us": makespan(d[order], slots),
                     "sim_longest_first_us": makespan(np.sort(d)[::-1], slots)}
    print(json.dumps(res, indent=1))
