"""One GPU, the driver's 20-frame C2 call: the whole frame against each of the 8 bands of the
N = 8 partition that bench.py's rebalance converges to (profiles/r02_shard_balance_rt.json),
each band rendered as cg_rt_render_frames_dist renders a rank's share (RGB24 rows).  Wall time
per cold call, median of N, measured (a) warm: calls back to back after warm-up, synchronised
before each; (b) post-idle: the GPU idle 100 ms, one 5-frame warm-up call, then the timed call
(bench.py's shape).  The N = 8 estimate is the slowest band plus a modelled tail: the last
frame's band (RGB24, the wire's visible columns) over one xGMI link at 50 GB/s, the other frames'
transfers overlapping the render (the signalled pipeline); then the bands the bench's warm-up
rebalance converges to from these times (cgdist.rebalance, twice), measured again.  Both with the metric's fixed camera and with a moving one
(cameraPos.z = -3 + 0.005 k for frame k, the UP key at a twentieth of its stride): no figure
may depend on a repeated camera.  Usage: python scripts/band_balanced.py [N] [fixed|moving]"""
import ctypes
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "computer-graphics_amd"))
import cgamd  # noqa: E402
import cgdist  # noqa: E402

W, H, F, K = 1920, 1080, 1080.0, 20
N = int(sys.argv[1]) if len(sys.argv) > 1 else 15
PATH = sys.argv[2] if len(sys.argv) > 2 else "fixed"
BANDS = [(0, 177), (177, 188), (365, 164), (529, 142), (671, 90), (761, 86), (847, 94), (941, 139)]
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
stream = torch.cuda.Stream(dev)
res = {"K": K, "calls": N, "bands": BANDS, "camera_path": PATH,
       "cert_single_max": os.environ.get("CG_CERT_SINGLE_MAX", "0")}
with cgamd.Context(0) as ctx:
    tris, n, sph = cgamd.rt_scene()
    ctx.rt_set_scene(tris, n, sph, 1)
    cam = cgamd.rt_camera(W, H, F)
    if PATH == "moving":
        cams = (cgamd.RtCamera * 32)(*[cgamd.rt_camera(W, H, F, (0.0, 0.0, -3.0 + 0.005 * k, 1.0)) for k in range(32)])
    else:
        cams = (cgamd.RtCamera * 32)(*([cam] * 32))
    lights = cgamd.default_lights()
    buf = torch.zeros(32 * H * W, dtype=torch.int32, device=dev)
    lib, h = ctx.lib, ctx.h
    sp = ctypes.c_void_p(stream.cuda_stream)

    def call(shard, fmt, nf):
        rc = lib.cg_rt_render_frames_device(h, lights, len(lights), cams, nf, shard, ctypes.c_void_p(buf.data_ptr()),
                                            H * W, fmt, sp)
        assert rc == 0

    def timed(shard, fmt):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        call(shard, fmt, K)
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) * 1e6

    def measure(shard, fmt):
        for _ in range(5):
            timed(shard, fmt)
        warm = sorted(timed(shard, fmt) for _ in range(N))[N // 2]
        idle = []
        for _ in range(max(3, N // 3)):
            torch.cuda.synchronize(dev)
            time.sleep(0.1)
            call(shard, fmt, 5)
            idle.append(timed(shard, fmt))
        return {"warm_us": warm, "post_idle_us": sorted(idle)[len(idle) // 2]}

    # the RGB24 wire carries the columns the scene's box can be seen in (cg_rt_frame_columns)
    c0, c1 = cgamd.frame_columns(tris, n, sph, 1, cam)
    res["wire_columns"] = [c0, c1]

    def bands_run(bands):
        out = []
        for r0, rows in bands:
            sh = cgamd.RtShard(row0=r0, rows=rows)
            m = measure(ctypes.byref(sh), cgamd.PIX_RGB24)
            m["tail_us_model"] = rows * (c1 - c0) * 3 / 50e9 * 1e6
            out.append(m)
        return out

    res["whole"] = measure(None, cgamd.PIX_ARGB8888)
    res["band"] = bands_run(BANDS)
    for cond in ("warm_us", "post_idle_us"):
        worst = max(b[cond] + b["tail_us_model"] for b in res["band"])
        res[f"n8_ratio_{cond[:-3]}"] = res["whole"][cond] / worst
    # the bench's warm-up rebalance (cgdist.rebalance, as cg_dist_rebalance): twice from the
    # measured band times, then the bands it converged to
    bands = BANDS
    for _ in range(2):
        bands = [tuple(int(v) for v in b) for b in cgdist.rebalance(bands, [b["warm_us"] for b in res["band"]],
                                                                  [0.0] * len(bands), H)]
        res["band"] = bands_run(bands)
    res["rebalanced_bands"] = bands
    for cond in ("warm_us", "post_idle_us"):
        worst = max(b[cond] + b["tail_us_model"] for b in res["band"])
        res[f"n8_ratio_{cond[:-3]}_rebalanced"] = res["whole"][cond] / worst
print(json.dumps(res, indent=1))
