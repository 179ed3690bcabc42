"""One GPU: cold 20-frame C2 calls (synchronised before each, median of N) of the whole frame,
of the r04 rebalanced N = 8 bands, and of interleaved stripe shards (rank r of 8, stripe height
S) in the RGB24 wire format over the wire's columns -- is a rank's call cheaper when its rows mix
heavy and light tiles?  Usage: python scripts/stripe_probe.py [N]"""
import ctypes
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "computer-graphics_amd"))
import cgamd  # noqa: E402

W, H, F, K = 1920, 1080, 1080.0, 20
N = int(sys.argv[1]) if len(sys.argv) > 1 else 11
WHAT = sys.argv[2].split(",") if len(sys.argv) > 2 else ["whole", "bands", "stripes"]
BANDS = [(0, 194), (194, 181), (375, 157), (532, 137), (669, 89), (758, 89), (847, 102), (949, 131)]
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
stream = torch.cuda.Stream(dev)
res = {}
with cgamd.Context(0) as ctx:
    tris, n, sph = cgamd.rt_scene()
    ctx.rt_set_scene(tris, n, sph, 1)
    cam = cgamd.rt_camera(W, H, F)
    cams = (cgamd.RtCamera * 32)(*([cam] * 32))
    lights = cgamd.default_lights()
    buf = torch.zeros(32 * H * W, dtype=torch.int32, device=dev)
    lib, h = ctx.lib, ctx.h
    sp = ctypes.c_void_p(stream.cuda_stream)
    c0, c1 = cgamd.frame_columns(tris, n, sph, 1, cam)

    def timed(shard, fmt):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        rc = lib.cg_rt_render_frames_device(h, lights, len(lights), cams, K, shard, ctypes.c_void_p(buf.data_ptr()),
                                            H * W, fmt, sp)
        assert rc == 0, rc
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) * 1e6

    def measure(shard, fmt):
        for _ in range(4):
            timed(shard, fmt)
        return sorted(timed(shard, fmt) for _ in range(N))[N // 2]

    res["whole_us"] = measure(None, cgamd.PIX_ARGB8888)
    if "bands" in WHAT:
        res["bands_us"] = [measure(ctypes.byref(cgamd.RtShard(row0=a, rows=b, col0=c0, cols=c1 - c0)), cgamd.PIX_RGB24)
                           for a, b in BANDS]
    for S in ((15, 30, 60) if "stripes" in WHAT else ()):
        res[f"stripes{S}_us"] = [measure(ctypes.byref(cgamd.RtShard(r, 8, S, 0, 0, c0, c1 - c0)), cgamd.PIX_RGB24)
                                 for r in range(8)]
    for k in list(res):
        v = res[k]
        if isinstance(v, list):
            res[k.replace("_us", "_ratio")] = res["whole_us"] / max(v)
print(json.dumps(res, indent=1))
