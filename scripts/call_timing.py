"""Cold 20-frame C2 call, timed the way bench.py's timed region is (synchronise, perf_counter,
call, synchronise), with and without the stripe shard and the HIP events bench.py records
around the call.  Median and spread of N calls per variant.  Usage: python scripts/call_timing.py [N]"""
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
N = int(sys.argv[1]) if len(sys.argv) > 1 else 30
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
    stripe = cgamd.RtShard(0, 1, cgdist.LATTICE_STRIPE)

    def one(shard, events):
        a = b = None
        if events:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        if events:
            a.record(stream)
        rc = lib.cg_rt_render_frames_device(h, lights, len(lights), cams, K, shard, ctypes.c_void_p(buf.data_ptr()),
                                            H * W, cgamd.PIX_ARGB8888, sp)
        if events:
            b.record(stream)
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        assert rc == 0
        return (t1 - t0) * 1e6, (a.elapsed_time(b) * 1e3 if events else None)

    for name, shard, events in (("stripe_events", ctypes.byref(stripe), True), ("none_events", None, True),
                                ("stripe_plain", ctypes.byref(stripe), False), ("none_plain", None, False)):
        for _ in range(5):
            one(shard, events)
        v = [one(shard, events) for _ in range(N)]
        walls = sorted(x[0] for x in v)
        devs = sorted(x[1] for x in v if x[1] is not None)
        res[name] = {"wall_us_median": walls[N // 2], "wall_us_min": walls[0], "wall_us_max": walls[-1],
                     "device_us_median": devs[N // 2] if devs else None,
                     "fps_median": K / (walls[N // 2] * 1e-6)}
    # the bench's shape: the GPU idle for a while, one 5-frame warm-up call, then the timed call
    def warm5():
        lib.cg_rt_render_frames_device(h, lights, len(lights), cams, 5, ctypes.byref(stripe),
                                       ctypes.c_void_p(buf.data_ptr()), H * W, cgamd.PIX_ARGB8888, sp)
    for idle in (0.0, 0.05, 0.5):
        v = []
        for _ in range(8):
            torch.cuda.synchronize(dev)
            time.sleep(idle)
            warm5()
            v.append(one(ctypes.byref(stripe), True))
        walls = sorted(x[0] for x in v)
        res[f"after_idle_{idle}s_warm5"] = {"wall_us_median": walls[len(walls) // 2], "wall_us_min": walls[0],
                                           "device_us_median": sorted(x[1] for x in v)[len(v) // 2]}
print(json.dumps(res, indent=1))
