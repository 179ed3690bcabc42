"""One GPU: where a cold C2 call's wall time goes on the host side -- the API call's own time
(t_api: cg_rt_render_frames_device returns), the synchronise after it, and the device span
(HIP events around the call on its stream) -- for the whole frame and a 1/8 band (RGB24,
the wire's columns).  Usage: python scripts/host_overhead.py [N] [spin|ktime]
(ktime: the library's live kernel timing on, as in bench.py's timed region)"""
import ctypes
import json
import os
import statistics
import sys
import time

SPIN = len(sys.argv) > 2 and sys.argv[2] == "spin"
KTIME = len(sys.argv) > 2 and sys.argv[2] == "ktime"
if SPIN:   # hipDeviceScheduleSpin before any HIP context exists
    hip = ctypes.CDLL("libamdhip64.so")
    assert hip.hipSetDeviceFlags(ctypes.c_uint(1)) == 0
import torch  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "computer-graphics_amd"))
import cgamd  # noqa: E402

W, H, F, K = 1920, 1080, 1080.0, 20
N = int(sys.argv[1]) if len(sys.argv) > 1 else 21
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
stream = torch.cuda.Stream(dev)
res = {"spin": SPIN, "ktime": KTIME}
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
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    cgamd.kernel_timing(KTIME)

    def one(shard, fmt):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        e0.record(stream)
        rc = lib.cg_rt_render_frames_device(h, lights, len(lights), cams, K, shard, ctypes.c_void_p(buf.data_ptr()),
                                            H * W, fmt, sp)
        e1.record(stream)
        t1 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        assert rc == 0
        return (t1 - t0) * 1e6, (t2 - t0) * 1e6, e0.elapsed_time(e1) * 1e3

    for name, sh, fmt in (("whole", None, cgamd.PIX_ARGB8888),
                          ("band_floor", ctypes.byref(cgamd.RtShard(row0=758, rows=89, col0=c0, cols=c1 - c0)),
                           cgamd.PIX_RGB24),
                          ("band_top", ctypes.byref(cgamd.RtShard(row0=0, rows=194, col0=c0, cols=c1 - c0)),
                           cgamd.PIX_RGB24)):
        for _ in range(5):
            one(sh, fmt)
        v = [one(sh, fmt) for _ in range(N)]
        res[name] = {k: statistics.median(x[i] for x in v) for i, k in enumerate(("api_us", "wall_us", "device_us"))}
print(json.dumps(res, indent=1))
