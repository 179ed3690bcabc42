"""Per-call cost of the C2 raytracer on one GPU: a whole-frame call of K frames
against a call of K frames restricted to one band of H/8 rows (the share of
one rank of 8, RGB24 wire format, window-cropped as cg_dist renders it).
Prints host submission time, wall time per call (cold: synchronised after the
previous call, as the driver's 20-frame bench does; and back-to-back) and the
device span.  Usage: python scripts/band_cost.py [K] [calls]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "computer-graphics_amd"))
import cgamd  # noqa: E402

W, H, F = 1920, 1080, 1080.0
K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
N = int(sys.argv[2]) if len(sys.argv) > 2 else 30
ONLY = sys.argv[3] if len(sys.argv) > 3 else None   # "whole" / "band": one configuration (for a trace)
COLD_ONLY = ONLY is not None
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
st = torch.cuda.current_stream(dev)
res = {"K": K, "calls": N}
with cgamd.Context(0) as ctx:
    tris, n, sph = cgamd.rt_scene()
    ctx.rt_set_scene(tris, n, sph, 1)
    cam = cgamd.rt_camera(W, H, F)
    cams = (cgamd.RtCamera * K)(*([cam] * K))
    lights = cgamd.default_lights()
    whole = torch.zeros(K * H * W, dtype=torch.int32, device=dev)
    band = torch.zeros(K * H * W, dtype=torch.int32, device=dev)

    def run(shard, out, fmt, n_calls, cold):
        host, wall, dspan = [], [], []
        for _ in range(n_calls):
            if cold:
                torch.cuda.synchronize(dev)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            a.record(st)
            ctx.rt_render_frames_device(cams, out.data_ptr(), shard=shard, stream=st.cuda_stream, lights=lights,
                                        pix_format=fmt)
            b.record(st)
            t1 = time.perf_counter()
            if cold:
                torch.cuda.synchronize(dev)
                t2 = time.perf_counter()
                wall.append(t2 - t0)
                dspan.append(a.elapsed_time(b) * 1e-3)
            host.append(t1 - t0)
        if not cold:
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(n_calls):
                ctx.rt_render_frames_device(cams, out.data_ptr(), shard=shard, stream=st.cuda_stream, lights=lights,
                                            pix_format=fmt)
            torch.cuda.synchronize(dev)
            wall = [(time.perf_counter() - t0) / n_calls]
        med = lambda v: sorted(v)[len(v) // 2] * 1e6 if v else None   # noqa: E731
        return {"host_us": med(host), "wall_us": med(wall), "device_us": med(dspan)}

    for name, shard, out, fmt in (("whole", None, whole, 0),) if ONLY in (None, "whole") else ():
        run(shard, out, fmt, 5, True)
        res[name] = {"cold": run(shard, out, fmt, N, True)}
        if not COLD_ONLY:
            res[name]["b2b"] = run(shard, out, fmt, N, False)
    rows = H // 8
    for r0 in (0, 3 * rows, 5 * rows) if ONLY is None else ((5 * rows,) if ONLY == "band" else ()):
        shard = cgamd.RtShard(row0=r0, rows=rows)
        name = f"band_{r0}"
        run(shard, band, 1, 5, True)
        res[name] = {"cold": run(shard, band, 1, N, True)}
        if not COLD_ONLY:
            res[name]["b2b"] = run(shard, band, 1, N, False)
print(json.dumps(res, indent=1))
