"""One GPU: the single host-buffer Draw (cg_rt_render: render, D2H into a pageable buffer,
synchronise), N calls, each followed by either nothing (back to back) or the golden hash of the
frame on the host (bench.py's measure_draw shape: the GPU idles meanwhile).  Prints the median
wall time per call; run under rocprofv3 --kernel-trace --memory-copy-trace to split it.
Usage: python scripts/draw_trace.py [N] [hash|b2b]"""
import ctypes
import hashlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "computer-graphics_amd"))
import cgamd  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 30
MODE = sys.argv[2] if len(sys.argv) > 2 else "hash"
W, H, F = 1920, 1080, 1080.0
with cgamd.Context(0) as ctx:
    tris, n, sph = cgamd.rt_scene()
    ctx.rt_set_scene(tris, n, sph, 1)
    cam = cgamd.rt_camera(W, H, F)
    lights = cgamd.default_lights()
    buf = np.zeros(W * H, np.uint32)
    lat = []
    for i in range(N + 5):
        t0 = time.perf_counter()
        rc = ctx.lib.cg_rt_render(ctx.h, lights, len(lights), ctypes.byref(cam), buf.ctypes.data_as(ctypes.c_void_p),
                                  None)
        dt = time.perf_counter() - t0
        assert rc == 0
        if i >= 5:
            lat.append(dt * 1e6)
        if MODE == "hash":
            hashlib.sha256(buf.tobytes()).hexdigest()
    print(json.dumps({"mode": MODE, "median_us": float(np.median(lat)), "min_us": float(np.min(lat))}))
