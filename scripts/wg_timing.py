"""Per-workgroup timing of the driver's 20-frame C2 call (diagnostic build only:
CGAMD_LIB=computer-graphics_amd/_build_wgt/libcgamd.so, built with
`make OUT=_build_wgt EXTRA=-DCG_WG_TIMING`).  For the whole frame and for the bands of
scripts/band_balanced.py, one cold call (GPU idle 100 ms, a 5-frame warm-up call, then the
recorded call, as bench.py) and one warm call; every workgroup of rt_tile_cert_kernel (kind 1:
entry, super-tile masks, phase 1, end) and rt_lattice_kernel (kind 2: entry, end; per tile when the
launch draws tiles from queues) with its workgroup id is written to
gpurun_out/wgt/<case>.npy, 100 MHz wall-clock stamps.  scripts/wg_analyze.py reads them.
Usage: python scripts/wg_timing.py [band indices, default all]"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "computer-graphics_amd"))
import cgamd  # noqa: E402

W, H, F, K = 1920, 1080, 1080.0, 20
BANDS = [(0, 177), (177, 188), (365, 164), (529, 142), (671, 90), (761, 86), (847, 94), (941, 139)]
PICK = [int(a) for a in sys.argv[1:]] or list(range(len(BANDS)))
OUT = os.path.join(ROOT, "gpurun_out", "wgt")
os.makedirs(OUT, exist_ok=True)
CAP = 800_000
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
stream = torch.cuda.Stream(dev)
with cgamd.Context(0) as ctx:
    lib, h = ctx.lib, ctx.h
    assert hasattr(lib, "cg_diag_wg_timing"), "needs the CG_WG_TIMING build (CGAMD_LIB)"
    lib.cg_diag_wg_timing.argtypes = [ctypes.c_void_p, ctypes.c_uint]
    lib.cg_diag_wg_count.argtypes = [ctypes.POINTER(ctypes.c_uint)]
    tris, n, sph = cgamd.rt_scene()
    ctx.rt_set_scene(tris, n, sph, 1)
    cams = (cgamd.RtCamera * 32)(*([cgamd.rt_camera(W, H, F)] * 32))
    lights = cgamd.default_lights()
    buf = torch.zeros(32 * H * W, dtype=torch.int32, device=dev)
    rec = torch.zeros(CAP * 6, dtype=torch.int64, device=dev)
    sp = ctypes.c_void_p(stream.cuda_stream)

    def call(shard, fmt, nf):
        rc = lib.cg_rt_render_frames_device(h, lights, len(lights), cams, nf, shard, ctypes.c_void_p(buf.data_ptr()),
                                            H * W, fmt, sp)
        assert rc == 0

    def recorded(name, shard, fmt, cold):
        for _ in range(5):
            call(shard, fmt, K)
        torch.cuda.synchronize(dev)
        if cold:
            time.sleep(0.1)
            call(shard, fmt, 5)
            torch.cuda.synchronize(dev)
        rec.zero_()
        torch.cuda.synchronize(dev)
        assert lib.cg_diag_wg_timing(ctypes.c_void_p(rec.data_ptr()), CAP) == 0
        t0 = time.perf_counter()
        call(shard, fmt, K)
        torch.cuda.synchronize(dev)
        wall = (time.perf_counter() - t0) * 1e6
        assert lib.cg_diag_wg_timing(None, 0) == 0
        r = rec.view(CAP, 6).cpu().numpy().view(np.uint64)
        r = r[r[:, 1] != 0]
        m = len(r)
        np.save(os.path.join(OUT, f"{name}.npy"), r)
        print(f"{name}: wall {wall:.1f} us, {m} workgroups", flush=True)

    for cold in (True, False):
        tag = "cold" if cold else "warm"
        recorded(f"whole_{tag}", None, cgamd.PIX_ARGB8888, cold)
        for b in PICK:
            r0, rows = BANDS[b]
            sh = cgamd.RtShard(row0=r0, rows=rows)
            recorded(f"band{b}_{tag}", ctypes.byref(sh), cgamd.PIX_RGB24, cold)
