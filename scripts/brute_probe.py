"""Time cg_rt_render_brute_device on C5 (1M triangles, 1920x1080) for a few 8-row bands, to size the
whole-frame defect-detector test (tests/test_rt_brute_gpu.py) before running it."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "computer-graphics_amd")]
import torch  # noqa: E402

import cgamd  # noqa: E402

W, H, n = 1920, 1080, 1_000_000
with cgamd.Context(0) as ctx:
    ctx.rt_set_scene(cgamd.random_scene(n, 0x5EED), n, None, 0)
    cam = cgamd.rt_camera(W, H, 1080.0)
    out = torch.zeros(32 * W, dtype=torch.int32, device="cuda")
    tot = 0.0
    for r0 in (0, 256, 528, 800, 1048):
        t0 = time.perf_counter()
        ctx.rt_render_brute_device(cam, r0, 32, out.data_ptr())
        dt = time.perf_counter() - t0
        tot += dt
        print(f"rows {r0}..{r0 + 31}: {dt:.3f} s", flush=True)
    print(f"estimate for the frame: {tot / 5 * H / 32:.1f} s", flush=True)
