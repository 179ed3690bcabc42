"""C5 (1920x1080, 1M random triangles) frame time with the large-scene walk in grid order
(CG_WALK_ORDER=0, read by launch_rt_big on every launch) against heavy-first order (default):
rounds alternate the two, each round warm-up frames then 20 timed frames (HIP events on the
render stream); both images must be equal (the order only schedules the walk)."""
import json
import os
import sys

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "computer-graphics_amd"))
import cgamd  # noqa: E402

W, H, F, N = 1920, 1080, 1080.0, 1_000_000
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
stream = torch.cuda.Stream(dev)
res = {}
with cgamd.Context(0) as ctx:
    ctx.rt_set_scene(cgamd.random_scene(N, 0x5EED), N, None, 0)
    cams = [cgamd.rt_camera(W, H, F)]
    ref = None
    for rnd in range(3):
        for mode in ("0", "1"):
            os.environ["CG_WALK_ORDER"] = mode
            buf = torch.zeros(H * W, dtype=torch.int32, device=dev)
            for _ in range(3):
                ctx.rt_render_frames_device(cams, buf.data_ptr(), None, stream.cuda_stream)
            torch.cuda.synchronize(dev)
            if ref is None:
                ref = buf.clone()
            same = bool(torch.equal(buf, ref))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(20):
                ctx.rt_render_frames_device(cams, buf.data_ptr(), None, stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            ms = e0.elapsed_time(e1) / 20
            res.setdefault(mode, []).append({"ms": round(ms, 4), "fps": round(1000 / ms, 2), "same": same})
            print("order" if mode == "1" else "grid ", rnd, f"{ms:.4f} ms {1000 / ms:.2f} fps same={same}", flush=True)
print(json.dumps(res))
