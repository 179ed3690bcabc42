"""One process, one rank: a workload's frames through the library's multi-GPU path
(cg_rt_render_frames_dist via cgdist.join) against the single-GPU call, timed per call;
run it under rocprofv3 --kernel-trace to see what the dist path launches.  Each path runs with
a fixed camera and with a moving one (cameraPos.z stepping 0.005 per frame, the reference's UP
key at a twentieth of its stride, skeleton.cpp:216-218): no rate may depend on a repeated camera.
Usage: python scripts/dist_probe.py [c5|rt] [frames]"""
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "computer-graphics_amd"))
import cgamd  # noqa: E402
import cgdist  # noqa: E402

WL = sys.argv[1] if len(sys.argv) > 1 else "c5"
NF = int(sys.argv[2]) if len(sys.argv) > 2 else 10
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29541")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
W, H, F = 1920, 1080, 1080.0
with cgamd.Context(0) as ctx:
    if WL == "c5":
        ctx.rt_set_scene(cgamd.random_scene(1_000_000, 0x5EED), 1_000_000, None, 0)
    else:
        tris, n, sph = cgamd.rt_scene()
        ctx.rt_set_scene(tris, n, sph, 1)
    fixed = [cgamd.rt_camera(W, H, F)] * NF
    moving = [cgamd.rt_camera(W, H, F, (0.0, 0.0, -3.0 + 0.005 * k, 1.0)) for k in range(NF)]
    lights = cgamd.default_lights()
    frames = torch.zeros(NF * H * W, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    for label in ("single", "dist"):
        d = cgdist.join(ctx) if label == "dist" else None
        for path, cl in (("fixed", fixed), ("moving", moving)):
            cams = (cgamd.RtCamera * NF)(*cl)
            times = []
            for it in range(4):
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                if d is None:
                    ctx.rt_render_frames_device(cams, frames.data_ptr(), stream=st, lights=lights)
                else:
                    d.render_frames(cams, frames.data_ptr(), stream=st, lights=lights)
                torch.cuda.synchronize(dev)
                times.append(time.perf_counter() - t0)
            print(label, path, "fps per call:", [round(NF / t, 1) for t in times], flush=True)
        if d is not None:
            print("bands", d.bands(), "last_times", d.last_times(), flush=True)
            d.close()
dist.destroy_process_group()
