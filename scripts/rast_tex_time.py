"""Device time per C3 frame (1920x1080, focal 768) per texture setting, on
seeded synthetic maps (cg_rast_draw_device, HIP events, median of 50)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "computer-graphics_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import cgamd  # noqa: E402


def main():
    rng = np.random.default_rng(3)
    maps = {k: rng.integers(0, 256, cgamd.TEXTURE_SHAPES.get(k, (1024, 1024, 3)), dtype=np.uint8)
            for k in cgamd.TEXTURE_MAPS}
    st = torch.cuda.Stream()
    torch.cuda.set_stream(st)
    ctx = cgamd.Context(0)
    ctx.rast_set_textures(maps)
    W, H = 1920, 1080
    p = cgamd.rast_params(W, H, 768.0)
    argb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    depth = torch.zeros(W * H, dtype=torch.float32, device="cuda")
    shadow = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    res = {}
    for s, b in ((0, 0), (2, 0), (3, 0), (1, 0), (2, 3)):
        ctx.rast_set_scene(*cgamd.rast_scene(s, b))
        call = lambda: ctx.rast_draw_device(p, argb.data_ptr(), depth.data_ptr(), shadow.data_ptr(), st.cuda_stream)
        for _ in range(5):
            call()
        ts = []
        for _ in range(50):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            call()
            e1.record(st)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        res[f"setting{s}_boxes{b}_us"] = round(float(np.median(ts)) * 1e3, 1)
    print(json.dumps(res), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
