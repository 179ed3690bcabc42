"""C3 single-Draw latency per kernel: cg_rast_draw_device one frame at a time
(synchronised), for rocprofv3 --kernel-trace --stats.  Usage:
  rocprofv3 --kernel-trace --stats --output-format csv -d OUT -o rast -- python scripts/rast_lat.py [frames]
(CG_RAST_CM=1|2: colour mode)"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "computer-graphics_amd"))
import cgamd  # noqa: E402

W, H, F = 1920, 1080, 768.0
n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
with cgamd.Context(0) as ctx:
    p = cgamd.rast_params(W, H, F, colour_mode=int(os.environ.get("CG_RAST_CM", "0")))
    ctx.rast_set_scene()
    argb = torch.zeros(W * H, dtype=torch.int32, device=dev)
    depth = torch.zeros(W * H, dtype=torch.float32, device=dev)
    st = torch.cuda.current_stream(dev)
    lat = []
    for i in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        ctx.rast_draw_device(p, argb.data_ptr(), depth.data_ptr(), None, st.cuda_stream)
        b.record(st)
        b.synchronize()
        lat.append(a.elapsed_time(b))
    lat.sort()
    print(f"single Draw: median {lat[len(lat) // 2] * 1e3:.1f} us, min {lat[0] * 1e3:.1f} us over {n}")
