"""Render the C2 frame N times on one stream (a profiling target: PC sampling, counters)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "computer-graphics_amd")]
import torch
import cgamd

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
st = torch.cuda.Stream()
torch.cuda.set_stream(st)
ctx = cgamd.Context(0)
t, nt, s = cgamd.rt_scene()
ctx.rt_set_scene(t, nt, s, 1)
cam = cgamd.rt_camera(1920, 1080, 1080.0)
buf = torch.zeros(1920 * 1080, dtype=torch.int32, device="cuda")
for _ in range(n):
    ctx.rt_render_device(cam, buf.data_ptr(), None, st.cuda_stream)
st.synchronize()
print("frames", n)
