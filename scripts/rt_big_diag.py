import sys, os, time
sys.path[:0] = ['computer-graphics_amd', 'tests/golden', 'oracle']
import torch, cgamd
ctx = cgamd.Context(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
ctx.rt_set_scene(cgamd.random_scene(n, 0x5EED), n, None, 0)
cam = cgamd.rt_camera(1920, 1080, 1080.0)
for i in range(2):
    t = time.time(); argb, st = ctx.rt_render(cam); print("frame", time.time() - t, st.kernel_ms, flush=True)
