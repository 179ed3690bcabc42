"""Large-scene RT diagnostics: render the C5 scene (or n random triangles)
twice and print frame times; with CG_RT_BIG_DIAG=1 the library also prints
bin-list and walk statistics to stderr."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "computer-graphics_amd")]
import torch  # noqa: E402,F401  (one HIP runtime in the process)
import cgamd  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
ctx = cgamd.Context(0)
ctx.rt_set_scene(cgamd.random_scene(n, 0x5EED), n, None, 0)
cam = cgamd.rt_camera(1920, 1080, 1080.0)
for i in range(2):
    t = time.time()
    argb, st = ctx.rt_render(cam)
    print("frame", time.time() - t, st.kernel_ms, flush=True)
