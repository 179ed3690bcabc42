import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["CGAMD_LIB"] = os.path.join(ROOT, "computer-graphics_amd/_build_diag/libcgamd.so")
sys.path[:0] = [os.path.join(ROOT, "computer-graphics_amd")]
import torch  # noqa: F401
import numpy as np, cgamd
ctx = cgamd.Context(0); t, n, s = cgamd.rt_scene(); ctx.rt_set_scene(t, n, s, 1)
a, _ = ctx.rt_render(cgamd.rt_camera(1920, 1080, 1080.0))
a = a.reshape(1080, 1920)
pm, sm = (a >> 8) & 0xff, a & 0xff
print("primary survivors per wave: mean %.2f  hist %s" % (pm.mean(), np.bincount(pm.ravel(), minlength=29)[:29].tolist()))
print("shadow survivors per wave:  mean %.2f  hist %s" % (sm.mean(), np.bincount(sm.ravel(), minlength=29)[:29].tolist()))
