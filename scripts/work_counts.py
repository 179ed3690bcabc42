"""The reference's own arithmetic the kernels perform per frame, from the
counting build of the library:

    make -C computer-graphics_amd OUT=_build_wc EXTRA=-DCG_WORK_COUNT _build_wc/libcgamd.so
    python scripts/work_counts.py [--out gpurun_out/work_counts.json]   (then copied to profiles/rNN_work_counts.json)

Every triangle t stage, u/v stage (only when the distance tests pass, as in the reference), sphere
test, ray and DirectLight the kernels execute is counted (cg_rt_dev.h WorkKind; wave-aggregated
atomics), primary and shadow rays apart, for C2 (one 20-frame call, per frame), C4 and C5 (one
frame each).  Weighted with SURVEY.md 8d's op counts (t stage 33, u/v stage 37, sphere 29, ray
setup 11, DirectLight 40) they are the useful work bench.py divides by the dominant kernel's time
for roofline.useful_frac.  Everything else a kernel executes -- FP64 certificates, masks, index
math, packing -- is overhead by this measure.  The counts are deterministic (same frame, same
work)."""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("CGAMD_LIB", os.path.join(ROOT, "computer-graphics_amd", "_build_wc", "libcgamd.so"))
sys.path[:0] = [os.path.join(ROOT, "computer-graphics_amd")]

import torch  # noqa: E402

import cgamd  # noqa: E402

KINDS = ("t_pri", "uv_pri", "sph_pri", "ray_pri", "t_sh", "uv_sh", "sph_sh", "ray_sh", "dl")
WEIGHTS = {"t_pri": 33, "uv_pri": 37, "sph_pri": 29, "ray_pri": 11, "t_sh": 33, "uv_sh": 37, "sph_sh": 29,
           "ray_sh": 11, "dl": 40}
# the counters the dominant kernel of each workload owns (bench.py's roofline kernel): the lattice
# kernels do the whole frame's per-ray work; C5's walk only the primary rays (its shadow rays are
# the hints', the pending search's and the shading kernel's, its DirectLights the shading kernel's)
DOMINANT = {"rt": ("rt_lattice_kernel", KINDS), "c4": ("rt_lattice_lights_kernel", KINDS),
            "c5": ("rt_big_primary_kernel", ("t_pri", "uv_pri", "sph_pri", "ray_pri"))}


def useful_ops(counts, kinds=KINDS):
    return sum(WEIGHTS[k] * counts[k] for k in kinds)


def read(lib, reset=True):
    tot = dict.fromkeys(KINDS, 0)
    for fn in ("cg_diag_work_counts_rt", "cg_diag_work_counts_big"):
        buf = (C.c_ulonglong * len(KINDS))()
        f = getattr(lib, fn)
        f.restype = C.c_int
        f.argtypes = [C.c_void_p, C.c_int]
        if f(buf, 1 if reset else 0) != 0:
            raise RuntimeError(fn)
        for k, v in zip(KINDS, buf):
            tot[k] += int(v)
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "work_counts.json"))
    args = ap.parse_args()
    res = {"note": __doc__.strip().splitlines()[0], "weights": WEIGHTS, "library": os.environ["CGAMD_LIB"],
           "workloads": {}}
    with cgamd.Context(0) as ctx:
        lib = ctx.lib
        dev = torch.device("cuda", 0)
        # C2: one 20-frame call (the driver's), per frame
        tris, n, sph = cgamd.rt_scene()
        ctx.rt_set_scene(tris, n, sph, 1)
        cam = cgamd.rt_camera(1920, 1080, 1080.0)
        out = torch.zeros(20 * 1920 * 1080, dtype=torch.int32, device=dev)
        read(lib)
        ctx.rt_render_frames_device([cam] * 20, out.data_ptr())
        torch.cuda.synchronize()
        c = {k: v / 20 for k, v in read(lib).items()}
        res["workloads"]["rt"] = {"frames": 20, "counts_per_frame": c}
        del out
        # C4: 3840x2160, 8x8 area light, one frame
        cam4 = cgamd.rt_camera(3840, 2160, 2160.0)
        ctx.rt_render(cam4, cgamd.area_lights(None, 0.1, 8))
        res["workloads"]["c4"] = {"frames": 1, "counts_per_frame": read(lib)}
        # C5: 1920x1080 over 1M random triangles, one frame (after a sizing frame)
        nb = 1_000_000
        ctx.rt_set_scene(cgamd.random_scene(nb, 0x5EED), nb, None, 0)
        ctx.rt_render(cam)
        read(lib)
        ctx.rt_render(cam)
        res["workloads"]["c5"] = {"frames": 1, "counts_per_frame": read(lib)}
    for name, w in res["workloads"].items():
        kern, kinds = DOMINANT[name]
        w["dominant_kernel"] = kern
        w["dominant_kinds"] = list(kinds)
        w["useful_ops_per_frame"] = useful_ops(w["counts_per_frame"], kinds)
        w["useful_ops_per_frame_all_kernels"] = useful_ops(w["counts_per_frame"])
        print(name, json.dumps(w), flush=True)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
