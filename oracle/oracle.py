"""TEST INFRASTRUCTURE ONLY -- ctypes binding of the CPU restatement.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker / CPU baseline.  See
cg_oracle.h for what it restates and how it is pinned.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libcgoracle.so")


class V3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


class V4(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float), ("w", C.c_float)]


class RtTri(C.Structure):
    _fields_ = [("v0", V4), ("v1", V4), ("v2", V4), ("normal", V4), ("color", V3)]


class Sphere(C.Structure):
    _fields_ = [("radius", C.c_float), ("radiusSquared", C.c_float), ("centre", V3), ("color", V3),
                ("normal", V3)]


class Isect(C.Structure):
    _fields_ = [("position", V4), ("distance", C.c_float), ("triangleIndex", C.c_int),
                ("sphereIndex", C.c_int)]


class Light(C.Structure):
    _fields_ = [("position", V4), ("colour", V3)]


class RtParams(C.Structure):
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("focal", C.c_float), ("camera", V4),
                ("R", C.c_float * 16), ("indirect", C.c_float), ("n_lights", C.c_int),
                ("lights", Light * 128)]   # CGO_MAX_LIGHTS


class RtCounters(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("n_ray", "n_t", "n_uv", "n_sph", "n_dl")]


class RastTri(C.Structure):
    _fields_ = [("v0", V4), ("v1", V4), ("v2", V4), ("normal", V4), ("color", V3),
                ("texture", C.c_int), ("index", C.c_int)]


class Pixel(C.Structure):
    _fields_ = [("x", C.c_int), ("y", C.c_int), ("zinv", C.c_float), ("pos3d", V4)]


class RastParams(C.Structure):
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("focal", C.c_float), ("camera", V4),
                ("R", C.c_float * 16), ("light_scene", V4), ("light_power", V3),
                ("indirect_first", C.c_float), ("colour_mode", C.c_int), ("yaw", C.c_float),
                ("rand_offset", C.c_uint64), ("setting", C.c_int), ("setting_boxes", C.c_int)]


TEXTURE_MAPS = ("marble", "woven", "woven_ao", "woven_opacity", "woven_normal",
                "grill", "grill_opacity", "grill_normal")


class RastTextures(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in TEXTURE_MAPS]


class RastCounters(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("n_tris", "n_spans", "n_frags", "n_shaded", "n_shadow")]


_lib = None


def build(quiet=True):
    """Compile the restatement (gcc, -O3, no -march, -ffp-contract=off)."""
    r = subprocess.run(["make", "-C", HERE], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + r.stdout + r.stderr)
    if not quiet:
        print(r.stdout)


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    lib = C.CDLL(LIB_PATH)
    P = C.c_void_p
    sigs = {
        "cgo_rt_load_scene": (C.c_int, [C.POINTER(RtTri), C.c_int, C.POINTER(Sphere)]),
        "cgo_rt_default_params": (None, [C.POINTER(RtParams), C.c_int, C.c_int]),
        "cgo_rt_draw": (None, [C.POINTER(RtParams), C.POINTER(RtTri), C.c_int, C.POINTER(Sphere),
                               C.c_int, P, C.c_int, C.c_int, C.POINTER(RtCounters)]),
        "cgo_rt_draw_mt": (C.c_int, [C.POINTER(RtParams), C.POINTER(RtTri), C.c_int,
                                     C.POINTER(Sphere), C.c_int, P, C.c_int, C.c_int, C.c_int]),
        "cgo_rt_closest": (C.c_int, [V4, V4, C.POINTER(RtTri), C.c_int, C.POINTER(Sphere), C.c_int,
                                     C.POINTER(Isect), C.POINTER(RtCounters)]),
        "cgo_rt_direct_light": (V3, [C.POINTER(Isect), C.POINTER(RtTri), C.c_int, C.POINTER(Sphere),
                                     C.c_int, C.POINTER(Light), C.POINTER(RtCounters)]),
        "cgo_sphere_solve_quadratic": (C.c_int, [C.c_float, C.c_float, C.c_float,
                                                 C.POINTER(C.c_float), C.POINTER(C.c_float)]),
        "cgo_put_pixel": (C.c_uint32, [V3]),
        "cgo_rt_draw_pixels": (None, [C.POINTER(RtParams), C.POINTER(RtTri), C.c_int, C.POINTER(Sphere),
                                      C.c_int, P, C.c_int, P, C.c_int]),
        "cgo_rt_draw_pixels_timed": (None, [C.POINTER(RtParams), C.POINTER(RtTri), C.c_int, C.POINTER(Sphere),
                                            C.c_int, P, C.c_int, P, C.c_int, C.POINTER(C.c_double)]),
        "cgo_rt_area_lights": (C.c_int, [Light, C.c_float, C.c_int, C.POINTER(Light)]),
        "cgo_rt_random_scene": (C.c_int, [C.c_uint64, C.c_int, C.POINTER(RtTri)]),
        "cgo_rast_load_scene": (C.c_int, [C.POINTER(RastTri), C.POINTER(C.c_int),
                                          C.POINTER(RastTri), C.POINTER(C.c_int)]),
        "cgo_rast_default_params": (None, [C.POINTER(RastParams), C.c_int, C.c_int]),
        "cgo_rast_geometry": (C.c_int, [C.POINTER(RastParams), C.POINTER(RastTri), C.c_int,
                                        C.POINTER(V4)]),
        "cgo_rast_polygon_rows": (C.c_int, [C.POINTER(Pixel), C.POINTER(Pixel), C.POINTER(Pixel),
                                            C.c_int]),
        "cgo_rast_interpolate": (None, [Pixel, Pixel, C.POINTER(Pixel), C.c_int]),
        "cgo_rast_draw": (None, [C.POINTER(RastParams), P, P, P, P, P, P,
                                 C.POINTER(RastCounters)]),
        "cgo_glibc_rand": (None, [C.c_uint64, C.c_int, P]),
        "cgo_rast_set_textures": (None, [C.POINTER(RastTextures)]),
        "cgo_rast_opacity_map": (None, [P, C.c_int, P]),
        "cgo_mat4_inverse": (None, [P, P]),
        "cgo_jpeg_info": (C.c_int, [P, C.c_size_t, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                    C.POINTER(C.c_int)]),
        "cgo_jpeg_decode": (C.c_int, [P, C.c_size_t, P, C.c_size_t]),
        "cgo_starfield_init": (None, [P, C.c_int]),
        "cgo_starfield_update": (None, [P, C.c_int, C.c_float]),
        "cgo_starfield_draw": (None, [P, C.c_int, C.c_int, C.c_int, P]),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def rt_scene():
    lib = load()
    tris = (RtTri * 64)()
    sph = Sphere()
    n = lib.cgo_rt_load_scene(tris, 64, C.byref(sph))
    return tris, n, sph


def rt_params(width, height, focal=256.0, cam=(0.0, 0.0, -3.0, 1.0), R=None, indirect=0.5,
              lights=None):
    lib = load()
    p = RtParams()
    lib.cgo_rt_default_params(C.byref(p), width, height)
    p.focal = focal
    p.camera = V4(*cam)
    if R is not None:
        p.R = (C.c_float * 16)(*list(R))
    p.indirect = indirect
    if lights is not None:
        p.n_lights = len(lights)
        for i, (pos, col) in enumerate(lights):
            p.lights[i].position = V4(*pos)
            p.lights[i].colour = V3(*col)
    return p


def rt_draw(p, rows=None, counters=False, threads=1, scene=None):
    """Render rows [r0, r1) of the RT frame (ARGB uint32, W*H, untouched rows 0).
    scene = (tris, n, sphere pointer or None, n_sph); default LoadTestModel."""
    lib = load()
    if scene is None:
        tris, n, sph1 = rt_scene()
        scene = (tris, n, C.pointer(sph1), 1)
    tris, n, sph, n_sph = scene
    out = np.zeros(p.width * p.height, np.uint32)
    r0, r1 = rows if rows is not None else (0, p.height)
    cnt = RtCounters()
    if threads > 1:
        lib.cgo_rt_draw_mt(C.byref(p), tris, n, sph, n_sph, out.ctypes.data_as(C.c_void_p),
                           r0, r1, threads)
    else:
        lib.cgo_rt_draw(C.byref(p), tris, n, sph, n_sph, out.ctypes.data_as(C.c_void_p), r0, r1,
                        C.byref(cnt) if counters else None)
    return (out, cnt) if counters else out


def rt_area_lights(pos, colour, side, n):
    """C4 area light (build-defined, see cg_oracle.h): list of (pos, colour) tuples."""
    lib = load()
    out = (Light * (n * n))()
    k = lib.cgo_rt_area_lights(Light(V4(*pos), V3(*colour)), side, n, out)
    assert k == n * n
    return [((l.position.x, l.position.y, l.position.z, l.position.w),
             (l.colour.x, l.colour.y, l.colour.z)) for l in out]


def rt_random_scene(seed, n):
    """C5 random scene (build-defined, see cg_oracle.h): ctypes RtTri array."""
    lib = load()
    tris = (RtTri * max(n, 1))()
    assert lib.cgo_rt_random_scene(seed, n, tris) == n
    return tris


def rt_draw_pixels(p, xy, scene=None, threads=1, worker_cpu=False):
    """Pixels xy (int array (k, 2) of (u, v)) of the RT frame; scene as in rt_draw.  With
    worker_cpu: (pixels, the workers' summed own CPU seconds -- no other thread counted)."""
    lib = load()
    if scene is None:
        tris1, n1, sph1 = rt_scene()
        scene = (tris1, n1, C.pointer(sph1), 1)
    tris, n_tris, sph, n_sph = scene
    xy = np.ascontiguousarray(np.asarray(xy, np.int32).reshape(-1, 2))
    out = np.zeros(len(xy), np.uint32)
    cpu = C.c_double(0.0)
    lib.cgo_rt_draw_pixels_timed(C.byref(p), tris, n_tris, sph, n_sph, xy.ctypes.data_as(C.c_void_p),
                                 len(xy), out.ctypes.data_as(C.c_void_p), threads, C.byref(cpu))
    return (out, cpu.value) if worker_cpu else out


def glibc_rand(offset, n):
    """n values of libc rand() after `offset` calls from srand(1) (the reference's RNG)."""
    lib = load()
    out = np.zeros(n, np.int32)
    lib.cgo_glibc_rand(offset, n, out.ctypes.data_as(C.c_void_p))
    return out


def starfield_init(n=1000):
    lib = load()
    st = np.zeros((n, 3), np.float32)
    lib.cgo_starfield_init(st.ctypes.data_as(C.c_void_p), n)
    return st


def starfield_update(stars, dt):
    load().cgo_starfield_update(stars.ctypes.data_as(C.c_void_p), len(stars), dt)


def starfield_draw(stars, W=320, H=256):
    out = np.zeros(W * H, np.uint32)
    load().cgo_starfield_draw(stars.ctypes.data_as(C.c_void_p), len(stars), W, H, out.ctypes.data_as(C.c_void_p))
    return out


def rast_params(width, height, focal=512.0, cam=(0.0, 0.0, -3.001, 1.0), R=None,
                light=(0.0, -0.5, 0.0, 1.0), indirect_first=0.2, colour_mode=0, rand_offset=0,
                setting=0, setting_boxes=0, yaw=0.0):
    lib = load()
    p = RastParams()
    lib.cgo_rast_default_params(C.byref(p), width, height)
    p.focal = focal
    p.camera = V4(*cam)
    if R is not None:
        p.R = (C.c_float * 16)(*list(R))
    p.light_scene = V4(*light)
    p.indirect_first = indirect_first
    p.colour_mode = colour_mode
    p.rand_offset = rand_offset
    p.setting = setting
    p.setting_boxes = setting_boxes
    p.yaw = yaw
    return p


_textures_keepalive = None


def rast_set_textures(maps):
    """maps: {name: uint8 array (H, W, 3) BGR} for names in TEXTURE_MAPS (missing = not
    loaded); None clears.  The arrays must stay alive while frames are drawn."""
    global _textures_keepalive
    lib = load()
    if maps is None:
        lib.cgo_rast_set_textures(None)
        _textures_keepalive = None
        return
    arrs = {k: np.ascontiguousarray(v, dtype=np.uint8) for k, v in maps.items()}
    t = RastTextures(**{k: a.ctypes.data for k, a in arrs.items()})
    _textures_keepalive = (arrs, t)
    lib.cgo_rast_set_textures(C.byref(t))


def opacity_map(bgr):
    a = np.ascontiguousarray(bgr, dtype=np.uint8)
    out = np.zeros(a.size // 3, np.uint8)
    load().cgo_rast_opacity_map(a.ctypes.data_as(C.c_void_p), out.size, out.ctypes.data_as(C.c_void_p))
    return out


def mat4_inverse(R):
    m = np.ascontiguousarray(R, dtype=np.float32).reshape(16)
    out = np.zeros(16, np.float32)
    load().cgo_mat4_inverse(m.ctypes.data_as(C.c_void_p), out.ctypes.data_as(C.c_void_p))
    return out


def jpeg_decode(data: bytes) -> np.ndarray:
    """cv::imread(..., CV_LOAD_IMAGE_UNCHANGED) of JPEG bytes as the reference's OpenCV 3.4 +
    libjpeg 9 build returns it: uint8 (H, W, 3) BGR or (H, W) gray."""
    lib = load()
    buf = np.frombuffer(data, np.uint8)
    w, h, nc = C.c_int(), C.c_int(), C.c_int()
    if lib.cgo_jpeg_info(buf.ctypes.data, buf.size, C.byref(w), C.byref(h), C.byref(nc)) != 0:
        raise ValueError("not a JPEG")
    out = np.zeros((h.value, w.value, nc.value), np.uint8)
    r = lib.cgo_jpeg_decode(buf.ctypes.data, buf.size, out.ctypes.data, out.size)
    if r != 0:
        raise ValueError(f"cgo_jpeg_decode failed: {r}")
    return out if nc.value == 3 else out[:, :, 0]


def rast_geometry(p):
    lib = load()
    out = (RastTri * 8192)()
    light = V4()
    n = lib.cgo_rast_geometry(C.byref(p), out, 8192, C.byref(light))
    return out, n, light


def rast_draw(p, counters=False):
    """Full RAST frame: (argb uint32, depth float32, shadow int32) planes of W*H."""
    lib = load()
    npx = p.width * p.height
    argb = np.zeros(npx, np.uint32)
    depth = np.zeros(npx, np.float32)
    shadow = np.zeros(npx, np.int32)
    cnt = RastCounters()
    vp = C.c_void_p
    lib.cgo_rast_draw(C.byref(p), argb.ctypes.data_as(vp), depth.ctypes.data_as(vp),
                      shadow.ctypes.data_as(vp), None, None, None, C.byref(cnt))
    return (argb, depth, shadow, cnt) if counters else (argb, depth, shadow)
