"""ctypes binding of the MI355X renderer's C-ABI (include/cg_render.h).

This is harness plumbing for tests/ and bench.py; the product host surface is
the C++ in host/ (the reference's Draw(screen*) shape).  Loading fails loudly
when libcgamd.so is missing: there is no CPU fallback anywhere on the product
path.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CGAMD_LIB") or os.path.join(HERE, "_build", "libcgamd.so")

CG_OK, CG_E_INVALID, CG_E_NODEVICE, CG_E_HIP, CG_E_NOSCENE, CG_E_CAPACITY, CG_E_TIMEOUT = 0, -1, -2, -3, -4, -5, -6


class Vec3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


class Vec4(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float), ("w", C.c_float)]


class Tri(C.Structure):        # raytracer Triangle, 76 B
    _fields_ = [("v0", Vec4), ("v1", Vec4), ("v2", Vec4), ("normal", Vec4), ("color", Vec3)]


class Sphere(C.Structure):     # 44 B
    _fields_ = [("radius", C.c_float), ("radiusSquared", C.c_float), ("centre", Vec3),
                ("color", Vec3), ("normal", Vec3)]


class Light(C.Structure):      # 28 B
    _fields_ = [("position", Vec4), ("colour", Vec3)]


class Isect(C.Structure):      # Intersection, 28 B
    _fields_ = [("position", Vec4), ("distance", C.c_float), ("triangleIndex", C.c_int),
                ("sphereIndex", C.c_int)]


class RtCamera(C.Structure):
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("focal", C.c_float), ("camera", Vec4),
                ("R", C.c_float * 16), ("indirect", C.c_float)]


class RtShard(C.Structure):
    """Stripes (rows == 0): RtShard(rank, nranks, stripe_h).  Band: RtShard(row0=a, rows=n).
    RGB24 window: col0=, cols= (see cg_render.h)."""
    _fields_ = [("rank", C.c_int), ("nranks", C.c_int), ("stripe_h", C.c_int), ("row0", C.c_int),
                ("rows", C.c_int), ("col0", C.c_int), ("cols", C.c_int)]


PIX_ARGB8888, PIX_RGB24 = 0, 1   # cg_render.h CG_PIX_*


class RTri(C.Structure):       # rasteriser Triangle, 84 B
    _fields_ = [("v0", Vec4), ("v1", Vec4), ("v2", Vec4), ("normal", Vec4), ("color", Vec3),
                ("texture", C.c_int), ("index", C.c_int)]


class RastParams(C.Structure):
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("focal", C.c_float), ("camera", Vec4),
                ("R", C.c_float * 16), ("light_scene", Vec4), ("light_power", Vec3),
                ("indirect_first", C.c_float), ("colour_mode", C.c_int), ("yaw", C.c_float),
                ("rand_offset", C.c_uint64)]


class Stats(C.Structure):
    _fields_ = [("kernel_ms", C.c_double), ("total_ms", C.c_double), ("n_tris", C.c_int),
                ("n_spans", C.c_int), ("n_shaded", C.c_longlong)]


assert C.sizeof(Tri) == 76 and C.sizeof(Sphere) == 44 and C.sizeof(Light) == 28
assert C.sizeof(Isect) == 28 and C.sizeof(RTri) == 84

P = C.c_void_p
TEXTURE_MAPS = ("marble", "woven", "woven_ao", "woven_opacity", "woven_normal",
                "grill", "grill_opacity", "grill_normal")
TEXTURE_SHAPES = {"marble": (2000, 2000, 3)}   # the rest 1024 x 1024 x 3 (BGR)


class RastTextures(C.Structure):   # cg_rast_textures
    _fields_ = [(n, C.c_void_p) for n in TEXTURE_MAPS]


_SIGS = {
    "cg_create": (C.c_int, [C.c_int, C.POINTER(P)]),
    "cg_destroy": (None, [P]),
    "cg_last_error": (C.c_char_p, [P]),
    "cg_device_count": (C.c_int, []),
    "cg_rt_load_test_model": (C.c_int, [C.POINTER(Tri), C.c_int, C.POINTER(Sphere)]),
    "cg_glibc_rand": (C.c_int, [C.c_uint64, C.c_int, P]),
    "cg_starfield_init": (C.c_int, [P, C.c_int]),
    "cg_starfield_update": (C.c_int, [P, C.c_int, C.c_float]),
    "cg_starfield_draw": (C.c_int, [P, P, C.c_int, C.c_int, C.c_int, P]),
    "cg_rt_area_lights": (C.c_int, [C.POINTER(Light), C.c_float, C.c_int, C.POINTER(Light), C.c_int]),
    "cg_rt_random_scene": (C.c_int, [C.c_uint64, C.c_int, C.POINTER(Tri)]),
    "cg_rt_set_scene": (C.c_int, [P, C.POINTER(Tri), C.c_int, C.POINTER(Sphere), C.c_int]),
    "cg_rt_set_pending_cap": (C.c_int, [P, C.c_int]),
    "cg_rt_scratch_info": (C.c_int, [P, C.POINTER(C.c_uint64)]),
    "cg_rt_pool_demand": (C.c_int, [P, C.POINTER(C.c_uint64)]),
    "cg_rt_route": (C.c_int, [C.POINTER(RtCamera), C.c_int, C.c_int, C.c_int, C.c_void_p]),
    "cg_rt_set_pool_caps": (C.c_int, [P, C.c_longlong, C.c_longlong, C.c_longlong, C.c_longlong]),
    "cg_rt_render_brute_device": (C.c_int, [P, C.POINTER(Light), C.c_int, C.POINTER(RtCamera), C.c_int, C.c_int, P, P]),
    "cg_rt_render": (C.c_int, [P, C.POINTER(Light), C.c_int, C.POINTER(RtCamera), P, C.POINTER(Stats)]),
    "cg_rt_render_frames": (C.c_int, [P, C.POINTER(Light), C.c_int, C.POINTER(RtCamera), C.c_int, P,
                                      C.c_size_t, C.c_int, C.POINTER(Stats)]),
    "cg_kernel_timing": (C.c_int, [C.c_int]),
    "cg_kernel_time": (C.c_int, [C.c_char_p, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_longlong)]),
    "cg_rt_render_device": (C.c_int, [P, C.POINTER(Light), C.c_int, C.POINTER(RtCamera),
                                      C.POINTER(RtShard), P, P]),
    "cg_rt_render_frames_device": (C.c_int, [P, C.POINTER(Light), C.c_int, C.POINTER(RtCamera), C.c_int,
                                             C.POINTER(RtShard), P, C.c_size_t, C.c_int, P]),
    "cg_rt_assemble_device": (C.c_int, [P, P, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_int, C.c_int,
                                        C.c_int, C.c_int, P, C.c_size_t, C.c_int, C.c_int, P]),
    "cg_rt_frame_columns": (C.c_int, [C.POINTER(Tri), C.c_int, C.POINTER(Sphere), C.c_int, C.POINTER(RtCamera),
                                      C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "cg_rt_shard_rows": (C.c_int, [C.c_int, C.POINTER(RtShard)]),
    "cg_rt_unstripe_device": (C.c_int, [P, P, C.c_int, C.c_int, C.c_int, C.c_int, P, P]),
    "cg_rt_unstripe_batch_device": (C.c_int, [P, P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, P, P]),
    "cg_rt_probe_closest": (C.c_int, [P, C.POINTER(Vec4), C.POINTER(Vec4), C.c_int,
                                      C.POINTER(Isect), C.POINTER(C.c_int)]),
    "cg_rt_probe_direct_light": (C.c_int, [P, C.POINTER(Isect), C.POINTER(Light), C.c_int,
                                           C.POINTER(Vec3)]),
    "cg_rt_probe_div3_device": (C.c_int, [P, P, C.c_int, P, P]),
    "cg_rast_load_test_model": (C.c_int, [C.POINTER(RTri), C.c_int, C.POINTER(C.c_int),
                                          C.POINTER(RTri), C.c_int, C.POINTER(C.c_int)]),
    "cg_rast_prepare": (C.c_int, [C.POINTER(RastParams), C.POINTER(RTri), C.c_int, C.POINTER(RTri),
                                  C.c_int, C.POINTER(RTri), C.c_int, C.POINTER(Vec4)]),
    "cg_rast_render": (C.c_int, [P, C.POINTER(RTri), C.c_int, C.POINTER(RastParams), Vec4, P, P, P,
                                 C.POINTER(Stats)]),
    "cg_rast_render_device": (C.c_int, [P, P, C.c_int, C.POINTER(RastParams), Vec4, P, P, P, P]),
    "cg_rast_set_scene": (C.c_int, [P, C.POINTER(RTri), C.c_int, C.POINTER(RTri), C.c_int]),
    "cg_rast_set_textures": (C.c_int, [P, C.POINTER(RastTextures)]),
    "cg_rast_opacity_map": (C.c_int, [P, C.c_int, P]),
    "cg_rast_draw": (C.c_int, [P, C.POINTER(RastParams), P, P, P, C.POINTER(Stats)]),
    "cg_rast_draw_device": (C.c_int, [P, C.POINTER(RastParams), P, P, P, P]),
    "cg_rast_draw_frames_device": (C.c_int, [P, C.POINTER(RastParams), C.c_int, P, P, P, C.c_size_t, P]),
    "cg_dist_unique_id": (C.c_int, [P]),
    "cg_dist_create": (C.c_int, [P, C.c_int, C.c_int, P, C.POINTER(P)]),
    "cg_dist_create_timed": (C.c_int, [P, C.c_int, C.c_int, P, C.c_int, C.POINTER(P)]),
    "cg_dist_set_timeout": (C.c_int, [P, C.c_int]),
    "cg_dist_wait": (C.c_int, [P, P]),
    "cg_dist_create_local": (C.c_int, [C.POINTER(P), C.c_int, C.POINTER(P)]),
    "cg_dist_destroy": (None, [P]),
    "cg_dist_set_bands": (C.c_int, [P, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "cg_dist_get_bands": (C.c_int, [P, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "cg_dist_set_chunk": (C.c_int, [P, C.c_int]),
    "cg_dist_set_pipeline": (C.c_int, [P, C.c_int]),
    "cg_dist_rebalance": (C.c_int, [P]),
    "cg_dist_last_times": (C.c_int, [P, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "cg_rt_render_frames_dist": (C.c_int, [P, C.POINTER(Light), C.c_int, C.POINTER(RtCamera), C.c_int, P,
                                           C.c_size_t, P]),
    "cg_dist_band_partition": (C.c_int, [P, C.c_int, C.c_int, P, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "cg_image_jpeg_info": (C.c_int, [P, C.c_size_t, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "cg_image_jpeg_check": (C.c_int, [P, C.c_size_t]),
    "cg_image_decode_jpeg": (C.c_int, [P, P, C.c_size_t, P, C.c_size_t]),
    "cg_image_decode_jpeg_device": (C.c_int, [P, P, C.c_size_t, P, C.c_size_t, P]),
}
EXPORTS = tuple(_SIGS)

# skeleton.cpp:135-146: the file each cg_rast_textures map is read from
TEXTURE_FILES = {"marble": "Marble2000x2000.jpg", "woven": "woven1024x1024.jpg",
                 "woven_ao": "Wood_wicker_003_ambientOcclusion.jpg",
                 "woven_opacity": "Wood_wicker_003_opacity.jpg", "woven_normal": "Wood_wicker_003_normal.jpg",
                 "grill": "Metal_Grill_002_basecolor.jpg", "grill_opacity": "Metal_Grill_002_opacity.jpg",
                 "grill_normal": "Metal_Grill_002_normal.jpg"}

_lib = None


def load(path: str = LIB_PATH):
    """Load libcgamd.so (raises if it was not built: no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"libcgamd.so not built at {path}; run __graft_entry__.build()")
    try:   # one HIP runtime per process: torch's (it bundles libamdhip64) must load first
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def identity16():
    return (C.c_float * 16)(*[1.0 if k % 5 == 0 else 0.0 for k in range(16)])


def yaw_matrix(yaw: float):
    """R for a yaw angle exactly as Update() sets it (RT skeleton.cpp:236-238):
    R[0][0]=cos R[0][2]=-sin R[2][0]=sin R[2][2]=cos, float32 cos/sin."""
    y = np.float32(yaw)
    c, s = np.cos(y, dtype=np.float32), np.sin(y, dtype=np.float32)
    m = [1.0 if k % 5 == 0 else 0.0 for k in range(16)]
    m[0 * 4 + 0], m[0 * 4 + 2] = float(c), float(-s)
    m[2 * 4 + 0], m[2 * 4 + 2] = float(s), float(c)
    return (C.c_float * 16)(*m)


ROUTES = ("pixel", "lattice", "lattice_yaw", "lights", "lights_yaw", "big_pixel", "big_lattice", "big_lattice_yaw")


def rt_route(cam, n_tris, n_spheres, n_lights, shard=None):
    """cg_rt_route: the kernels a frame of this shape takes (host-only; no GPU
    needed), as a name from ROUTES."""
    lib = load()
    rc = lib.cg_rt_route(C.byref(cam), n_tris, n_spheres, n_lights, C.cast(C.byref(shard), C.c_void_p) if shard else None)
    if rc < 0:
        raise ValueError(f"cg_rt_route: {rc}")
    return ROUTES[rc]


def rt_camera(width, height, focal=256.0, cam=(0.0, 0.0, -3.0, 1.0), R=None, indirect=0.5):
    c = RtCamera()
    c.width, c.height, c.focal = width, height, focal
    c.camera = Vec4(*cam)
    c.R = R if R is not None else identity16()
    c.indirect = indirect
    return c


def default_lights():
    """skeleton.cpp:86-89: one light at (0,-0.5,-0.7), colour 14*(1,1,1)."""
    arr = (Light * 1)()
    arr[0].position = Vec4(0.0, -0.5, -0.7, 1.0)
    f = float(np.float32(14.0) * np.float32(1.0))
    arr[0].colour = Vec3(f, f, f)
    return arr


def area_lights(centre=None, side=0.1, n=8):
    """C4 soft-shadow light set (cg_rt_area_lights): n*n lights, default around
    the reference light (skeleton.cpp:86-89)."""
    lib = load()
    c = default_lights()[0] if centre is None else centre
    out = (Light * (n * n))()
    k = lib.cg_rt_area_lights(C.byref(c), side, n, out, n * n)
    if k != n * n:
        raise RuntimeError(f"cg_rt_area_lights failed: {k}")
    return out


def glibc_rand(offset, n):
    """cg_glibc_rand: n values of glibc rand() from call `offset` (seed 1)."""
    lib = load()
    out = np.zeros(max(n, 1), np.int32)
    rc = lib.cg_glibc_rand(offset, n, out.ctypes.data_as(C.c_void_p))
    if rc:
        raise RuntimeError(f"cg_glibc_rand failed: {rc}")
    return out[:n]


def starfield_init(n=1000):
    """cg_starfield_init: (n, 3) float32 stars (starfield/Source/skeleton.cpp:41-46)."""
    st = np.zeros((n, 3), np.float32)
    rc = load().cg_starfield_init(st.ctypes.data_as(C.c_void_p), n)
    if rc:
        raise RuntimeError(f"cg_starfield_init failed: {rc}")
    return st


def starfield_update(stars, dt):
    rc = load().cg_starfield_update(stars.ctypes.data_as(C.c_void_p), len(stars), dt)
    if rc:
        raise RuntimeError(f"cg_starfield_update failed: {rc}")


def random_scene(n, seed=0x5EED):
    """C5 random triangles (cg_rt_random_scene): ctypes Tri array of n."""
    lib = load()
    tris = (Tri * max(n, 1))()
    k = lib.cg_rt_random_scene(seed, n, tris)
    if k != n:
        raise RuntimeError(f"cg_rt_random_scene failed: {k}")
    return tris


def rast_params(width, height, focal=512.0, cam=(0.0, 0.0, -3.001, 1.0), R=None,
                light=(0.0, -0.5, 0.0, 1.0), indirect_first=0.2, colour_mode=0, rand_offset=0, yaw=0.0):
    p = RastParams()
    p.width, p.height, p.focal = width, height, focal
    p.camera = Vec4(*cam)
    p.R = (C.c_float * 16)(*R) if R is not None else identity16()
    p.light_scene = Vec4(*light)
    f = float(np.float32(20.0) * np.float32(1.0))
    p.light_power = Vec3(f, f, f)
    p.indirect_first = indirect_first
    p.colour_mode = colour_mode
    p.rand_offset = rand_offset
    p.yaw = yaw
    return p


def opacity_map(bgr):
    """cg_rast_opacity_map (host-only): BGR texels -> 0/255 bytes."""
    a = np.ascontiguousarray(bgr, dtype=np.uint8)
    out = np.zeros(a.size // 3, np.uint8)
    rc = load().cg_rast_opacity_map(a.ctypes.data_as(P), out.size, out.ctypes.data_as(P))
    if rc != CG_OK:
        raise RuntimeError(f"cg_rast_opacity_map failed with {rc}")
    return out


def frame_columns(tris, n, sph, n_sph, cam):
    """cg_rt_frame_columns: the columns [c0, c1) an unrotated camera can see anything in."""
    lib = load()
    c0, c1 = C.c_int(), C.c_int()
    rc = lib.cg_rt_frame_columns(tris, n, sph, n_sph, C.byref(cam), C.byref(c0), C.byref(c1))
    if rc != CG_OK:
        raise RuntimeError(f"cg_rt_frame_columns failed with {rc}")
    return c0.value, c1.value


def probe_div3_device(d_x, d_den, n, d_q, stream=None):
    """cg_rt_probe_div3_device: d_q[3i + k] = d_x[3i + k] / d_den[i] as the light-set sweep divides
    (device pointers; asynchronous on `stream`)."""
    if load().cg_rt_probe_div3_device(P(d_x), P(d_den), n, P(d_q), P(stream) if stream else None) != CG_OK:
        raise RuntimeError("cg_rt_probe_div3_device failed")


def kernel_timing(enable: bool):
    """cg_kernel_timing: start (reset) or stop the live per-kernel HIP-event timing."""
    if load().cg_kernel_timing(1 if enable else 0) != CG_OK:
        raise RuntimeError("cg_kernel_timing failed")


def kernel_time(kernel: str):
    """(total ms, busy ms, launches) of one timed kernel since kernel_timing(True); busy counts
    overlapping launches (two frames in flight) once."""
    ms, busy, n = C.c_double(), C.c_double(), C.c_longlong()
    if load().cg_kernel_time(kernel.encode(), C.byref(ms), C.byref(busy), C.byref(n)) != CG_OK:
        raise ValueError(f"cg_kernel_time: {kernel} is not a timed kernel")
    return ms.value, busy.value, n.value


def rt_scene():
    lib = load()
    tris = (Tri * 64)()
    sph = Sphere()
    n = lib.cg_rt_load_test_model(tris, 64, C.byref(sph))
    if n < 0:
        raise RuntimeError(f"cg_rt_load_test_model failed: {n}")
    return tris, n, sph


def rast_scene(setting=0, setting_boxes=0):
    """LoadTestModel; setting / setting_boxes are the texture selectors of the
    room and the boxes (TestModelH.h:9-10: 0 none, 1 marble, 2 grill, 3 woven)."""
    lib = load()
    room, boxes = (RTri * 16)(), (RTri * 32)()
    nr, nb = C.c_int(), C.c_int()
    rc = lib.cg_rast_load_test_model(room, 16, C.byref(nr), boxes, 32, C.byref(nb))
    if rc < 0:
        raise RuntimeError(f"cg_rast_load_test_model failed: {rc}")
    for i in range(nr.value):
        room[i].texture = setting
    for i in range(nb.value):
        boxes[i].texture = setting_boxes
    return room, nr.value, boxes, nb.value


def rast_prepare(params, room=None, nr=None, boxes=None, nb=None):
    """Host geometry (clip etc.): returns (clipped RTri array, n, light Vec4)."""
    lib = load()
    if room is None:
        room, nr, boxes, nb = rast_scene()
    light = Vec4()
    n = lib.cg_rast_prepare(C.byref(params), room, nr, boxes, nb, None, 0, C.byref(light))
    if n < 0:
        raise RuntimeError(f"cg_rast_prepare failed: {n}")
    out = (RTri * max(n, 1))()
    n = lib.cg_rast_prepare(C.byref(params), room, nr, boxes, nb, out, n, C.byref(light))
    return out, n, light



def jpeg_info(data: bytes):
    """(width, height, channels) of a JPEG file's bytes (host-only, no GPU)."""
    lib = load()
    buf = np.frombuffer(data, np.uint8)
    w, h, ch = C.c_int(), C.c_int(), C.c_int()
    if lib.cg_image_jpeg_info(buf.ctypes.data_as(P), buf.size, C.byref(w), C.byref(h), C.byref(ch)) != 0:
        raise ValueError("not a supported JPEG")
    return w.value, h.value, ch.value

DIST_ID_BYTES = 128   # cg_dist_id (an RCCL unique id)
DIST_SIGNALLED, DIST_CHUNKED = 0, 1   # cg_dist_set_pipeline


def dist_unique_id() -> bytes:
    """cg_dist_unique_id: rank 0 creates the id every rank passes to Dist."""
    buf = (C.c_char * DIST_ID_BYTES)()
    rc = load().cg_dist_unique_id(buf)
    if rc != CG_OK:
        raise RuntimeError(f"cg_dist_unique_id failed with {rc}")
    return bytes(buf.raw)


def band_partition_native(row_cost, nranks, overhead=None):
    """cg_dist_band_partition (host-only): [(row0, rows)] per rank."""
    c = np.ascontiguousarray(row_cost, dtype=np.float64)
    o = None if overhead is None else np.ascontiguousarray(overhead, dtype=np.float64)
    r0, rs = (C.c_int * nranks)(), (C.c_int * nranks)()
    rc = load().cg_dist_band_partition(c.ctypes.data_as(P), len(c), nranks, o.ctypes.data_as(P) if o is not None
                                       else None, r0, rs)
    if rc != CG_OK:
        raise RuntimeError(f"cg_dist_band_partition failed with {rc}")
    return [(r0[r], rs[r]) for r in range(nranks)]


class DistTimeout(RuntimeError):
    """A multi-GPU wait passed its deadline (CG_E_TIMEOUT); the communicator was aborted."""


class Dist:
    """Multi-GPU raytracer frames (cg_dist_*): one rank's handle.  Dist(ctx,
    nranks, rank, id) joins an RCCL communicator; Dist.local(ctxs) builds an
    in-process group (tests) and returns one handle per rank."""

    def __init__(self, ctx, nranks=1, rank=0, uid: bytes = None, _handle=None, timeout_ms=0):
        """timeout_ms: deadline of every host wait on this handle, init included (0: the
        library's default, CG_DIST_TIMEOUT_MS or 60 s); a passed deadline raises
        DistTimeout after the library aborted the communicator."""
        self.ctx, self.lib, self.nranks, self.rank = ctx, ctx.lib, nranks, rank
        if _handle is not None:
            self.h = _handle
            return
        h = P()
        idb = (C.c_char * DIST_ID_BYTES).from_buffer_copy(uid)
        self._check(self.lib.cg_dist_create_timed(ctx.h, nranks, rank, idb, int(timeout_ms), C.byref(h)),
                    "cg_dist_create")
        self.h = h

    def _check(self, rc, what):
        if rc == CG_E_TIMEOUT:
            msg = self.lib.cg_last_error(self.ctx.h)
            raise DistTimeout(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
        self.ctx._check(rc, what)

    def set_timeout(self, ms):
        self._check(self.lib.cg_dist_set_timeout(self.h, int(ms)), "cg_dist_set_timeout")

    def wait(self, stream=None):
        """cg_dist_wait: bounded host wait for this rank's enqueued work (raises on a
        timeout or an RCCL error, after the library aborted the communicator)."""
        self._check(self.lib.cg_dist_wait(self.h, P(stream) if stream else None), "cg_dist_wait")

    @classmethod
    def local(cls, ctxs):
        n = len(ctxs)
        hs, outs = (P * n)(*[c.h for c in ctxs]), (P * n)()
        ctxs[0]._check(ctxs[0].lib.cg_dist_create_local(hs, n, outs), "cg_dist_create_local")
        return [cls(ctxs[r], n, r, _handle=P(outs[r])) for r in range(n)]

    def close(self):
        if getattr(self, "h", None):
            self.lib.cg_dist_destroy(self.h)
            self.h = None

    def set_bands(self, height, bands):
        r0 = (C.c_int * self.nranks)(*[b[0] for b in bands])
        rs = (C.c_int * self.nranks)(*[b[1] for b in bands])
        self.ctx._check(self.lib.cg_dist_set_bands(self.h, height, r0, rs), "cg_dist_set_bands")

    def bands(self):
        r0, rs = (C.c_int * self.nranks)(), (C.c_int * self.nranks)()
        rc = self.lib.cg_dist_get_bands(self.h, r0, rs)
        if rc < 0:
            return None
        return [(r0[r], rs[r]) for r in range(self.nranks)]

    def set_chunk(self, frames):
        self.ctx._check(self.lib.cg_dist_set_chunk(self.h, frames), "cg_dist_set_chunk")

    def set_pipeline(self, mode):
        """DIST_SIGNALLED / DIST_CHUNKED (cg_dist_set_pipeline)."""
        self.ctx._check(self.lib.cg_dist_set_pipeline(self.h, mode), "cg_dist_set_pipeline")

    def rebalance(self):
        self._check(self.lib.cg_dist_rebalance(self.h), "cg_dist_rebalance")

    def last_times(self):
        """(render ms per frame, assembly ms per frame) of this rank's last call."""
        a, b = C.c_double(), C.c_double()
        self._check(self.lib.cg_dist_last_times(self.h, C.byref(a), C.byref(b)), "cg_dist_last_times")
        return a.value, b.value

    def render_frames(self, cams, d_frames, stream=None, lights=None, frame_stride=0):
        """cg_rt_render_frames_dist: len(cams) frames, assembled on rank 0 at d_frames."""
        lights = default_lights() if lights is None else lights
        arr = (RtCamera * len(cams))(*cams)
        self._check(self.lib.cg_rt_render_frames_dist(self.h, lights, len(lights), arr, len(cams),
                                                          P(d_frames) if d_frames else None, frame_stride,
                                                          P(stream) if stream else None),
                        "cg_rt_render_frames_dist")


class Context:
    """One GPU context (cg_create/cg_destroy)."""

    def __init__(self, device: int = 0):
        self.lib = load()
        h = P()
        rc = self.lib.cg_create(device, C.byref(h))
        if rc != CG_OK:
            raise RuntimeError(f"cg_create({device}) failed with {rc} (no usable HIP device?)")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.lib.cg_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != CG_OK:
            msg = self.lib.cg_last_error(self.h)
            raise RuntimeError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")

    # -- RT --
    def rt_set_scene(self, tris, n, sph=None, n_sph=1):
        sp = C.byref(sph) if sph is not None else None
        self._check(self.lib.cg_rt_set_scene(self.h, tris, n, sp, n_sph if sph is not None else 0),
                    "cg_rt_set_scene")

    def rt_set_pending_cap(self, cap):
        """Test hook: capacity of the large-scene pending shadow-ray queue (0 = default)."""
        self._check(self.lib.cg_rt_set_pending_cap(self.h, cap), "cg_rt_set_pending_cap")

    def rt_set_pool_caps(self, sup=0, bin=0, sbin=0, sorted=0):
        """Test hook: pin the large-scene pool capacities (all 0 = automatic)."""
        self._check(self.lib.cg_rt_set_pool_caps(self.h, sup, bin, sbin, sorted), "cg_rt_set_pool_caps")

    def rt_render_brute_device(self, cam, row0, rows, d_out, lights=None, stream=None):
        """Test hook cg_rt_render_brute_device: rows row0 .. row0 + rows - 1 of cam's frame into the
        device buffer d_out by the reference's unaccelerated loop (synchronous)."""
        lights = default_lights() if lights is None else lights
        self._check(self.lib.cg_rt_render_brute_device(self.h, lights, len(lights), C.byref(cam), row0, rows, P(d_out),
                                                       P(stream) if stream else None), "cg_rt_render_brute_device")

    def rt_scratch_info(self):
        """Large-scene scratch after the latest frame: dict(bytes, listed, capacity, overflows)."""
        out = (C.c_uint64 * 4)()
        self._check(self.lib.cg_rt_scratch_info(self.h, out), "cg_rt_scratch_info")
        return dict(bytes=out[0], listed=out[1], capacity=out[2], overflows=out[3])

    def rt_pool_demand(self):
        """Entries the latest large-scene frame listed per pool: dict(sup, bin, sbin, sorted)."""
        out = (C.c_uint64 * 4)()
        self._check(self.lib.cg_rt_pool_demand(self.h, out), "cg_rt_pool_demand")
        return dict(sup=out[0], bin=out[1], sbin=out[2], sorted=out[3])

    def rt_render(self, cam, lights=None, n_lights=None):
        lights = default_lights() if lights is None else lights
        n_lights = len(lights) if n_lights is None else n_lights
        out = np.zeros(cam.width * cam.height, np.uint32)
        st = Stats()
        self._check(self.lib.cg_rt_render(self.h, lights, n_lights, C.byref(cam),
                                          out.ctypes.data_as(P), C.byref(st)), "cg_rt_render")
        return out, st

    def rt_render_frames(self, cams, out=None, chunk=0, lights=None, frame_stride=0):
        """cg_rt_render_frames: len(cams) frames into host memory `out` at f * frame_stride pixels
        (uint32; pageable or pinned, allocated pageable when None; frame_stride 0 = W * H),
        downloads overlapped with later renders."""
        lights = default_lights() if lights is None else lights
        arr = (RtCamera * len(cams))(*cams)
        npx = cams[0].width * cams[0].height
        stride = frame_stride or npx
        if stride < npx:
            raise ValueError(f"frame_stride {stride} < W*H = {npx}")
        if out is None:
            out = np.zeros(len(cams) * stride, np.uint32)
        # the C entry has no capacity argument: the last frame ends at (n - 1) * stride + W * H
        # pixels, and a caller's buffer shorter than that would be written past its end
        need = (len(cams) - 1) * stride + npx
        have = (out.nbytes if isinstance(out, np.ndarray) else out.numel() * out.element_size()) // 4
        if have < need:
            raise ValueError(f"out holds {have} pixels, {len(cams)} frames at stride {stride} need {need}")
        ptr = out.ctypes.data if isinstance(out, np.ndarray) else out.data_ptr()
        st = Stats()
        self._check(self.lib.cg_rt_render_frames(self.h, lights, len(lights), arr, len(cams), P(ptr), stride, chunk,
                                                 C.byref(st)), "cg_rt_render_frames")
        return out, st

    def rt_render_device(self, cam, d_out, shard=None, stream=None, lights=None):
        lights = default_lights() if lights is None else lights
        sh = C.byref(shard) if shard is not None else None
        self._check(self.lib.cg_rt_render_device(self.h, lights, len(lights), C.byref(cam), sh,
                                                 P(d_out), P(stream) if stream else None),
                    "cg_rt_render_device")

    def rt_render_frames_device(self, cams, d_out, shard=None, stream=None, lights=None, frame_stride=0,
                                pix_format=PIX_ARGB8888):
        """cg_rt_render_frames_device: len(cams) frames into d_out + f * frame_stride pixels."""
        lights = default_lights() if lights is None else lights
        arr = (RtCamera * len(cams))(*cams)
        sh = C.byref(shard) if shard is not None else None
        self._check(self.lib.cg_rt_render_frames_device(self.h, lights, len(lights), arr, len(cams), sh, P(d_out),
                                                        frame_stride, pix_format, P(stream) if stream else None),
                    "cg_rt_render_frames_device")

    def rt_assemble_device(self, d_src, pix_format, row0, rows, width, height, nframes, d_frames, frame_stride=0,
                           stream=None, col0=0, cols=0):
        """cg_rt_assemble_device: row blocks (row0[b], rows[b]) of nframes frames -> frames."""
        n = len(rows)
        r0, rs = (C.c_int * n)(*row0), (C.c_int * n)(*rows)
        self._check(self.lib.cg_rt_assemble_device(self.h, P(d_src), pix_format, r0, rs, n, width, height, nframes,
                                                   P(d_frames), frame_stride, col0, cols,
                                                   P(stream) if stream else None),
                    "cg_rt_assemble_device")

    def rt_unstripe_device(self, d_gathered, width, height, nranks, stripe_h, d_frame, stream=None):
        self._check(self.lib.cg_rt_unstripe_device(self.h, P(d_gathered), width, height, nranks,
                                                   stripe_h, P(d_frame), P(stream) if stream else None),
                    "cg_rt_unstripe_device")

    def rt_unstripe_batch_device(self, d_gathered, width, height, nranks, stripe_h, nframes, d_frames,
                                 stream=None):
        self._check(self.lib.cg_rt_unstripe_batch_device(self.h, P(d_gathered), width, height, nranks, stripe_h,
                                                         nframes, P(d_frames), P(stream) if stream else None),
                    "cg_rt_unstripe_batch_device")

    def rt_probe_closest(self, starts, dirs):
        n = len(starts)
        S, D = (Vec4 * n)(*[Vec4(*s) for s in starts]), (Vec4 * n)(*[Vec4(*d) for d in dirs])
        out, hit = (Isect * n)(), (C.c_int * n)()
        self._check(self.lib.cg_rt_probe_closest(self.h, S, D, n, out, hit), "cg_rt_probe_closest")
        return out, list(hit)

    def rt_probe_direct_light(self, isects, light):
        n = len(isects)
        arr = (Isect * n)(*isects)
        out = (Vec3 * n)()
        self._check(self.lib.cg_rt_probe_direct_light(self.h, arr, C.byref(light), n, out),
                    "cg_rt_probe_direct_light")
        return out

    # -- RAST --
    def starfield_draw(self, stars, width=320, height=256):
        out = np.zeros(width * height, np.uint32)
        self._check(self.lib.cg_starfield_draw(self.h, stars.ctypes.data_as(P), len(stars), width, height,
                                               out.ctypes.data_as(P)), "cg_starfield_draw")
        return out

    def rast_render(self, tris, n, params, light, want_depth=True, want_shadow=True):
        npx = params.width * params.height
        argb = np.zeros(npx, np.uint32)
        depth = np.zeros(npx, np.float32) if want_depth else None
        shadow = np.zeros(npx, np.int32) if want_shadow else None
        st = Stats()
        self._check(self.lib.cg_rast_render(
            self.h, tris, n, C.byref(params), light, argb.ctypes.data_as(P),
            depth.ctypes.data_as(P) if depth is not None else None,
            shadow.ctypes.data_as(P) if shadow is not None else None, C.byref(st)), "cg_rast_render")
        return argb, depth, shadow, st

    def rast_set_scene(self, room=None, nr=None, boxes=None, nb=None):
        if room is None:
            room, nr, boxes, nb = rast_scene()
        self._check(self.lib.cg_rast_set_scene(self.h, room, nr, boxes, nb), "cg_rast_set_scene")

    def rast_set_textures(self, maps):
        """maps: {name: uint8 (H, W, 3) BGR array} over TEXTURE_MAPS (absent = not
        loaded), as cv::imread returns them; None unloads."""
        if maps is None:
            self._check(self.lib.cg_rast_set_textures(self.h, None), "cg_rast_set_textures")
            return
        arrs = {}
        for k, v in maps.items():
            a = np.ascontiguousarray(v, dtype=np.uint8)
            if a.shape != TEXTURE_SHAPES.get(k, (1024, 1024, 3)):
                raise ValueError(f"texture {k}: shape {a.shape}")
            arrs[k] = a
        t = RastTextures(**{k: a.ctypes.data for k, a in arrs.items()})
        self._check(self.lib.cg_rast_set_textures(self.h, C.byref(t)), "cg_rast_set_textures")

    def decode_jpeg(self, data: bytes) -> np.ndarray:
        """cv::imread(..., CV_LOAD_IMAGE_UNCHANGED) of JPEG bytes (skeleton.cpp:135-146) on
        this context's GPU: uint8 (H, W, 3) BGR or (H, W) gray."""
        w, h, ch = jpeg_info(data)
        buf = np.frombuffer(data, np.uint8)
        out = np.zeros((h, w, ch), np.uint8)
        self._check(self.lib.cg_image_decode_jpeg(self.h, buf.ctypes.data_as(P), buf.size, out.ctypes.data_as(P),
                                                  out.size), "cg_image_decode_jpeg")
        return out if ch == 3 else out[:, :, 0]

    def load_textures_jpeg(self, directory: str) -> dict:
        """Decode the reference's texture files found in `directory` (names as
        skeleton.cpp:135-146) -> {map name: BGR array}, ready for rast_set_textures."""
        maps = {}
        for name, fn in TEXTURE_FILES.items():
            path = os.path.join(directory, fn)
            if os.path.exists(path):
                with open(path, "rb") as f:
                    maps[name] = self.decode_jpeg(f.read())
        return maps

    def rast_draw(self, params, want_depth=True, want_shadow=True):
        """Whole Draw on the device (geometry + fill + post)."""
        npx = params.width * params.height
        argb = np.zeros(npx, np.uint32)
        depth = np.zeros(npx, np.float32) if want_depth else None
        shadow = np.zeros(npx, np.int32) if want_shadow else None
        st = Stats()
        self._check(self.lib.cg_rast_draw(
            self.h, C.byref(params), argb.ctypes.data_as(P),
            depth.ctypes.data_as(P) if depth is not None else None,
            shadow.ctypes.data_as(P) if shadow is not None else None, C.byref(st)), "cg_rast_draw")
        return argb, depth, shadow, st

    def rast_draw_device(self, params, d_argb, d_depth=None, d_shadow=None, stream=None):
        self._check(self.lib.cg_rast_draw_device(self.h, C.byref(params), P(d_argb), P(d_depth) if d_depth else None,
                                                 P(d_shadow) if d_shadow else None, P(stream) if stream else None),
                    "cg_rast_draw_device")

    def rast_draw_frames_device(self, params_list, d_argb, d_depth=None, d_shadow=None, frame_stride=0,
                                stream=None):
        """len(params_list) colour-mode-0 Draws, frame f at d_argb + f * stride pixels,
        overlapped on the context's internal streams; `stream` waits for them."""
        arr = (RastParams * len(params_list))(*params_list)
        self._check(self.lib.cg_rast_draw_frames_device(
            self.h, arr, len(params_list), P(d_argb), P(d_depth) if d_depth else None,
            P(d_shadow) if d_shadow else None, frame_stride, P(stream) if stream else None),
            "cg_rast_draw_frames_device")

    def rast_render_device(self, d_tris, n, params, light, d_argb, d_depth=None, d_shadow=None,
                           stream=None):
        self._check(self.lib.cg_rast_render_device(
            self.h, P(d_tris), n, C.byref(params), light, P(d_argb),
            P(d_depth) if d_depth else None, P(d_shadow) if d_shadow else None,
            P(stream) if stream else None), "cg_rast_render_device")
