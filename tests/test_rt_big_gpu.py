"""GPU: the large-scene path (n_tris > 64, cg_rt_big.hip) in every mode it
has, against the live oracle's whole frame, bit-exact (tolerance 0):

* lattice mode, unrotated camera (shared half-pixel columns): one light
  (C5's shape) and 16 lights (one verdict word per lattice point);
* lattice mode, yawed camera (raytracer/Source/skeleton.cpp:233-244; per-pixel
  lattice columns, rows shared): one light and 16 lights;
* per-pixel mode: a pitched camera (R turns y: no lattice) with one light, and
  the many-light path (certified per-bin shadow lists) for 16 lights under the
  pitch and for 81 lights (more than a lattice word holds);
* the camera inside the cloud (triangles behind the eye, one straddling the
  eye plane around the eye, and one with a vertex exactly on it: the culling
  projections' unbounded and singular cases), unrotated, yawed and pitched,
  and over 2 x 2 super-bins;
* each also with the pools pinned far too small (every list overflows: the
  consumers' fallback over all triangles) and with a one-entry pending queue
  (the shading kernel's per-lane lit search)."""
import os

import numpy as np
import pytest

import cgamd
import make_golden as mg
import oracle

pytestmark = pytest.mark.gpu

L0 = [[0.0, -0.5, -0.7, 1.0], [14.0, 14.0, 14.0]]
SCENE = dict(random=500, seed=0x5EED)
YAW = mg.yaw_R(np.float32(0.0) - np.float32(0.174533))


def _pitch(a):
    """Rotation about x (column-major m[4 c + r]), float32 cos/sin."""
    c, sn = float(np.cos(np.float32(a), dtype=np.float32)), float(np.sin(np.float32(a), dtype=np.float32))
    m = [1.0 if k % 5 == 0 else 0.0 for k in range(16)]
    m[1 * 4 + 1], m[1 * 4 + 2], m[2 * 4 + 1], m[2 * 4 + 2] = c, sn, -sn, c
    return m


PITCH = _pitch(0.15)
# random_scene(500, 0x5EED)'s first triangle has z in [0.0299, 0.0467] around
# (x, y) = (-0.2249, 0.1385): an eye at z 0.04 sits inside its span; EYE_V0 puts
# the eye plane exactly through its vertex v0 (z 0.029914677, a float)
EYE_IN = [-0.2249, 0.1385, 0.04, 1.0]
EYE_V0 = [-0.2249, 0.1385, float(np.float32(0.029914677)), 1.0]
CASES = {
    "lat_1": dict(R=None, lights=[L0]),
    "lat_area16": dict(R=None, lights=[L0], area=dict(side=0.1, n=4)),
    "yawlat_1": dict(R=YAW, lights=[L0]),
    "yawlat_area16": dict(R=YAW, lights=[L0], area=dict(side=0.1, n=4)),
    "pix_pitch_1": dict(R=PITCH, lights=[L0]),
    "pix_pitch_area16": dict(R=PITCH, lights=[L0], area=dict(side=0.1, n=4)),
    "pix_area81": dict(R=None, lights=[L0], area=dict(side=0.1, n=9)),
    "inside_lat_1": dict(R=None, lights=[L0], cam=EYE_IN),
    "inside_yawlat_area16": dict(R=YAW, lights=[L0], area=dict(side=0.1, n=4), cam=EYE_IN),
    "inside_pix_pitch_1": dict(R=PITCH, lights=[L0], cam=EYE_IN),
    "vertex_plane_lat_1": dict(R=None, lights=[L0], cam=EYE_V0),
    "vertex_plane_yawlat_1": dict(R=YAW, lights=[L0], cam=EYE_V0),
    # 2 x 2 super-bins (512 x 128 pixels each) around the eye
    "inside_lat_wide": dict(R=None, lights=[L0], cam=EYE_IN, width=640, height=160, focal=160.0),
}


def _cfg(case):
    return dict(dict(width=64, height=48, focal=48.0, cam=[0, 0, -3.0, 1], scene=SCENE), **CASES[case])


_REF = {}


def _oracle(case):
    if case not in _REF:
        cfg = _cfg(case)
        _REF[case] = oracle.rt_draw(mg.rt_params_of(cfg), scene=mg.rt_oracle_scene(cfg),
                                    threads=min(16, os.cpu_count() or 8))
    return _REF[case]


def _render(ctx, cfg):
    import ctypes as C
    lights = (cgamd.Light * 1)()
    lights[0].position = cgamd.Vec4(*cfg["lights"][0][0])
    lights[0].colour = cgamd.Vec3(*cfg["lights"][0][1])
    if "area" in cfg:
        lights = cgamd.area_lights(lights[0], cfg["area"]["side"], cfg["area"]["n"])
    R = (C.c_float * 16)(*cfg["R"]) if cfg["R"] is not None else None
    cam = cgamd.rt_camera(cfg["width"], cfg["height"], cfg["focal"], tuple(cfg["cam"]), R)
    argb, _ = ctx.rt_render(cam, lights)
    return argb


@pytest.fixture(scope="module")
def big(ctx):
    sc = SCENE
    ctx.rt_set_scene(cgamd.random_scene(sc["random"], sc["seed"]), sc["random"], None, 0)
    yield ctx
    tris, n, sph = cgamd.rt_scene()
    ctx.rt_set_scene(tris, n, sph, 1)


@pytest.mark.parametrize("case", list(CASES))
@pytest.mark.parametrize("stress", ["sized", "pools_overflow", "sorted_overflow", "pending_cap1"])
def test_big_scene_modes_match_oracle(big, case, stress):
    cfg = _cfg(case)
    try:
        if stress == "pools_overflow":
            big.rt_set_pool_caps(1, 1, 1, 1)
        elif stress == "sorted_overflow":   # bin lists fit, their bucketed copies do not
            big.rt_set_pool_caps(1 << 20, 1 << 20, 1 << 20, 64)
        elif stress == "pending_cap1":
            big.rt_set_pending_cap(1)
        argb = _render(big, cfg)
        info = big.rt_scratch_info()
    finally:
        big.rt_set_pool_caps(0, 0, 0)
        big.rt_set_pending_cap(0)
    ref = _oracle(case)
    bad = np.flatnonzero(argb != ref)
    assert bad.size == 0, f"{case}/{stress}: {bad.size} pixels differ, first {bad[:6]}"
    assert (ref != 0x80000000).sum() > 100          # the frame does see the cloud
    if stress in ("pools_overflow", "sorted_overflow"):
        assert info["overflows"] >= 1, info
    elif stress == "sized":
        assert info["overflows"] == 0 and info["capacity"] <= 2 * info["listed"] + 5 * 4096, info


@pytest.mark.parametrize("case", ["lat_1", "pix_pitch_1", "inside_lat_wide"])
def test_big_walk_order_does_not_change_pixels(big, case, monkeypatch):
    """The walk's heavy-first workgroup order (rt_walk_order_kernel) only
    schedules it: grid order (CG_WALK_ORDER=0) renders the same frame, and
    both equal the oracle."""
    cfg = _cfg(case)
    ordered = _render(big, cfg)
    monkeypatch.setenv("CG_WALK_ORDER", "0")
    grid = _render(big, cfg)
    assert np.array_equal(ordered, grid)
    assert np.array_equal(ordered, _oracle(case))


def _degenerate_scene(n=500, around_eye=False):
    """random_scene(n) with edge-case triangles written over its first ones:
    a point, two collinear forms, a repeated vertex, a sliver, a 10 x 10
    backdrop behind the cloud (every bin lists it, every pixel can hit it), a
    triangle in the eye's plane z = -3 beside the eye (or around it: every
    camera ray meets it at its origin) and one behind the eye.
    Normals as ComputeNormal makes them (NaN for the zero-area ones, which no
    ray can hit: their determinant is 0)."""
    a = np.frombuffer(bytes(cgamd.random_scene(n, 0x5EED)), np.float32).reshape(n, 19).copy()
    v = lambda k: a[k, 0:12].reshape(3, 4)                               # noqa: E731
    p = v(1)[0].copy()
    v(1)[1], v(1)[2] = p, p                                              # a point
    v(2)[2, :3] = v(2)[0, :3] + np.float32(2) * (v(2)[1, :3] - v(2)[0, :3])   # collinear (float)
    v(3)[2, :3] = v(3)[0, :3] + np.float32(0.5) * (v(3)[1, :3] - v(3)[0, :3])
    v(4)[1] = v(4)[0]                                                    # repeated vertex
    v(5)[2, :3] = v(5)[1, :3] + np.float32(1e-6)                         # sliver
    v(6)[:, :3] = [[-5, -5, 1.5], [5, -5, 1.5], [0, 5, 1.5]]             # backdrop
    v(7)[:, :3] = [[-1, -1, -3], [1, -1, -3], [0, 1, -3]] if around_eye else \
        [[0.5, -1, -3], [2, -1, -3], [1, 1, -3]]                          # in the eye plane
    v(8)[:, :3] = [[-1, -1, -4], [1, -1, -4], [0, 1, -4]]                # behind the eye
    with np.errstate(invalid="ignore", divide="ignore"):
        for k in range(1, 9):
            t = v(k)
            e1, e2 = t[1, :3] - t[0, :3], t[2, :3] - t[0, :3]
            c = np.cross(e2, e1).astype(np.float32)
            a[k, 12:15] = c / np.float32(np.sqrt(np.float32((c * c).sum())))
            a[k, 15] = 1.0
    raw = a.tobytes()
    return (cgamd.Tri * n).from_buffer_copy(raw), (oracle.RtTri * n).from_buffer_copy(raw)


@pytest.mark.parametrize("case,around_eye", [("lat_1", False), ("yawlat_area16", False), ("pix_pitch_1", False),
                                             ("pix_area81", False), ("inside_lat_wide", False), ("lat_1", True),
                                             ("pix_pitch_1", True)])
@pytest.mark.parametrize("n", [40, 500])      # 40: the small-scene kernels (n_tris <= 64)
def test_big_scene_degenerate_triangles(ctx, case, around_eye, n):
    gtris, otris = _degenerate_scene(n, around_eye)
    cfg = _cfg(case)
    try:
        ctx.rt_set_scene(gtris, n, None, 0)
        argb = _render(ctx, cfg)
    finally:
        tris, n1, sph = cgamd.rt_scene()
        ctx.rt_set_scene(tris, n1, sph, 1)
    ref = oracle.rt_draw(mg.rt_params_of(cfg), scene=(otris, n, None, 0), threads=min(16, os.cpu_count() or 8))
    bad = np.flatnonzero(argb != ref)
    assert bad.size == 0, f"{case}: {bad.size} pixels differ, first {bad[:6]}: gpu {argb[bad[:3]]} ref {ref[bad[:3]]}"
    assert (ref != 0x80000000).sum() > ref.size // 2                      # the backdrop fills the frame


@pytest.mark.parametrize("lights_n", [1, 16])
def test_big_frames_two_in_flight_equal_single_frames(ctx, lights_n):
    """cg_rt_render_frames_device over a large scene alternates consecutive frames between
    two slots on two streams (two independent frames in flight): a dolly camera path and a
    second call right after it (slot parity and the slots' buffers reused across calls) give
    exactly the frames cg_rt_render renders one at a time."""
    import torch
    W, H, F = 160, 96, 120.0
    n = 4000
    ctx.rt_set_scene(cgamd.random_scene(n, 0x5EED), n, None, 0)
    try:
        lights = cgamd.default_lights() if lights_n == 1 else cgamd.area_lights(None, 0.1, 4)
        cams = [cgamd.rt_camera(W, H, F, (0.0, 0.0, float(np.float32(-3.0 + 0.05 * k)), 1.0)) for k in range(5)]
        want = [ctx.rt_render(c, lights)[0] for c in cams]
        dev = torch.device("cuda", 0)
        s = torch.cuda.Stream(dev)
        for call in range(2):
            out = torch.zeros(len(cams) * W * H, dtype=torch.int32, device=dev)
            order = cams if call == 0 else cams[::-1]
            ctx.rt_render_frames_device(order, out.data_ptr(), stream=s.cuda_stream, lights=lights)
            s.synchronize()
            got = out.cpu().numpy().view(np.uint32).reshape(len(cams), W * H)
            exp = want if call == 0 else want[::-1]
            for k in range(len(cams)):
                assert np.array_equal(got[k], exp[k]), f"call {call} frame {k}"
        assert len({w.tobytes() for w in want}) == len(want)      # the path's frames differ
    finally:
        tris, nt, sph = cgamd.rt_scene()
        ctx.rt_set_scene(tris, nt, sph, 1)
