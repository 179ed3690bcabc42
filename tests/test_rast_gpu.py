"""GPU: the rasteriser fill + post-pass against the oracle.  Colour, depth
(z-buffer) and shadow planes must be bit-exact."""
import ctypes as C

import numpy as np
import pytest

import cgamd
import make_golden as mg
import oracle

pytestmark = pytest.mark.gpu


def _params(cfg):
    R = (C.c_float * 16)(*cfg["R"]) if cfg["R"] else None
    return cgamd.rast_params(cfg["width"], cfg["height"], cfg["focal"], tuple(cfg["cam"]), R,
                             tuple(cfg["light"]), cfg["indirect_first"], cfg.get("colour_mode", 0),
                             cfg.get("rand_offset", 0))


def _render(ctx, cfg):
    p = _params(cfg)
    tris, n, light = cgamd.rast_prepare(p)
    argb, depth, shadow, st = ctx.rast_render(tris, n, p, light)
    return argb, depth, shadow, n


@pytest.mark.parametrize("name", list(mg.rast_configs()))
def test_rast_configs_match_golden(ctx, golden, name):
    cfg = mg.rast_configs()[name]
    argb, depth, shadow, n = _render(ctx, cfg)
    e = golden["rast"][name]
    assert n == e["counters"]["n_tris"]
    assert mg.sha(shadow) == e["shadow_sha256"], "shadow plane"
    assert mg.sha(depth) == e["depth_sha256"], "depth plane"
    assert mg.sha(argb) == e["argb_sha256"], "colour plane"


def test_rast_vs_live_oracle_diff_report(ctx):
    cfg = mg.rast_configs()["rast_900x720"]
    argb, depth, shadow, _ = _render(ctx, cfg)
    ra, rd, rs = oracle.rast_draw(mg.rast_params_of(cfg))
    for nm, a, b in (("shadow", shadow, rs), ("depth", depth.view(np.uint32), rd.view(np.uint32)),
                     ("argb", argb, ra)):
        bad = np.flatnonzero(a != b)
        assert bad.size == 0, f"{nm}: {bad.size} differ, first {bad[:6]} gpu {a[bad[:3]]} ref {b[bad[:3]]}"


def test_rast_empty_list(ctx):
    """No triangles: depth 0, no shadow, interior pixels black with alpha 128."""
    p = cgamd.rast_params(64, 48, 64.0)
    argb, depth, shadow, _ = ctx.rast_render((cgamd.RTri * 1)(), 0, p, cgamd.Vec4(0, 0, 0, 1))
    img = argb.reshape(48, 64)
    assert np.all(img[1:-1, 1:-1] == 0x80000000) and not img[0].any()
    assert not depth.any() and not shadow.any()


@pytest.mark.parametrize("name", list(mg.rast_configs()))
def test_rast_device_geometry_draw_matches_golden(ctx, golden, name):
    """cg_rast_draw: geometry (shadow volumes + clip) on the GPU too."""
    cfg = mg.rast_configs()[name]
    ctx.rast_set_scene()
    argb, depth, shadow, st = ctx.rast_draw(_params(cfg))
    e = golden["rast"][name]
    assert st.n_tris == e["counters"]["n_tris"]
    if cfg.get("colour_mode", 0):   # rand() calls consumed: 3 per shaded fragment
        assert st.n_shaded == e["counters"]["n_shaded"]
    assert mg.sha(shadow) == e["shadow_sha256"], "shadow plane"
    assert mg.sha(depth) == e["depth_sha256"], "depth plane"
    assert mg.sha(argb) == e["argb_sha256"], "colour plane"


def test_rast_draw_frames_device_overlapped(ctx):
    """cg_rast_draw_frames_device: 6 frames with their own camera / light /
    first-frame indirect, overlapped on the context's lanes, each bit-exact
    against the oracle (colour, depth, shadow); colour modes 1-2 refused."""
    import torch
    W, H, F = 320, 240, 180.0
    f32 = lambda x: float(np.float32(x))
    ctx.rast_set_scene()
    cfgs = [dict(cam=(0.0, 0.0, -3.001 + 0.05 * k, 1.0), light=(f32(0.1 * (k % 3) - 0.1), -0.5, 0.0, 1.0),
                 indirect_first=f32(0.15) if k == 0 else f32(0.2)) for k in range(6)]
    ps = [cgamd.rast_params(W, H, F, c["cam"], None, c["light"], c["indirect_first"]) for c in cfgs]
    npx, stride = W * H, W * H + 256
    a = torch.zeros(6 * stride, dtype=torch.int32, device="cuda")
    d = torch.zeros(6 * stride, dtype=torch.float32, device="cuda")
    s = torch.zeros(6 * stride, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    ctx.rast_draw_frames_device(ps, a.data_ptr(), d.data_ptr(), s.data_ptr(), stride, st.cuda_stream)
    st.synchronize()
    A = a.cpu().numpy().view(np.uint32)
    D = d.cpu().numpy().view(np.uint32)
    S = s.cpu().numpy()
    for k, c in enumerate(cfgs):
        ra, rd, rs = oracle.rast_draw(oracle.rast_params(W, H, F, c["cam"], light=c["light"],
                                                         indirect_first=c["indirect_first"]))
        o = k * stride
        assert np.array_equal(A[o:o + npx], ra), f"frame {k} colour"
        assert np.array_equal(D[o:o + npx], rd.view(np.uint32)), f"frame {k} depth"
        assert np.array_equal(S[o:o + npx], rs), f"frame {k} shadow"
    with pytest.raises(RuntimeError):
        ctx.rast_draw_frames_device([cgamd.rast_params(W, H, F, colour_mode=1)], a.data_ptr())


_f = lambda x: float(np.float32(x))   # noqa: E731
# Camera and light poses the golden configs do not reach (TestModelH boxes: the
# short one spans x [-0.05, 0.70], y [0.41, 1], z [-0.77, -0.02]; the tall one
# x [-0.70, 0.05], y [-0.19, 1], z [-0.11, 0.64]): the eye inside a box, the
# light inside a box (every shadow volume cast from inside), looking away from
# the room, the eye behind the back wall, the eye and the light on a wall's
# plane, the light outside the room.
POSES = {
    "eye_in_short_box": dict(cam=(_f(0.33), _f(0.7), _f(-0.4), 1.0)),
    "eye_light_in_tall_box": dict(cam=(_f(-0.33), _f(0.4), _f(0.27), 1.0), light=(_f(-0.3), _f(0.2), _f(0.3), 1.0)),
    "light_in_short_box": dict(light=(_f(0.33), _f(0.7), _f(-0.4), 1.0)),
    "looking_back": dict(cam=(0.0, 0.0, _f(-0.5), 1.0), yaw=_f(3.14159)),
    "behind_back_wall": dict(cam=(0.0, 0.0, _f(1.5), 1.0)),
    "eye_on_left_wall": dict(cam=(-1.0, 0.0, _f(-0.5), 1.0)),
    "light_on_right_wall": dict(light=(1.0, 0.0, 0.0, 1.0)),
    "light_outside_front": dict(light=(0.0, _f(-0.5), -2.0, 1.0)),
}


@pytest.mark.parametrize("pose", list(POSES))
def test_rast_edge_poses_vs_live_oracle(ctx, pose):
    """Both Draw entry points (host geometry + device fill, whole Draw on the
    device) against the oracle's Draw for the pose, all three planes bit-exact."""
    c = dict(dict(cam=(0.0, 0.0, _f(-3.001), 1.0), light=(0.0, _f(-0.5), 0.0, 1.0), yaw=0.0), **POSES[pose])
    W, H, F = 160, 120, 90.0
    R = mg.yaw_R(np.float32(0.0) - np.float32(c["yaw"])) if c["yaw"] else None
    ra, rd, rs = oracle.rast_draw(oracle.rast_params(W, H, F, c["cam"], R, light=c["light"], yaw=c["yaw"]))
    p = cgamd.rast_params(W, H, F, c["cam"], (C.c_float * 16)(*R) if R else None, c["light"], yaw=c["yaw"])
    tris, n, light = cgamd.rast_prepare(p)
    ctx.rast_set_scene()
    for how, (a, d, s) in (("render", ctx.rast_render(tris, n, p, light)[:3]), ("draw", ctx.rast_draw(p)[:3])):
        for nm, x, y in (("shadow", s, rs), ("depth", d.view(np.uint32), rd.view(np.uint32)), ("argb", a, ra)):
            bad = np.flatnonzero(x != y)
            assert bad.size == 0, f"{pose}/{how} {nm}: {bad.size} differ, first {bad[:6]} gpu {x[bad[:3]]} ref {y[bad[:3]]}"
