"""GPU: rasteriser texture modes 1-3 (skeleton.cpp:588-645) against the oracle,
bit-exact in colour, depth and shadow.

Two sets of maps: seeded synthetic maps (every mode, including marble, whose
Marble2000x2000.jpg is missing from the reference tree), and the reference's
own grill and woven-wood JPEGs (tests/golden/textures), decoded on the GPU by
cg_image_decode_jpeg -- bit-equal to IJG libjpeg 9, which OpenCV 3.4's imread
uses -- and thresholded as skeleton.cpp:138-155 does.  The grill mode with
the real maps is also pinned to the reference's rasteriser/screenshot.bmp
(tests/test_rast_screenshot.py); woven wood (mode 3, :622-645) has no
reference-rendered frame, so it is pinned through the restatement."""
import ctypes as C

import numpy as np
import pytest

import cgamd
import oracle

pytestmark = pytest.mark.gpu

W, H, F = 320, 240, 256.0


def _maps(seed=7, marble=False):
    rng = np.random.default_rng(seed)
    u = np.arange(1024)
    block = (((u[:, None] // 48) + (u[None, :] // 48)) % 2 == 0)   # big opaque / transparent blocks
    speck = rng.random((1024, 1024)) < 0.1                           # and isolated flipped texels
    op = np.where(block ^ speck, 230, 40).astype(np.uint8)
    op3 = np.repeat(op[:, :, None], 3, axis=2)
    m = {"grill": rng.integers(0, 256, (1024, 1024, 3), dtype=np.uint8),
         "grill_opacity": op3,
         "grill_normal": rng.integers(0, 256, (1024, 1024, 3), dtype=np.uint8),
         "woven": rng.integers(0, 256, (1024, 1024, 3), dtype=np.uint8),
         "woven_ao": rng.integers(0, 256, (1024, 1024, 3), dtype=np.uint8),
         "woven_opacity": op3[::-1].copy(),
         "woven_normal": rng.integers(0, 256, (1024, 1024, 3), dtype=np.uint8)}
    if marble:
        m["marble"] = rng.integers(0, 256, (2000, 2000, 3), dtype=np.uint8)
    return m


@pytest.fixture(scope="module")
def tex_ctx(ctx):
    maps = _maps(marble=True)
    ctx.rast_set_textures(maps)
    oracle.rast_set_textures(maps)
    yield ctx, maps
    ctx.rast_set_textures(None)
    oracle.rast_set_textures(None)
    ctx.rast_set_scene()


def _check(got, ref, what):
    for nm, a, b in zip(("argb", "depth", "shadow"), got, ref):
        a = a.view(np.uint32) if a.dtype == np.float32 else a
        b = b.view(np.uint32) if b.dtype == np.float32 else b
        bad = np.flatnonzero(a != b)
        assert bad.size == 0, f"{what} {nm}: {bad.size} differ, first {bad[:5]} gpu {a[bad[:3]]} ref {b[bad[:3]]}"


CASES = [(2, 0, 0.2, 0.0), (3, 0, 0.2, 0.0), (0, 2, 0.2, 0.0), (0, 3, 0.2, 0.0), (2, 3, 0.2, 0.0),
         (3, 2, 0.15, 0.0), (2, 0, 0.15, 0.0), (1, 0, 0.2, 0.0), (1, 3, 0.15, 0.0), (2, 3, 0.2, 0.35),
         (3, 1, 0.2, -0.35)]


@pytest.mark.parametrize("setting,boxes,ind,yaw", CASES)
def test_textured_draw_matches_oracle(tex_ctx, setting, boxes, ind, yaw):
    ctx, _ = tex_ctx
    R = cgamd.yaw_matrix(yaw) if yaw else None
    p = cgamd.rast_params(W, H, F, R=R, indirect_first=ind, yaw=yaw)
    po = oracle.rast_params(W, H, F, R=list(R) if R is not None else None, indirect_first=ind,
                            setting=setting, setting_boxes=boxes, yaw=yaw)
    ref = oracle.rast_draw(po)
    ctx.rast_set_scene(*cgamd.rast_scene(setting, boxes))
    a, d, s, _ = ctx.rast_draw(p)                       # device geometry
    _check((a, d, s), ref, f"draw {setting}/{boxes}")
    room, nr, bx, nb = cgamd.rast_scene(setting, boxes)
    tris, n, light = cgamd.rast_prepare(p, room, nr, bx, nb)
    a, d, s, _ = ctx.rast_render(tris, n, p, light)     # host geometry, caller's list
    _check((a, d, s), ref, f"render {setting}/{boxes}")


def test_textures_change_the_frame(tex_ctx):
    """The textured path is exercised: frames differ from texture 0, and some
    pixels of a grill room are see-through (depth 0 inside the box)."""
    ctx, _ = tex_ctx
    p = cgamd.rast_params(W, H, F)
    ctx.rast_set_scene(*cgamd.rast_scene(0, 0))
    a0, d0, _, _ = ctx.rast_draw(p)
    ctx.rast_set_scene(*cgamd.rast_scene(2, 0))
    a2, d2, _, _ = ctx.rast_draw(p)
    assert (a0 != a2).mean() > 0.3
    assert (d2 == 0).sum() > (d0 == 0).sum() + 1000


def test_colour_modes_ignore_textures(tex_ctx):
    """randColourSelect 1-2 switch before the texture branches (:575-662)."""
    ctx, _ = tex_ctx
    for mode in (1, 2):
        p = cgamd.rast_params(W, H, F, colour_mode=mode, rand_offset=12_000_000)
        po = oracle.rast_params(W, H, F, colour_mode=mode, rand_offset=12_000_000, setting=3, setting_boxes=2)
        ref = oracle.rast_draw(po)
        ctx.rast_set_scene(*cgamd.rast_scene(3, 2))
        a, d, s, _ = ctx.rast_draw(p)
        _check((a, d, s), ref, f"colour mode {mode}")


def test_missing_maps_and_bad_selector_fail_loudly(ctx):
    ctx.rast_set_textures(None)
    try:
        p = cgamd.rast_params(64, 48, 64.0)
        ctx.rast_set_scene(*cgamd.rast_scene(3, 0))
        with pytest.raises(RuntimeError):
            ctx.rast_draw(p)
        maps = _maps(seed=3)
        ctx.rast_set_textures({k: v for k, v in maps.items() if k.startswith("grill")})
        ctx.rast_set_scene(*cgamd.rast_scene(2, 0))
        ctx.rast_draw(p)                                 # grill loaded: fine
        ctx.rast_set_scene(*cgamd.rast_scene(3, 0))
        with pytest.raises(RuntimeError):                # woven still missing
            ctx.rast_draw(p)
        ctx.rast_set_scene(*cgamd.rast_scene(5, 0))
        with pytest.raises(RuntimeError):                # no texture 5
            ctx.rast_draw(p)
    finally:
        ctx.rast_set_textures(None)
        ctx.rast_set_scene()


def test_device_list_with_unloaded_texture_shades_as_texture_0(ctx):
    """cg_rast_render_device does not inspect a device list: a triangle whose
    texture maps are not loaded must not be read from (no fault) and shades as
    texture 0."""
    import torch
    W2, H2, F2 = 160, 120, 96.0
    maps = _maps(seed=5)
    ctx.rast_set_textures({k: v for k, v in maps.items() if k.startswith("grill")})
    try:
        p = cgamd.rast_params(W2, H2, F2)
        room, nr, bx, nb = cgamd.rast_scene(3, 0)                 # woven room, woven not loaded
        tris, n, light = cgamd.rast_prepare(p, room, nr, bx, nb)
        d_tris = torch.frombuffer(bytearray(tris), dtype=torch.uint8)[:n * C.sizeof(cgamd.RTri)].cuda()
        a = torch.zeros(W2 * H2, dtype=torch.int32, device="cuda")
        d = torch.zeros(W2 * H2, dtype=torch.float32, device="cuda")
        s = torch.zeros(W2 * H2, dtype=torch.int32, device="cuda")
        ctx.rast_render_device(d_tris.data_ptr(), n, p, light, a.data_ptr(), d.data_ptr(), s.data_ptr())
        torch.cuda.synchronize()
        ra, rd, rs = oracle.rast_draw(oracle.rast_params(W2, H2, F2))
        _check((a.cpu().numpy().view(np.uint32), d.cpu().numpy(), s.cpu().numpy()), (ra, rd, rs), "device list")
    finally:
        ctx.rast_set_textures(None)


@pytest.fixture(scope="module")
def real_maps(ctx):
    """The reference's JPEG maps decoded on the GPU, and the oracle's decode of the same files."""
    import make_golden as mg
    jp = mg.texture_jpegs()
    gpu = {k: ctx.decode_jpeg(v) for k, v in jp.items()}
    ref = {k: oracle.jpeg_decode(v) for k, v in jp.items()}
    for k in jp:
        assert np.array_equal(gpu[k], ref[k]), k
    return gpu, ref


REAL_CASES = [(3, 3, 0.2, 0.0), (3, 0, 0.2, 0.35), (0, 3, 0.15, 0.1745), (2, 3, 0.2, -0.52),
              (3, 2, 0.2, 0.0), (2, 2, 0.15, -0.1745)]


@pytest.mark.parametrize("setting,boxes,ind,yaw", REAL_CASES)
def test_real_maps_draw_matches_oracle(ctx, real_maps, setting, boxes, ind, yaw):
    """Woven-wood (mode 3) and grill (mode 2) rooms and boxes with the reference's maps,
    yawed cameras included (findU/findV through inverse(R), :1756-1825)."""
    gpu, ref = real_maps
    R = cgamd.yaw_matrix(yaw) if yaw else None
    p = cgamd.rast_params(W, H, F, R=R, indirect_first=ind, yaw=yaw)
    po = oracle.rast_params(W, H, F, R=list(R) if R is not None else None, indirect_first=ind,
                            setting=setting, setting_boxes=boxes, yaw=yaw)
    oracle.rast_set_textures(ref)
    ctx.rast_set_textures(gpu)
    try:
        want = oracle.rast_draw(po)
        ctx.rast_set_scene(*cgamd.rast_scene(setting, boxes))
        got = ctx.rast_draw(p)[:3]
    finally:
        oracle.rast_set_textures(None)
        ctx.rast_set_textures(None)
        ctx.rast_set_scene()
    _check(got, want, f"real maps {setting}/{boxes} yaw {yaw}")
    # the textures matter: the frame differs from texture 0's
    ref0 = oracle.rast_draw(oracle.rast_params(W, H, F, R=list(R) if R is not None else None, indirect_first=ind,
                                               yaw=yaw))
    assert (got[0] != ref0[0]).mean() > 0.05
