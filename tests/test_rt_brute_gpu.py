"""GPU: a defect detector for the certificate machinery.

cg_rt_render_brute_device renders with the reference's own loop and no
acceleration at all (every sub-ray against every triangle, every shadow ray
against every triangle until its first blocker; csrc/cg_rt_brute.hip).  It is
pinned here against the oracle on whole small frames (the Cornell box with its
sphere, large-scene clouds under every camera kind, 16 lights) and on SURVEY
8d's 1,024-pixel stratified sample of the full C5 frame; then the product's
accelerated C5 frame (1920x1080 over 1M random triangles: FP64 interval
certificates, grazing-triangle bin / half-bin masks, the certified lit search,
the pools) is compared with it on every one of its 2,073,600 pixels.
Reference semantics: raytracer/Source/skeleton.cpp:120-166, 263-415."""
import ctypes as C
import os
import time

import numpy as np
import pytest

import cgamd
import make_golden as mg
import oracle

pytestmark = pytest.mark.gpu

L0 = [[0.0, -0.5, -0.7, 1.0], [14.0, 14.0, 14.0]]


def _lights(cfg):
    arr = (cgamd.Light * len(cfg["lights"]))()
    for i, (p, c) in enumerate(cfg["lights"]):
        arr[i].position = cgamd.Vec4(*p)
        arr[i].colour = cgamd.Vec3(*c)
    if "area" in cfg:
        return cgamd.area_lights(arr[0], cfg["area"]["side"], cfg["area"]["n"])
    return arr


def _cam(cfg):
    R = (C.c_float * 16)(*cfg["R"]) if cfg.get("R") else None
    return cgamd.rt_camera(cfg["width"], cfg["height"], cfg["focal"], tuple(cfg["cam"]), R)


def _set_scene(ctx, cfg):
    if "scene" in cfg:
        sc = cfg["scene"]
        ctx.rt_set_scene(cgamd.random_scene(sc["random"], sc["seed"]), sc["random"], None, 0)
    else:
        tris, n, sph = cgamd.rt_scene()
        ctx.rt_set_scene(tris, n, sph, 1)


def _brute(ctx, cfg, rows=None, band=120):
    """The brute-force frame (or rows (row0, n)) as uint32 pixels, band by band."""
    import torch
    W, H = cfg["width"], cfg["height"]
    r0, nr = rows or (0, H)
    out = torch.zeros(nr * W, dtype=torch.int32, device="cuda")
    cam, lights = _cam(cfg), _lights(cfg)
    for a in range(r0, r0 + nr, band):
        n = min(band, r0 + nr - a)
        ctx.rt_render_brute_device(cam, a, n, out.data_ptr() + (a - r0) * W * 4, lights=lights)
    return out.cpu().numpy().view(np.uint32).reshape(nr, W)


SMALL = {
    "cornell_320x256": dict(width=320, height=256, focal=256.0, cam=[0, 0, -2.9, 1], R=None, lights=[L0]),
    "cornell_area16": dict(width=96, height=72, focal=72.0, cam=[0, 0, -3.0, 1], R=None, lights=[L0],
                           area=dict(side=0.1, n=4)),
    "cloud_lat": dict(width=64, height=48, focal=48.0, cam=[0, 0, -3.0, 1], R=None, lights=[L0],
                      scene=dict(random=500, seed=0x5EED)),
    "cloud_yaw_area16": dict(width=64, height=48, focal=48.0, cam=[0, 0, -3.0, 1],
                             R=mg.yaw_R(np.float32(0.0) - np.float32(0.174533)), lights=[L0],
                             area=dict(side=0.1, n=4), scene=dict(random=500, seed=0x5EED)),
    "cloud_inside": dict(width=64, height=48, focal=48.0, cam=[-0.2249, 0.1385, 0.04, 1.0], R=None, lights=[L0],
                         scene=dict(random=500, seed=0x5EED)),
    "c5_256x144": dict(width=256, height=144, focal=144.0, cam=[0, 0, -3.0, 1], R=None, lights=[L0],
                       scene=dict(random=2000, seed=0x5EED)),
}


@pytest.mark.parametrize("name", list(SMALL))
def test_brute_matches_oracle_whole_frame(ctx, name):
    cfg = SMALL[name]
    _set_scene(ctx, cfg)
    try:
        got = _brute(ctx, cfg, band=16).reshape(-1)
    finally:
        _set_scene(ctx, {})
    ref = oracle.rt_draw(mg.rt_params_of(cfg), scene=mg.rt_oracle_scene(cfg),
                         threads=min(16, os.cpu_count() or 8))
    bad = np.flatnonzero(got != ref)
    assert bad.size == 0, f"{name}: {bad.size} pixels differ, first {bad[:6]}"
    assert (ref != 0x80000000).sum() > 100


C5_FULL = dict(width=1920, height=1080, focal=1080.0, cam=[0, 0, -3.0, 1], R=None, lights=[L0],
               scene=dict(random=1_000_000, seed=0x5EED))


def _stratified(W, H, n_side):
    """bench.py's fixed stratified sample: the centre of each cell of an n_side grid."""
    xs = ((np.arange(n_side) + 0.5) * W / n_side).astype(np.int64)
    ys = ((np.arange(n_side) + 0.5) * H / n_side).astype(np.int64)
    return np.stack(np.meshgrid(xs, ys), -1).reshape(-1, 2)


def test_c5_full_frame_every_pixel_vs_brute_force(ctx):
    """The accelerated C5 frame == the brute-force frame on all 2,073,600 pixels; the brute
    force itself == the oracle on the 1,024-pixel stratified sample."""
    cfg = C5_FULL
    W, H = cfg["width"], cfg["height"]
    _set_scene(ctx, cfg)
    try:
        fast, _ = ctx.rt_render(_cam(cfg), _lights(cfg))
        t0 = time.perf_counter()
        brute = _brute(ctx, cfg)
        dt = time.perf_counter() - t0
    finally:
        _set_scene(ctx, {})
    print(f"\nC5 brute-force frame: {dt:.1f} s on the GPU")
    xy = _stratified(W, H, 32)
    ref = oracle.rt_draw_pixels(mg.rt_params_of(cfg), xy, scene=mg.rt_oracle_scene(cfg),
                                threads=min(16, os.cpu_count() or 8))
    bs = brute[xy[:, 1], xy[:, 0]]
    bad = np.flatnonzero(bs != ref)
    assert bad.size == 0, f"brute force vs oracle: {bad.size} of 1024 differ, first at {xy[bad[:4]]}"
    fast = fast.reshape(H, W)
    diff = np.argwhere(fast != brute)
    assert diff.size == 0, f"{len(diff)} pixels differ from the brute force, first (y, x) {diff[:6].tolist()}"
    assert (brute != 0x80000000).sum() > W * H // 4            # the frame sees the cloud
