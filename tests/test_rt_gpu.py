"""GPU: the raytracer hot path (rt_pixel_kernel via cg_rt_render) against the
oracle, bit-exact (integer ARGB output: the tolerance is 0), plus the
reference's own screenshot.bmp and the SURVEY.md 8c fingerprints."""
import ctypes as C
import os

import numpy as np
import pytest

import cgamd
import cgdist
import make_golden as mg
import oracle

pytestmark = pytest.mark.gpu


def _lights(cfg):
    arr = (cgamd.Light * len(cfg["lights"]))()
    for i, (p, c) in enumerate(cfg["lights"]):
        arr[i].position = cgamd.Vec4(*p)
        arr[i].colour = cgamd.Vec3(*c)
    if "area" in cfg:   # C4: the library's own area-light expansion
        return cgamd.area_lights(arr[0], cfg["area"]["side"], cfg["area"]["n"])
    return arr


def _set_scene(ctx, cfg):
    if "scene" in cfg:
        sc = cfg["scene"]
        ctx.rt_set_scene(cgamd.random_scene(sc["random"], sc["seed"]), sc["random"], None, 0)
    else:
        tris, n, sph = cgamd.rt_scene()
        ctx.rt_set_scene(tris, n, sph, 1)


def _cam(cfg):
    R = (C.c_float * 16)(*cfg["R"]) if cfg["R"] else None
    return cgamd.rt_camera(cfg["width"], cfg["height"], cfg["focal"], tuple(cfg["cam"]), R)


@pytest.fixture(scope="module")
def rt(ctx):
    tris, n, sph = cgamd.rt_scene()
    ctx.rt_set_scene(tris, n, sph, 1)
    return ctx


def test_rt_screenshot_golden(rt):
    """GPU frame == raytracer/screenshot.bmp, every pixel."""
    cfg = mg.rt_configs()["rt_320x256_z-2.9"]
    argb, st = rt.rt_render(_cam(cfg), _lights(cfg))
    assert int((argb != mg.screenshot_argb()).sum()) == 0
    assert st.kernel_ms > 0


@pytest.mark.parametrize("name", list(mg.rt_configs()))
def test_rt_configs_match_golden(rt, golden, name):
    cfg = mg.rt_configs()[name]
    _set_scene(rt, cfg)
    try:
        argb, _ = rt.rt_render(_cam(cfg), _lights(cfg))
    finally:
        _set_scene(rt, {})
    h = mg.sha(argb)
    assert h == golden["rt"][name]["argb_sha256"], name
    ref = mg.REFERENCE_FINGERPRINTS.get(name)
    if ref:
        assert h.startswith(ref["argb"])


def test_rt_vs_live_oracle_diff_report(rt):
    """Independent live oracle run at an odd size; on mismatch report the diff."""
    p = oracle.rt_params(200, 120, 150.0, (0.05, -0.1, -2.7, 1.0))
    ref = oracle.rt_draw(p, threads=os.cpu_count() or 8)
    cam = cgamd.rt_camera(200, 120, 150.0, (0.05, -0.1, -2.7, 1.0))
    argb, _ = rt.rt_render(cam)
    bad = np.flatnonzero(argb != ref)
    assert bad.size == 0, f"{bad.size} pixels differ, first {bad[:8]} gpu {argb[bad[:4]]} ref {ref[bad[:4]]}"


_LIGHT_SET = [((0.0, -0.5, -0.7, 1.0), (14.0, 14.0, 14.0)), ((0.3, -0.6, 0.2, 1.0), (3.0, 1.5, 0.5)),
              ((-0.5, -0.2, -0.3, 1.0), (0.25, 2.0, 1.0)), ((0.2, 0.1, -0.9, 1.0), (1.0, 1.0, 6.0)),
              ((0.0, -0.9, 0.0, 1.0), (2.5, 2.5, 2.5))]


_SET_YAWS = {"yaw5": 0.1, "yaw64": 0.1, "yaw2_5": 2.0, "yawneg_64": -0.52}


@pytest.mark.parametrize("case", ["lattice5", "lattice64", "yaw5", "yaw64", "yaw2_5", "yawneg_64"])
def test_rt_light_sets_vs_oracle(rt, case):
    """Light sets against the live oracle at a ragged size (partial lattice
    tiles on both edges): rt_lattice_lights_kernel, unrotated cameras with
    shared lattice columns, yawed ones (also past 90 degrees, dir.x decreasing)
    with per-pixel columns.  5 lights (not a multiple of the fold's 4-light
    vector reads) and C4's 8 x 8 area light."""
    W, H, f = 200, 118, 150.0
    if case.endswith("64"):
        lights = oracle.rt_area_lights((0.0, -0.5, -0.7, 1.0), (14.0, 14.0, 14.0), 0.1, 8)
    else:
        lights = _LIGHT_SET
    R = cgamd.yaw_matrix(_SET_YAWS[case]) if case.startswith("yaw") else None
    cam_pos = (0.05, -0.1, -2.7, 1.0)
    p = oracle.rt_params(W, H, f, cam_pos, list(R) if R is not None else None, lights=lights)
    ref = oracle.rt_draw(p, threads=os.cpu_count() or 8)
    arr = (cgamd.Light * len(lights))()
    for i, (pos, col) in enumerate(lights):
        arr[i].position = cgamd.Vec4(*pos)
        arr[i].colour = cgamd.Vec3(*col)
    argb, _ = rt.rt_render(cgamd.rt_camera(W, H, f, cam_pos, R), arr)
    bad = np.flatnonzero(argb != ref)
    assert bad.size == 0, f"{case}: {bad.size} pixels differ, first {bad[:8]}"


def _three_spheres():
    """LoadTestModel's sphere plus two more (TestModelH.h:275-277 shape): the
    lattice paths store sphere q's hits as -1 - q, so sphere 1's are -2."""
    _, _, s0 = cgamd.rt_scene()
    sph = (cgamd.Sphere * 3)(s0, s0, s0)
    for q, (c, r, col) in enumerate((((0.4, 0.55, -0.3), 0.25, (0.2, 0.8, 0.3)),
                                     ((0.05, -0.15, 0.1), 0.15, (0.9, 0.4, 0.1))), 1):
        sph[q].radius, sph[q].radiusSquared = r, np.float32(r) * np.float32(r)
        sph[q].centre = cgamd.Vec3(*c)
        sph[q].color = cgamd.Vec3(*col)
    return sph


@pytest.mark.parametrize("case", ["lattice5", "lattice64", "yaw5", "one"])
def test_rt_three_spheres_vs_oracle(rt, case):
    """Three spheres under light sets (rt_lattice_units_kernel's per-unit sole-hit
    object must not confuse sphere 1's hit index -2 with 'no hit'), a yawed
    light set and the one-light lattice, against the live oracle."""
    tris, n, _ = cgamd.rt_scene()
    sph = _three_spheres()
    W, H, f = 200, 118, 150.0
    lights = {"lattice64": oracle.rt_area_lights((0.0, -0.5, -0.7, 1.0), (14.0, 14.0, 14.0), 0.1, 8),
              "one": _LIGHT_SET[:1]}.get(case, _LIGHT_SET)
    R = cgamd.yaw_matrix(0.3) if case.startswith("yaw") else None
    cam_pos = (0.05, -0.1, -2.7, 1.0)
    osph = (oracle.Sphere * 3).from_buffer_copy(sph)
    otris = (oracle.RtTri * len(tris)).from_buffer_copy(tris)
    p = oracle.rt_params(W, H, f, cam_pos, list(R) if R is not None else None, lights=lights)
    ref = oracle.rt_draw(p, threads=os.cpu_count() or 8, scene=(otris, n, osph, 3))
    arr = (cgamd.Light * len(lights))()
    for i, (pos, col) in enumerate(lights):
        arr[i].position = cgamd.Vec4(*pos)
        arr[i].colour = cgamd.Vec3(*col)
    rc = rt.lib.cg_rt_set_scene(rt.h, tris, n, sph, 3)
    assert rc == 0
    try:
        argb, _ = rt.rt_render(cgamd.rt_camera(W, H, f, cam_pos, R), arr)
    finally:
        _set_scene(rt, {})
    bad = np.flatnonzero(argb != ref)
    assert bad.size == 0, f"{case}: {bad.size} pixels differ, first {bad[:8]}"
    # the extra spheres are in view: the frame differs from the one-sphere scene's
    ref1 = oracle.rt_draw(p, threads=os.cpu_count() or 8)
    assert int((ref1 != ref).sum()) > 500


@pytest.mark.parametrize("yaw", [0.1745, -0.52, 0.9, 2.0, -1.5707964, 3.1415927])
def test_rt_yaw_lattice_vs_oracle(rt, yaw):
    """A yawed one-light camera (skeleton.cpp:233-244) takes the lattice
    kernel's per-pixel-column form (cg_rt.hip lat_yaw): dir.x = fl(c x + s f)
    per pixel, rows shared.  Ragged size (partial tiles on both edges); yaws
    past 90 degrees make dir.x decrease along a row (the certificates' x extent
    comes from the end pixels either way); -90 degrees makes c ~ 0."""
    W, H, f = 200, 118, 150.0
    R = cgamd.yaw_matrix(yaw)
    cam_pos = (0.05, -0.1, -2.7, 1.0)
    ref = oracle.rt_draw(oracle.rt_params(W, H, f, cam_pos, list(R)), threads=os.cpu_count() or 8)
    argb, _ = rt.rt_render(cgamd.rt_camera(W, H, f, cam_pos, R))
    bad = np.flatnonzero(argb != ref)
    assert bad.size == 0, f"yaw {yaw}: {bad.size} pixels differ, first {bad[:8]}"


@pytest.mark.parametrize("W,H,yaw,nl", [(1, 1, 0.3, 1), (17, 9, -2.5, 1), (33, 31, 0.3, 5), (15, 16, 1.2, 5)])
def test_rt_yaw_lattice_small_frames(rt, W, H, yaw, nl):
    """Yawed lattice kernels on frames smaller than / not multiples of a
    16 x 15 tile (a single pixel, partial tiles only), one light and a
    5-light set, against the live oracle."""
    f = 40.0
    R = cgamd.yaw_matrix(yaw)
    cam_pos = (0.02, -0.05, -2.8, 1.0)
    lights = _LIGHT_SET[:nl]
    ref = oracle.rt_draw(oracle.rt_params(W, H, f, cam_pos, list(R), lights=lights), threads=4)
    arr = (cgamd.Light * nl)()
    for i, (pos, col) in enumerate(lights):
        arr[i].position = cgamd.Vec4(*pos)
        arr[i].colour = cgamd.Vec3(*col)
    argb, _ = rt.rt_render(cgamd.rt_camera(W, H, f, cam_pos, R), arr)
    assert np.array_equal(argb, ref), f"{W}x{H} yaw {yaw}: {int((argb != ref).sum())} pixels differ"


def test_rt_yaw_lattice_stripes_vs_oracle(rt):
    """Yawed lattice on 15-row stripes (2 and 3 ranks), reassembled, against
    the oracle's whole frame."""
    torch = pytest.importorskip("torch")
    W, H, f = 192, 150, 140.0
    R = cgamd.yaw_matrix(-0.3)
    cam_pos = (0.1, 0.05, -2.8, 1.0)
    ref = oracle.rt_draw(oracle.rt_params(W, H, f, cam_pos, list(R)), threads=os.cpu_count() or 8)
    cam = cgamd.rt_camera(W, H, f, cam_pos, R)
    full, _ = rt.rt_render(cam)
    assert int((full != ref).sum()) == 0
    st = torch.cuda.Stream()
    for n in (2, 3):
        S = cgdist.LATTICE_STRIPE
        rows = cgdist.shard_rows(H, n, S)
        g = torch.zeros(n * rows * W, dtype=torch.int32, device="cuda")
        for r in range(n):
            rt.rt_render_device(cam, g.data_ptr() + r * rows * W * 4, cgamd.RtShard(r, n, S), st.cuda_stream)
        frame = torch.zeros(H * W, dtype=torch.int32, device="cuda")
        rt.rt_unstripe_device(g.data_ptr(), W, H, n, S, frame.data_ptr(), st.cuda_stream)
        st.synchronize()
        assert np.array_equal(frame.cpu().numpy().view(np.uint32), ref), n


def test_rt_probe_closest_and_direct_light(rt, golden):
    rays = golden["rt_rays"]
    out, hit = rt.rt_probe_closest([r["start"] for r in rays], [r["dir"] for r in rays])
    isects = []
    for r, o, h in zip(rays, out, hit):
        assert h == r["hit"]
        if h:
            e = r["isect"]
            assert [o.position.x, o.position.y, o.position.z, o.position.w] == e["position"]
            assert o.distance == e["distance"]
            assert (o.triangleIndex, o.sphereIndex) == (e["triangleIndex"], e["sphereIndex"])
            isects.append((o, r["direct_light"]))
    light = cgamd.Light(cgamd.Vec4(0.0, -0.5, -0.7, 1.0), cgamd.Vec3(14.0, 14.0, 14.0))
    dl = rt.rt_probe_direct_light([i for i, _ in isects], light)
    for got, (_, want) in zip(dl, isects):
        assert [got.x, got.y, got.z] == want


def test_rt_sharded_device_path_reassembles(rt):
    """cg_rt_render_device per shard + cg_rt_unstripe_device == whole frame."""
    torch = pytest.importorskip("torch")
    W, H = 320, 256
    cam = cgamd.rt_camera(W, H)
    full, _ = rt.rt_render(cam)
    st = torch.cuda.Stream()
    torch.cuda.set_stream(st)
    # 8-row stripes (general kernel's tiles), 15-row (lattice kernel's tiles: the
    # unrotated one-light camera), and a height that matches neither
    for S in (cgdist.DEFAULT_STRIPE, cgdist.LATTICE_STRIPE, 12):
        for n in (2, 3, 8):
            rows = cgdist.shard_rows(H, n, S)
            g = torch.zeros(n * rows * W, dtype=torch.int32, device="cuda")
            for r in range(n):
                sh = cgamd.RtShard(r, n, S)
                rt.rt_render_device(cam, g.data_ptr() + r * rows * W * 4, sh, st.cuda_stream)
            frame = torch.zeros(H * W, dtype=torch.int32, device="cuda")
            rt.rt_unstripe_device(g.data_ptr(), W, H, n, S, frame.data_ptr(), st.cuda_stream)
            st.synchronize()
            assert np.array_equal(frame.cpu().numpy().view(np.uint32), full), (S, n)


def test_rt_batched_unstripe(rt):
    """cg_rt_unstripe_batch_device: per-rank shards of several frames (frame-major
    per rank, as one gather of K frames lays them out) == each frame rendered whole."""
    torch = pytest.importorskip("torch")
    W, H, n, S = 320, 256, 3, cgdist.DEFAULT_STRIPE
    cams = [cgamd.rt_camera(W, H, 256.0, (0.0, 0.0, z, 1.0)) for z in (-3.0, -2.9, -2.6)]
    fulls = [rt.rt_render(c)[0] for c in cams]
    st = torch.cuda.Stream()
    rows = cgdist.shard_rows(H, n, S)
    K = len(cams)
    g = torch.zeros(n * K * rows * W, dtype=torch.int32, device="cuda")
    for r in range(n):
        for k, cam in enumerate(cams):
            off = ((r * K + k) * rows * W) * 4
            rt.rt_render_device(cam, g.data_ptr() + off, cgamd.RtShard(r, n, S), st.cuda_stream)
    frames = torch.zeros(K * H * W, dtype=torch.int32, device="cuda")
    rt.rt_unstripe_batch_device(g.data_ptr(), W, H, n, S, K, frames.data_ptr(), st.cuda_stream)
    st.synchronize()
    got = frames.cpu().numpy().view(np.uint32).reshape(K, H * W)
    for k in range(K):
        assert np.array_equal(got[k], fulls[k]), k


def test_rt_render_frames_batched(rt, golden):
    """cg_rt_render_frames_device: a camera path (cameraPos moving as the UP/DOWN
    keys move it) rendered as one batched launch per 16 frames, whole and
    sharded, == each frame rendered alone; the z = -3 / -2.9 frames also equal
    the golden fingerprint / screenshot.bmp."""
    torch = pytest.importorskip("torch")
    W, H = 320, 256
    zs = [-3.0, mg.CAM_UP] + [-3.0 + 0.05 * k for k in range(1, 18)]   # 19 frames: two launches
    cams = [cgamd.rt_camera(W, H, 256.0, (0.0, 0.0, z, 1.0)) for z in zs]
    singles = [rt.rt_render(c)[0] for c in cams]
    assert np.array_equal(singles[1], mg.screenshot_argb())
    st = torch.cuda.Stream()
    for S, n in ((cgdist.LATTICE_STRIPE, 1), (cgdist.LATTICE_STRIPE, 3), (60, 2)):
        rows = cgdist.shard_rows(H, n, S)
        stride = rows * W + 96                       # a padded frame stride
        g = torch.zeros(n * len(cams) * stride, dtype=torch.int32, device="cuda")
        for r in range(n):
            rt.rt_render_frames_device(cams, g.data_ptr() + r * len(cams) * stride * 4, cgamd.RtShard(r, n, S),
                                       st.cuda_stream, frame_stride=stride)
        st.synchronize()
        got = g.cpu().numpy().view(np.uint32).reshape(n, len(cams), stride)[:, :, :rows * W]
        for k in range(len(cams)):
            frame = cgdist.unstripe_np(got[:, k].reshape(n, rows, W), H, n, S).reshape(-1)
            assert np.array_equal(frame, singles[k]), (S, n, k)


@pytest.mark.parametrize("nl", [1, 4])
def test_rt_render_frames_lateral_windows(rt, nl):
    """A batch's lattice launches cover only the union of its cameras' column windows (the
    scene box's projection, cg_shim.hip rt_enqueue_lattice_batch): cameraPos moving sideways
    -- windows at either edge, one camera that sees nothing at all (an empty window), one
    centred -- rendered as one batched launch (the edge workgroups store the columns outside
    the union black) == each frame rendered alone (no window), one light and a light set."""
    torch = pytest.importorskip("torch")
    W, H = 320, 256
    xs = [-40.0, -1.6, -0.7, 0.0, 0.35, 1.1, 2.4, 40.0]
    cams = [cgamd.rt_camera(W, H, 256.0, (x, 0.1 * k - 0.3, -3.0, 1.0)) for k, x in enumerate(xs)]
    lights = cgamd.default_lights() if nl == 1 else cgamd.area_lights(cgamd.default_lights()[0], 0.1, 2)
    singles = [rt.rt_render(c, lights)[0] for c in cams]
    tris, n, sph = cgamd.rt_scene()
    cols = [cgamd.frame_columns(tris, n, sph, 1, c) for c in cams]
    assert cols[0][0] >= cols[0][1] and cols[-1][0] >= cols[-1][1]     # these two see nothing
    assert not singles[0].any() or (singles[0] == singles[0][0]).all()  # a uniform (black) frame
    assert any(0 < c0 < c1 < W for c0, c1 in cols)                     # a window inside the frame
    g = torch.zeros(len(cams) * W * H, dtype=torch.int32, device="cuda")
    st = torch.cuda.Stream()
    for sel in (list(range(len(cams))), [1, 2], [0], [3, 7]):          # whole path, narrow unions, empty
        sub = [cams[k] for k in sel]
        g.zero_()
        rt.rt_render_frames_device(sub, g.data_ptr(), None, st.cuda_stream, lights=lights)
        st.synchronize()
        got = g.cpu().numpy().view(np.uint32).reshape(len(cams), W * H)
        for i, k in enumerate(sel):
            assert np.array_equal(got[i], singles[k]), (sel, k)


@pytest.mark.parametrize("window", [False, True])
@pytest.mark.parametrize("kind", ["lattice", "yaw", "yaw_batch", "c4", "c4yaw"])
def test_rt_bands_rgb24_assemble(rt, kind, window):
    """bench.py's N > 1 layout on one GPU: uneven bands, rank 0's band rendered
    ARGB straight into the frames, the others in the RGB24 wire format into
    one buffer, cg_rt_assemble_device expands them: == each frame whole."""
    torch = pytest.importorskip("torch")
    W, H = 320, 256
    if kind == "lattice":   # batched lattice launches, RGB24 stored by the kernel
        cams = [cgamd.rt_camera(W, H, 256.0, (0.0, 0.0, z, 1.0)) for z in (-3.0, -2.95, -2.8)]
        lights = cgamd.default_lights()
    elif kind == "yaw":     # yawed lattice, one frame at a time (R differs between the frames)
        cams = [cgamd.rt_camera(W, H, 256.0, (0.0, 0.0, -3.0, 1.0), cgamd.yaw_matrix(y)) for y in (0.05, -0.1)]
        lights = cgamd.default_lights()
    elif kind == "yaw_batch":   # yawed lattice, one batched launch (same R, cameraPos moving)
        cams = [cgamd.rt_camera(W, H, 256.0, (0.0, 0.0, z, 1.0), cgamd.yaw_matrix(0.12)) for z in (-3.0, -2.9, -2.75)]
        lights = cgamd.default_lights()
    elif kind == "c4":      # light set (light-set lattice kernel)
        cams = [cgamd.rt_camera(W, H, 256.0)]
        lights = cgamd.area_lights(None, 0.1, 3)
    else:                   # light set under a yaw (light-set lattice, per-pixel columns)
        cams = [cgamd.rt_camera(W, H, 256.0, (0.0, 0.0, z, 1.0), cgamd.yaw_matrix(-0.2)) for z in (-3.0, -2.85)]
        lights = cgamd.area_lights(None, 0.1, 3)
    singles = [rt.rt_render(c, lights)[0] for c in cams]
    K = len(cams)
    bands = cgdist.rebalance(cgdist.equal_bands(H, 4), [1.0, 2.5, 1.2, 0.6], [0.4, 0, 0, 0], H)
    assert len({nr for _, nr in bands}) > 1          # uneven
    st = torch.cuda.Stream()
    frames = torch.zeros(K * H * W, dtype=torch.int32, device="cuda")
    r0, nr = bands[0]
    # RGB24 window: the columns the camera can see anything in (cg_rt_frame_columns)
    c0, cols = 0, 0
    if window:
        t_, n_, s_ = cgamd.rt_scene()
        c0, c1 = cgamd.frame_columns(t_, n_, s_, 1, cams[0])
        cols = c1 - c0 if c1 - c0 < W else 0
        if "yaw" not in kind:
            assert 0 < cols < W
    pitch = cols or W
    frames.fill_(-1)                                  # the assembly must write every pixel
    rt.rt_render_frames_device(cams, frames.data_ptr() + 4 * r0 * W, cgamd.RtShard(row0=r0, rows=nr),
                               st.cuda_stream, lights, frame_stride=H * W)
    rbuf = torch.zeros(K * H * W * 3 + 64, dtype=torch.uint8, device="cuda")
    off = 0
    for a, n in bands[1:]:
        rt.rt_render_frames_device(cams, rbuf.data_ptr() + off, cgamd.RtShard(row0=a, rows=n, col0=c0, cols=cols),
                                   st.cuda_stream, lights, pix_format=cgamd.PIX_RGB24)
        off += K * n * pitch * 3
    rt.rt_assemble_device(rbuf.data_ptr(), cgamd.PIX_RGB24, [a for a, _ in bands[1:]], [n for _, n in bands[1:]],
                          W, H, K, frames.data_ptr(), 0, st.cuda_stream, col0=c0, cols=cols)
    st.synchronize()
    got = frames.cpu().numpy().view(np.uint32).reshape(K, -1)
    for k in range(K):
        assert np.array_equal(got[k], singles[k]), (kind, window, k)
    # the wire bytes are exactly the low three bytes of each pixel (of the window)
    a, n = bands[1]
    wire = rbuf[:K * n * pitch * 3].cpu().numpy()
    want = np.concatenate([cgdist.pack_rgb24_np(cgdist.window_np(s_[a * W:(a + n) * W], W, c0, pitch))
                           for s_ in singles])
    assert np.array_equal(wire, want)


def test_rt_window_validation(rt):
    """Windows only for RGB24, 16-aligned, inside the frame."""
    torch = pytest.importorskip("torch")
    cam = cgamd.rt_camera(320, 256, 256.0)
    buf = torch.zeros(320 * 256, dtype=torch.int32, device="cuda")
    for sh, fmt in ((cgamd.RtShard(row0=0, rows=8, col0=16, cols=64), cgamd.PIX_ARGB8888),
                    (cgamd.RtShard(row0=0, rows=8, col0=8, cols=64), cgamd.PIX_RGB24),
                    (cgamd.RtShard(row0=0, rows=8, col0=16, cols=20), cgamd.PIX_RGB24),
                    (cgamd.RtShard(row0=0, rows=8, col0=304, cols=32), cgamd.PIX_RGB24)):
        with pytest.raises(RuntimeError):
            rt.rt_render_frames_device([cam], buf.data_ptr(), sh, None, pix_format=fmt)
    with pytest.raises(RuntimeError):
        rt.rt_render_device(cam, buf.data_ptr(), cgamd.RtShard(row0=0, rows=8, col0=16, cols=64))


def test_rt_assemble_argb_and_ragged(rt):
    """cg_rt_assemble_device with ARGB blocks, a width that is not a multiple of
    4 and a block running past the frame's last row."""
    torch = pytest.importorskip("torch")
    W, H = 37, 11
    rng = np.random.default_rng(9)
    ref = (0x80000000 | rng.integers(0, 1 << 24, H * W, dtype=np.uint32)).astype(np.uint32)
    bands = [(0, 4), (4, 5), (9, 4)]                 # last block: rows 9..12, 11.. are padding
    for fmt, bpp in ((cgamd.PIX_ARGB8888, 4), (cgamd.PIX_RGB24, 3)):
        blocks = []
        for a, n in bands:
            blk = np.zeros(n * W, np.uint32)
            m = min(n, H - a)
            blk[:m * W] = ref[a * W:(a + m) * W]
            blocks.append(blk.view(np.uint8) if bpp == 4 else cgdist.pack_rgb24_np(blk))
        src = torch.from_numpy(np.concatenate(blocks)).cuda()
        out = torch.zeros(H * W, dtype=torch.int32, device="cuda")
        rt.rt_assemble_device(src.data_ptr(), fmt, [a for a, _ in bands], [n for _, n in bands], W, H, 1,
                              out.data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().view(np.uint32), ref), fmt


def test_rt_render_frames_fallback(rt):
    """Frames that cannot share a launch (yaw-rotated R, two lights) go one by one."""
    torch = pytest.importorskip("torch")
    W, H = 256, 192
    cams = [cgamd.rt_camera(W, H, 200.0, (0.0, 0.0, -3.0, 1.0), cgamd.yaw_matrix(y)) for y in (0.0, 0.1)]
    two = (cgamd.Light * 2)(*cgamd.default_lights(), *cgamd.default_lights())
    two[1].position = cgamd.Vec4(0.3, -0.5, -0.2, 1.0)
    for lights in (cgamd.default_lights(), two):
        singles = [rt.rt_render(c, lights)[0] for c in cams]
        g = torch.zeros(len(cams) * W * H, dtype=torch.int32, device="cuda")
        st = torch.cuda.Stream()
        rt.rt_render_frames_device(cams, g.data_ptr(), None, st.cuda_stream, lights)
        st.synchronize()
        got = g.cpu().numpy().view(np.uint32).reshape(len(cams), -1)
        for k in range(len(cams)):
            assert np.array_equal(got[k], singles[k]), k


def test_rt_full_1080p_vs_oracle(rt, golden):
    """North-star config C2 at full size: the oracle's frame hash, itself pinned
    to the reference build's fingerprint."""
    cfg = mg.rt_configs()["rt_1920x1080_f1080"]
    argb, _ = rt.rt_render(_cam(cfg), _lights(cfg))
    assert mg.sha(argb) == golden["rt"]["rt_1920x1080_f1080"]["argb_sha256"]


def _sample_xy(W, H, n, seed):
    """n pixels: the four corners, a stratified grid and uniform random ones."""
    rng = np.random.default_rng(seed)
    g = int(np.sqrt(n // 2))
    gx, gy = np.meshgrid(np.linspace(0, W - 1, g).astype(int), np.linspace(0, H - 1, g).astype(int))
    xy = [np.array([[0, 0], [W - 1, 0], [0, H - 1], [W - 1, H - 1]]),
          np.stack([gx.ravel(), gy.ravel()], 1),
          np.stack([rng.integers(0, W, n - 4 - g * g), rng.integers(0, H, n - 4 - g * g)], 1)]
    return np.concatenate(xy).astype(np.int32)


C4_FULL = dict(width=3840, height=2160, focal=2160.0, cam=[0, 0, -3.0, 1], R=None,
               lights=[[[0.0, -0.5, -0.7, 1.0], [14.0, 14.0, 14.0]]], area=dict(side=0.1, n=8))


@pytest.mark.parametrize("mode", ["2", "1"])
def test_rt_measured_order_bands_exact(rt, golden, mode):
    """The measured lattice dispatch order (cg_internal.h LatOrder; band-sized launches take it
    from the previous call's per-tile durations): the N = 8 bands of C2, 20-frame calls repeated
    on one context (call 1 records, later calls run in the sorted order) with a fixed and a moving
    camera, RGB24 over the wire's columns: every frame's band == the golden 1080p frame's rows
    (fixed camera) or == the frame rendered alone (moving camera).  Run in a child process per
    order mode (CG_LAT_ORDER is read once per process)."""
    import json
    import subprocess
    import sys
    code = r"""
import hashlib, json, os, sys
import numpy as np, torch
sys.path[:0] = [os.path.join(os.environ["CG_ROOT"], "computer-graphics_amd"), os.path.join(os.environ["CG_ROOT"], "tests", "golden")]
import cgamd, cgdist
W, H, F = 1920, 1080, 1080.0
ctx = cgamd.Context(0)
tris, n, sph = cgamd.rt_scene()
ctx.rt_set_scene(tris, n, sph, 1)
cam = cgamd.rt_camera(W, H, F)
whole = ctx.rt_render(cam)[0]
c0, c1 = cgamd.frame_columns(tris, n, sph, 1, cam)
moving = [cgamd.rt_camera(W, H, F, (0.0, 0.0, -3.0 + 0.005 * k, 1.0)) for k in range(20)]
alone = {k: ctx.rt_render(moving[k])[0] for k in (0, 7, 19)}
bands = [(0, 194), (194, 181), (375, 157), (532, 137), (669, 89), (758, 89), (847, 102), (949, 131)]
bad = []
buf = torch.zeros(20 * 194 * (c1 - c0) * 3 + 64, dtype=torch.uint8, device="cuda")
for path, cams in (("fixed", [cam] * 20), ("moving", moving)):
    for a, nr in bands:
        sh = cgamd.RtShard(row0=a, rows=nr, col0=c0, cols=c1 - c0)
        for call in range(3):
            buf.zero_()
            ctx.rt_render_frames_device(cams, buf.data_ptr(), sh, None, pix_format=cgamd.PIX_RGB24)
            torch.cuda.synchronize()
            got = buf[:20 * nr * (c1 - c0) * 3].cpu().numpy().reshape(20, -1)
            for k in range(20):
                ref = whole if path == "fixed" else alone.get(k)
                if ref is None:
                    continue
                want = cgdist.pack_rgb24_np(cgdist.window_np(ref[a * W:(a + nr) * W], W, c0, c1 - c0))
                if not np.array_equal(got[k], want):
                    bad.append((path, a, call, k))
print("RESULT " + json.dumps({"bad": bad[:10], "nbad": len(bad), "whole_sha": hashlib.sha256(whole.tobytes()).hexdigest()}))
"""
    env = dict(os.environ, CG_ROOT=os.path.dirname(os.path.dirname(os.path.abspath(__file__))), CG_LAT_ORDER=mode)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=110, env=env)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
    assert r.returncode == 0 and lines, f"rc {r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-3000:]}"
    res = json.loads(lines[-1][7:])
    assert res["whole_sha"] == golden["rt"]["rt_1920x1080_f1080"]["argb_sha256"]
    assert res["nbad"] == 0, res["bad"]


def test_rt_c4_4k_soft_shadows_sampled(rt):
    """C4 at full size (3840x2160, f=2160, 8x8 area light = 64 lights): the
    whole GPU frame, 65,536 of its pixels checked bit-exactly against the
    oracle (the whole frame: test_rt_c4_4k_whole_frame_vs_oracle; the 480x270
    C4 frame is checked whole in test_rt_configs_match_golden)."""
    cfg = C4_FULL
    W, H = cfg["width"], cfg["height"]
    argb, st = rt.rt_render(_cam(cfg), _lights(cfg))
    xy = _sample_xy(W, H, 65536, 4)
    ref = oracle.rt_draw_pixels(mg.rt_params_of(cfg), xy, threads=min(16, os.cpu_count() or 8))
    got = argb.reshape(H, W)[xy[:, 1], xy[:, 0]]
    bad = np.flatnonzero(got != ref)
    assert bad.size == 0, f"{bad.size} differ, first at {xy[bad[:4]]}: gpu {got[bad[:4]]} ref {ref[bad[:4]]}"
    assert (got >> 24 == 0x80).all()


def test_rt_c4_4k_whole_frame_vs_oracle(rt):
    """C4 at full size, every one of the 8,294,400 pixels bit-exact against the oracle (about
    5 CPU-minutes of oracle work: ~20 s on the GPU box's 16 usable cores)."""
    cfg = C4_FULL
    W, H = cfg["width"], cfg["height"]
    argb, _ = rt.rt_render(_cam(cfg), _lights(cfg))
    yy, xx = np.mgrid[0:H, 0:W]
    xy = np.stack([xx.ravel(), yy.ravel()], 1).astype(np.int32)
    ref = oracle.rt_draw_pixels(mg.rt_params_of(cfg), xy, threads=min(16, os.cpu_count() or 8))
    bad = np.flatnonzero(argb != ref)
    assert bad.size == 0, f"{bad.size} differ, first at {xy[bad[:4]]}: gpu {argb[bad[:4]]} ref {ref[bad[:4]]}"


def test_rt_c4_sharded_matches_whole(rt):
    """C4's multi-GPU form: 8 row-stripe shards + unstripe == the whole frame."""
    torch = pytest.importorskip("torch")
    cfg = dict(C4_FULL, width=960, height=540, focal=540.0)
    W, H = cfg["width"], cfg["height"]
    cam, lights = _cam(cfg), _lights(cfg)
    full, _ = rt.rt_render(cam, lights)
    st = torch.cuda.Stream()
    n = 8
    rows = cgdist.shard_rows(H, n)
    g = torch.zeros(n * rows * W, dtype=torch.int32, device="cuda")
    for r in range(n):
        rt.rt_render_device(cam, g.data_ptr() + r * rows * W * 4, cgamd.RtShard(r, n, cgdist.DEFAULT_STRIPE),
                            st.cuda_stream, lights=lights)
    frame = torch.zeros(H * W, dtype=torch.int32, device="cuda")
    rt.rt_unstripe_device(g.data_ptr(), W, H, n, cgdist.DEFAULT_STRIPE, frame.data_ptr(), st.cuda_stream)
    st.synchronize()
    assert np.array_equal(frame.cpu().numpy().view(np.uint32), full)


C5_FULL = dict(width=1920, height=1080, focal=1080.0, cam=[0, 0, -3.0, 1], R=None,
               lights=[[[0.0, -0.5, -0.7, 1.0], [14.0, 14.0, 14.0]]], scene=dict(random=1_000_000, seed=0x5EED))


def test_rt_c5_1m_triangles_sampled(rt):
    """C5 at full size (1920x1080 over 1M random triangles, no sphere): the
    whole GPU frame through the binned path, 768 pixels checked bit-exactly
    against the brute-force oracle (each oracle pixel costs ~18M triangle
    tests); the 256x144 / 2000-triangle C5 frame is checked whole above."""
    cfg = C5_FULL
    W, H = cfg["width"], cfg["height"]
    _set_scene(rt, cfg)
    try:
        argb, st = rt.rt_render(_cam(cfg), _lights(cfg))
        again, _ = rt.rt_render(_cam(cfg), _lights(cfg))
        scratch = rt.rt_scratch_info()
    finally:
        _set_scene(rt, {})
    assert np.array_equal(again, argb)
    xy = _sample_xy(W, H, 768, 5)
    xy[-128:] = np.stack([np.random.default_rng(6).integers(W // 2 - 300, W // 2 + 300, 128),
                          np.random.default_rng(7).integers(H // 2 - 300, H // 2 + 300, 128)], 1)   # in the cloud
    ref = oracle.rt_draw_pixels(mg.rt_params_of(cfg), xy, scene=mg.rt_oracle_scene(cfg),
                                threads=min(16, os.cpu_count() or 8))
    got = argb.reshape(H, W)[xy[:, 1], xy[:, 0]]
    # the pools were sized on this first frame: capacity within 2x of what it listed
    info = scratch
    assert info["capacity"] <= 2 * info["listed"], info
    assert info["bytes"] < (4 << 30), info
    bad = np.flatnonzero(got != ref)
    assert bad.size == 0, f"{bad.size} differ, first at {xy[bad[:4]]}: gpu {got[bad[:4]]} ref {ref[bad[:4]]}"
    assert (got != 0x80000000).sum() > 100      # the sample does see the cloud


@pytest.mark.parametrize("cap", [1, 64])
def test_rt_c5_pending_queue_overflow(rt, golden, cap):
    """Shadow rays past the pending queue take the shading kernel's per-lane
    certified lit search instead of the wave-per-ray one: the C5 golden frame
    (2000 triangles) and a 100k-triangle frame are unchanged."""
    cfg = mg.rt_configs()["rt_c5_256x144_rand2000"]
    big = dict(C5_FULL, width=320, height=180, focal=180.0, scene=dict(random=100_000, seed=0x5EED))
    try:
        _set_scene(rt, big)
        want, _ = rt.rt_render(_cam(big), _lights(big))
        _set_scene(rt, cfg)
        rt.rt_set_pending_cap(cap)
        argb, _ = rt.rt_render(_cam(cfg), _lights(cfg))
        assert mg.sha(argb) == golden["rt"]["rt_c5_256x144_rand2000"]["argb_sha256"]
        _set_scene(rt, big)
        got, _ = rt.rt_render(_cam(big), _lights(big))
        assert np.array_equal(got, want)
    finally:
        rt.rt_set_pending_cap(0)
        _set_scene(rt, {})


def test_rt_c5_sharded_matches_whole(rt):
    """C5's multi-GPU form (32-row stripes over 4 ranks) == the whole frame."""
    torch = pytest.importorskip("torch")
    cfg = dict(C5_FULL, width=480, height=270, focal=270.0, scene=dict(random=100_000, seed=0x5EED))
    W, H = cfg["width"], cfg["height"]
    _set_scene(rt, cfg)
    try:
        cam, lights = _cam(cfg), _lights(cfg)
        full, _ = rt.rt_render(cam, lights)
        st = torch.cuda.Stream()
        n, sh_h = 4, 32
        rows = cgdist.shard_rows(H, n, sh_h)
        g = torch.zeros(n * rows * W, dtype=torch.int32, device="cuda")
        for r in range(n):
            rt.rt_render_device(cam, g.data_ptr() + r * rows * W * 4, cgamd.RtShard(r, n, sh_h),
                                st.cuda_stream, lights=lights)
        frame = torch.zeros(H * W, dtype=torch.int32, device="cuda")
        rt.rt_unstripe_device(g.data_ptr(), W, H, n, sh_h, frame.data_ptr(), st.cuda_stream)
        st.synchronize()
    finally:
        _set_scene(rt, {})
    assert np.array_equal(frame.cpu().numpy().view(np.uint32), full)
    assert (full != 0x80000000).sum() > 1000


def test_rt_empty_scene_is_black(ctx):
    """No triangles, no spheres: every pixel is PutPixelSDL(black) = 0x80000000."""
    ctx.rt_set_scene(None, 0, None, 0)
    argb, _ = ctx.rt_render(cgamd.rt_camera(64, 32, 64.0))
    assert np.all(argb == 0x80000000)
    tris, n, sph = cgamd.rt_scene()
    ctx.rt_set_scene(tris, n, sph, 1)


def test_rt_errors(ctx):
    with pytest.raises(RuntimeError):
        ctx.rt_render(cgamd.rt_camera(0, 10))


_f = lambda x: float(np.float32(x))   # noqa: E731
_W = [14.0, 14.0, 14.0]
# Eye and light poses the golden configs do not reach (the sphere: centre
# (-0.45, 0.6, -0.6), radius 0.3; the short box spans x [-0.05, 0.70],
# y [0.41, 1], z [-0.77, -0.02]): the eye at and off the sphere's centre, the
# light inside the sphere or a box, looking away from the room, the eye behind
# the back wall, the eye and the light on a wall's plane, the light outside.
RT_POSES = {
    "eye_at_sphere_centre": dict(cam=[_f(-0.45), _f(0.6), _f(-0.6), 1]),
    "eye_in_sphere_yawed": dict(cam=[_f(-0.4), _f(0.55), _f(-0.65), 1], yaw=_f(0.5)),
    "light_in_sphere": dict(lights=[[[_f(-0.45), _f(0.6), _f(-0.6), 1.0], _W]]),
    "light_in_short_box_area16": dict(lights=[[[_f(0.33), _f(0.7), _f(-0.4), 1.0], _W]], area=dict(side=0.1, n=4)),
    "eye_in_short_box": dict(cam=[_f(0.33), _f(0.7), _f(-0.4), 1]),
    "looking_back": dict(cam=[0, 0, _f(-0.5), 1], yaw=_f(3.14159)),
    "behind_back_wall": dict(cam=[0, 0, _f(1.5), 1]),
    "eye_on_left_wall": dict(cam=[-1.0, 0, _f(-0.5), 1]),
    "light_on_right_wall": dict(lights=[[[1.0, 0.0, 0.0, 1.0], _W]]),
    "light_outside_front_area16": dict(lights=[[[0.0, _f(-0.5), -2.0, 1.0], _W]], area=dict(side=0.1, n=4)),
}


@pytest.mark.parametrize("pose", list(RT_POSES))
def test_rt_edge_poses_vs_live_oracle(rt, pose):
    """The Cornell-box frame (lattice kernels; per-pixel columns when yawed)
    for each pose against the oracle's whole frame, bit-exact."""
    c = dict(RT_POSES[pose])
    yaw = c.pop("yaw", 0.0)
    cfg = dict(dict(width=96, height=72, focal=72.0, cam=[0, 0, -3.0, 1], lights=[[[0.0, -0.5, -0.7, 1.0], _W]],
                    R=mg.yaw_R(np.float32(0.0) - np.float32(yaw)) if yaw else None), **c)
    argb, _ = rt.rt_render(_cam(cfg), _lights(cfg))
    ref = oracle.rt_draw(mg.rt_params_of(cfg), threads=min(16, os.cpu_count() or 8))
    bad = np.flatnonzero(argb != ref)
    assert bad.size == 0, f"{pose}: {bad.size} differ, first {bad[:6]} gpu {argb[bad[:3]]} ref {ref[bad[:3]]}"


def test_rt_div3_shared_reciprocal_is_ieee(ctx):
    """The light-set sweep's three divides by one area (:412) through one refined reciprocal
    (cg_rt_dev.h div3_by, inside its range guard; IEEE x / d outside) == numpy's IEEE float32
    x / d, bit for bit: 6M quotients over C4's operand ranges (area 4 pi |r|^2 of nearby
    lights, numerators colour x light x cos), log-uniform operands across the whole float range,
    both ends of the guard, zeros of both signs, denormals, infinities and NaN."""
    import torch
    rng = np.random.default_rng(0xD1B3)
    n = 2_000_000

    def logu(k, lo, hi):
        return np.exp2(rng.uniform(lo, hi, k)).astype(np.float32)

    den = np.concatenate([logu(n // 2, -8, 12),                                   # C4-like areas
                          logu(n // 4, -140, 127) * rng.choice([-1, 1], n // 4).astype(np.float32),
                          np.float32(2.0) ** rng.integers(-42, 43, n // 4).astype(np.float32)])
    x = np.concatenate([logu(3 * (n // 2), -30, 6),                               # C4-like numerators
                        logu(3 * (n // 4), -150, 127) * rng.choice([-1, 1], 3 * (n // 4)).astype(np.float32),
                        np.float32(2.0) ** rng.integers(-90, 43, 3 * (n // 4)).astype(np.float32)])
    specials = np.array([0.0, -0.0, 1e-45, -1e-45, 1e-39, np.inf, -np.inf, np.nan, 2.0 ** -86, 2.0 ** -87,
                         2.0 ** 40, 2.0 ** 41, 2.0 ** -40, 2.0 ** -41, 3.4e38], dtype=np.float32)
    k = len(specials)
    den[:k * k] = np.repeat(specials, k)
    x[:3 * k * k] = np.tile(specials, 3 * k)
    with np.errstate(all="ignore"):
        want = x.reshape(-1, 3) / den[:, None]
    dx = torch.from_numpy(x).cuda()
    dd = torch.from_numpy(den).cuda()
    dq = torch.empty_like(dx)
    cgamd.probe_div3_device(dx.data_ptr(), dd.data_ptr(), n, dq.data_ptr())
    torch.cuda.synchronize()
    got = dq.cpu().numpy().reshape(-1, 3)
    same = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
    bad = np.argwhere(~same)
    assert bad.size == 0, f"{len(bad)} quotients differ, first {[(x.reshape(-1, 3)[i, j], den[i], got[i, j], want[i, j]) for i, j in bad[:5]]}"
