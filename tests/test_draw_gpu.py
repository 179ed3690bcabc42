"""GPU: the host-buffer boundary -- cg_rt_render_frames (frames delivered into HOST
memory, the reference's Draw(screen*) loop, raytracer/Source/skeleton.cpp:91-94,
104-169) equals cg_rt_render frame by frame, which tests/test_rt_gpu.py pins to the
oracle.  ADVICE r04: pageable and pinned output, a frame stride larger than W*H (the
gaps untouched), a frame count that is not a multiple of the chunk, the large-scene
(multi-slot) path, and an error return that leaves no copy running."""
import numpy as np
import pytest
import torch

import cgamd

pytestmark = pytest.mark.gpu


def _cams(W, H, f, n):
    return [cgamd.rt_camera(W, H, f, (0.01 * k, -0.004 * k, -3.0 + 0.015 * k, 1.0)) for k in range(n)]


def _per_frame(ctx, cams, lights):
    return np.stack([ctx.rt_render(c, lights)[0] for c in cams])


def _host(n, pinned):
    if pinned:
        t = torch.full((n,), 0x5A5A5A5A, dtype=torch.int32, pin_memory=True)
        return t, t.numpy().view(np.uint32)
    a = np.full(n, 0x5A5A5A5A, np.uint32)
    return a, a


@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("scene", ["cornell", "big"])
@pytest.mark.parametrize("n,chunk,pad", [(7, 3, 0), (5, 8, 37), (9, 2, 320)])
def test_render_frames_host_matches_per_frame(ctx, pinned, scene, n, chunk, pad):
    W, H = (320, 256) if scene == "cornell" else (200, 120)
    if scene == "big":
        nt = 20000
        ctx.rt_set_scene(cgamd.random_scene(nt, 0x5EED), nt, None, 0)
    else:
        tris, nt, sph = cgamd.rt_scene()
        ctx.rt_set_scene(tris, nt, sph, 1)
    cams = _cams(W, H, float(H), n)
    lights = cgamd.default_lights()
    want = _per_frame(ctx, cams, lights)
    stride = W * H + pad
    out, view = _host(n * stride, pinned)
    ctx.rt_render_frames(cams, out, chunk=chunk, lights=lights, frame_stride=stride)
    got = view.reshape(n, stride)
    assert np.array_equal(got[:, :W * H], want)
    assert (got[:, W * H:] == 0x5A5A5A5A).all(), "bytes between frames written"
    # back to back on the same context (slots and copy stream reused)
    out2, view2 = _host(n * stride, pinned)
    ctx.rt_render_frames(cams[::-1], out2, chunk=chunk, lights=lights, frame_stride=stride)
    assert np.array_equal(view2.reshape(n, stride)[:, :W * H], want[::-1])


def test_render_frames_host_error_returns_cleanly(ctx):
    """A call with a camera of another size in a later chunk is refused (CG_E_INVALID,
    before anything is enqueued: the slots hold W x H frames); the next call on the
    context still delivers exact frames."""
    tris, nt, sph = cgamd.rt_scene()
    ctx.rt_set_scene(tris, nt, sph, 1)
    W, H = 160, 128
    cams = _cams(W, H, 128.0, 6)
    bad = list(cams)
    bad[4] = cgamd.rt_camera(W + 16, H, 128.0)
    with pytest.raises(RuntimeError):
        ctx.rt_render_frames(bad, np.zeros(6 * W * H, np.uint32), chunk=2)
    want = _per_frame(ctx, cams, cgamd.default_lights())
    out, _ = ctx.rt_render_frames(cams, None, chunk=2)
    assert np.array_equal(out.reshape(6, W * H), want)


def test_render_host_window_columns_exact(ctx):
    """Only the columns the camera can see anything in cross PCIe (cg_rt_frame_columns); the
    host stores the rest as PutPixelSDL(0, 0, 0).  Cameras moving sideways (windows at either
    edge, none at all), a yawed camera (whole rows) and a light set: cg_rt_render and
    cg_rt_render_frames (pageable and pinned) == the device-resident frame, every pixel."""
    W, H = 320, 256
    tris, nt, sph = cgamd.rt_scene()
    ctx.rt_set_scene(tris, nt, sph, 1)
    xs = [-40.0, -1.6, -0.7, 0.0, 0.35, 1.1, 2.4, 40.0]
    cams = [cgamd.rt_camera(W, H, 256.0, (x, 0.1 * k - 0.3, -3.0, 1.0)) for k, x in enumerate(xs)]
    cams.append(cgamd.rt_camera(W, H, 256.0, (0.0, 0.0, -3.0, 1.0), cgamd.yaw_matrix(0.3)))
    cols = [cgamd.frame_columns(tris, nt, sph, 1, c) for c in cams]
    assert any(0 < c0 < c1 < W for c0, c1 in cols) and cols[0][0] >= cols[0][1]
    for lights in (cgamd.default_lights(), cgamd.area_lights(cgamd.default_lights()[0], 0.1, 2)):
        want = []
        for c in cams:
            d = torch.zeros(W * H, dtype=torch.int32, device="cuda")
            ctx.rt_render_frames_device([c], d.data_ptr(), lights=lights)
            torch.cuda.synchronize()
            want.append(d.cpu().numpy().view(np.uint32).copy())
        for k, c in enumerate(cams):
            got, _ = ctx.rt_render(c, lights)
            assert np.array_equal(got, want[k]), ("cg_rt_render", k)
        for pinned in (False, True):
            out, view = _host(len(cams) * W * H, pinned)
            ctx.rt_render_frames(cams, out, chunk=3, lights=lights)
            assert np.array_equal(view.reshape(len(cams), -1), np.stack(want)), ("frames", pinned)
