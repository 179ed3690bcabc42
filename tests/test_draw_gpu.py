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
