"""GPU: the live kernel timing the bench's rooflines read (cg_kernel_timing / cg_kernel_time,
csrc/cg_ktime.hip): while timing is on, each launch of a timed kernel carries one start / stop
event pair on its own dispatch; the totals count every launch once, a kernel's busy time never
exceeds its summed time, switching timing on resets the totals, and while it is off nothing is
recorded."""
import pytest

import cgamd

pytestmark = pytest.mark.gpu


def _times(*names):
    return {k: cgamd.kernel_time(k) for k in names}


def test_kernel_time_counts_each_timed_launch(ctx, monkeypatch):
    torch = pytest.importorskip("torch")
    tris, n, sph = cgamd.rt_scene()
    ctx.rt_set_scene(tris, n, sph, 1)
    W, H, calls = 640, 360, 3
    cams = [cgamd.rt_camera(W, H, 360.0, (0.0, 0.0, -3.0 + 0.01 * k, 1.0)) for k in range(5)]
    g = torch.zeros(len(cams) * W * H, dtype=torch.int32, device="cuda")
    st = torch.cuda.Stream()
    ctx.rt_render_frames_device(cams, g.data_ptr(), None, st.cuda_stream)      # warm, untimed
    st.synchronize()
    ref = g.clone()
    monkeypatch.setenv("CG_KTIME_ALL", "1")        # the certificate launches timed too
    cgamd.kernel_timing(True)
    try:
        for _ in range(calls):
            ctx.rt_render_frames_device(cams, g.data_ptr(), None, st.cuda_stream)
        st.synchronize()
        t = _times("rt_lattice_kernel", "rt_tile_cert_kernel", "rt_prepare_kernel", "rast_fill_kernel")
        cgamd.kernel_timing(True)                  # a new session starts from zero
        assert cgamd.kernel_time("rt_lattice_kernel") == (0.0, 0.0, 0)
    finally:
        cgamd.kernel_timing(False)
    assert torch.equal(g, ref)                     # timing changes nothing in the frames
    tot, busy, nl = t["rt_lattice_kernel"]
    assert nl == calls and tot > 0 and 0 < busy <= tot * (1 + 1e-9)
    cert_launches = t["rt_tile_cert_kernel"][2] + t["rt_prepare_kernel"][2]
    assert calls <= cert_launches <= 2 * calls     # fused certificates: one launch per call, split: two
    assert t["rast_fill_kernel"] == (0.0, 0.0, 0)  # kernels that did not run record nothing
    # by default only the kernels a roofline reads are timed: the certificate launches ride plain
    monkeypatch.delenv("CG_KTIME_ALL")
    cgamd.kernel_timing(True)
    try:
        ctx.rt_render_frames_device(cams, g.data_ptr(), None, st.cuda_stream)
        st.synchronize()
        t2 = _times("rt_lattice_kernel", "rt_tile_cert_kernel", "rt_prepare_kernel")
    finally:
        cgamd.kernel_timing(False)
    assert t2["rt_lattice_kernel"][2] == 1 and t2["rt_tile_cert_kernel"][2] == 0 and t2["rt_prepare_kernel"][2] == 0
    # off: nothing is recorded
    ctx.rt_render_frames_device(cams, g.data_ptr(), None, st.cuda_stream)
    st.synchronize()
    assert cgamd.kernel_time("rt_lattice_kernel")[2] == 0
    with pytest.raises(ValueError):
        cgamd.kernel_time("no_such_kernel")


def test_kernel_time_rasteriser_and_large_scene(ctx):
    torch = pytest.importorskip("torch")
    W, H = 320, 240
    d = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    ctx.rast_set_scene()
    p = cgamd.rast_params(W, H, 240.0)
    ctx.rast_draw_device(p, d.data_ptr())
    torch.cuda.synchronize()
    cgamd.kernel_timing(True)
    try:
        for _ in range(2):
            ctx.rast_draw_device(p, d.data_ptr())
        torch.cuda.synchronize()
        r = _times("rast_fill_kernel", "rast_post_kernel")
    finally:
        cgamd.kernel_timing(False)
    for k in ("rast_fill_kernel", "rast_post_kernel"):
        tot, busy, nl = r[k]
        assert nl == 2 and 0 < busy <= tot * (1 + 1e-9), k
    # a large scene (more than 64 triangles): the walk, its hints and the whole frame, per frame
    ntri = 20000
    ctx.rt_set_scene(cgamd.random_scene(ntri, 0x5EED), ntri, None, 0)
    try:
        cams = [cgamd.rt_camera(W, H, 240.0, (0.0, 0.0, -3.0, 1.0))] * 2
        g = torch.zeros(len(cams) * W * H, dtype=torch.int32, device="cuda")
        ctx.rt_render_frames_device(cams, g.data_ptr())
        torch.cuda.synchronize()
        cgamd.kernel_timing(True)
        try:
            ctx.rt_render_frames_device(cams, g.data_ptr())
            torch.cuda.synchronize()
            b = _times("rt_big_primary_kernel", "rt_big_frame")
        finally:
            cgamd.kernel_timing(False)
    finally:
        tris, n, sph = cgamd.rt_scene()
        ctx.rt_set_scene(tris, n, sph, 1)
    assert b["rt_big_primary_kernel"][2] == len(cams) and b["rt_big_primary_kernel"][0] > 0
    assert b["rt_big_frame"][2] == len(cams)
    assert b["rt_big_frame"][0] >= b["rt_big_primary_kernel"][0]   # the frame contains its walk
