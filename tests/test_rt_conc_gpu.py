"""GPU: certificates published beside the lattice launch (cg_internal.h LatReady /
LatPublish, CG_CERT_CONC=1; VERDICT r05 item 1 -- built, measured slower, off by
default, cg_shim.hip cert_concurrent).  A whole-frame batched call starts its
lattice launch beside its certificate launch; each lattice workgroup waits only
for its own super-tile's publication word, or -- past its bound, or forced with
CG_LAT_FORCE_UNCERT=1 -- renders its tile uncertified (every triangle and the
sphere as candidates, the frame's RtTri formed by the workgroup itself).  Every
path must give the reference's image bit for bit: the golden 1080p frame
(SURVEY 8c fingerprint) for every frame of a call, and per-frame renders for
moving and yawed cameras.  The forced uncertified path is the test that the
certificates only ever remove candidates that cannot change a pixel.
Reference: raytracer/Source/skeleton.cpp:104-169."""
import hashlib

import numpy as np
import pytest

import cgamd

pytestmark = pytest.mark.gpu

W, H, F = 1920, 1080, 1080.0


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def c2(ctx):
    tris, n, sph = cgamd.rt_scene()
    ctx.rt_set_scene(tris, n, sph, 1)
    return ctx


def _call(ctx, cams, out=None):
    import torch
    n = len(cams)
    out = torch.zeros(n * W * H, dtype=torch.int32, device="cuda") if out is None else out
    s = torch.cuda.Stream()
    ctx.rt_render_frames_device(cams, out.data_ptr(), None, s.cuda_stream)
    s.synchronize()
    return out.cpu().numpy().view(np.uint32).reshape(-1, W * H)[:n]


@pytest.mark.parametrize("mode", ["published", "uncertified", "serial"])
def test_conc_whole_calls_golden(c2, golden, monkeypatch, mode):
    """Calls of 20, 5, 32 and 20 frames back to back (both certificate slots, rising
    generations): every frame == the golden 1080p fingerprint."""
    monkeypatch.setenv("CG_CERT_CONC", "0" if mode == "serial" else "1")
    if mode == "uncertified":
        monkeypatch.setenv("CG_LAT_FORCE_UNCERT", "1")
    want = golden["rt"]["rt_1920x1080_f1080"]["argb_sha256"]
    cam = cgamd.rt_camera(W, H, F)
    for nf in (20, 5, 32, 20):
        frames = _call(c2, [cam] * nf)
        bad = [k for k in range(nf) if _sha(frames[k]) != want]
        assert not bad, f"{mode}: {nf}-frame call, frames {bad} differ from the golden frame"


@pytest.mark.parametrize("mode", ["published", "uncertified"])
@pytest.mark.parametrize("path", ["dolly", "yaw"])
def test_conc_moving_cameras_equal_single_frames(c2, monkeypatch, mode, path):
    """A 20-frame call whose every frame has its own camera (cameraPos dolly, or a yaw per
    frame as the LEFT key turns it) == each frame rendered alone (cg_rt_render)."""
    monkeypatch.setenv("CG_CERT_CONC", "1")
    if mode == "uncertified":
        monkeypatch.setenv("CG_LAT_FORCE_UNCERT", "1")
    if path == "dolly":
        cams = [cgamd.rt_camera(W, H, F, (0.0, 0.0, float(np.float32(-3.0 + 0.005 * k)), 1.0)) for k in range(20)]
    else:   # one batch needs one R: the yaw is shared, cameraPos moves
        R = cgamd.yaw_matrix(0.1745)
        cams = [cgamd.rt_camera(W, H, F, (0.002 * k, 0.0, -3.0, 1.0), R) for k in range(20)]
    frames = _call(c2, cams)
    monkeypatch.delenv("CG_LAT_FORCE_UNCERT", raising=False)
    monkeypatch.delenv("CG_CERT_CONC", raising=False)
    for k in range(20):
        alone = c2.rt_render(cams[k])[0]
        assert np.array_equal(frames[k], alone), f"{path}/{mode}: frame {k}"
    assert len({_sha(f) for f in frames}) == 20       # the path's frames differ

