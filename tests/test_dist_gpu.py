"""GPU: the library's multi-GPU raytracer (cg_rt_render_frames_dist,
csrc/cg_dist.hip) assembles on rank 0 exactly the frames one GPU renders.

Ranks run in one process through the in-process transport
(cg_dist_create_local: N contexts on cuda:0, bands moved by device copies --
the same band, window, chunk and assembly logic as the RCCL transport), and
the RCCL transport itself with one rank.  Frames are compared bit for bit
with cg_rt_render_frames_device on a single context, itself pinned to the
oracle by tests/test_rt_gpu.py."""
import numpy as np
import pytest
import torch

import cgamd

pytestmark = pytest.mark.gpu


def _ctxs(n, scene=None):
    out = []
    for _ in range(n):
        c = cgamd.Context(0)
        tris, nt, sph = scene or cgamd.rt_scene()
        c.rt_set_scene(tris, nt, sph, 1 if sph is not None else 0)
        out.append(c)
    return out


def _single(ctx, cams, lights):
    W, H = cams[0].width, cams[0].height
    buf = torch.zeros(len(cams) * W * H, dtype=torch.int32, device="cuda")
    ctx.rt_render_frames_device(cams, buf.data_ptr(), lights=lights, frame_stride=W * H)
    torch.cuda.synchronize()
    return buf.cpu().numpy().view(np.uint32).reshape(len(cams), H * W)


def _dist_render(ds, cams, lights):
    W, H = cams[0].width, cams[0].height
    frames = torch.zeros(len(cams) * W * H, dtype=torch.int32, device="cuda")
    for d in reversed(ds):                 # ranks > 0 enqueue first (local transport)
        d.render_frames(cams, frames.data_ptr() if d.rank == 0 else None, lights=lights)
    torch.cuda.synchronize()
    return frames.cpu().numpy().view(np.uint32).reshape(len(cams), H * W)


def _cams(W, H, f, n, R=None):
    # the camera moves from frame to frame (the reference's Update(), skeleton.cpp:195-252)
    return [cgamd.rt_camera(W, H, f, (0.01 * k, -0.005 * k, -3.0 + 0.02 * k, 1.0), R) for k in range(n)]


@pytest.mark.parametrize("pipeline", [cgamd.DIST_SIGNALLED, cgamd.DIST_CHUNKED])
@pytest.mark.parametrize("nranks,chunk", [(2, 4), (3, 1), (8, 3)])
def test_dist_local_matches_single_gpu(nranks, chunk, pipeline):
    W, H = 320, 256
    cams = _cams(W, H, 256.0, 7)
    lights = cgamd.default_lights()
    ctxs = _ctxs(nranks)
    ds = cgamd.Dist.local(ctxs)
    try:
        for d in ds:
            d.set_chunk(chunk)
            d.set_pipeline(pipeline)
        want = _single(ctxs[0], cams, lights)
        got = _dist_render(ds, cams, lights)
        assert np.array_equal(got, want)
        bands = ds[0].bands()
        assert bands[0][0] == 0 and sum(n for _, n in bands) == H
        # uneven bands (one rank empty) and a rebalance from the measured times
        if nranks >= 3:
            rows = [(H - 100) * (r + 1) // (nranks - 2) - (H - 100) * r // (nranks - 2) for r in range(nranks - 2)]
            b = [(0, 100), (100, 0)] + [(100 + (H - 100) * r // (nranks - 2), rows[r]) for r in range(nranks - 2)]
            for d in ds:
                d.set_bands(H, b)
            assert np.array_equal(_dist_render(ds, cams, lights), want)
        ds[0].rebalance()
        nb = ds[0].bands()
        assert all(d.bands() == nb for d in ds) and sum(n for _, n in nb) == H
        assert np.array_equal(_dist_render(ds, cams, lights), want)
        r, a = ds[0].last_times()
        assert r > 0 and (a > 0 or nranks == 1)
    finally:
        for d in ds:
            d.close()
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("pipeline", [cgamd.DIST_SIGNALLED, cgamd.DIST_CHUNKED])
def test_dist_local_back_to_back_calls(pipeline):
    """Several calls on the same streams with no synchronisation in between,
    each with its own cameras and output buffer (a call's slot
    counters are reused two calls later; a wait that passed on the stale
    counts would ship a half-written band).  Every call's frames must equal
    the single-GPU render of its cameras."""
    W, H, calls, nf = 320, 256, 5, 6
    lights = cgamd.default_lights()
    ctxs = _ctxs(3)
    ds = cgamd.Dist.local(ctxs)
    try:
        for d in ds:
            d.set_chunk(2)
            d.set_pipeline(pipeline)
        cams = [[cgamd.rt_camera(W, H, 256.0, (0.03 * (c - 2) + 0.002 * k, 0.01 * c, -3.0 + 0.05 * c + 0.01 * k, 1.0))
                 for k in range(nf)] for c in range(calls)]
        outs = [torch.zeros(nf * W * H, dtype=torch.int32, device="cuda") for _ in range(calls)]
        for c in range(calls):
            for d in reversed(ds):
                d.render_frames(cams[c], outs[c].data_ptr() if d.rank == 0 else None, lights=lights)
        torch.cuda.synchronize()
        for c in range(calls):
            want = _single(ctxs[0], cams[c], lights)
            got = outs[c].cpu().numpy().view(np.uint32).reshape(nf, H * W)
            assert np.array_equal(got, want), f"call {c}"
    finally:
        for d in ds:
            d.close()
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("kind", ["c4", "yaw", "big"])
def test_dist_local_light_set_and_rotated_camera(kind):
    """The light-set lattice kernel (C4's 8x8 area light), the general kernel
    (yawed camera: full-width rows, pack pass) and the large-scene pipeline
    (C5's random scene, here 20k triangles) through the bands."""
    W, H = 240, 120   # whole frames: a multiple of the 8-row tile (no padding rows)
    scene = None
    if kind == "c4":
        cams, lights = _cams(W, H, 135.0, 3), cgamd.area_lights(None, 0.1, 8)
    elif kind == "big":
        n = 20000
        scene = (cgamd.random_scene(n, 0x5EED), n, None)
        cams, lights = _cams(W, H, 135.0, 3), cgamd.default_lights()
    else:
        cams, lights = _cams(W, H, 135.0, 3, cgamd.yaw_matrix(0.1745)), cgamd.default_lights()
    ctxs = _ctxs(4, scene)
    ds = cgamd.Dist.local(ctxs)
    try:
        want = _single(ctxs[0], cams, lights)
        assert np.array_equal(_dist_render(ds, cams, lights), want)
    finally:
        for d in ds:
            d.close()
        for c in ctxs:
            c.close()


def test_dist_rccl_one_rank():
    """The RCCL transport with one rank: own id, communicator, frames."""
    W, H = 320, 256
    cams = _cams(W, H, 256.0, 5)
    (ctx,) = _ctxs(1)
    d = cgamd.Dist(ctx, 1, 0, cgamd.dist_unique_id())
    try:
        want = _single(ctx, cams, cgamd.default_lights())
        got = _dist_render([d], cams, cgamd.default_lights())
        assert np.array_equal(got, want)
        d.rebalance()
    finally:
        d.close()
        ctx.close()


def test_dist_errors():
    ctxs = _ctxs(2)
    ds = cgamd.Dist.local(ctxs)
    try:
        with pytest.raises(RuntimeError):
            ds[0].set_bands(100, [(0, 60), (50, 50)])      # overlapping
        with pytest.raises(RuntimeError):
            ds[0].set_chunk(0)
        with pytest.raises(RuntimeError):
            ds[0].set_pipeline(7)
        with pytest.raises(RuntimeError):                  # rank 0 before its peer (local transport)
            ds[0].render_frames(_cams(64, 48, 48.0, 2), torch.zeros(2 * 64 * 48, dtype=torch.int32,
                                                                    device="cuda").data_ptr())
    finally:
        for d in ds:
            d.close()
        for c in ctxs:
            c.close()


_MISSING_PEER = r"""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.environ["CG_ROOT"], "computer-graphics_amd"))
import cgamd
ctx = cgamd.Context(0)
uid = cgamd.dist_unique_id()
t0 = time.monotonic()
res = {}
try:
    cgamd.Dist(ctx, 2, 0, uid, timeout_ms=int(os.environ["CG_T_MS"]))
    res["raised"] = None
except cgamd.DistTimeout as e:
    res["raised"], res["msg"] = "timeout", str(e)
except RuntimeError as e:
    res["raised"], res["msg"] = "other", str(e)
res["elapsed"] = time.monotonic() - t0
# the context itself stays usable after the aborted communicator
tris, n, sph = cgamd.rt_scene()
ctx.rt_set_scene(tris, n, sph, 1)
argb, _ = ctx.rt_render(cgamd.rt_camera(64, 48, 48.0))
res["frame_ok"] = bool(argb.any())
print("RESULT " + json.dumps(res), flush=True)
ctx.close()
"""


def test_dist_rccl_missing_peer_fails_within_deadline():
    """rank 0 of a world of two calls cg_dist_create alone (its peer
    never joins).  The non-blocking init is polled against the deadline; past it the
    communicator is aborted and the call returns CG_E_TIMEOUT (cgamd.DistTimeout) instead
    of blocking the job forever.  Run in a child process under its own time limit, so a
    regression fails this test rather than hanging the suite."""
    import json
    import os
    import subprocess
    import sys
    t_ms = 3000
    env = dict(os.environ, CG_ROOT=os.path.dirname(os.path.dirname(os.path.abspath(__file__))), CG_T_MS=str(t_ms))
    r = subprocess.run([sys.executable, "-c", _MISSING_PEER], capture_output=True, text=True, timeout=100, env=env)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
    assert r.returncode == 0 and lines, f"rc {r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-3000:]}"
    res = json.loads(lines[-1][7:])
    assert res["raised"] == "timeout", res
    # the deadline, plus at most the 10 s the library gives ncclCommAbort
    assert t_ms / 1e3 * 0.9 <= res["elapsed"] <= t_ms / 1e3 + 12.0, res
    assert res["frame_ok"], res


def test_dist_rccl_one_rank_bounded_waits():
    """The bounded host waits on a healthy communicator: cg_dist_wait, a short deadline,
    rebalance and last_times all succeed, and the frames are the single-GPU render."""
    W, H = 320, 256
    cams = _cams(W, H, 256.0, 4)
    (ctx,) = _ctxs(1)
    d = cgamd.Dist(ctx, 1, 0, cgamd.dist_unique_id(), timeout_ms=20000)
    try:
        d.set_timeout(5000)
        want = _single(ctx, cams, cgamd.default_lights())
        frames = torch.zeros(len(cams) * W * H, dtype=torch.int32, device="cuda")
        for _ in range(3):
            d.render_frames(cams, frames.data_ptr(), lights=cgamd.default_lights())
        d.wait()
        got = frames.cpu().numpy().view(np.uint32).reshape(len(cams), H * W)
        assert np.array_equal(got, want)
        d.rebalance()
        r, _ = d.last_times()
        assert r > 0
        with pytest.raises(RuntimeError):
            d.set_timeout(0)
    finally:
        d.close()
        ctx.close()
