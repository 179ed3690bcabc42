"""CPU: the build-defined workloads of SURVEY.md 8d (C4 area light, C5 random
scene).  The library's host helpers (cg_rt_area_lights, cg_rt_random_scene,
no device work) must produce the same bytes as the oracle's independent
restatement of their definition (include/cg_render.h)."""
import ctypes as C

import numpy as np

import cgamd
import oracle


def test_area_lights_match_oracle():
    for side, n in ((0.1, 8), (0.25, 3), (0.0, 1)):
        got = cgamd.area_lights(None, side, n)
        want = oracle.rt_area_lights((0.0, -0.5, -0.7, 1.0), (14.0, 14.0, 14.0), side, n)
        assert len(got) == len(want) == n * n
        for g, (p, c) in zip(got, want):
            assert (g.position.x, g.position.y, g.position.z, g.position.w) == p
            assert (g.colour.x, g.colour.y, g.colour.z) == c
    # 8x8: colour share 14/64 is exact, positions symmetric about the centre
    L = cgamd.area_lights(None, 0.1, 8)
    xs = sorted({l.position.x for l in L})
    assert len(xs) == 8 and xs[0] == -xs[-1] and all(l.colour.x == 14.0 / 64 for l in L)


def test_random_scene_matches_oracle():
    n = 50000
    got = cgamd.random_scene(n, 0x5EED)
    want = oracle.rt_random_scene(0x5EED, n)
    assert bytes(got) == bytes(want)
    a = np.frombuffer(bytes(got), np.float32).reshape(n, 19)
    v = a[:, :12].reshape(n, 3, 4)
    assert np.all(v[:, :, 3] == 1.0) and np.all(np.abs(v[:, :, :3]) <= 1.02)
    assert np.all((a[:, 16:19] >= 0.15) & (a[:, 16:19] <= 0.75))
    assert np.all(a[:, 15] == 1.0)   # normal.w
    assert bytes(cgamd.random_scene(16, 1)) != bytes(cgamd.random_scene(16, 2))


def test_random_scene_rejects_bad_args():
    lib = cgamd.load()
    assert lib.cg_rt_random_scene(1, -1, None) < 0
    assert lib.cg_rt_area_lights(None, 0.1, 8, None, 0) < 0
    out = (cgamd.Light * 4)()
    assert lib.cg_rt_area_lights(C.byref(cgamd.default_lights()[0]), 0.1, 8, out, 4) < 0


def test_glibc_rand_restatement_matches_libc():
    """cg_glibc_rand (jump-ahead restatement used by colour modes 1-2) against
    the C library's own rand(), the reference's RNG, at several offsets."""
    for off in (0, 1, 30, 31, 344, 10_007, 1_234_567):
        assert np.array_equal(cgamd.glibc_rand(off, 200), oracle.glibc_rand(off, 200)), off


def test_starfield_init_and_update_match_oracle():
    """starfield/Source/skeleton.cpp:41-46 (glibc rand, double intermediates) and
    Update :93-100 (z drift in double), library vs oracle, bytes."""
    a, b = cgamd.starfield_init(1000), oracle.starfield_init(1000)
    assert a.tobytes() == b.tobytes()
    for dt in (0.0, 16.0, 33.0, 1000.0, 2500.0):
        cgamd.starfield_update(a, dt)
        oracle.starfield_update(b, dt)
        assert a.tobytes() == b.tobytes(), dt


def test_frame_columns_only_black_outside():
    """cg_rt_frame_columns (host-only): every pixel outside the returned columns
    of the oracle's frame is PutPixelSDL(0,0,0) = 0x80000000 -- the contract the
    multi-GPU RGB24 window relies on -- at several cameras, focal lengths and a
    random scene; rotated cameras get the whole width."""
    import os
    tris, n, sph = cgamd.rt_scene()
    threads = min(8, os.cpu_count() or 1)
    cases = [(320, 256, 256.0, (0.0, 0.0, -3.0, 1.0)), (480, 270, 270.0, (0.0, 0.0, -3.0, 1.0)),
             (320, 256, 400.0, (0.2, -0.1, -2.5, 1.0)), (256, 144, 144.0, (0.0, 0.0, -3.0, 1.0))]
    for W, H, f, c in cases:
        c0, c1 = cgamd.frame_columns(tris, n, sph, 1, cgamd.rt_camera(W, H, f, c))
        assert 0 <= c0 < c1 <= W and c0 % 16 == 0 and (c1 % 16 == 0 or c1 == W)
        frame = oracle.rt_draw(oracle.rt_params(W, H, f, c), threads=threads).reshape(H, W)
        outside = np.concatenate([frame[:, :c0].ravel(), frame[:, c1:].ravel()])
        assert np.all(outside == 0x80000000), (W, H, f, c)
        assert c0 > 0 or c1 < W or f >= 400.0      # it does crop the default framings
    rs = cgamd.random_scene(2000, 0x5EED)
    c0, c1 = cgamd.frame_columns(rs, 2000, None, 0, cgamd.rt_camera(256, 144, 144.0))
    ors = oracle.rt_random_scene(0x5EED, 2000)
    frame = oracle.rt_draw(oracle.rt_params(256, 144, 144.0), scene=(ors, 2000, None, 0), threads=threads)
    frame = frame.reshape(144, 256)
    assert np.all(frame[:, :c0] == 0x80000000) and np.all(frame[:, c1:] == 0x80000000)
    assert cgamd.frame_columns(tris, n, sph, 1, cgamd.rt_camera(320, 256, 256.0, R=cgamd.yaw_matrix(0.1))) == (0, 320)
    # camera inside the box: no crop
    assert cgamd.frame_columns(tris, n, sph, 1, cgamd.rt_camera(320, 256, 256.0, (0.0, 0.0, 0.0, 1.0))) == (0, 320)
