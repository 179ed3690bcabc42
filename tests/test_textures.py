"""CPU: the texture-mode host pieces -- the opacity maps (OpenCV 3.4 BGR2GRAY +
threshold, skeleton.cpp:149-155) of the product's host entry against the
oracle and the fixed-point formula, and the oracle's glm::inverse against a
float64 inverse."""
import math

import numpy as np

import cgamd
import oracle


def test_opacity_map_matches_oracle_and_formula():
    rng = np.random.default_rng(5)
    bgr = rng.integers(0, 256, (4096, 3), dtype=np.uint8)
    bgr[:256] = np.arange(256, dtype=np.uint8)[:, None]          # every gray level
    got = cgamd.opacity_map(bgr)
    assert np.array_equal(got, oracle.opacity_map(bgr))
    b, g, r = (bgr[:, k].astype(np.int64) for k in range(3))
    y = (b * 1868 + g * 9617 + r * 4899 + (1 << 13)) >> 14
    assert np.array_equal(got, np.where(y > 100, 255, 0).astype(np.uint8))
    assert got[100] == 0 and got[101] == 255                      # threshold is strict


def test_glm_inverse_restatement():
    for yaw in (0.174533, -0.523599, 1.2):
        R = np.array(list(cgamd.yaw_matrix(yaw)), np.float32)
        inv = oracle.mat4_inverse(R).reshape(4, 4).T                # column-major -> rows
        M = R.reshape(4, 4).T
        assert np.abs(inv.astype(np.float64) @ M.astype(np.float64) - np.eye(4)).max() < 1e-6
    assert np.array_equal(oracle.mat4_inverse(np.eye(4, dtype=np.float32).reshape(16)),
                          np.eye(4, dtype=np.float32).reshape(16))


def test_textured_oracle_frames_are_deterministic_and_differ():
    rng = np.random.default_rng(1)
    maps = {k: rng.integers(0, 256, (1024, 1024, 3), dtype=np.uint8)
            for k in oracle.TEXTURE_MAPS if k != "marble"}
    oracle.rast_set_textures(maps)
    try:
        base = oracle.rast_draw(oracle.rast_params(96, 72, 72.0))[0]
        a = oracle.rast_draw(oracle.rast_params(96, 72, 72.0, setting=3))[0]
        b = oracle.rast_draw(oracle.rast_params(96, 72, 72.0, setting=3))[0]
        assert np.array_equal(a, b) and (a != base).mean() > 0.2
        assert math.isfinite(float(a.mean()))
    finally:
        oracle.rast_set_textures(None)
