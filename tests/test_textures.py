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


def _crafted_jpeg(segs):
    """SOI, the (marker, payload) segments, 64 entropy bytes after SOS, EOI."""
    j = bytearray(b"\xff\xd8")
    for m, pay in segs:
        j += bytes([0xFF, m, (len(pay) + 2) >> 8, (len(pay) + 2) & 0xFF]) + bytes(pay)
        if m == 0xDA:
            j += bytes(0x5A ^ k for k in range(64))
    return bytes(j + b"\xff\xd9")


def test_huffman_table_with_all_ones_code_is_rejected():
    """libjpeg 9 jdhuff.c jpeg_make_d_derived_tbl rejects a table whose codes of
    length l reach 2^l -- no code word may be all ones (JERR_BAD_HUFF_TABLE).
    Two 1-bit codes use '1': the product's parser and the oracle both refuse it;
    one 1-bit code is fine."""
    sof1 = [8, 0, 16, 0, 16, 1, 1, 0x11, 0]
    dqt = [0] + [1] * 64
    dht_dc = [0x00, 1] + [0] * 15 + [0]
    dht_ac = [0x10, 1] + [0] * 15 + [0]
    dht_all_ones = [0x10, 2] + [0] * 15 + [0, 1]
    sos1 = [1, 1, 0x00, 0, 63, 0]
    good = _crafted_jpeg([(0xDB, dqt), (0xC0, sof1), (0xC4, dht_dc), (0xC4, dht_ac), (0xDA, sos1)])
    bad = _crafted_jpeg([(0xDB, dqt), (0xC0, sof1), (0xC4, dht_dc), (0xC4, dht_all_ones), (0xDA, sos1)])
    lib = cgamd.load()
    gb, bb = np.frombuffer(good, np.uint8), np.frombuffer(bad, np.uint8)
    assert lib.cg_image_jpeg_check(gb.ctypes.data, gb.size) == 0
    assert lib.cg_image_jpeg_check(bb.ctypes.data, bb.size) == cgamd.CG_E_INVALID
    oracle.jpeg_decode(good)
    try:
        oracle.jpeg_decode(bad)
    except ValueError:
        pass
    else:
        raise AssertionError("the oracle accepted a Huffman table with an all-ones code")
