"""CPU: the oracle (test infrastructure) against the reference's own goldens.

Pins: raytracer/screenshot.bmp bit-exact, SURVEY.md 8c fingerprints of the
reference build, the ComputePolygonRows KAT (rasteriser skeleton.cpp:183-199)
and the work counters of SURVEY.md 8d.
"""
import ctypes as C

import numpy as np
import pytest

import make_golden as mg
import oracle


def test_rt_screenshot_bit_exact():
    """raytracer/screenshot.bmp == restatement at cameraPos.z = -3 + 0.1 (one UP key)."""
    p = oracle.rt_params(320, 256, 256.0, (0.0, 0.0, mg.CAM_UP, 1.0))
    argb = oracle.rt_draw(p)
    shot = mg.screenshot_argb()
    assert shot.shape == argb.shape
    assert int((shot != argb).sum()) == 0


def test_rt_default_fingerprint_and_counters():
    p = oracle.rt_params(320, 256)
    argb, cnt = oracle.rt_draw(p, counters=True)
    assert mg.sha(argb).startswith(mg.REFERENCE_FINGERPRINTS["rt_320x256_z-3"]["argb"])
    # SURVEY.md 8d, C1 default
    assert (cnt.n_ray, cnt.n_t, cnt.n_uv, cnt.n_dl) == (1327103, 37158884, 18950531, 589823)


def test_rt_golden_hashes_small(golden):
    for name, e in golden["rt"].items():
        cfg = e["config"]
        if cfg["width"] * cfg["height"] > 320 * 256:
            continue
        argb = oracle.rt_draw(mg.rt_params_of(cfg), scene=mg.rt_oracle_scene(cfg), threads=8)
        assert mg.sha(argb) == e["argb_sha256"], name


def test_rt_multithreaded_equals_serial():
    p = oracle.rt_params(160, 128, 128.0)
    a = oracle.rt_draw(p)
    b = oracle.rt_draw(p, threads=4)
    assert np.array_equal(a, b)


def test_polygon_rows_kat(golden):
    lib = oracle.load()
    vp = (oracle.Pixel * 3)()
    for i, (x, y) in enumerate(golden["kat_polygon_rows"]["vertices"]):
        vp[i].x, vp[i].y = x, y
    L, R = (oracle.Pixel * 64)(), (oracle.Pixel * 64)()
    rows = lib.cgo_rast_polygon_rows(vp, L, R, 64)
    assert [[L[i].x, R[i].x] for i in range(rows)] == golden["kat_polygon_rows"]["rows"]
    assert [L[i].y for i in range(rows)] == list(range(5, 16))


@pytest.mark.parametrize("name", ["rast_900x720", "rast_1920x1080_f768"])
def test_rast_reference_fingerprints(name):
    cfg = mg.rast_configs()[name]
    argb, depth, shadow, cnt = oracle.rast_draw(mg.rast_params_of(cfg), counters=True)
    ref = mg.REFERENCE_FINGERPRINTS[name]
    assert mg.sha(argb).startswith(ref["argb"])
    assert mg.sha(depth).startswith(ref["depth"])
    assert mg.sha(shadow).startswith(ref["shadow"])
    assert cnt.n_tris == 303
    if name == "rast_1920x1080_f768":   # SURVEY.md 8a/8d counts
        assert (cnt.n_spans, cnt.n_shaded, cnt.n_shadow) == (112168, 692207, 3883089)


def test_rast_golden_hashes(golden):
    for name, e in golden["rast"].items():
        argb, depth, shadow = oracle.rast_draw(mg.rast_params_of(e["config"]))
        assert mg.sha(argb) == e["argb_sha256"], name
        assert mg.sha(depth) == e["depth_sha256"], name
        assert mg.sha(shadow) == e["shadow_sha256"], name


def test_rast_border_and_alpha():
    """Border pixels are never written (0x00000000); interior alpha is 128."""
    argb, _, _ = oracle.rast_draw(oracle.rast_params(320, 240, 180.0))
    img = argb.reshape(240, 320)
    assert not img[0].any() and not img[-1].any() and not img[:, 0].any() and not img[:, -1].any()
    assert np.all((img[1:-1, 1:-1] >> 24) == 128)


def test_solve_quadratic_cases():
    lib = oracle.load()
    x0, x1 = C.c_float(), C.c_float()
    assert lib.cgo_sphere_solve_quadratic(1.0, 0.0, 1.0, C.byref(x0), C.byref(x1)) == 0   # disc < 0
    assert lib.cgo_sphere_solve_quadratic(1.0, -2.0, 1.0, C.byref(x0), C.byref(x1)) == 1  # disc == 0
    assert x0.value == x1.value == 1.0
    assert lib.cgo_sphere_solve_quadratic(1.0, -3.0, 2.0, C.byref(x0), C.byref(x1)) == 1
    assert (x0.value, x1.value) == (1.0, 2.0)


def test_put_pixel_packing():
    lib = oracle.load()
    assert lib.cgo_put_pixel(oracle.V3(0, 0, 0)) == 0x80000000
    assert lib.cgo_put_pixel(oracle.V3(1, 1, 1)) == 0x80FFFFFF
    assert lib.cgo_put_pixel(oracle.V3(-1, 2, 0.5)) == 0x8000FF7F
