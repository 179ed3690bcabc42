"""CPU: the product C-ABI library loads, exports every symbol include/cg_render.h
declares, and its host-side code (scene loaders, RAST host geometry) matches
the oracle bit for bit.  No compute call needs a GPU here."""
import ctypes as C
import os
import re

import numpy as np

import cgamd
import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "cg_render.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(cg_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_header_symbols():
    lib = cgamd.load()
    syms = header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), s
    assert sorted(cgamd.EXPORTS) == syms


def test_struct_layouts_match_reference():
    # raytracer Triangle 76 B, Sphere 44 B, Light 28 B, Intersection 28 B;
    # rasteriser Triangle 84 B
    assert C.sizeof(cgamd.Tri) == 76 and cgamd.Tri.color.offset == 64
    assert C.sizeof(cgamd.Sphere) == 44
    assert C.sizeof(cgamd.Light) == 28 and C.sizeof(cgamd.Isect) == 28
    assert C.sizeof(cgamd.RTri) == 84


def _bytes(arr, n, T):
    return bytes(C.string_at(C.addressof(arr), n * C.sizeof(T)))


def test_rt_scene_matches_oracle():
    tris, n, sph = cgamd.rt_scene()
    otris, on, osph = oracle.rt_scene()
    assert n == on == 28
    assert _bytes(tris, n, cgamd.Tri) == _bytes(otris, on, oracle.RtTri)
    assert bytes(sph) == bytes(osph)


def test_rast_scene_matches_oracle():
    room, nr, boxes, nb = cgamd.rast_scene()
    lib = oracle.load()
    oroom, oboxes = (oracle.RastTri * 16)(), (oracle.RastTri * 32)()
    onr, onb = C.c_int(), C.c_int()
    lib.cgo_rast_load_scene(oroom, C.byref(onr), oboxes, C.byref(onb))
    assert (nr, nb) == (onr.value, onb.value) == (10, 20)
    assert _bytes(room, nr, cgamd.RTri) == _bytes(oroom, nr, oracle.RastTri)
    assert _bytes(boxes, nb, cgamd.RTri) == _bytes(oboxes, nb, oracle.RastTri)


def _geometry_cases():
    import make_golden as mg
    return [c for c in mg.rast_configs().values()] + [
        dict(width=900, height=720, focal=512.0, cam=[0.35, 0.2, -1.9, 1.0], R=mg.yaw_R(-0.52),
             light=[0.2, -0.4, -0.3, 1.0], indirect_first=0.2),
        dict(width=400, height=300, focal=150.0, cam=[-0.6, 0.0, -0.4, 1.0], R=mg.yaw_R(0.9),
             light=[0, -0.5, 0, 1.0], indirect_first=0.2),
    ]


def test_rast_host_geometry_matches_oracle():
    """cg_rast_prepare (camera space, shadow volumes, rotation, 6 clip planes
    with the reference's plane-6 quirks) == oracle, bitwise, incl. order."""
    for cfg in _geometry_cases():
        p = cgamd.rast_params(cfg["width"], cfg["height"], cfg["focal"], tuple(cfg["cam"]),
                              (C.c_float * 16)(*cfg["R"]) if cfg["R"] else None, tuple(cfg["light"]))
        out, n, light = cgamd.rast_prepare(p)
        op = oracle.rast_params(cfg["width"], cfg["height"], cfg["focal"], tuple(cfg["cam"]), cfg["R"],
                                tuple(cfg["light"]))
        oout, on, olight = oracle.rast_geometry(op)
        assert n == on, cfg
        a = np.frombuffer(_bytes(out, n, cgamd.RTri), np.uint8).reshape(n, 84)
        b = np.frombuffer(_bytes(oout, on, oracle.RastTri), np.uint8).reshape(on, 84)
        # index of a shadow-volume triangle is uninitialised in the reference: compare v0..texture
        assert np.array_equal(a[:, :80], b[:, :80]), cfg
        assert bytes(light) == bytes(olight)


def test_no_gpu_fails_loudly():
    """Without a usable device cg_create must fail (no CPU fallback)."""
    lib = cgamd.load()
    if lib.cg_device_count() > 0:
        return
    h = C.c_void_p()
    assert lib.cg_create(0, C.byref(h)) == cgamd.CG_E_NODEVICE
    try:
        cgamd.Context(0)
    except RuntimeError:
        pass
    else:
        raise AssertionError("Context() must raise without a GPU")


def test_shard_rows_abi_matches_python():
    import cgdist
    lib = cgamd.load()
    for H in (256, 720, 1080, 2160, 1001):
        for n in (1, 2, 3, 4, 8):
            sh = cgamd.RtShard(0, n, 8)
            assert lib.cg_rt_shard_rows(H, C.byref(sh)) == cgdist.shard_rows(H, n, 8)
