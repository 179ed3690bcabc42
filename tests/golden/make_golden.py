"""Generate tests/golden/golden.json from the CPU restatement (oracle/).

The restatement is pinned before any vector is written:
  * RT: bit-exact against the reference's own raytracer/screenshot.bmp
    (copied here as rt_screenshot_320x256.bmp, the reference's data file);
  * RT and RAST frames: the SHA-256 prefixes SURVEY.md section 8c recorded
    from the reference build (REFERENCE_FINGERPRINTS below);
  * RAST ComputePolygonRows: the reference's first-party KAT
    (rasteriser/Source/skeleton.cpp:183-199) with the survey's values.
Configs without a reference fingerprint (yaw/focal/light variants) are
pinned only transitively through the restatement ("parity unpinned" beyond
it) and are marked so in the JSON.

Usage: python tests/golden/make_golden.py   (writes golden.json next to it)
"""
from __future__ import annotations

import ctypes as C
import hashlib
import math
import json
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

# SURVEY.md section 8c, "Oracle fingerprints" (SHA-256 prefix of the raw
# little-endian planes of the reference build).
REFERENCE_FINGERPRINTS = {
    "rt_320x256_z-3": {"argb": "ae6dc7a534ca7b36"},
    "rt_320x256_z-2.9": {"argb": "a9a5d6e3b54cfcb5"},
    "rt_1920x1080_f1080": {"argb": "491ccd1a7aa74e31"},
    "rast_900x720": {"argb": "d263c345ede70be0", "depth": "1b41f904e60498b4",
                     "shadow": "e44df4a2df118261"},
    "rast_1920x1080_f768": {"argb": "51edb980fd402f9e", "depth": "4ea2dc05607151eb",
                            "shadow": "b3d6df4122de334e"},
}

# skeleton.cpp:183-199 KAT, expected rows from SURVEY.md section 4.
KAT_ROWS = {"vertices": [[10, 5], [5, 10], [15, 15]],
            "rows": [[10, 10], [9, 10], [8, 11], [7, 11], [6, 12], [5, 12], [7, 13], [9, 13],
                     [11, 14], [13, 14], [15, 15]]}


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def f32(x) -> float:
    return float(np.float32(x))


def yaw_R(yaw):
    """R as Update() builds it for a yaw (RT skeleton.cpp:236-238), float32."""
    y = np.float32(yaw)
    c, s = float(np.cos(y, dtype=np.float32)), float(np.sin(y, dtype=np.float32))
    m = [1.0 if k % 5 == 0 else 0.0 for k in range(16)]
    m[0], m[2], m[8], m[10] = c, -s, s, c
    return [f32(v) for v in m]


CAM_UP = f32(np.float32(-3.0) + np.float32(0.1))   # one UP keypress (:216-217)


def rt_configs():
    L0 = [[0.0, -0.5, -0.7, 1.0], [14.0, 14.0, 14.0]]
    return {
        "rt_320x256_z-3": dict(width=320, height=256, focal=256.0, cam=[0, 0, -3.0, 1], R=None, lights=[L0]),
        "rt_320x256_z-2.9": dict(width=320, height=256, focal=256.0, cam=[0, 0, CAM_UP, 1], R=None, lights=[L0]),
        "rt_1920x1080_f1080": dict(width=1920, height=1080, focal=1080.0, cam=[0, 0, -3.0, 1], R=None, lights=[L0]),
        "rt_320x256_yaw": dict(width=320, height=256, focal=256.0, cam=[0, 0, -3.0, 1],
                               R=yaw_R(np.float32(0.0) - np.float32(0.174533)), lights=[L0]),
        "rt_320x256_light_focal": dict(width=320, height=256, focal=266.0, cam=[f32(0.1), 0, -3.0, 1], R=None,
                                       lights=[[[f32(0.1), f32(-0.6), f32(-0.6), 1.0], [14.0, 14.0, 14.0]]]),
        "rt_256x192_2lights": dict(width=256, height=192, focal=200.0, cam=[0, 0, -3.0, 1], R=None,
                                   lights=[L0, [[0.3, -0.8, -0.2, 1.0], [6.0, 3.0, 9.0]]]),
        # build-defined workloads, small sizes of C4 and C5
        "rt_c4_480x270_soft8x8": dict(width=480, height=270, focal=270.0, cam=[0, 0, -3.0, 1], R=None,
                                      lights=[L0], area=dict(side=0.1, n=8)),
        "rt_c5_256x144_rand2000": dict(width=256, height=144, focal=144.0, cam=[0, 0, -3.0, 1], R=None,
                                       lights=[L0], scene=dict(random=2000, seed=0x5EED)),
    }


def rast_configs():
    return {
        "rast_900x720": dict(width=900, height=720, focal=512.0, cam=[0, 0, f32(-3.001), 1], R=None,
                             light=[0, -0.5, 0, 1], indirect_first=f32(0.2)),
        "rast_900x720_first": dict(width=900, height=720, focal=512.0, cam=[0, 0, f32(-3.001), 1], R=None,
                                   light=[0, -0.5, 0, 1], indirect_first=f32(0.15)),
        "rast_1920x1080_f768": dict(width=1920, height=1080, focal=768.0, cam=[0, 0, f32(-3.001), 1], R=None,
                                    light=[0, -0.5, 0, 1], indirect_first=f32(0.2)),
        "rast_640x480_yaw": dict(width=640, height=480, focal=360.0, cam=[f32(0.2), f32(-0.1), f32(-2.6), 1],
                                 R=yaw_R(np.float32(0.0) + np.float32(0.174533)),
                                 light=[f32(0.1), -0.5, f32(-0.2), 1], indirect_first=f32(0.2)),
        "rast_320x240_close": dict(width=320, height=240, focal=180.0, cam=[0, 0, f32(-1.2), 1], R=None,
                                   light=[0, -0.5, 0, 1], indirect_first=f32(0.2)),
        # colour modes 1-2 (randColourSelect, skeleton.cpp:647-662): libc rand() from the oracle
        "rast_640x480_colour1": dict(width=640, height=480, focal=360.0, cam=[0, 0, f32(-3.001), 1], R=None,
                                     light=[0, -0.5, 0, 1], indirect_first=f32(0.2), colour_mode=1,
                                     rand_offset=0),
        "rast_900x720_colour2_offset": dict(width=900, height=720, focal=512.0, cam=[0, 0, f32(-3.001), 1],
                                            R=None, light=[0, -0.5, 0, 1], indirect_first=f32(0.2),
                                            colour_mode=2, rand_offset=3_000_001),
        "rast_320x240_colour1_first": dict(width=320, height=240, focal=180.0, cam=[0, 0, f32(-3.001), 1],
                                           R=None, light=[0, -0.5, 0, 1], indirect_first=f32(0.15),
                                           colour_mode=1, rand_offset=0),
    }


def rt_lights_of(cfg):
    """Light list of a config: explicit, or the C4 area light around lights[0]."""
    if "area" in cfg:
        (p, c), a = cfg["lights"][0], cfg["area"]
        return oracle.rt_area_lights(tuple(p), tuple(c), a["side"], a["n"])
    return [(tuple(p), tuple(c)) for p, c in cfg["lights"]]


def rt_params_of(cfg):
    return oracle.rt_params(cfg["width"], cfg["height"], cfg["focal"], tuple(cfg["cam"]), cfg["R"], 0.5,
                            rt_lights_of(cfg))


def rt_oracle_scene(cfg):
    """(tris, n, sph pointer or None, n_sph) for oracle.rt_draw*: LoadTestModel or the C5 scene."""
    if "scene" in cfg:
        sc = cfg["scene"]
        return oracle.rt_random_scene(sc["seed"], sc["random"]), sc["random"], None, 0
    tris, n, sph = oracle.rt_scene()
    return tris, n, C.pointer(sph), 1


def rast_params_of(cfg):
    return oracle.rast_params(cfg["width"], cfg["height"], cfg["focal"], tuple(cfg["cam"]), cfg["R"],
                              tuple(cfg["light"]), cfg["indirect_first"], cfg.get("colour_mode", 0),
                              cfg.get("rand_offset", 0))


def screenshot_argb(path=os.path.join(HERE, "rt_screenshot_320x256.bmp")) -> np.ndarray:
    b = open(path, "rb").read()
    off = struct.unpack_from("<I", b, 10)[0]
    w, h = struct.unpack_from("<ii", b, 18)
    img = np.frombuffer(b[off:off + 4 * w * abs(h)], np.uint32).reshape(abs(h), w)
    if h > 0:
        img = img[::-1]          # BMP rows are bottom-up
    return np.ascontiguousarray(img).reshape(-1)


# ---- rasteriser/screenshot.bmp (the reference's own RAST output, 900 x 720) ----
# TestModelH.h:9-10 as committed: setting = 2 (metal grill room), settingBoxes = 1
# (marble boxes; Marble2000x2000.jpg is absent from the reference tree).  The
# camera/light state was recovered by a silhouette fit of the room followed by a
# search over Update()'s key counts and orders (rasteriser/Source/skeleton.cpp:
# 334-409); every screenshot pixel that does not depend on the marble texels
# then matches the restatement bit for bit.  Key letters as the host app's
# --keys: n/m yaw, L/R/U/D camera x/z, a/d/q/e/w/s light.
RAST_SCREENSHOT_KEYS = "m" + "n" * 6 + "L" * 20 + "R" * 2 + "U" * 14 + "d" * 3 + "a" * 13 + "e" * 8 + "s" * 4
RAST_SCREENSHOT_PATH = os.path.join(HERE, "rast_screenshot_900x720.bmp.xz")
TEXTURE_DIR = os.path.join(HERE, "textures")


def rast_replay_keys(keys):
    """Update() (rasteriser skeleton.cpp:334-409) over scripted keys: the globals after them.
    float32 vec4 adds; yaw -= 0.174533 is a double subtraction rounded to float; R from
    cos/sin of the float yaw (correctly rounded)."""
    f = np.float32
    cam = [f(0), f(0), f(-3.001), f(1)]
    light = [f(0), f(-0.5), f(0), f(1)]
    yaw, focal = f(0), f(512)
    step = {"U": (cam, 2, 0.1), "D": (cam, 2, -0.1), "L": (cam, 0, -0.1), "R": (cam, 0, 0.1),
            "z": (cam, 1, -0.1), "x": (cam, 1, 0.1), "w": (light, 2, 0.1), "s": (light, 2, -0.1),
            "a": (light, 0, -0.1), "d": (light, 0, 0.1), "q": (light, 1, -0.1), "e": (light, 1, 0.1)}
    for k in keys:
        if k in step:
            vec, i, d = step[k]
            vec[i] = f(vec[i] + f(d))
        elif k in "nm":
            yaw = f(float(yaw) + (0.174533 if k == "m" else -0.174533))
        elif k in "fg":
            focal = f(focal + (5 if k == "f" else -5))
    R = None
    if any(k in "nm" for k in keys):
        c, s_ = f(math.cos(float(yaw))), f(math.sin(float(yaw)))
        R = [1.0 if i % 5 == 0 else 0.0 for i in range(16)]
        R[0], R[2], R[8], R[10] = float(c), -float(s_), float(s_), float(c)
    return dict(cam=[float(v) for v in cam], light=[float(v) for v in light], yaw=float(yaw),
                focal=float(focal), R=R)


def rast_screenshot_argb() -> np.ndarray:
    import lzma
    with open(RAST_SCREENSHOT_PATH, "rb") as fh:
        raw = lzma.decompress(fh.read())
    tmp = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"cg_rast_shot_{os.getpid()}.bmp")
    with open(tmp, "wb") as fh:
        fh.write(raw)
    try:
        return screenshot_argb(tmp)
    finally:
        os.unlink(tmp)


def rast_screenshot_params(width=900, height=720):
    st = rast_replay_keys(RAST_SCREENSHOT_KEYS)
    return oracle.rast_params(width, height, st["focal"], tuple(st["cam"]), st["R"], tuple(st["light"]),
                              f32(0.2), 0, 0, setting=2, setting_boxes=1, yaw=st["yaw"])


def texture_jpegs():
    """{map name: JPEG bytes} of the reference texture files kept in tests/golden/textures."""
    files = {"woven": "woven1024x1024.jpg", "woven_ao": "Wood_wicker_003_ambientOcclusion.jpg",
             "woven_opacity": "Wood_wicker_003_opacity.jpg", "woven_normal": "Wood_wicker_003_normal.jpg",
             "grill": "Metal_Grill_002_basecolor.jpg", "grill_opacity": "Metal_Grill_002_opacity.jpg",
             "grill_normal": "Metal_Grill_002_normal.jpg"}
    out = {}
    for k, fn in files.items():
        with open(os.path.join(TEXTURE_DIR, fn), "rb") as fh:
            out[k] = fh.read()
    return out


def mg_sha_ok(a, want):
    return sha(a) == want


def main():
    oracle.build()
    out = {"generator": "tests/golden/make_golden.py", "reference_fingerprints": REFERENCE_FINGERPRINTS,
           "kat_polygon_rows": KAT_ROWS, "rt": {}, "rast": {}}
    shot = screenshot_argb()
    for name, cfg in rt_configs().items():
        p = rt_params_of(cfg)
        scene = rt_oracle_scene(cfg)
        small = cfg["width"] <= 320 and "area" not in cfg and "scene" not in cfg
        argb, cnt = oracle.rt_draw(p, counters=True, threads=1) if small else \
            (oracle.rt_draw(p, threads=os.cpu_count() or 8, scene=scene), None)
        e = {"config": cfg, "argb_sha256": sha(argb)}
        if cnt is not None:
            e["counters"] = {k: int(getattr(cnt, k)) for k in ("n_ray", "n_t", "n_uv", "n_sph", "n_dl")}
        ref = REFERENCE_FINGERPRINTS.get(name)
        if ref:
            assert e["argb_sha256"].startswith(ref["argb"]), (name, e["argb_sha256"])
            e["pinned_by"] = "SURVEY.md 8c reference fingerprint"
        elif "area" in cfg or "scene" in cfg:
            e["pinned_by"] = "build-defined workload (SURVEY.md 8d C4/C5, not in the reference): restatement only"
        else:
            e["pinned_by"] = "restatement only (parity unpinned beyond the oracle)"
        if name == "rt_320x256_z-2.9":
            assert np.array_equal(argb, shot), "restatement differs from raytracer/screenshot.bmp"
            e["pinned_by"] += " + raytracer/screenshot.bmp (bit-exact)"
        out["rt"][name] = e
        print(name, e["argb_sha256"][:16], e["pinned_by"])
    for name, cfg in rast_configs().items():
        p = rast_params_of(cfg)
        argb, depth, shadow, cnt = oracle.rast_draw(p, counters=True)
        e = {"config": cfg, "argb_sha256": sha(argb), "depth_sha256": sha(depth),
             "shadow_sha256": sha(shadow),
             "counters": {k: int(getattr(cnt, k)) for k in ("n_tris", "n_spans", "n_frags", "n_shaded", "n_shadow")}}
        ref = REFERENCE_FINGERPRINTS.get(name)
        if ref:
            for plane in ("argb", "depth", "shadow"):
                assert e[plane + "_sha256"].startswith(ref[plane]), (name, plane)
            e["pinned_by"] = "SURVEY.md 8c reference fingerprint"
        elif cfg.get("colour_mode", 0):
            e["pinned_by"] = "restatement + the C library's own rand() (no reference fingerprint for colour modes)"
        else:
            e["pinned_by"] = "restatement only (parity unpinned beyond the oracle)"
        out["rast"][name] = e
        print(name, e["argb_sha256"][:16], e["pinned_by"])
    # per-function vectors: ClosestIntersection / DirectLight on sampled rays
    lib = oracle.load()
    tris, n, sph = oracle.rt_scene()
    rng = np.random.default_rng(20241015)
    rays = []
    light = oracle.Light(oracle.V4(0.0, -0.5, -0.7, 1.0), oracle.V3(14.0, 14.0, 14.0))
    for k in range(64):
        if k < 48:   # camera rays through random pixels
            s = [0.0, 0.0, -3.0, 1.0]
            d = [f32(rng.integers(-160, 160) + 0.5 * rng.integers(-1, 2)),
                 f32(rng.integers(-128, 128) + 0.5 * rng.integers(-1, 2)), 256.0, 1.0]
        else:        # generic rays from inside the box
            s = [f32(v) for v in rng.uniform(-0.9, 0.9, 3)] + [1.0]
            d = [f32(v) for v in rng.uniform(-1, 1, 3)] + [0.0]
        ci = oracle.Isect()
        hit = lib.cgo_rt_closest(oracle.V4(*s), oracle.V4(*d), tris, n, C.byref(sph), 1, C.byref(ci), None)
        e = {"start": s, "dir": d, "hit": int(hit)}
        if hit:
            e["isect"] = {"position": [ci.position.x, ci.position.y, ci.position.z, ci.position.w],
                          "distance": ci.distance, "triangleIndex": ci.triangleIndex,
                          "sphereIndex": ci.sphereIndex}
            dl = lib.cgo_rt_direct_light(C.byref(ci), tris, n, C.byref(sph), 1, C.byref(light), None)
            e["direct_light"] = [dl.x, dl.y, dl.z]
        rays.append(e)
    out["rt_rays"] = rays
    # per-row work counters of the north-star config C2 (bench.py roofline basis)
    cfg = rt_configs()["rt_1920x1080_f1080"]
    p = rt_params_of(cfg)
    names = ("n_ray", "n_t", "n_uv", "n_sph", "n_dl")
    rowc = {k: np.zeros(cfg["height"], np.int64) for k in names}
    tris, n, sph = oracle.rt_scene()
    scratch = np.zeros(cfg["width"] * cfg["height"], np.uint32)
    for y in range(cfg["height"]):
        cnt = oracle.RtCounters()
        lib.cgo_rt_draw(C.byref(p), tris, n, C.byref(sph), 1, scratch.ctypes.data_as(C.c_void_p), y, y + 1,
                        C.byref(cnt))
        for k in names:
            rowc[k][y] = getattr(cnt, k)
    assert mg_sha_ok(scratch, out["rt"]["rt_1920x1080_f1080"]["argb_sha256"])
    np.savez(os.path.join(HERE, "rt_1080p_row_counters.npz"), **rowc)
    out["rt"]["rt_1920x1080_f1080"]["counters"] = {k: int(v.sum()) for k, v in rowc.items()}
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote golden.json")


if __name__ == "__main__":
    main()
