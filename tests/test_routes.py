"""CPU: cg_rt_route -- which kernels a frame of a given shape takes (host
logic only, no GPU).  The lattice kernels need R to leave y alone with dir.x a
function of x alone (raytracer/Source/skeleton.cpp:126-137): the identity
shares half-pixel columns, a yaw (:236-238) shares rows only; anything else,
more than 64 lights or stripes not on the 15-row lattice tile take the
per-pixel kernels.  Every route renders the reference's image (the GPU tests
check each against the oracle)."""
import math

import numpy as np
import pytest

import cgamd


def cam(R=None, W=1920, H=1080, f=1080.0):
    return cgamd.rt_camera(W, H, f, R=R)


def pitch(a):
    c, s = float(np.cos(np.float32(a), dtype=np.float32)), float(np.sin(np.float32(a), dtype=np.float32))
    m = [1.0 if k % 5 == 0 else 0.0 for k in range(16)]
    m[5], m[6], m[9], m[10] = c, s, -s, c
    return (cgamd.C.c_float * 16)(*m)


def raw(vals):
    return (cgamd.C.c_float * 16)(*vals)


@pytest.mark.parametrize("R,n_tris,n_sph,n_lights,want", [
    (None, 28, 1, 1, "lattice"),                      # C2
    (None, 28, 1, 64, "lights"),                      # C4
    (None, 28, 1, 65, "pixel"),                       # more lights than a lattice word
    (None, 28, 9, 1, "pixel"),                        # more spheres than the LDS table
    (None, 63, 0, 1, "pixel"),                        # > 62 triangles: no lattice mask room
    ("yaw", 28, 1, 1, "lattice_yaw"),                 # C2 after the LEFT key
    ("yaw", 28, 1, 16, "lights_yaw"),
    ("yaw2", 28, 1, 1, "lattice_yaw"),                # past 90 degrees: dir.x decreasing
    ("pitch", 28, 1, 1, "pixel"),                     # R turns y
    ("nan", 28, 1, 1, "pixel"),                       # a non-finite x row
    ("huge", 28, 1, 1, "pixel"),                      # entries past the monotone-x bound
    (None, 1_000_000, 0, 1, "big_lattice"),           # C5
    ("yaw", 1_000_000, 0, 1, "big_lattice_yaw"),
    ("yaw", 1_000_000, 0, 81, "big_pixel"),
    ("pitch", 1_000_000, 0, 1, "big_pixel"),
])
def test_route_by_camera_and_scene(R, n_tris, n_sph, n_lights, want):
    Rm = {None: None, "yaw": cgamd.yaw_matrix(0.1745), "yaw2": cgamd.yaw_matrix(2.0), "pitch": pitch(0.2)}.get(R)
    if R == "nan":
        Rm = raw([math.nan if k == 0 else (1.0 if k % 5 == 0 else 0.0) for k in range(16)])
    if R == "huge":
        Rm = raw([1e9 if k == 0 else (1.0 if k % 5 == 0 else 0.0) for k in range(16)])
    assert cgamd.rt_route(cam(Rm), n_tris, n_sph, n_lights) == want


def test_route_by_shard():
    c = cam()
    assert cgamd.rt_route(c, 28, 1, 1, cgamd.RtShard(0, 2, 15)) == "lattice"      # stripes on the tile height
    assert cgamd.rt_route(c, 28, 1, 1, cgamd.RtShard(1, 3, 8)) == "pixel"         # 8-row stripes
    band = cgamd.RtShard(0, 1, 15)
    band.row0, band.rows = 135, 270                                              # a band: contiguous rows
    assert cgamd.rt_route(c, 28, 1, 1, band) == "lattice"
    assert cgamd.rt_route(c, 1_000_000, 0, 1, cgamd.RtShard(0, 2, 32)) == "big_pixel"   # stripes: per-pixel mode


def test_route_rejects_bad_shapes():
    with pytest.raises(ValueError):
        cgamd.rt_route(cam(W=0), 28, 1, 1)
    with pytest.raises(ValueError):
        cgamd.rt_route(cam(), -1, 1, 1)
    with pytest.raises(ValueError):
        cgamd.rt_route(cam(), 28, 1, 1, cgamd.RtShard(2, 2, 8))                     # rank >= nranks
