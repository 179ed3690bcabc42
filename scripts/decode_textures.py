"""Decode the reference's texture JPEGs into the raw BGR maps the framework
takes (cg_rast_set_textures, `rasteriser --textures DIR`): DIR/NAME.bgr, row-
major, 3 bytes per texel in B, G, R order -- what cv::imread(...,
CV_LOAD_IMAGE_UNCHANGED) hands the reference (rasteriser/Source/skeleton.cpp:135-146).

Decoded with Pillow's libjpeg.  The reference was built against OpenCV 3.4's
JPEG reader, whose libjpeg may round some texels differently: frames drawn
from these maps are parity-checked against the CPU restatement on the same
maps, not against a reference-rendered textured frame (none exists; the
marble map is missing from the reference tree).
usage: python scripts/decode_textures.py [SRC_DIR] OUT_DIR
"""
import os
import sys

import numpy as np
from PIL import Image

FILES = {"marble": "Marble2000x2000.jpg",
         "woven": "woven1024x1024.jpg",
         "woven_ao": "Wood_wicker_003_ambientOcclusion.jpg",
         "woven_opacity": "Wood_wicker_003_opacity.jpg",
         "woven_normal": "Wood_wicker_003_normal.jpg",
         "grill": "Metal_Grill_002_basecolor.jpg",
         "grill_opacity": "Metal_Grill_002_opacity.jpg",
         "grill_normal": "Metal_Grill_002_normal.jpg"}
SIZES = {"marble": 2000}


def decode(src_dir):
    """{name: (H, W, 3) uint8 BGR} for the maps present in src_dir."""
    maps = {}
    for name, fn in FILES.items():
        path = os.path.join(src_dir, fn)
        if not os.path.exists(path):
            continue
        rgb = np.asarray(Image.open(path).convert("RGB"), dtype=np.uint8)
        n = SIZES.get(name, 1024)
        if rgb.shape != (n, n, 3):
            raise ValueError(f"{fn}: {rgb.shape}, the reference indexes it as {n} x {n}")
        maps[name] = np.ascontiguousarray(rgb[:, :, ::-1])
    return maps


def main():
    args = sys.argv[1:]
    src = args[0] if len(args) > 1 else "/root/reference/rasteriser/Textures"
    out = args[-1]
    os.makedirs(out, exist_ok=True)
    for name, a in decode(src).items():
        a.tofile(os.path.join(out, name + ".bgr"))
        print(name, a.shape)


if __name__ == "__main__":
    main()
