#!/usr/bin/env python3
"""Builds compact fixtures from the reference's OWN output images (data files in
/root/reference/generated_images, rendered by older revisions of the reference with an
unseeded RNG). Run once in the build container; the outputs are committed because
/root/reference does not exist on the GPU box.

  ref_earth_400x225.png       earth.ppm (main.rs:370-387 scene, 400x225), lossless
  ref_cornell_smoke_blocks.npy cornell_box.ppm (600x600; it is the cornell_box_smoke
                               scene, main.rs:138-171, 40 spp per the preset main.rs:424-441)
                               as 20x20-pixel block means of the 8-bit channels (30x30x3)
"""
import os

import numpy as np
from PIL import Image

SRC = "/root/reference/generated_images"
OUT = os.path.dirname(os.path.abspath(__file__))


def read_ppm(path):
    toks = open(path).read().split()
    assert toks[0] == "P3"
    w, h = int(toks[1]), int(toks[2])
    return np.array(toks[4:4 + w * h * 3], dtype=np.uint8).reshape(h, w, 3)


def blocks(a, b=20):
    h, w, _ = a.shape
    return a[: h // b * b, : w // b * b].astype(np.float64).reshape(h // b, b, w // b, b, 3).mean(axis=(1, 3))


if __name__ == "__main__":
    Image.fromarray(read_ppm(os.path.join(SRC, "earth.ppm"))).save(os.path.join(OUT, "ref_earth_400x225.png"))
    np.save(os.path.join(OUT, "ref_cornell_smoke_blocks.npy"), blocks(read_ppm(os.path.join(SRC, "cornell_box.ppm"))))
