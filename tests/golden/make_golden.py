#!/usr/bin/env python3
"""Golden vectors of the CPU oracle (oracle/oracle.c): small renders of every reference
scene at fixed seeds, f64 mean radiance. They pin the oracle against regressions and
are the fixtures the GPU tests compare the megakernel with.

usage: python tests/golden/make_golden.py   (writes tests/golden/oracle_renders.npz)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from tests import oracle_binding as ob  # noqa: E402

# (scene, W, H, spp, depth, scene_seed, render_seed)
CASES = [
    (0, 40, 24, 6, 50, 1, 1),
    (0, 33, 17, 3, 8, 4, 5),
    (1, 32, 18, 4, 50, 1, 1),
    (2, 32, 18, 4, 50, 1, 1),
    (3, 32, 18, 4, 50, 1, 1),
    (4, 32, 18, 6, 50, 1, 1),
    (5, 24, 24, 6, 50, 1, 1),
    (6, 24, 24, 6, 50, 1, 1),
    (7, 32, 18, 6, 50, 1, 1),
    (7, 16, 9, 4, 50, 3, 2),
]


def key(c):
    return "s%d_%dx%dx%d_d%d_ss%d_rs%d" % c


if __name__ == "__main__":
    out = {}
    for c in CASES:
        s, w, h, spp, d, ss, rs = c
        out[key(c)] = ob.render(s, w, h, spp, d, ss, rs, threads=4)
    np.savez_compressed(os.path.join(HERE, "oracle_renders.npz"), **out)
    print("wrote", len(out), "renders")
