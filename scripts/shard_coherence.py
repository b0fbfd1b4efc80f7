#!/usr/bin/env python3
"""Per-sample cost of one rank's row shard vs the whole frame (C2 geometry).

A rank of N renders rows y = r + k*N; its 8x8 work tiles then span 8 columns x 8N image
rows, i.e. camera rays over a taller solid angle. This times rank 0's shard for N = 1, 2, 4,
8 on one GPU (kernel ms per shard, Msamples/s of the shard), so the multi-GPU scaling loss
from tile coherence can be read apart from the gather.

usage: python scripts/shard_coherence.py [--spp 500] [--reps 3]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--block-samples", type=int, nargs="*", default=[], help="per-sample pool block sizes to sweep")
    ap.add_argument("--row-blocks", type=int, nargs="*", default=[1, 8], help="rt_render_params.row_block values to sweep")
    ap.add_argument("--tiles", action="store_true", help="also rank 0's 8x8-tile shard (rt_render_params.tile_shard)")
    a = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401  (one HIP runtime: torch's)
    import __graft_entry__ as ge
    rt = ge.import_binding()
    W, H = 1200, 800
    world = rt.World(1).build_scene(0)
    cam, bg = rt.scene_camera(0, W, H)
    cases = [(n, block, None) for block in a.row_blocks for n in ((1, 2, 4, 8) if block == 1 else (2, 4, 8))]
    cases += [(n, 1, bs) for bs in a.block_samples for n in (1, 8)]
    if a.tiles:
        cases += [(n, "tiles", None) for n in (2, 4, 8)]
    renderers = {}
    for n, block, bs in cases:
        if bs not in renderers:
            renderers[bs] = rt.Renderer(0)
            if bs:
                renderers[bs].set_option(rt.RT_OPT_BLOCK_SAMPLES, bs)
            renderers[bs].upload(world)
        r = renderers[bs]
        if block == "tiles":
            p = rt.Renderer.params(W, H, a.spp, 50, bg, 1, row_begin=0, row_stride=n, out_format=rt.RT_OUT_F32,
                                   tile_shard=1)
        else:
            p = rt.Renderer.params(W, H, a.spp, 50, bg, 1, row_begin=0, row_stride=n, out_format=rt.RT_OUT_F32,
                                   row_block=block)
        rows, width = rt.shard_shape(p)
        out = np.empty((rows, width, 3), np.float32)
        r.render(cam, p, out)
        ms = []
        for _ in range(a.reps):
            r.render(cam, p, out)
            ms.append(r.stats().kernel_ms)
        k = float(np.median(ms))
        print(json.dumps({"n": n, "row_block": block, "block_samples": bs, "rows": rows, "pixels": rows * width,
                          "kernel_ms": round(k, 3), "msamples_per_s": round(rows * width * a.spp / k / 1e3, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
