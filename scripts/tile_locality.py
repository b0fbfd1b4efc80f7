#!/usr/bin/env python3
"""Does a tile shard lose to the whole frame through locality?

A rank of an N-way round-robin tile partition holds every N-th tile, so the waves it runs at one
time work on tiles spread over the whole image, where one GPU's waves work on a band of
neighbouring tiles. This times, through tile orders (rt_ctx_set_tile_order; no kernel change):
  - one GPU: the frame as one tile shard in raster order, and in a scattered order (every
    --stride-th tile first, then the next residue, ...), which spreads it as an N-way shard is;
  - N ranks: round-robin single tiles (the default deal), and runs of G consecutive raster tiles
    dealt round-robin (rank r takes runs r, r + N, ...), for each --groups G.
kernel + reduce ms, median of --reps.

usage: python scripts/tile_locality.py [--configs c4 c2] [--spp 256] [--n 8] [--groups 8 30 120]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

CONFIGS = {"c2": (0, 1200, 800), "c4": (7, 1920, 1080), "c5": (0, 4096, 4096)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="*", default=["c4", "c2"])
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--stride", type=int, default=8)
    ap.add_argument("--groups", type=int, nargs="*", default=[8, 30, 120])
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import __graft_entry__ as ge
    rt = ge.import_binding()
    r = rt.Renderer(0)

    def timed(cam, p):
        out = np.empty(rt.shard_shape(p) + (3,), np.float32)
        r.render(cam, p, out)
        ms = []
        for _ in range(a.reps):
            r.render(cam, p, out)
            st = r.stats()
            ms.append(st.kernel_ms + st.reduce_ms)
        return float(np.median(ms))

    for name in a.configs:
        scene, W, H = CONFIGS[name]
        spp = a.spp
        r.upload(rt.World(1).build_scene(scene))
        cam, bg = rt.scene_camera(scene, W, H)
        n_tiles = ((W + 7) // 8) * ((H + 7) // 8)

        def params(rank=0, n=1, tile=1):
            return rt.Renderer.params(W, H, spp, 50, bg, 1, row_begin=rank, row_stride=n, tile_shard=tile,
                                      out_format=rt.RT_OUT_F32)

        r.set_tile_order(None)
        t_rows = timed(cam, params(tile=0))
        t_raster = timed(cam, params())
        r.set_tile_order(rt.scattered_tile_order(n_tiles, a.stride))
        t_scatter = timed(cam, params())
        # Z-order (Morton) of the tile grid: the waves in flight work on a compact square of tiles
        tx, ty = (W + 7) // 8, (H + 7) // 8

        def morton(x, y):
            z = 0
            for b in range(16):
                z |= ((x >> b) & 1) << (2 * b) | ((y >> b) & 1) << (2 * b + 1)
            return z
        keys = [morton(t % tx, t // tx) for t in range(n_tiles)]
        r.set_tile_order(np.argsort(np.array(keys), kind="stable").astype(np.uint32))
        t_morton = timed(cam, params())
        print(json.dumps({"config": name, "spp": spp, "n": 1, "frame_rows_ms": round(t_rows, 3),
                          "tile_shard_raster_ms": round(t_raster, 3),
                          "tile_shard_scattered_ms": round(t_scatter, 3), "stride": a.stride,
                          "tile_shard_morton_ms": round(t_morton, 3)}), flush=True)
        for g in [1] + a.groups:
            r.set_tile_order(None if g == 1 else rt.grouped_tile_order(n_tiles, a.n, g))
            per = [timed(cam, params(k, a.n)) for k in range(a.n)]
            mx, mean = max(per), sum(per) / a.n
            print(json.dumps({"config": name, "spp": spp, "n": a.n, "group": g, "max_ms": round(mx, 3),
                              "mean_ms": round(mean, 3), "max_over_mean": round(mx / mean, 4),
                              "implied_eff": round(t_rows / (a.n * mx), 4), "sum_over_t1": round(sum(per) / t_rows, 4),
                              "per_rank_ms": [round(x, 3) for x in per]}), flush=True)
        r.set_tile_order(None)
    r.close()


if __name__ == "__main__":
    main()
