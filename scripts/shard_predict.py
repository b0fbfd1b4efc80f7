#!/usr/bin/env python3
"""The multi-GPU curve predicted from one GPU: every rank's tile shard of
C2, C4 and C5 at N = 2, 4, 8, rendered one after another on this GPU exactly as that rank
would render it (rt_render_params.tile_shard = 1, tiles r, r + N, ...).

Per N: each rank's kernel + reduce ms (median of --reps), max and mean over ranks, max/mean,
the implied efficiency T1 / (N * max) against the whole frame on one GPU, and the bytes each
rank's f64 slab sends to rank 0 in bench.py's gather. The gather itself (RCCL over xGMI) is
not timed here; its bytes are reported.

usage: python scripts/shard_predict.py [--configs c2 c4 c5] [--reps 3] [--c5-spp 256]
C5 runs at --c5-spp samples (its 4096 spp frame takes 10.6 s per pass): a rank's cost is
linear in spp, so max/mean and efficiency do not depend on it; say so where quoted.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

CONFIGS = {"c2": (0, 1200, 800, 500), "c4": (7, 1920, 1080, 1000), "c5": (0, 4096, 4096, 4096)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="*", default=["c2", "c4", "c5"])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--c5-spp", type=int, default=256)
    ap.add_argument("--ns", type=int, nargs="*", default=[2, 4, 8])
    ap.add_argument("--order", nargs="*", default=["raster"], choices=["raster", "cost"],
                    help="tile orders to time: raster, or cost (rt_ctx_set_tile_order from a count_work pass "
                         "of --cost-spp samples per pixel, most expensive tiles first)")
    ap.add_argument("--cost-spp", type=int, default=8)
    ap.add_argument("--ring", type=int, default=None, help="RT_OPT_POOL_RING for every render (default: the library's)")
    ap.add_argument("--block", type=int, default=None, help="RT_OPT_BLOCK_SAMPLES for every render (default: automatic)")
    a = ap.parse_args()
    import numpy as np
    import __graft_entry__ as ge
    rt = ge.import_binding()
    r = rt.Renderer(0)
    if a.ring is not None:
        r.set_option(rt.RT_OPT_POOL_RING, a.ring)
    if a.block is not None:
        r.set_option(rt.RT_OPT_BLOCK_SAMPLES, a.block)

    def timed(cam, p):
        rows, width = rt.shard_shape(p)
        out = np.empty((rows, width, 3), np.float32)
        r.render(cam, p, out)
        ms = []
        for _ in range(a.reps):
            r.render(cam, p, out)
            st = r.stats()
            ms.append(st.kernel_ms + st.reduce_ms)
        return float(np.median(ms)), rows * width

    for name in a.configs:
        scene, W, H, spp = CONFIGS[name]
        if name == "c5":
            spp = a.c5_spp
        world = rt.World(1).build_scene(scene)
        cam, bg = rt.scene_camera(scene, W, H)
        r.upload(world)
        t1, _ = timed(cam, rt.Renderer.params(W, H, spp, 50, bg, 1, out_format=rt.RT_OUT_F32))
        print(json.dumps({"config": name, "spp": spp, "n": 1, "frame_ms": round(t1, 3)}), flush=True)
        for order_kind in a.order:
            r.set_tile_order(None)
            if order_kind == "cost":
                import time
                t0 = time.perf_counter()
                r.render(cam, rt.Renderer.params(W, H, a.cost_spp, 50, bg, 1, out_format=rt.RT_OUT_F32, count_work=1))
                order = rt.cost_tile_order(r.tile_costs())
                r.set_tile_order(order)
                print(json.dumps({"config": name, "order": "cost", "cost_pass_spp": a.cost_spp,
                                    "cost_pass_wall_ms": round((time.perf_counter() - t0) * 1e3, 2)}), flush=True)
            for n in a.ns:
                per = []
                for rank in range(n):
                    p = rt.Renderer.params(W, H, spp, 50, bg, 1, row_begin=rank, row_stride=n, tile_shard=1,
                                           out_format=rt.RT_OUT_F32)
                    ms, px = timed(cam, p)
                    st = r.stats()
                    per.append({"rank": rank, "ms": round(ms, 3), "pixels": px, "slab_bytes_f64": px * 24,
                                "ring": st.ring_bytes > 0, "reduce_ms": round(st.reduce_ms, 3)})
                mx = max(q["ms"] for q in per)
                mean = sum(q["ms"] for q in per) / n
                print(json.dumps({"config": name, "order": order_kind, "spp": spp, "n": n, "max_ms": round(mx, 3), "mean_ms": round(mean, 3),
                                  "max_over_mean": round(mx / mean, 4), "implied_eff": round(t1 / (n * mx), 4),
                                  "sum_over_t1": round(sum(q["ms"] for q in per) / t1, 4),
                                  "gather_bytes_to_rank0": sum(q["slab_bytes_f64"] for q in per[1:]),
                                  "per_rank": per}), flush=True)
        r.set_tile_order(None)
    r.close()


if __name__ == "__main__":
    main()
