#!/usr/bin/env python3
"""Where a rank's time goes, per rank of an N-way tile partition (C4's ranks
differ by ~2.7 % in time at N = 8, whatever the tile order, while their measured lane work is
balanced). For every rank's shard: the timed render (kernel + reduce ms, median of --reps), then
a count_work render of the same shard, whose counters give the lane work (casts, node visits,
primitive tests, summed lane-cycles of the samples) and the wave work (bounce-loop, node-loop
and leaf-loop iterations of the waves, summed wave lifetimes).

usage: python scripts/shard_counts.py [--config c4] [--n 8] [--spp 256] [--order raster|cost]
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
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--order", default="raster", choices=["raster", "cost"])
    a = ap.parse_args()
    import numpy as np
    import __graft_entry__ as ge
    rt = ge.import_binding()
    scene, W, H = CONFIGS[a.config]
    r = rt.Renderer(0)
    r.upload(rt.World(1).build_scene(scene))
    cam, bg = rt.scene_camera(scene, W, H)
    if a.order == "cost":
        r.render(cam, rt.Renderer.params(W, H, 8, 50, bg, 1, out_format=rt.RT_OUT_F32, count_work=1))
        r.set_tile_order(rt.cost_tile_order(r.tile_costs()))
    rows = []
    for rank in range(a.n):
        p = rt.Renderer.params(W, H, a.spp, 50, bg, 1, row_begin=rank, row_stride=a.n, tile_shard=1,
                               out_format=rt.RT_OUT_F32)
        shape = rt.shard_shape(p)
        out = np.empty(shape + (3,), np.float32)
        r.render(cam, p, out)
        ms = []
        for _ in range(a.reps):
            r.render(cam, p, out)
            st = r.stats()
            ms.append(st.kernel_ms + st.reduce_ms)
        pc = rt.Renderer.params(W, H, a.spp, 50, bg, 1, row_begin=rank, row_stride=a.n, tile_shard=1,
                                out_format=rt.RT_OUT_F32, count_work=1)
        r.render(cam, pc, out)
        st = r.stats()
        c = r.counters(32)
        lane_cycles = int(r.tile_costs().sum())
        rows.append({"rank": rank, "ms": float(np.median(ms)), "count_ms": st.kernel_ms, "casts": int(st.casts),
                     "nodes": int(st.node_visits), "prims": int(st.prim_tests), "lane_cycles": lane_cycles,
                     "wave_steps": int(st.wave_steps), "wave_node_steps": int(st.wave_node_steps),
                     "wave_leaf_steps": int(st.wave_leaf_steps), "wave_life": int(c[21]),
                     "max_life_cycles": int(c[25]), "waves": int(c[26]),
                     "slot_use": int(c[21]) / max(1, int(c[26]) * int(c[25])),
                     "occupancy": st.casts / max(1, 64 * st.wave_steps)})
    # the whole frame (rows, one launch) with the same counters: the ranks' sums against it
    pf = rt.Renderer.params(W, H, a.spp, 50, bg, 1, out_format=rt.RT_OUT_F32)
    fo = np.empty(rt.shard_shape(pf) + (3,), np.float32)
    r.set_tile_order(None)
    r.render(cam, pf, fo)
    fms = []
    for _ in range(a.reps):
        r.render(cam, pf, fo)
        st = r.stats()
        fms.append(st.kernel_ms + st.reduce_ms)
    r.render(cam, rt.Renderer.params(W, H, a.spp, 50, bg, 1, out_format=rt.RT_OUT_F32, count_work=1), fo)
    st = r.stats()
    c = r.counters(32)
    whole = {"ms": float(np.median(fms)), "count_ms": st.kernel_ms, "casts": int(st.casts), "nodes": int(st.node_visits),
             "prims": int(st.prim_tests), "lane_cycles": int(r.tile_costs().sum()), "wave_steps": int(st.wave_steps),
             "wave_node_steps": int(st.wave_node_steps), "wave_leaf_steps": int(st.wave_leaf_steps),
             "wave_life": int(c[21]), "max_life_cycles": int(c[25]), "waves": int(c[26]),
             "slot_use": int(c[21]) / max(1, int(c[26]) * int(c[25])),
             "occupancy": st.casts / max(1, 64 * st.wave_steps)}
    print(json.dumps({"whole_frame": whole}), flush=True)
    keys = ["ms", "count_ms", "casts", "nodes", "prims", "lane_cycles", "wave_steps", "wave_node_steps",
            "wave_leaf_steps", "wave_life", "max_life_cycles", "slot_use", "occupancy"]
    print("sum over ranks / whole frame: " + json.dumps(
        {k: round(sum(q[k] for q in rows) / whole[k], 4) for k in keys if k not in ("occupancy", "slot_use", "max_life_cycles")}), flush=True)
    for q in rows:
        print(json.dumps(q), flush=True)
    mean = {k: sum(q[k] for q in rows) / len(rows) for k in keys}
    print("rank " + " ".join(f"{k:>15s}" for k in keys))
    for q in rows:   # each quantity relative to the mean over ranks
        print(f"{q['rank']:4d} " + " ".join(f"{q[k] / mean[k]:15.4f}" for k in keys))
    ms = np.array([q["ms"] for q in rows])
    for k in keys[1:]:
        v = np.array([q[k] for q in rows], dtype=np.float64)
        print(f"corr(ms, {k}) = {np.corrcoef(ms, v)[0, 1]:+.3f}")
    r.close()


if __name__ == "__main__":
    main()
