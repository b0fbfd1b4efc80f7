#!/usr/bin/env python3
"""A/B of the wavefront schedule (RT_SCHED_WAVEFRONT) against the per-sample pool on one
config: kernel ms per frame (median of --reps after one warm-up), the path-pool sizes given,
and whether each whole frame equals the pool's bit for bit.

usage: python scripts/wf_sweep.py [--scene 7 --width 1920 --height 1080 --spp 100]
                                  [--paths 0,524288,1048576,4194304] [--reps 3]
"""
import argparse
import hashlib
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", type=int, default=7)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=100)
    ap.add_argument("--paths", default="0")
    ap.add_argument("--refill", default="0", help="RT_OPT_WF_REFILL values (0: the default)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--count", action="store_true", help="also a count_work render per schedule (work and occupancy)")
    a = ap.parse_args()
    import __graft_entry__ as ge
    rt = ge.import_binding()
    W, H, spp = a.width, a.height, a.spp
    world = rt.World(1).build_scene(a.scene)
    cam, bg = rt.scene_camera(a.scene, W, H)
    r = rt.Renderer(0)
    r.upload(world)
    p = rt.Renderer.params(W, H, spp, 50, bg, 1, out_format=rt.RT_OUT_F64)
    out = np.empty((H, W, 3), np.float64)
    runs = [("pool", rt.RT_SCHED_POOL, 0, 0)] + [("wavefront", rt.RT_SCHED_WAVEFRONT, int(x), int(f))
                                                 for x in a.paths.split(",") for f in a.refill.split(",")]
    res = {k: [] for k in runs}
    frames = {}
    stats = {}
    for _ in range(a.rounds):
        for run in runs:
            name, sched, paths, refill = run
            r.set_schedule(sched)
            r.set_option(rt.RT_OPT_WF_PATHS, paths)
            r.set_option(rt.RT_OPT_WF_REFILL, refill)
            r.render(cam, p, out)   # warm-up
            for _ in range(a.reps):
                r.render(cam, p, out)
                res[run].append(r.stats().kernel_ms)
            st = r.stats()
            stats[run] = (st.schedule, st.wf_iterations, st.waves_per_simd)
            frames[run] = hashlib.sha1(out.tobytes()).hexdigest()
            print(f"  {name} paths={paths} refill={refill}: {['%.2f' % m for m in res[run][-a.reps:]]}", flush=True)
    base = frames[runs[0]]
    n = W * H * spp
    for run in runs:
        ms = sorted(res[run])[len(res[run]) // 2]
        sch, its, wps = stats[run]
        print(f"{run[0]} paths={run[2]} refill={run[3]}: median {ms:.2f} ms -> {n / ms / 1e3:.1f} Msamples/s  schedule {sch} "
              f"iterations {its} waves/SIMD {wps}  frame == pool: {frames[run] == base}", flush=True)
    if a.count:
        cp = rt.Renderer.params(W, H, min(spp, 16), 50, bg, 1, out_format=rt.RT_OUT_F32, count_work=1)
        for run in runs[:2]:
            r.set_schedule(run[1])
            r.set_option(rt.RT_OPT_WF_PATHS, run[2])
            r.set_option(rt.RT_OPT_WF_REFILL, run[3])
            r.render(cam, cp)
            s = r.stats()
            c = r.counters(24)
            d = {"casts": s.casts, "node_visits": s.node_visits, "prim_tests": s.prim_tests,
                 "wave_steps": int(c[6]), "wave_node_steps": int(c[7]), "wave_leaf_steps": int(c[10]),
                 "node_lane_occupancy": s.node_visits / max(64 * int(c[7]), 1),
                 "leaf_lane_occupancy": s.prim_tests / max(64 * int(c[10]), 1)}
            if run[1] == rt.RT_SCHED_WAVEFRONT:
                d["busy_lane_occupancy"] = int(c[13]) / max(64 * int(c[6]), 1)
                tot = max(int(c[21]), 1)   # wave-cycles summed over waves
                d["phase_shares"] = {k: round(int(c[i]) / tot, 4) for k, i in
                                     (("refill", 20), ("fetch", 16), ("ray_load_setup", 15), ("nodes", 8), ("leaves", 9),
                                                    ("blas_start", 22), ("hit_write", 17))}
            print("count", run[0], json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
