#!/usr/bin/env python3
"""Where a small shard's extra time goes: the count_work variant of rank 0's
tile shard at N = 1, 2, 4, 8 (C2 or C4 geometry), with the phase shares of scripts/phases.py and
the launch's wave-slot use: the waves' summed lifetimes over (waves x the longest lifetime), so
1 - that is the share of the launch's wave slots left idle while its last waves finish (its tail).

usage: python scripts/shard_tail.py [--scene 7 --width 1920 --height 1080 --spp 64]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", type=int, default=7)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--ns", type=int, nargs="*", default=[1, 2, 4, 8])
    a = ap.parse_args()
    import __graft_entry__ as ge
    rt = ge.import_binding()
    world = rt.World(1).build_scene(a.scene)
    cam, bg = rt.scene_camera(a.scene, a.width, a.height)
    r = rt.Renderer(0)
    r.upload(world)
    for n in a.ns:
        p = rt.Renderer.params(a.width, a.height, a.spp, 50, bg, 1, row_begin=0, row_stride=n, tile_shard=int(n > 1),
                               count_work=1)
        r.render(cam, p)
        st = r.stats()
        c = [int(x) for x in r.counters(32)]
        tot = max(c[21], 1)
        util = c[21] / max(c[25] * c[26], 1)
        print(json.dumps({"n": n, "spp": a.spp, "kernel_ms": round(st.kernel_ms, 3), "samples": st.samples,
                          "waves": c[26], "wave_slot_use": round(util, 4), "tail_idle": round(1 - util, 4),
                          "casts_per_sample": round(st.casts / max(st.samples, 1), 4),
                          "refill": round(c[20] / tot, 4), "raygen": round(c[3] / tot, 4),
                          "nodes": round(c[8] / tot, 4), "leaves": round(c[9] / tot, 4), "defer": round(c[22] / tot, 4),
                          "lane_occ_bounce": round(st.casts / max(64 * st.wave_steps, 1), 4),
                          "schedule": st.schedule, "ring_bytes": st.ring_bytes}), flush=True)
    r.close()


if __name__ == "__main__":
    main()
