#!/usr/bin/env python3
"""Where a trace kernel's wave-cycles go: the count_work variant's s_memtime phase timers
(rt_last_counters) and lane occupancies, for one config.

usage: python scripts/phases.py [--scene 7 --width 1920 --height 1080 --spp 16]
Shares are of the summed per-wave kernel time (counter 21); the timers themselves cost ~10 %.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

PHASES = [("refill", 20), ("ray generation (camera + scatter draws)", 3), ("ray set-up (finish_ray)", 15),
          ("walk prologue (pre-leaf test)", 16), ("node loops", 8), ("leaf tests", 9),
          ("deferred instance walks", 22), ("hit record", 17),
          ("shading (emission)", 5)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", type=int, default=0)
    ap.add_argument("--width", type=int, default=1200)
    ap.add_argument("--height", type=int, default=800)
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--precision", default="f64")
    ap.add_argument("--ring", type=int, default=1, help="RT_OPT_POOL_RING (2: the ring whenever blocks allow)")
    ap.add_argument("--buf-mb", type=int, default=0, help="RT_OPT_TRACE_BUF_BYTES in MB (0: default)")
    a = ap.parse_args()
    import __graft_entry__ as ge
    rt = ge.import_binding()
    world = rt.World(1).build_scene(a.scene)
    cam, bg = rt.scene_camera(a.scene, a.width, a.height)
    r = rt.Renderer(0)
    r.upload(world)
    if a.precision == "f32":
        r.set_precision(rt.RT_PREC_F32)
    r.set_option(rt.RT_OPT_POOL_RING, a.ring)
    if a.buf_mb:
        r.set_option(rt.RT_OPT_TRACE_BUF_BYTES, a.buf_mb << 20)
    p = rt.Renderer.params(a.width, a.height, a.spp, a.depth, bg, 1, count_work=1)
    r.render(cam, p)
    st = r.stats()
    c = [int(x) for x in r.counters()]
    tot = max(c[21], 1)
    print(f"scene {a.scene} {a.width}x{a.height}x{a.spp} depth {a.depth} {a.precision} ring {st.ring_bytes > 0} "
          f"schedule {st.schedule} chunk {st.spp_chunk}: waves/SIMD {st.waves_per_simd}, "
          f"casts/sample {st.casts / st.samples:.3f}, nodes/cast {st.node_visits / max(st.casts, 1):.2f}, "
          f"prims/cast {st.prim_tests / max(st.casts, 1):.2f}")
    acc = 0
    for name, i in PHASES:
        acc += c[i]
        extra = ""
        if i == 9:
            extra = f"  (media {c[18] / tot:.3f}, instances {c[19] / tot:.3f})"
        if i == 3 and len(c) > 24:
            extra = (f"  (seeding + jitter {c[23] / tot:.3f}, rejection loop {c[24] / tot:.3f}, "
                     f"camera_end / scatter {(c[3] - c[23] - c[24]) / tot:.3f})")
        print(f"  {name:42s} {c[i] / tot:6.3f}{extra}")
    print(f"  {'unattributed':42s} {(tot - acc) / tot:6.3f}")
    slots = max(64 * st.wave_steps, 1)
    print(f"bounce-loop lane slots: casting {st.casts / slots:.3f}, idle at the tail {c[27] / slots:.3f}, "
          f"idle for a ring slot {c[28] / slots:.3f}, path absorbed in its scatter {c[29] / slots:.3f}, "
          f"depth cap {c[30] / slots:.3f}, rejection loop carried over {c[31] / slots:.3f}, "
          f"unaccounted {1 - (st.casts + sum(c[27:32])) / slots:.3f}")
    print(f"lane occupancy: bounce loop {st.casts / max(64 * st.wave_steps, 1):.3f}  node loop "
          f"{st.node_visits / max(64 * st.wave_node_steps, 1):.3f}  leaf loop {st.prim_tests / max(64 * st.wave_leaf_steps, 1):.3f}  "
          f"per wave iteration: {st.wave_node_steps / max(st.wave_steps, 1):.2f} node steps, "
          f"{st.wave_leaf_steps / max(st.wave_steps, 1):.2f} leaf steps")
    r.close()


if __name__ == "__main__":
    main()
