#!/usr/bin/env python3
"""Interleaved A/B of render paths on one config, in one process (round 6): the whole frame
through rt_render against the same frame as a world-1 tile shard (rt_render_gather's layout),
and the per-sample pool with its in-kernel ring reduction against the per-sample buffer
(RT_OPT_POOL_RING 2 / 0 under a bound the buffer fits in one batch).

usage: python scripts/ab_paths.py --scene 0 --width 1200 --height 800 --spp 500 [--precision f32]
       [--paths plain,tile,ring,buffer] [--rounds 5]
Prints per path the median / min of kernel ms and of kernel + reduce ms, and checks that every
path renders the same image bit for bit."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", type=int, default=0)
    ap.add_argument("--width", type=int, default=1200)
    ap.add_argument("--height", type=int, default=800)
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--precision", default="f64")
    ap.add_argument("--paths", default="plain,tile,ring,buffer")
    a = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401  (the HIP runtime bench.py shares)
    import __graft_entry__ as ge
    rt = ge.import_binding()
    W, H = a.width, a.height
    r = rt.Renderer(0)
    r.upload(rt.World(1).build_scene(a.scene))
    if a.precision == "f32":
        r.set_precision(rt.RT_PREC_F32)
    cam, bg = rt.scene_camera(a.scene, W, H)
    big = 96 << 30   # the per-sample buffer of C4 (49.8 GB) in one batch

    def run(path):
        r.set_option(rt.RT_OPT_TRACE_BUF_BYTES, big if path == "buffer" else 0)
        r.set_option(rt.RT_OPT_POOL_RING, {"ring": 2, "buffer": 0}.get(path, 1))
        if path == "tile":
            p = rt.Renderer.params(W, H, a.spp, a.depth, bg, 1, out_format=rt.RT_OUT_F64, tile_shard=1)
            slab = r.render(cam, p)
            img = rt.assemble_tiles([slab], W, H, 1)
        else:
            img = r.render(cam, rt.Renderer.params(W, H, a.spp, a.depth, bg, 1, out_format=rt.RT_OUT_F64))
        st = r.stats()
        return img, st.kernel_ms, st.kernel_ms + st.reduce_ms, st

    paths = a.paths.split(",")
    times = {p: ([], []) for p in paths}
    ref = None
    for i in range(a.rounds + 1):
        for p in paths:
            img, k, kr, st = run(p)
            if ref is None:
                ref = img
            assert np.array_equal(img, ref), p
            if i == 0:
                print(f"{p}: schedule {st.schedule} ring {st.ring_bytes} trace_buf {st.trace_buf_bytes} "
                      f"batches {st.n_batches} waves/SIMD {st.waves_per_simd}", flush=True)
                continue   # warm-up round
            times[p][0].append(k)
            times[p][1].append(kr)
    for p in paths:
        k, kr = times[p]
        print(f"{p:8s} kernel median {np.median(k):9.3f} min {min(k):9.3f} | kernel+reduce median {np.median(kr):9.3f} "
              f"min {min(kr):9.3f} ms  ({len(k)} runs)", flush=True)
    print("images bit-identical across paths")
    r.close()


if __name__ == "__main__":
    main()
