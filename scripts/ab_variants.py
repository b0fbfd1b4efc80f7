#!/usr/bin/env python3
"""A/B the megakernel's variant knobs in ONE process (interleaved rounds), on a bench config.

usage: python scripts/ab_variants.py [--scene 0] [--width 1200] [--height 800] [--spp 500] [--rounds 3]
Prints per-variant kernel ms (median, min) and checks the variants render identical images.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def bvh_options(rt, world, b):
    """(c_isect, max_leaf, force_leaf) as rt_world_set_build_option values (0: the default)."""
    world.set_build_option(rt.RT_BUILD_C_ISECT, float(b[0]))
    world.set_build_option(rt.RT_BUILD_MAX_LEAF, float(b[1]))
    world.set_build_option(rt.RT_BUILD_FORCE_LEAF, float(b[2]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", type=int, default=0)
    ap.add_argument("--width", type=int, default=1200)
    ap.add_argument("--height", type=int, default=800)
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="1:1:1,1:1:0", help="slab32:lds_stack:lds_nodes tuples")
    ap.add_argument("--sched", default="", help="comma list of schedules to A/B: 0 chunks, 1 pool")
    ap.add_argument("--chunks", default="", help="comma list of spp_chunk values to A/B")
    ap.add_argument("--accel", default="", help="comma list of accel modes to A/B: 0 SAH, 1 LINEAR, 2 MEDIAN")
    ap.add_argument("--bvh", default="", help="comma list of CI:MAXLEAF[:LEAFN] BVH builds to A/B (default variant)")
    args = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401  (same HIP runtime as bench.py)
    import __graft_entry__ as ge
    rt = ge.import_binding()

    W, H = args.width, args.height
    world = rt.World(1).build_scene(args.scene)
    cam, bg = rt.scene_camera(args.scene, W, H)
    r = rt.Renderer(0)
    r.upload(world)
    variants = [tuple(int(x) for x in v.split(":")) for v in args.variants.split(",")]
    # identity check on a small f64 render
    imgs = {}
    for v in variants:
        r.set_variant(*v)
        imgs[v] = r.render(cam, rt.Renderer.params(W, H, 2, args.depth, bg, 1, row_stride=8, out_format=rt.RT_OUT_F64))
    base = imgs[variants[0]]
    for v in variants[1:]:
        same = np.array_equal(imgs[v], base)
        print(f"variant {v} identical to {variants[0]}: {same}" +
              ("" if same else f" (max diff {np.max(np.abs(imgs[v] - base)):.3e}, "
                               f"{int(np.sum(np.any(imgs[v] != base, axis=2)))} px)"))
    times = {v: [] for v in variants}
    p = rt.Renderer.params(W, H, args.spp, args.depth, bg, 1, out_format=rt.RT_OUT_F32)
    out = np.empty((H, W, 3), np.float32)
    for rnd in range(args.rounds + 1):
        for v in variants:
            r.set_variant(*v)
            r.render(cam, p, out)
            st = r.stats()
            if rnd > 0:
                times[v].append(st.kernel_ms)
            used = (st.variant_features, st.slab32, st.lds_stack, st.lds_nodes)
    for v in variants:
        t = times[v]
        ms = float(np.median(t))
        print(f"variant {v}: median {ms:.2f} ms  min {min(t):.2f} ms  "
              f"-> {W * H * args.spp / ms / 1e3:.1f} Msamples/s")
    print("last variant features/slab32/lds_stack:", used)
    if args.sched:
        scheds = [int(x) for x in args.sched.split(",")]
        r.set_variant(*variants[0])
        st_t, st_img, occ = {m: [] for m in scheds}, {}, {}
        for m in scheds:
            r.set_schedule(m)
            st_img[m] = r.render(cam, rt.Renderer.params(W, H, 4, args.depth, bg, 1, row_stride=8,
                                                         out_format=rt.RT_OUT_F64))
            ck = max(1, (args.spp + 15) // 16)
            r.render(cam, rt.Renderer.params(W, H, min(args.spp, 2 * ck), args.depth, bg, 1, spp_chunk=ck,
                                             count_work=1))
            q = r.stats()
            occ[m] = q.casts / max(64 * q.wave_steps, 1)
        for rnd in range(args.rounds + 1):
            for m in scheds:
                r.set_schedule(m)
                r.render(cam, p, out)
                if rnd > 0:
                    st_t[m].append(r.stats().kernel_ms)
        for m in scheds:
            ms = float(np.median(st_t[m]))
            print(f"schedule {m}: median {ms:.2f} ms -> {W * H * args.spp / ms / 1e3:.1f} Msamples/s  "
                  f"bounce-loop occupancy {occ[m]:.3f}  image == schedule {scheds[0]}: "
                  f"{np.array_equal(st_img[m], st_img[scheds[0]])}")
        r.set_schedule(1)
    if args.accel:
        modes = [int(x) for x in args.accel.split(",")]
        names = {0: "SAH", 1: "LINEAR", 2: "MEDIAN"}
        r.set_variant(*variants[0])
        at, work, ims = {m: [] for m in modes}, {}, {}
        for m in modes:
            r.upload(world, m)
            ims[m] = r.render(cam, rt.Renderer.params(W, H, 2, args.depth, bg, 1, row_stride=8,
                                                      out_format=rt.RT_OUT_F64))
            r.render(cam, rt.Renderer.params(W, H, 4, args.depth, bg, 1, row_stride=4, count_work=1))
            st = r.stats()
            work[m] = (st.node_visits / st.casts, st.prim_tests / st.casts)
        for rnd in range(args.rounds + 1):
            for m in modes:
                r.upload(world, m)
                r.render(cam, p, out)
                if rnd > 0:
                    at[m].append(r.stats().kernel_ms)
        for m in modes:
            soa = world.flatten(m)
            ms = float(np.median(at[m]))
            print(f"accel {names[m]}: nodes={soa.n_nodes} stack={soa.tlas_depth}/{soa.blas_depth} "
                  f"node visits/cast {work[m][0]:.2f} prim tests/cast {work[m][1]:.2f}  "
                  f"median {ms:.2f} ms -> {W * H * args.spp / ms / 1e3:.1f} Msamples/s  "
                  f"image == SAH: {np.array_equal(ims[m], ims[modes[0]])}")
        r.upload(world)
    if args.bvh:
        builds = [tuple((x + ":2").split(":")[:3]) if x.count(":") == 1 else tuple(x.split(":"))
                  for x in args.bvh.split(",")]
        bt = {b: [] for b in builds}
        r.set_variant(*variants[0])
        for rnd in range(args.rounds + 1):
            for b in builds:
                bvh_options(rt, world, b)
                r.upload(world)
                r.render(cam, p, out)
                if rnd > 0:
                    bt[b].append(r.stats().kernel_ms)
        for b in builds:
            bvh_options(rt, world, b)
            soa = world.flatten()
            print(f"bvh ci={b[0]} maxleaf={b[1]} leafn={b[2]} nodes={soa.n_nodes} depth={soa.tlas_depth}/{soa.blas_depth}: "
                  f"median {float(np.median(bt[b])):.2f} ms")
        bvh_options(rt, world, ("0", "0", "0"))   # the defaults
        r.upload(world)
    # phase shares from the diagnostic count_work variant (first variant's knobs), at the
    # timed run's chunk size so the lane-occupancy figures describe the same waves
    r.set_variant(*variants[0])
    chunk = max(1, (args.spp + 15) // 16)
    r.render(cam, rt.Renderer.params(W, H, min(args.spp, 2 * chunk), args.depth, bg, 1, spp_chunk=chunk,
                                     count_work=1))
    st = r.stats()
    tot = st.cycles_camera + st.cycles_trace + st.cycles_shade
    if tot:
        print(f"phase shares (wave-cycles): camera {st.cycles_camera / tot:.3f}  trace {st.cycles_trace / tot:.3f} "
              f"(node loops {st.cycles_nodes / tot:.3f}, leaves {st.cycles_leaves / tot:.3f})  "
              f"shade {st.cycles_shade / tot:.3f};  casts/sample {st.casts / st.samples:.3f}  "
              f"nodes/cast {st.node_visits / max(st.casts, 1):.2f}  prims/cast {st.prim_tests / max(st.casts, 1):.2f}")
        print(f"lane occupancy (spp_chunk {chunk}): bounce loop {st.casts / max(64 * st.wave_steps, 1):.3f}  "
              f"node-visit loop {st.node_visits / max(64 * st.wave_node_steps, 1):.3f}  "
              f"leaf loop {st.prim_tests / max(64 * st.wave_leaf_steps, 1):.3f}  "
              f"camera {st.camera_lanes / max(64 * st.camera_steps, 1):.3f} ({st.camera_steps / max(st.wave_steps, 1):.3f} of iterations)  "
              f"shade {st.shade_lanes / max(64 * st.shade_steps, 1):.3f} ({st.shade_steps / max(st.wave_steps, 1):.3f} of iterations)")
        print(f"per wave iteration: node steps {st.wave_node_steps / max(st.wave_steps, 1):.2f}  "
              f"leaf steps {st.wave_leaf_steps / max(st.wave_steps, 1):.2f}")
    if args.chunks:
        cks = [int(x) for x in args.chunks.split(",")]
        ct = {k: [] for k in cks}
        for rnd in range(args.rounds + 1):
            for k in cks:
                q = rt.Renderer.params(W, H, args.spp, args.depth, bg, 1, spp_chunk=k, out_format=rt.RT_OUT_F32)
                r.render(cam, q, out)
                if rnd > 0:
                    ct[k].append(r.stats().kernel_ms)
        for k in cks:
            q = rt.Renderer.params(W, H, min(args.spp, 4 * k), args.depth, bg, 1, spp_chunk=k, count_work=1)
            r.render(cam, q)
            st = r.stats()
            print(f"spp_chunk {k}: median {float(np.median(ct[k])):.2f} ms  bounce-loop occupancy "
                  f"{st.casts / max(64 * st.wave_steps, 1):.3f}")


if __name__ == "__main__":
    main()
