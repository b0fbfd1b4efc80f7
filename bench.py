#!/usr/bin/env python3
"""Headline benchmark: Msamples/s (pixels x spp per second) on the 1200x800 random-spheres
scene, 500 spp, max depth 50 (BASELINE.json configs[1] = SURVEY C2), at N GPUs.

One step = one full render of the frame through the library's multi-GPU entry point,
rt_render_gather (C ABI, librtiow_amd.so): every rank traces its 8x8 tile shard (the tiles at
positions rank + k*N of the frame's tile order) through the HIP megakernel, the library's own
RCCL communicator gathers the slabs to rank 0 and a reorder kernel writes the frame there —
inside the timed region; at N = 1 the same call over a world-1 communicator. torch.distributed
(gloo, on the host) only hands out the RCCL unique id and runs the barriers and the MAX
all-reduce of the step time. The scene is built and uploaded, and the tile order's cost pass
run, before timing; the cost pass's time is amortised into `value` (value_steady without).

Prints ONE JSON line (rank 0). Besides the contract fields it carries
  roofline:     the binding resource, VALU issue: the issue cycles the launch's VALU
                instruction mix needs (per-class counts from a rocprofv3 PMC pass of THIS
                build and workload, profiles/pmc.json keyed by the source hash; cycles
                per instruction class calibrated on the box, scripts/calib) against the
                SIMD-cycles of the live-timed kernel; `traffic` = DRAM bytes per launch from
                the same PMC pass; the DRAM fraction and the SURVEY §8(d) algorithmic
                (LDS/L1/L2-served) bytes are reported beside it;
  cpu_baseline: the CPU oracle (reference-faithful C restatement, linear list scan like
                hittable.rs:43-55) on this host's usable cores, rank 0 at N=1 only, on a
                bounded row subset of the same workload, plus the reference's own 10-thread
                sample split (main.rs:497-551) for comparison with README.md:6;
  parity:       the GPU render of exactly the rows and samples the CPU baseline rendered,
                against the oracle's image, per pixel (north_star: L_inf <= 1e-3).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
N_SIMDS = 1024                 # 256 CUs x 4 SIMDs
PMC_JSON = os.path.join(REPO, "profiles", "pmc.json")
ROW_BLOCK = 1                  # multi-GPU shards: single rows round-robin over the ranks


# BASELINE.json configs (SURVEY §8 shorthand). The headline metric is C2; the others are
# reachable for measurement with --config (C4/C5 are quoted on 8 GPUs).
CONFIGS = {
    "C1": dict(scene=0, width=1200, height=800, spp=10, depth=8),
    "C2": dict(scene=0, width=1200, height=800, spp=500, depth=50),
    "C3": dict(scene=5, width=800, height=800, spp=1000, depth=50),
    "C4": dict(scene=7, width=1920, height=1080, spp=1000, depth=50),
    "C5": dict(scene=0, width=4096, height=4096, spp=4096, depth=50),
}
SCHEDULES = {"chunks": 0, "pool": 1, "items": 2, "auto": 3}
SCENE_NAMES = {0: "random_scene (main.rs:245-289)", 5: "cornell_box_scene (main.rs:107-136)",
               7: "final_scene (main.rs:173-243)"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS), help="BASELINE.json config preset")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", type=int, default=None)
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--depth", type=int, default=None)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--t10-seconds", type=float, default=10.0, help="CPU time of the reference 10-thread split run")
    ap.add_argument("--count-spp", type=int, default=16, help="spp of the untimed count_work pass")
    ap.add_argument("--spp-chunk", type=int, default=0, help="samples per chunk (0: the library's automatic choice)")
    ap.add_argument("--no-count", action="store_true", help="skip the count_work pass (profiling runs)")
    ap.add_argument("--ppm", default="", help="write the rendered frame (rank 0) as a P3 PPM")
    ap.add_argument("--frame-npy", default="", help="save the rendered f64 frame (rank 0) as .npy")
    ap.add_argument("--transport", default="rccl", choices=["rccl", "gloo", "none"],
                    help="rccl (default, every N): the library's multi-GPU render, rt_render_gather — the rank's "
                         "8x8 tile shard, one RCCL gather to rank 0 over the library's own communicator, the "
                         "on-device reorder kernel (at N = 1 a world-1 communicator: the same code path); gloo: "
                         "tile (or row) slabs staged through the host and gathered by torch.distributed gloo, so "
                         "several ranks can share one GPU (tests of the N > 1 path on a 1-GPU box); none: N = 1 "
                         "only, rt_render straight into the frame")
    ap.add_argument("--shard", default="tiles", choices=["tiles", "rows"],
                    help="partition: the frame's 8x8 tiles round-robin (rt_render_params.tile_shard) or, with "
                         "--transport gloo only, single rows round-robin")
    ap.add_argument("--tile-order", default="auto", choices=["auto", "raster", "cost"],
                    help="tile shards: cost (every rank counts its raster shard at --cost-spp samples per "
                         "pixel, one all-reduce of the per-tile lane-cycles, the tiles sorted by cost: "
                         "rt_comm_tile_order; shards then deal their blocks tile-major), raster, or auto "
                         "(default: cost at N > 1, raster at N = 1). The pass runs before the timed steps and "
                         "its time is amortised into the headline value (value_steady leaves it out)")
    ap.add_argument("--cost-spp", type=int, default=8, help="spp of the --tile-order cost pass")
    ap.add_argument("--comm-direct", type=int, default=1, choices=[0, 1],
                    help="RT_OPT_COMM_DIRECT: 1 (default) a world of one in raster order renders straight into "
                         "the frame inside rt_render_gather; 0 the tile shard + RCCL gather + reorder as at N > 1")
    ap.add_argument("--device", type=int, default=None,
                    help="GPU index for every rank (default: LOCAL_RANK); with --transport gloo, ranks may share one")
    ap.add_argument("--force-dist", action="store_true",
                    help="take the distributed branch (torch.distributed control plane, unique-id broadcast, "
                         "barriers, MAX all-reduce) even at world size 1: launch as torch.distributed.run "
                         "--nproc-per-node 1 ... --gpus 1 --force-dist")
    ap.add_argument("--precision", default="f64", choices=["f64", "f32"],
                    help="f64: the reference's arithmetic (the headline); f32: the fast mode (SURVEY §8 f3)")
    ap.add_argument("--schedule", default="auto", choices=sorted(SCHEDULES),
                    help="work schedule (rt_ctx_set_schedule); images are bit-identical under all of them")
    ap.add_argument("--buf-mb", type=int, default=0,
                    help="trace-output buffer bound in MB (rt_ctx_set_option RT_OPT_TRACE_BUF_BYTES; 0: default)")
    ap.add_argument("--no-overlap", action="store_true", help="buffer batches in order in one buffer")
    args = ap.parse_args()
    for k, v in CONFIGS[args.config].items():
        if getattr(args, k) is None:
            setattr(args, k, v)
    return args


def usable_cores():
    """CPU threads this process may really run: its affinity mask, capped by a cgroup CPU
    quota (the GPU box gives one GPU's job a 16-CPU share of a larger machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, math.ceil(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    return (min(n, quota) if quota else n), n, quota


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def pmc_entry(src_hash, workload):
    """The PMC record of this build (source hash) and workload, or None."""
    if not os.path.exists(PMC_JSON):
        return None, None
    doc = json.load(open(PMC_JSON))
    for e in doc.get("entries", []):
        if e.get("src_hash") == src_hash and e.get("workload") == workload:
            return e, doc.get("calibration")
    return None, doc.get("calibration")


ISA_JSON = os.path.join(REPO, "profiles", "isa_mix.json")
VARIANT_NAMES = {0: "spheres", 35: "rectinst", 103: "media", 287: "final", 4095: "all"}


def isa_prices(src_hash, variant_features, schedule, slab32=1, nall=1, ring=False):
    """Per-class issue prices from the trace kernel's own instruction mix (scripts/isa_mix.py,
    profiles/isa_mix.json) for this build and kernel: {counter or 'other': (price, lo, hi)}.
    ring: the per-sample pool's in-kernel-reduction kernel (rt_stats.ring_bytes > 0)."""
    if not os.path.exists(ISA_JSON):
        return None
    kind = "items" if schedule == 2 else "ring" if ring else "pool"
    e = json.load(open(ISA_JSON)).get(src_hash, {}).get(
        "%s/%s/s%dn%d" % (VARIANT_NAMES.get(variant_features, "?"), kind, slab32, nall))
    if not e:
        return None
    return {c: (v["price"], v["range"][0], v["range"][1]) for c, v in e["classes"].items()}


KMIX_OF = {0: "kmix_c2", 287: "kmix_c4", 35: "kmix_c3"}   # variant -> calibration replay of its VALU mix (scripts/calib/gen_kmix.py)


def replay_price(calib, variant_features):
    """Cycles per VALU instruction of the variant's own instruction mix replayed as a saturated
    calibration stream (KMIX_*), or None."""
    k = (calib.get("kmix") or {}).get(KMIX_OF.get(variant_features, ""))
    return k["measured"] if k else None


def valu_issue_cycles(counts, calib, other=None, isa=None, bound=0):
    """Issue cycles (summed over SIMDs) the launch's VALU instruction mix needs at the
    calibrated saturated rates: sum over classes of count x cycles per wave-instruction; the
    instructions no class counter covers (moves, compares, selects, bit ops) at the measured
    rate of those (calib 'other', or `other` to price the bounds). With `isa` (isa_prices),
    every class — "other" included — is priced from the kernel's own static instruction mix
    over the calibrated per-opcode costs; bound -1 / +1 takes each class's low / high price."""
    cyc = dict(calib["cycles_per_inst"])
    if other is not None:
        cyc["other"] = other
    by_counter = {}
    if isa:
        k = {0: 0, -1: 1, 1: 2}[bound]
        by_counter = {c: v[k] for c, v in isa.items()}
        if "other" in isa:
            cyc["other"] = isa["other"][k]
    total = counts["SQ_INSTS_VALU"]
    known, need = 0.0, 0.0
    for cls, key in calib["class_counters"].items():
        n = counts.get(key)
        if n is None:
            continue
        known += n
        need += n * by_counter.get(key[len("SQ_INSTS_VALU_"):], cyc[cls])
    need += max(0.0, total - known) * cyc["other"]
    return need


class stdout_to_stderr:
    """fd 1 -> fd 2 for a block (native libraries print there; the bench's stdout is its JSON line)."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one rank per GPU)")
    # the distributed branch: N > 1, or N = 1 under --force-dist
    dist_on = world > 1 or args.force_dist
    if args.force_dist and "MASTER_ADDR" not in os.environ:
        raise SystemExit("--force-dist needs torch.distributed.run (MASTER_ADDR / RANK / WORLD_SIZE in the env)")
    transport = args.transport
    gloo = transport == "gloo"
    if transport == "none" and world > 1:
        raise SystemExit("--transport none is the one-GPU path")
    if gloo and not dist_on:
        raise SystemExit("--transport gloo needs torch.distributed.run")
    if args.shard == "rows" and not gloo:
        raise SystemExit("--shard rows needs --transport gloo (rt_render_gather deals 8x8 tiles)")
    if args.device is not None:
        if world > 1 and not gloo:
            raise SystemExit("--device with N > 1 needs --transport gloo (RCCL needs one GPU per rank)")
        local = args.device
    torch.cuda.set_device(local)
    if dist_on:
        # torch.distributed is the control plane only (the unique-id broadcast, barriers, the MAX
        # all-reduce of the step time), on the host; with --transport rccl every frame byte moves
        # through the library's own RCCL communicator (rt_render_gather)
        dist.init_process_group("gloo")
    device = torch.device("cuda", local)

    import __graft_entry__ as ge
    rt = ge.import_binding()          # after torch: one HIP runtime in the process

    W, H, spp, depth = args.width, args.height, args.spp, args.depth
    t_build = time.perf_counter()
    scene = rt.World(args.seed).build_scene(args.scene)
    cam, bg = rt.scene_camera(args.scene, W, H)
    renderer = rt.Renderer(local)
    renderer.upload(scene)
    f32 = args.precision == "f32"
    if f32:
        renderer.set_precision(rt.RT_PREC_F32)
    renderer.set_schedule(SCHEDULES[args.schedule])
    if args.buf_mb:
        renderer.set_option(rt.RT_OPT_TRACE_BUF_BYTES, args.buf_mb << 20)
    if args.no_overlap:
        renderer.set_option(rt.RT_OPT_BATCH_OVERLAP, 0)
    renderer.set_option(rt.RT_OPT_COMM_DIRECT, args.comm_direct)
    comm = None
    if transport == "rccl":   # rank 0 makes the RCCL unique id, torch (gloo) hands it to the others
        with stdout_to_stderr():   # RCCL's version banner: stdout carries the one JSON line alone
            uid = [rt.Comm.unique_id() if rank == 0 else None]
            if dist_on:
                dist.broadcast_object_list(uid, src=0)
            comm = rt.Comm(renderer, rank, world, uid[0])
    t_build = time.perf_counter() - t_build

    def progress(msg):   # stderr, one line per step: long configs (C5) keep the run visibly alive
        if rank == 0:
            print(f"bench: {msg}", file=sys.stderr, flush=True)

    def max_over_ranks(x):
        if not dist_on:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    # Ranks take the frame's 8x8 tiles round-robin (tile shards: every work tile stays a compact
    # 8x8 block of the image and every rank gets the same tile count to within one). Rank 0's C2
    # shard at N = 8 runs at 6,202 Msamples/s in 8x8 tiles against 5,993 as single rows 8 apart
    # (scripts/shard_coherence.py, profiles/r03u_shard.log). --shard rows keeps the row partition.
    tiles = transport != "none" and args.shard == "tiles"
    if tiles:
        n_mine = rt.tiles_in_shard(W, H, rank, world)
        n_max = max(rt.tiles_in_shard(W, H, r, world) for r in range(world))
        px_mine, slab_shape = 64 * n_mine, (8, 8 * n_max, 3)
    elif gloo:
        rows = rt.rows_in_shard(H, rank, world, ROW_BLOCK)
        rows_max = max(rt.rows_in_shard(H, r, world, ROW_BLOCK) for r in range(world))
        px_mine, slab_shape = rows * W, (rows_max, W, 3)
    else:
        px_mine, slab_shape = W * H, None
    frame_params = rt.Renderer.params(W, H, spp, depth, bg, args.seed, spp_chunk=args.spp_chunk,
                                      out_format=rt.RT_OUT_F64)
    # Tile order: cost = the tiles sorted by the lane-cycles of a count_work pass, most
    # expensive first, dealt round-robin. Every rank counts its own raster shard (1/N of a cost_spp
    # frame), one all-reduce sums the per-tile costs, and every rank sorts the same vector
    # (rt_comm_tile_order: RCCL, in the library; --transport gloo: the same steps over gloo here).
    # The pass is setup like the upload but not free: its time is amortised into `value`.
    order_mode = args.tile_order if args.tile_order != "auto" else ("cost" if world > 1 else "raster")
    tile_order, t_order, gloo_order = None, 0.0, None
    if tiles and order_mode == "cost":
        t0 = time.perf_counter()
        if comm is not None:
            try:   # a failed pass leaves every rank in raster order (RT_ERR_PEER on the others)
                comm.tile_order(cam, rt.Renderer.params(W, H, spp, depth, bg, args.seed), args.cost_spp)
            except rt.RTError as e:
                progress(f"tile-order cost pass failed, raster order: {e}")
        else:   # gloo: f64 and a pool schedule for the count (the chunk schedule counts no tile costs)
            n_img_tiles = ((W + 7) // 8) * ((H + 7) // 8)
            costs, ok = np.zeros(n_img_tiles, dtype=np.int64), 1
            try:
                renderer.set_tile_order(None)
                renderer.set_precision(rt.RT_PREC_F64)
                renderer.set_schedule(rt.RT_SCHED_POOL if args.schedule == "chunks" else SCHEDULES[args.schedule])
                renderer.render(cam, rt.Renderer.params(W, H, args.cost_spp, depth, bg, args.seed, row_begin=rank,
                                                        row_stride=world, tile_shard=1, count_work=1))
                c = renderer.tile_costs()
                if len(c) == n_img_tiles:
                    costs[:] = c.astype(np.int64)
                else:
                    ok = 0
            except rt.RTError:
                ok = 0
            finally:
                renderer.set_precision(rt.RT_PREC_F32 if f32 else rt.RT_PREC_F64)
                renderer.set_schedule(SCHEDULES[args.schedule])
            v = torch.from_numpy(np.concatenate([costs if ok else np.zeros_like(costs), [1 - ok]]))
            dist.all_reduce(v)   # every rank takes part, failed or not: no rank waits forever
            if int(v[-1]) == 0:
                gloo_order = rt.cost_tile_order(v[:-1].numpy().astype(np.uint64))
                renderer.set_tile_order(gloo_order)
            else:
                order_mode = "raster (cost pass failed on %d rank(s))" % int(v[-1])
        st = comm.stats() if comm is not None else None
        if st is not None and not st.tile_order:
            order_mode = "raster (cost pass failed)"
        tile_order = order_mode
        t_order = max_over_ranks(time.perf_counter() - t0)
    frame = torch.empty((H, W, 3), dtype=torch.float64, device=device) if rank == 0 else None
    # gloo: the render writes its shard contiguously at the start of a slab padded to the largest
    # shard (a tile shard's 8 x 8n layout is then a prefix of the 8 x 8n_max buffer), staged through
    # pinned host memory and gathered by gloo; rank 0 puts the slabs back in image order
    slab = torch.zeros(slab_shape, dtype=torch.float64, device=device) if gloo else None
    stage = torch.empty(slab.shape, dtype=slab.dtype, pin_memory=True) if gloo else None
    gathered = [torch.empty_like(stage) for _ in range(world)] if (gloo and rank == 0) else None
    # A stream of our own: torch's default stream has the null handle, which the C ABI reads as
    # "the context's stream" (a non-blocking stream the default stream does not wait for), so a
    # torch op on the frame would not be ordered after the render. Every op of a step runs on it.
    stream = torch.cuda.Stream(device)
    shard_params = rt.Renderer.params(W, H, spp, depth, bg, args.seed, row_begin=rank, row_stride=world,
                                      spp_chunk=args.spp_chunk, out_format=rt.RT_OUT_F64,
                                      row_block=1 if tiles else ROW_BLOCK, tile_shard=int(tiles))

    def assemble(slabs):
        if tiles:
            views = [g.reshape(-1)[: 3 * 64 * rt.tiles_in_shard(W, H, r, world)].view(8, -1, 3)
                     for r, g in enumerate(slabs)]
            rt.assemble_tiles(views, W, H, world, out=frame, order=gloo_order)
        else:
            rt.assemble_rows(slabs, H, world, out=frame, row_block=ROW_BLOCK)
    kernel_ms, gather_ms, render_ms = [], [], []

    def step(timed=False):
        with torch.cuda.stream(stream):
            if comm is not None:   # the product path at every N: rt_render_gather
                comm.render_gather_device(cam, frame_params, frame.data_ptr() if rank == 0 else None,
                                          stream.cuda_stream)
            elif gloo:
                renderer.render_device(cam, shard_params, slab.data_ptr(), stream.cuda_stream)
                stage.copy_(slab, non_blocking=True)
                stream.synchronize()
                tg = time.perf_counter()
                dist.gather(stage, gathered if rank == 0 else None, dst=0)
                if timed:
                    gather_ms.append((time.perf_counter() - tg) * 1e3)
                if rank == 0:
                    assemble([g.to(device, non_blocking=True) for g in gathered])
            else:
                renderer.render_device(cam, frame_params, frame.data_ptr(), stream.cuda_stream)

    def record():   # after the step's synchronize: HIP-event times of this rank's step
        if comm is not None:
            cs = comm.stats()
            kernel_ms.append(cs.kernel_ms)
            gather_ms.append(cs.gather_ms)
            render_ms.append(cs.render_ms)
        else:
            kernel_ms.append(renderer.stats().kernel_ms)   # HIP events around the trace kernel on `stream`

    for i in range(args.warmup):
        step()
        torch.cuda.synchronize(device)
        progress(f"warmup {i + 1}/{args.warmup}")
    torch.cuda.synchronize(device)
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    step_ends = []
    for i in range(args.steps):
        step(timed=True)
        torch.cuda.synchronize(device)
        step_ends.append(time.perf_counter())
        record()
        progress(f"step {i + 1}/{args.steps}: kernel {kernel_ms[-1]:.1f} ms")
    torch.cuda.synchronize(device)
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(device)
    elapsed = max_over_ranks(time.perf_counter() - t0)
    per_rank = None
    if dist_on:
        # per-rank kernel, render and gather times, so a multi-GPU line says where its time went
        mine = torch.tensor([float(np.mean(kernel_ms)) if kernel_ms else float("nan"),
                             float(np.mean(gather_ms)) if gather_ms else float("nan"),
                             float(np.mean(render_ms)) if render_ms else float("nan"),
                             float(px_mine * spp)], dtype=torch.float64)
        allr = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per_rank = [{"rank": r, "kernel_ms": round(float(v[0]), 3), "gather_ms": round(float(v[1]), 3),
                     "render_ms": round(float(v[2]), 3), "samples": int(v[3])} for r, v in enumerate(allr)]
    last = renderer.stats()
    direct = comm is not None and comm.stats().slab_bytes == 0   # the world-1 direct render (RT_OPT_COMM_DIRECT)

    samples_per_step = W * H * spp
    # the headline: the timed steps plus the tile-order cost pass amortised over them (the pass is
    # per (scene, camera, frame) setup, like the upload, but it renders); value_steady leaves it out
    value_steady = samples_per_step * args.steps / elapsed / 1e6
    value = samples_per_step * args.steps / (elapsed + t_order) / 1e6
    ms_per_step = (elapsed + t_order) / args.steps * 1e3
    k_ms = float(np.mean(kernel_ms)) if kernel_ms else float("nan")
    step_ms = [(b - a) * 1e3 for a, b in zip([t0] + step_ends[:-1], step_ends)]

    # ---- roofline: VALU issue (the binding resource), from the PMC pass of this build. The build
    # is the LOADED library's (rt_build_info, compiled in from __graft_entry__.source_hash()); a
    # library that does not match the sources next to it is a stale build, and no PMC record is
    # quoted for it
    src_hash = rt.build_info()
    tree_hash = ge.source_hash()
    workload = [args.scene, W, H, spp, depth, world, last.schedule] + ([1] if f32 else [])
    pmc, calib = pmc_entry(src_hash, workload) if src_hash == tree_hash else (None, None)
    roofline = {"bound": "valu", "achieved": None, "peak": None, "unit": "G SIMD-cycles/s", "frac": None,
                "traffic": None, "src_hash": src_hash, "src_hash_from": "rt_build_info (the loaded library)"}
    if src_hash != tree_hash:
        roofline["note"] = ("stale library: built from sources %s, the tree is %s; no PMC record quoted"
                            % (src_hash, tree_hash))
    elif pmc is not None and calib is not None:
        isa = isa_prices(src_hash, last.variant_features, last.schedule, last.slab32, int(last.lds_nodes > 0),
                         ring=getattr(last, "ring_bytes", 0) > 0)
        additive = valu_issue_cycles(pmc["counters"], calib, isa=isa)   # SIMD-cycles of VALU issue per launch
        rp = replay_price(calib, last.variant_features)
        # the kernel's mix replayed at saturation issues below the sum of its classes' costs
        # (calibration 'kmix'): price the launch at the replay's measured rate when there is one
        # the PMC record is per trace dispatch; a render in n equal buffer batches (C5: 256 chunks in
        # batches of 4) dispatches n of them inside the frame's kernel time
        nb = max(1, int(last.n_batches))
        additive *= nb
        need = pmc["counters"]["SQ_INSTS_VALU"] * nb * rp if rp else additive
        clk = pmc["clock_ghz"]                                   # the clock the chip held in that pass
        achieved = need / (k_ms * 1e-3) / 1e9                    # per live-timed launch
        peak = N_SIMDS * clk
        dram = pmc["dram_bytes"] * nb
        if isa:   # each class at the low / high end of its static-mix price
            ests = [nb * valu_issue_cycles(pmc["counters"], calib, isa=isa, bound=b) for b in (-1, 0, 1)]
        else:
            ests = [nb * valu_issue_cycles(pmc["counters"], calib, o)
                    for o in calib.get("other_range", [calib["cycles_per_inst"]["other"]] * 2)]
        lo, hi = (x / (k_ms * 1e-3) / 1e9 / peak for x in (min(ests + [need]), max(ests + [need])))
        roofline.update({
            "achieved": round(achieved, 1), "peak": round(peak, 1), "frac": round(achieved / peak, 4),
            "traffic": int(dram),
            "valu_lane_util": round(pmc["counters"]["SQ_THREAD_CYCLES_VALU"] /
                                    (64.0 * pmc["counters"]["SQ_INSTS_VALU"]), 4),
            "hbm": {"achieved": round(dram / (k_ms * 1e-3) / 1e9, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(dram / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)},
            "frac_range": [round(lo, 4), round(hi, 4)],
            "useful_frac": round(achieved / peak * pmc["counters"]["SQ_THREAD_CYCLES_VALU"] /
                                 (64.0 * pmc["counters"]["SQ_INSTS_VALU"]), 4),
            "pricing": ("SQ_INSTS_VALU x the measured cycles per instruction of this kernel's VALU mix replayed "
                        "at saturation (%s, %.3f); frac_range spans it and the additive per-class model" %
                        (KMIX_OF[last.variant_features], rp) if rp else
                        "per-class prices from this kernel's instruction mix (profiles/isa_mix.json)" if isa
                        else "calibration class means, 'other' bounded by its cheapest / dearest op"),
            "additive_frac": round(additive / (k_ms * 1e-3) / 1e9 / peak, 4),
            "model_check": {"mix": calib.get("mix"),
                            **{k: round(v["ratio"], 4) for k, v in (calib.get("kmix") or {}).items()}},
            "pmc_tag": pmc.get("tag"), "pmc_kernel_ms": pmc.get("kernel_ms"), "clock_ghz": clk,
            "pmc_dispatches_per_frame": nb})
    else:
        roofline["note"] = "no PMC pass of this build (source hash) and workload in profiles/pmc.json"

    # ---- SURVEY §8(d) algorithmic bytes per sample (LDS/L1/L2-served; not an HBM figure)
    count_spp = min(args.count_spp, spp)
    cs = None
    if not args.no_count and not f32:   # count_work is an f64-mode diagnostic
        cp = rt.Renderer.params(W, H, count_spp, depth, bg, args.seed, row_begin=rank, row_stride=world,
                                row_block=1 if tiles else ROW_BLOCK, tile_shard=int(tiles),
                                spp_chunk=min(args.spp_chunk, count_spp), out_format=rt.RT_OUT_F32, count_work=1)
        renderer.render(cam, cp)
        cs = renderer.stats()
    alg = None
    if cs is not None:
        bytes_per_sample = (cs.node_visits * cs.node_bytes + cs.prim_tests * cs.prim_bytes +
                            cs.casts * cs.material_bytes) / max(cs.samples, 1)
        alg = {"bytes_per_sample": round(bytes_per_sample, 1),
               "gbs": round(bytes_per_sample * px_mine * spp / (k_ms * 1e-3) / 1e9, 1),
               "casts_per_sample": round(cs.casts / max(cs.samples, 1), 4),
               "nodes_per_cast": round(cs.node_visits / max(cs.casts, 1), 3),
               "prims_per_cast": round(cs.prim_tests / max(cs.casts, 1), 3),
               "bounce_lane_occupancy": round(cs.casts / max(64 * cs.wave_steps, 1), 3),
               "node_lane_occupancy": round(cs.node_visits / max(64 * cs.wave_node_steps, 1), 3),
               "leaf_lane_occupancy": round(cs.prim_tests / max(64 * cs.wave_leaf_steps, 1), 3)}

    frame_np = frame.cpu().numpy() if rank == 0 else None   # f64 mean radiance, row 0 = bottom
    if args.ppm and rank == 0:
        rt.write_ppm(frame_np, args.ppm)   # f64: rt_write_ppm_f64, the reference's bytes
    if args.frame_npy and rank == 0:
        np.save(args.frame_npy, frame_np)

    progress("timed steps done; count pass, CPU baseline and parity")
    # ---- CPU baseline + parity (rank 0, N = 1 only)
    cpu, parity = None, None
    if rank == 0 and not dist_on and not args.no_cpu_baseline:
        from tests import oracle_binding as ob
        cores, n_aff, quota = usable_cores()
        # calibrate on `cores` interleaved rows at low spp, then take an interleaved subset of the
        # real workload's rows worth ~cpu_seconds, at full spp: the oracle deals pixels round-robin
        # over its threads, so even one row keeps every core busy, and the timed frame's own rows
        # are then compared at full spp on every config
        cal_stride = max(1, H // cores)
        _, st1 = ob.render(args.scene, W, H, min(spp, 16), depth, args.seed, args.seed, row_begin=0,
                           row_stride=cal_stride, threads=cores, return_stats=True)
        rate = st1.samples / max(st1.seconds, 1e-9)
        target = args.cpu_seconds * rate            # samples worth ~cpu_seconds
        n_rows = max(1, min(H, int(target / (W * spp))))
        stride = max(1, H // n_rows)
        row0 = stride // 2                          # rows y = row0 + k * stride, centred in their bands
        n_rows = len(range(row0, H, stride))
        # a row worth more than ~3 budgets takes the first spp_cpu samples of every pixel instead
        spp_cpu = spp if W * spp <= 3 * target else int(max(1, target // (n_rows * W)))
        ref_img, st = ob.render(args.scene, W, H, spp_cpu, depth, args.seed, args.seed, row_begin=row0,
                                row_stride=stride, threads=cores, return_stats=True)
        spp_note = "" if spp_cpu == spp else f", samples 0..{spp_cpu - 1} of each pixel"
        cpu = {"value": st.samples / st.seconds / 1e6, "unit": "Msamples/s", "cores": cores, "kind": "port",
               "sample": f"oracle (C, f64, recursive ray_color, linear hit_hittables scan) on rows y % {stride} == "
                         f"{row0} of the same {W}x{H}x{spp} depth-{depth} frame{spp_note}: {st.samples} samples in "
                         f"{st.seconds:.1f} s on {cores} threads (pixels round-robin)",
               "cpu_model": cpu_model(), "nproc": os.cpu_count(), "affinity": n_aff, "cgroup_quota": quota}
        # the reference's own decomposition: 10 threads, each all pixels x spp/10 samples
        # (main.rs:497-551, spp/thread_count at :516), the figure comparable to README.md:6
        n10 = max(1, int(args.t10_seconds * rate * min(10, cores) / cores / (W * spp)))
        stride10 = max(1, H // n10)
        _, st10 = ob.render(args.scene, W, H, spp, depth, args.seed, args.seed, row_begin=0, row_stride=stride10,
                            threads=10, split=ob.SPLIT_SAMPLES, return_stats=True)
        cpu["ref_split_t10"] = {
            "value": st10.samples / st10.seconds / 1e6, "unit": "Msamples/s", "threads": 10,
            "sample": f"rows y % {stride10} == 0, all {spp} spp split over 10 threads ({spp // 10} each, "
                      f"main.rs:516): {st10.samples} samples in {st10.seconds:.1f} s",
            "comparable_to": "README.md:6 (1200x800x500 in 1 h 10 min on 10 threads = 0.114 Msamples/s; "
                             "older book-1 scene revision, unknown CPU)"}
        # parity: the GPU renders exactly those rows and samples (f64 output) and the timed
        # frame's same rows (full spp only) are compared as well
        gp = rt.Renderer.params(W, H, spp_cpu, depth, bg, args.seed, row_begin=row0, row_stride=stride,
                                out_format=rt.RT_OUT_F64)
        gimg = renderer.render(cam, gp)
        d = np.abs(gimg - ref_img)
        parity = {"linf": float(d.max()), "max_rel": float((d / np.maximum(np.abs(ref_img), 1e-300)).max()),
                  "rows": n_rows, "row_begin": row0, "row_stride": stride, "spp": spp_cpu, "max_depth": depth,
                  "samples": int(st.samples), "tolerance": 1e-3, "pass": bool(d.max() <= 1e-3),
                  "vs": "oracle image of the cpu_baseline sample (same rows, samples, seeds)"}
        if f32:   # the f32 mode's paths are its own: statistical parity (tests/test_gpu_f32.py)
            mean_rel = abs(float(gimg.mean()) / float(ref_img.mean()) - 1.0)
            parity.update({"mode": "statistical (f32)", "mean_rel": mean_rel, "tolerance": 0.01,
                           "pass": bool(mean_rel < 0.01)})
        if spp_cpu == spp and not f32:
            parity["linf_timed_frame"] = float(np.abs(frame_np[row0::stride] - ref_img).max())
            # the timed frame's PPM bytes (rt_write_color) against the oracle's write_color of its image
            parity["ppm_bytes_equal_on_rows"] = bool(np.array_equal(rt.write_color(frame_np[row0::stride]),
                                                                    ob.write_color(ref_img)))

    if rank == 0:
        out = {
            "metric": ("Msamples/s (pixels x spp) for 1200x800 random-spheres scene" if args.config == "C2"
                       else "Msamples/s (pixels x spp), %s" % args.config),
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": args.precision,
            "data": "synthetic (seeded scene builders, scene_seed=render_seed=%d)" % args.seed,
            "value_steady": round(value_steady, 3),
            "value_basis": ("timed steps + the tile-order cost pass (%.3f s) amortised over them; value_steady: "
                            "the timed steps alone" % t_order) if t_order > 0 else "timed steps (no cost pass)",
            "config": {"workload": "%s %s %dx%d, %d spp, max depth %d, %s-sharded over %d GPU"
                                   % (args.config, SCENE_NAMES.get(args.scene, "scene %d" % args.scene), W, H, spp,
                                      depth, "tile" if tiles and not direct else "row" if gloo else "not", world),
                       "scene": args.scene, "width": W, "height": H, "spp": spp, "max_depth": depth,
                       "tile_order": order_mode if tiles else None,
                       "parallelism": "%s interleaved over %d rank(s), %s"
                                      % (("8x8 tiles (%s order)" % order_mode) if tiles and not direct else
                                         "rows" if gloo else "whole frame", world,
                                         "gloo gather (host-staged)" if gloo else
                                         "rt_render_gather of a world of one: straight into the frame, no gather "
                                         "(RT_OPT_COMM_DIRECT)" if direct else
                                         "RCCL gather (library communicator, rt_render_gather)" if comm is not None
                                         else "no gather")},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "parity": parity,
            "detail": {"kernel_ms_mean": round(k_ms, 3), "kernel_ms_median": round(float(np.median(kernel_ms)), 3),
                       "kernel_ms_steps": [round(x, 3) for x in kernel_ms],
                       "step_ms_median": round(float(np.median(step_ms)), 3) if step_ms else None,
                       "value_at_median_step": (round(samples_per_step / (float(np.median(step_ms)) * 1e-3) / 1e6, 3)
                                                if step_ms else None),
                       "reduce_ms": round(last.reduce_ms, 3), "ring_bytes": int(getattr(last, "ring_bytes", 0)),
                       "schedule": last.schedule, "n_batches": last.n_batches, "waves_per_simd": last.waves_per_simd, "spp_chunk": last.spp_chunk,
                       "trace_buf_bytes": int(last.trace_buf_bytes), "batches_overlapped": bool(last.overlapped),
                       "scene_bytes": int(last.scene_bytes), "scene_build_upload_s": round(t_build, 3),
                       "tile_order_pass_s": round(t_order, 3) if tile_order is not None else None,
                       "render_ms_mean": round(float(np.mean(render_ms)), 3) if render_ms else None,
                       "gather_ms_mean": round(float(np.mean(gather_ms)), 3) if gather_ms else None,
                       "algorithmic_bytes_survey_8d": alg},
        }
        if per_rank is not None:
            out["per_rank"] = per_rank
            out["distributed"] = {"transport": "gloo (host-staged)" if gloo else "RCCL (library communicator)",
                                  "control_plane": "torch.distributed gloo", "world_size": world,
                                  "forced_at_world_1": bool(args.force_dist and world == 1)}
        print(json.dumps(out), flush=True)
    if dist_on:   # every rank done with the communicator before any destroys it
        dist.barrier()
    if comm is not None:   # the RCCL communicator before the process group and the context
        comm.close()
    renderer.close()
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
