"""GPU parity: the HIP megakernel (through the C ABI) against the CPU oracle.

Bar (BASELINE.json north_star): per-pixel L_inf <= 1e-3 on the linear mean radiance.
The kernel and the oracle follow the same paths (same seeded draws, same f64
operation order), so we also require a relative agreement of 1e-9: a single
diverged sample would move a pixel by ~1e-2, so this checks path identity; what is
left is only the summation order of the bounce loop (iterative on the GPU, recursive
in the reference).
"""
import os

import numpy as np
import pytest

from tests import oracle_binding as ob

pytestmark = pytest.mark.gpu

LINF = 1e-3          # north_star tolerance
REL = 1e-9           # path identity (f64 output)


def gpu_render(rt, renderer, scene_id, W, H, spp, depth=50, scene_seed=1, render_seed=1, row_begin=0,
               row_stride=1, spp_chunk=0, out_format=None):
    fmt = rt.RT_OUT_F64 if out_format is None else out_format
    img, _ = rt.render_scene(scene_id, W, H, spp, depth, scene_seed, render_seed, row_begin, row_stride, fmt,
                             spp_chunk, renderer=renderer)
    return img


def assert_parity(got, ref, label):
    assert got.shape == ref.shape, label
    assert np.all(np.isfinite(got)), label
    diff = np.abs(got - ref)
    linf = float(diff.max())
    assert linf <= LINF, f"{label}: L_inf {linf}"
    bad = diff > REL * np.maximum(1.0, np.abs(ref))
    assert not bad.any(), f"{label}: {int(bad.sum())} px differ beyond {REL} (max {linf})"


def test_device_numerics_bit_equal_host(rt, renderer):
    rng = np.random.default_rng(11)
    x = np.concatenate([rng.uniform(-50, 50, 4000), rng.uniform(-2e4, 2e4, 2000), [0.0, -0.0, np.inf, np.nan]])
    pos = np.concatenate([rng.uniform(0, 1, 4000), 2.0 ** -rng.uniform(0, 53, 2000), [0.0, 1.0, 5e-324, np.inf]])
    y = rng.normal(size=x.size)
    n = rng.normal(size=(3, 3000))
    n /= np.linalg.norm(n, axis=0)
    bits = rng.integers(0, 2 ** 63, size=5000, dtype=np.int64).astype(np.uint64).view(np.float64)
    # fn 13: the kernel's division through a correctly rounded reciprocal (div_rcp) against
    # IEEE division, incl. significands of all ones / powers of two, zeros and infinities
    ones = np.frombuffer(np.array([0x3FFFFFFFFFFFFFFF, 0x400FFFFFFFFFFFFF, 0x3FF0000000000000],
                                  dtype=np.uint64).tobytes(), dtype=np.float64)
    den = np.concatenate([y, rng.uniform(0.5, 3, 3000) * 2.0 ** rng.integers(-30, 30, 3000),
                          np.repeat(ones, 100) * 2.0 ** rng.integers(-20, 20, 300), [0.0, -0.0, np.inf, 1e-310]])
    num = np.concatenate([x, rng.uniform(-1e4, 1e4, 3000), rng.uniform(-10, 10, 300), [1.0, 0.0, 2.0, 3.0]])
    cases = {0: (x,), 1: (x,), 2: (pos,), 3: (x, y), 4: (np.clip(y / 3, -1, 1),), 5: tuple(n), 6: tuple(n),
             7: (pos,), 8: (np.abs(x),), 9: (x, y), 10: (bits,), 11: (bits,), 12: (x,), 13: (num, den)}
    for fn, args in cases.items():
        host = ob.evaluate(fn, *args)
        dev = renderer.device_eval(fn, *args)
        same = (host.view(np.uint64) == dev.view(np.uint64)) | (np.isnan(host) & np.isnan(dev))
        if fn == 13:  # a zero quotient may differ in sign (div_rcp's comment); any other value bit for bit
            same |= (host == 0.0) & (dev == 0.0)
        assert same.all(), f"fn {fn}: {int((~same).sum())} mismatches, e.g. {args[0][~same][:3]}"



def test_loaded_library_is_the_build_of_this_tree(built_from_tree):
    """The .so the GPU tier loads carries the source hash it was compiled from; it must be this
    tree's (a stale library would make every GPU result here evidence for another build)."""
    lib_hash, tree_hash = built_from_tree
    assert lib_hash == tree_hash, f"stale library: built from {lib_hash}, sources are {tree_hash}"


@pytest.mark.parametrize("scene_id,W,H,spp", [
    (0, 64, 48, 8),      # random spheres (C1/C2/C5 scene)
    (1, 48, 27, 4),      # two checker spheres
    (2, 48, 27, 4),      # perlin
    (3, 48, 27, 4),      # earth (image texture, sphere_uv)
    (4, 48, 27, 8),      # simple light
    (5, 40, 40, 8),      # cornell (C3 scene)
    (6, 40, 40, 8),      # cornell smoke (media with instanced box boundary)
    (7, 48, 27, 8),      # final scene (C4 scene)
])
def test_scene_parity(rt, renderer, scene_id, W, H, spp):
    got = gpu_render(rt, renderer, scene_id, W, H, spp)
    ref = ob.render(scene_id, W, H, spp)
    assert_parity(got, ref, f"scene {scene_id}")


def test_parity_other_seeds_and_depths(rt, renderer):
    for scene_seed, render_seed, depth in [(2, 9, 50), (3, 4, 8), (5, 77, 1), (1, 1, 2)]:
        got = gpu_render(rt, renderer, 0, 40, 24, 4, depth, scene_seed, render_seed)
        ref = ob.render(0, 40, 24, 4, depth, scene_seed, render_seed)
        assert_parity(got, ref, f"seeds {scene_seed}/{render_seed} depth {depth}")


def test_depth_zero_is_black(rt, renderer):
    got = gpu_render(rt, renderer, 0, 16, 8, 2, depth=0)
    assert np.all(got == 0.0)   # main.rs:21-23


def test_tiny_and_ragged_images(rt, renderer):
    for W, H, spp in [(2, 2, 1), (9, 7, 3), (67, 5, 2), (3, 65, 1)]:
        got = gpu_render(rt, renderer, 5, W, H, spp)
        ref = ob.render(5, W, H, spp)
        assert_parity(got, ref, f"{W}x{H}x{spp}")


def test_row_shards_reassemble_bit_exactly(rt, renderer):
    """Row sharding (the multi-GPU partition) does not change any pixel (keys are per pixel/sample)."""
    W, H, spp, G = 40, 30, 4, 4
    full = gpu_render(rt, renderer, 7, W, H, spp)
    for r in range(G):
        shard = gpu_render(rt, renderer, 7, W, H, spp, row_begin=r, row_stride=G)
        assert np.array_equal(shard, full[r::G]), r
    # bench.py's multi-GPU shards: 8-row bands round-robin (30 rows: the last band is cut)
    world = rt.World(1).build_scene(7)
    cam, bg = rt.scene_camera(7, W, H)
    renderer.upload(world)
    for G in (1, 2, 3):
        for r in range(G):
            p = rt.Renderer.params(W, H, spp, 50, bg, 1, row_begin=r, row_stride=G, row_block=8,
                                   out_format=rt.RT_OUT_F64)
            shard = renderer.render(cam, p)
            assert np.array_equal(shard, full[rt.shard_rows(H, r, G, 8)]), (G, r)


def test_tile_shards_reassemble_bit_exactly(rt, renderer):
    """Tile shards (rt_render_params.tile_shard: the frame's 8x8 tiles round-robin, bench.py's
    multi-GPU partition) reassemble into the full frame bit for bit, edge tiles included, under
    every schedule, on a wide and a tall frame."""
    world = rt.World(1).build_scene(7)
    renderer.upload(world)
    for (W, H, spp) in ((40, 30, 4), (17, 44, 2)):
        cam, bg = rt.scene_camera(7, W, H)
        full = renderer.render(cam, rt.Renderer.params(W, H, spp, 50, bg, 1, out_format=rt.RT_OUT_F64))
        for sched in (rt.RT_SCHED_POOL, rt.RT_SCHED_ITEMS, rt.RT_SCHED_CHUNKS):
            renderer.set_schedule(sched)
            for G in (1, 2, 3, 5):
                slabs = []
                for r in range(G):
                    p = rt.Renderer.params(W, H, spp, 50, bg, 1, row_begin=r, row_stride=G, tile_shard=1,
                                           out_format=rt.RT_OUT_F64)
                    slab = renderer.render(cam, p)
                    assert slab.shape == (8, 8 * rt.tiles_in_shard(W, H, r, G), 3)
                    slabs.append(slab)
                assert np.array_equal(rt.assemble_tiles(slabs, W, H, G), full), (W, H, sched, G)
    renderer.set_schedule(rt.RT_SCHED_AUTO)


def test_chunking_only_changes_rounding(rt, renderer):
    a = gpu_render(rt, renderer, 0, 32, 16, 12, spp_chunk=12)
    b = gpu_render(rt, renderer, 0, 32, 16, 12, spp_chunk=1)
    c = gpu_render(rt, renderer, 0, 32, 16, 12, spp_chunk=5)
    assert np.allclose(a, b, rtol=1e-12, atol=1e-14) and np.allclose(a, c, rtol=1e-12, atol=1e-14)
    ref = ob.render(0, 32, 16, 12, spp_chunk=5)
    assert np.array_equal(c, ref) or np.allclose(c, ref, rtol=REL, atol=0)


def test_f32_output_matches(rt, renderer):
    got = gpu_render(rt, renderer, 5, 32, 32, 4, out_format=rt.RT_OUT_F32)
    ref = ob.render(5, 32, 32, 4)
    assert got.dtype == np.float32
    assert np.max(np.abs(got - ref)) <= 1e-5 * max(1.0, float(np.abs(ref).max()))


def test_full_width_rows_c2_geometry(rt, renderer):
    """BASELINE config C2 geometry (1200x800, depth 50) on a bounded row subset at 2 spp."""
    W, H = 1200, 800
    got = gpu_render(rt, renderer, 0, W, H, 2, row_begin=5, row_stride=40)
    ref = ob.render(0, W, H, 2, row_begin=5, row_stride=40)
    assert_parity(got, ref, "C2 rows")


def test_count_work_mode(rt, renderer):
    world = rt.World(1).build_scene(0)
    cam, bg = rt.scene_camera(0, 120, 80)
    renderer.upload(world)
    p = rt.Renderer.params(120, 80, 8, 50, bg, 1, count_work=1, out_format=rt.RT_OUT_F64)
    counted = renderer.render(cam, p)
    st = renderer.stats()
    _, ost = ob.render(0, 120, 80, 8, return_stats=True)
    assert st.samples == 120 * 80 * 8
    assert st.casts == ost.casts            # same paths -> same number of hit_hittables calls
    assert st.node_visits > st.casts and st.prim_tests > st.casts
    p2 = rt.Renderer.params(120, 80, 8, 50, bg, 1, out_format=rt.RT_OUT_F64)
    assert np.array_equal(renderer.render(cam, p2), counted)


def test_custom_world_parity_against_preset(rt, renderer):
    """A world built through the constructor ABI renders like the same preset scene."""
    w = rt.World(1)
    red = w.lambertian(w.solid(0.65, 0.05, 0.05))
    white = w.lambertian(w.solid(0.73, 0.73, 0.73))
    green = w.lambertian(w.solid(0.12, 0.45, 0.15))
    light = w.diffuse_light(w.solid(15.0, 15.0, 15.0))
    w.push(w.yz_rect(green, 0, 555, 0, 555, 555))
    w.push(w.yz_rect(red, 0, 555, 0, 555, 0))
    w.push(w.xz_rect(light, 213, 343, 227, 332, 554))
    w.push(w.xz_rect(white, 0, 555, 0, 555, 0))
    w.push(w.xz_rect(white, 0, 555, 0, 555, 555))
    w.push(w.xy_rect(white, 0, 555, 0, 555, 555))
    w.push(w.translate(w.rotate_y(w.box((0, 0, 0), (165, 330, 165), white), 15.0), (265, 0, 295)))
    w.push(w.translate(w.rotate_y(w.box((0, 0, 0), (165, 165, 165), white), -18.0), (130, 0, 65)))
    cam, bg = rt.scene_camera(5, 32, 32)
    renderer.upload(w)
    got = renderer.render(cam, rt.Renderer.params(32, 32, 4, 50, bg, 1, out_format=rt.RT_OUT_F64))
    assert_parity(got, ob.render(5, 32, 32, 4), "custom cornell")


@pytest.mark.parametrize("scene_id,W,H", [(0, 48, 32), (5, 32, 32), (6, 32, 32), (7, 48, 27)])
def test_kernel_variants_identical(rt, renderer, scene_id, W, H):
    """The variant knobs (f32/f64 slab tests, LDS/scratch traversal stack, TLAS in LDS)
    only change speed: the image is bit-identical, and equal to the oracle's."""
    world = rt.World(1).build_scene(scene_id)
    cam, bg = rt.scene_camera(scene_id, W, H)
    renderer.upload(world)
    p = rt.Renderer.params(W, H, 4, 50, bg, 1, out_format=rt.RT_OUT_F64)
    imgs = []
    for v in [(1, 1, 1), (0, 0, 0), (1, 1, 0), (0, 1, 1), (1, 0, 1)]:
        renderer.set_variant(*v)
        imgs.append(renderer.render(cam, p))
    renderer.set_variant(1, 1, 1)
    for im in imgs[1:]:
        assert np.array_equal(im, imgs[0])
    assert_parity(imgs[0], ob.render(scene_id, W, H, 4), f"variants scene {scene_id}")


@pytest.mark.parametrize("scene_id,W,H,feat", [(0, 40, 24, 0), (5, 24, 24, 1 | 2 | 32), (6, 24, 24, 1 | 2 | 4 | 32 | 64),
                                              (7, 32, 18, 31 | 256)])
def test_feature_set_variants_identical(rt, renderer, scene_id, W, H, feat):
    """Each scene runs on the smallest feature-set variant covering it (final scene: instances
    over spheres only, media bounded by spheres); the all-features variant, which no reference
    scene selects, renders the same bits (RT_OPT_EXTRA_FEATURES forces it)."""
    world = rt.World(1).build_scene(scene_id)
    cam, bg = rt.scene_camera(scene_id, W, H)
    p = rt.Renderer.params(W, H, 4, 50, bg, 1, out_format=rt.RT_OUT_F64)
    renderer.upload(world)
    img = renderer.render(cam, p)
    assert renderer.stats().variant_features == feat
    big = rt.Renderer(0)
    big.set_option(rt.RT_OPT_EXTRA_FEATURES, 4095)   # incl. FEAT_NEST_MOVING: nested spheres as moving
    try:
        big.upload(world)
        img_all = big.render(cam, p)
        assert big.stats().variant_features == 4095
    finally:
        big.close()
    assert np.array_equal(img, img_all)
    assert_parity(img, ob.render(scene_id, W, H, 4), f"feature variant scene {scene_id}")


def test_cornell_variant_occupancy(rt, renderer):
    """The Cornell scenes have no BVH node (one top-level leaf; instances over one box): they
    run the f64-slab instantiation of the rects + instances variant without the nested BLAS
    walk, whose registers fit 4 waves per SIMD; the spheres variant with the whole TLAS in
    LDS and 16-bit stack entries (Stack16) runs at 6 (80 VGPRs, 768-thread workgroups; 5 until
    round 6); the final scene's variant (128 VGPRs) at 4, its deferred instance walk sharing the
    top-level walk's LDS stack (13 entries, not 25)."""
    for scene_id, waves in ((5, 4), (0, 6), (7, 4)):
        world = rt.World(1).build_scene(scene_id)
        cam, bg = rt.scene_camera(scene_id, 16, 16)
        renderer.upload(world)
        renderer.render(cam, rt.Renderer.params(16, 16, 2, 50, bg, 1, out_format=rt.RT_OUT_F64))
        st = renderer.stats()
        assert st.waves_per_simd == waves, (scene_id, st.waves_per_simd)
        assert st.slab32 == (0 if scene_id == 5 else 1)


def _golden_cases():
    from tests.golden import make_golden as mg
    return mg.CASES, mg.key


@pytest.mark.parametrize("case", _golden_cases()[0], ids=[_golden_cases()[1](c) for c in _golden_cases()[0]])
def test_kernel_matches_committed_golden(rt, renderer, case):
    """The committed oracle renders (tests/golden/oracle_renders.npz, make_golden.py)."""
    import os
    _, key = _golden_cases()
    gold = np.load(os.path.join(os.path.dirname(__file__), "golden", "oracle_renders.npz"))[key(case)]
    s, w, h, spp, d, ss, rs = case
    got = gpu_render(rt, renderer, s, w, h, spp, d, ss, rs)
    assert_parity(got, gold, key(case))


def test_earth_matches_reference_output_on_gpu(rt, renderer):
    """The megakernel's earth render against the reference's own earth.ppm (see test_oracle)."""
    import os
    from PIL import Image
    ref = np.asarray(Image.open(os.path.join(os.path.dirname(__file__), "golden", "ref_earth_400x225.png")),
                     dtype=np.int32)
    img = gpu_render(rt, renderer, 3, 400, 225, 100)
    mine = (256.0 * np.clip(np.sqrt(img[::-1]), 0.0, 0.999)).astype(np.int32)
    bg = (256.0 * np.clip(np.sqrt(np.array([0.7, 0.8, 1.0])), 0, 0.999)).astype(np.int32)
    sphere = np.any(mine != bg, axis=2)
    a, b = ref[sphere].astype(float), mine[sphere].astype(float)
    for c in range(3):
        assert np.corrcoef(a[:, c], b[:, c])[0, 1] > 0.99


@pytest.mark.parametrize("scene_id,W,H", [(0, 40, 24), (5, 24, 24), (6, 24, 24), (7, 32, 18)])
def test_accel_modes_render_identically(rt, renderer, scene_id, W, H):
    """the LINEAR (hit_hittables scan) and MEDIAN (reference BvhNode) hierarchies
    give the SAH image bit for bit (closest hit does not depend on the hierarchy), and all
    three match the oracle, which walks the reference's own median BVH."""
    imgs = {}
    for accel in (rt.RT_ACCEL_SAH, rt.RT_ACCEL_LINEAR, rt.RT_ACCEL_MEDIAN):
        imgs[accel], _ = rt.render_scene(scene_id, W, H, 4, out_format=rt.RT_OUT_F64, renderer=renderer, accel=accel)
    assert np.array_equal(imgs[rt.RT_ACCEL_LINEAR], imgs[rt.RT_ACCEL_SAH])
    assert np.array_equal(imgs[rt.RT_ACCEL_MEDIAN], imgs[rt.RT_ACCEL_SAH])
    assert_parity(imgs[rt.RT_ACCEL_MEDIAN], ob.render(scene_id, W, H, 4), f"median scene {scene_id}")


def test_linear_mode_tests_every_primitive_per_cast(rt, renderer):
    """A LINEAR walk is the reference's list scan: every cast visits every chain node and
    tests every top-level primitive (random scene: no instances or media)."""
    world = rt.World(1).build_scene(0)
    soa = rt.SceneSoA.from_buffer_copy(world.flatten(rt.RT_ACCEL_LINEAR))
    cam, bg = rt.scene_camera(0, 48, 32)
    renderer.upload(world, rt.RT_ACCEL_LINEAR)
    renderer.render(cam, rt.Renderer.params(48, 32, 4, 50, bg, 1, count_work=1, out_format=rt.RT_OUT_F64))
    st = renderer.stats()
    assert st.prim_tests == st.casts * soa.n_prims
    assert st.node_visits == st.casts * soa.n_nodes
    renderer.upload(world)


def _final_setup(rt, renderer, W=32, H=18):
    world = rt.World(1).build_scene(7)       # every feature, incl. media (keyed in-hit draws)
    cam, bg = rt.scene_camera(7, W, H)
    renderer.upload(world)
    return cam, bg


def test_progressive_batches_equal_one_render(rt, renderer):
    """batches split at chunk boundaries sum in rt_render's order (bit-identical);
    the progress callback sees every batch; the accumulator composes per row shard."""
    W, H, spp = 32, 18, 40                   # auto chunk = ceil(40/16) = 3
    cam, bg = _final_setup(rt, renderer, W, H)
    p = rt.Renderer.params(W, H, spp, 50, bg, 1, out_format=rt.RT_OUT_F64)
    one = renderer.render(cam, p)
    seen = []
    prog = renderer.render_progressive(cam, p, 5, lambda done, total: seen.append((done, total)))  # 5 -> 6
    assert np.array_equal(prog, one)
    assert seen == [(d, spp) for d in (6, 12, 18, 24, 30, 36, 40)]
    acc = renderer.accumulator(p)
    for n in (3, 9, 6, 22):
        acc.add(cam, p, n)
    assert acc.samples_done == 40
    assert np.array_equal(acc.resolve(out_format=rt.RT_OUT_F64), one)
    assert np.array_equal(acc.resolve(), one.astype(np.float32))
    assert_parity(one, ob.render(7, W, H, spp), "final 40 spp")


def test_accumulator_checkpoint_resume(rt, renderer):
    """Checkpoint after 12 samples, restore into a fresh accumulator (the resumable C5 run),
    finish: identical to the uninterrupted render."""
    W, H, spp = 32, 18, 24
    cam, bg = _final_setup(rt, renderer, W, H)
    p = rt.Renderer.params(W, H, spp, 50, bg, 7, row_begin=1, row_stride=2, out_format=rt.RT_OUT_F64)
    one = renderer.render(cam, p)
    a = renderer.accumulator(p)
    a.add(cam, p, 12)
    sums, done = a.checkpoint()
    a.close()
    b = renderer.accumulator(p)
    b.restore(sums, done)
    b.add(cam, p, spp - done)
    assert np.array_equal(b.resolve(out_format=rt.RT_OUT_F64), one)


def test_progressive_early_stop_and_divisor(rt, renderer):
    W, H = 24, 16
    cam, bg = _final_setup(rt, renderer, W, H)
    p = rt.Renderer.params(W, H, 32, 50, bg, 1, spp_chunk=4, out_format=rt.RT_OUT_F64)
    stop = renderer.render_progressive(cam, p, 8, lambda done, total: done >= 8)
    ref8 = ob.render(7, W, H, 8, spp_chunk=4)       # the first 8 samples of every pixel
    assert_parity(stop, ref8, "stopped after 8")
    # the reference's truncation (spp / thread_count samples per thread, divided by spp):
    acc = renderer.accumulator(p)
    acc.add(cam, p, 30)
    a = acc.resolve(out_format=rt.RT_OUT_F64)
    b = acc.resolve(32.0, out_format=rt.RT_OUT_F64)
    assert np.allclose(b, a * (30.0 / 32.0), rtol=1e-14, atol=0)
    q = rt.Renderer.params(W, H, 32, 50, bg, 1, row_begin=1, out_format=rt.RT_OUT_F64)
    with pytest.raises(rt.RTError):
        acc.add(cam, q, 2)                          # another shard


@pytest.mark.parametrize("scene_id,W,H,spp", [(0, 40, 24, 8), (5, 24, 24, 8), (6, 24, 24, 8), (7, 32, 18, 8)])
def test_schedules_render_identically(rt, scene_id, W, H, spp):
    """The three schedules give the same bits: chunks; the per-sample pool (persistent
    waves, per-lane refill, [sample][pixel] buffer); the item pool (persistent waves, a lane
    takes a whole (pixel, chunk) item). So do the pools split into many buffer batches
    (RT_OPT_TRACE_BUF_BYTES), at ragged sizes and with row shards."""
    world = rt.World(1).build_scene(scene_id)
    cam, bg = rt.scene_camera(scene_id, W, H)
    imgs = []
    small = rt.Renderer(0)
    small.set_option(rt.RT_OPT_TRACE_BUF_BYTES, 1 << 20)
    small.set_option(rt.RT_OPT_POOL_RING, 0)          # the per-sample buffer's batches (ring: test_gpu_ring.py)
    grouped = rt.Renderer(0)                         # item-pool blocks of 3 chunks, pool blocks of 5 samples
    grouped.set_option(rt.RT_OPT_BLOCK_CHUNKS, 3)
    grouped.set_option(rt.RT_OPT_BLOCK_SAMPLES, 5)
    serial = rt.Renderer(0)                          # buffer batches one after another in one buffer
    serial.set_option(rt.RT_OPT_TRACE_BUF_BYTES, 1 << 20)
    serial.set_option(rt.RT_OPT_BATCH_OVERLAP, 0)
    serial.set_option(rt.RT_OPT_POOL_RING, 0)
    r = rt.Renderer(0)
    runs = [(r, rt.RT_SCHED_CHUNKS), (r, rt.RT_SCHED_POOL), (r, rt.RT_SCHED_ITEMS), (small, rt.RT_SCHED_POOL),
            (small, rt.RT_SCHED_ITEMS), (grouped, rt.RT_SCHED_ITEMS), (r, rt.RT_SCHED_AUTO),
            (serial, rt.RT_SCHED_POOL), (serial, rt.RT_SCHED_ITEMS)]
    for rr, sched in runs:
        rr.set_schedule(sched)
        rr.upload(world)
        imgs.append(rr.render(cam, rt.Renderer.params(W, H, spp, 50, bg, 1, row_begin=1, row_stride=2,
                                                      out_format=rt.RT_OUT_F64)))
        # AUTO: the item pool for the Cornell box (scene 5), the per-sample pool otherwise
        auto = rt.RT_SCHED_ITEMS if scene_id == 5 else rt.RT_SCHED_POOL
        assert rr.stats().schedule == (sched if sched != rt.RT_SCHED_AUTO else auto)
    for im in imgs[1:]:
        assert np.array_equal(imgs[0], im)
    q = rt.Renderer.params(64, 48, 40, 50, bg, 1, out_format=rt.RT_OUT_F64)   # 73.7 KB per sample
    r.set_schedule(rt.RT_SCHED_ITEMS)
    one = r.render(cam, q)
    assert r.stats().n_batches == 1
    small.set_schedule(rt.RT_SCHED_POOL)
    batched = small.render(cam, q)
    # 256-thread-workgroup variants (Cornell scenes): overlapped, 5 x 7 + 5 samples in the bound's
    # halves, chunks of 3 straddle batches; the random and final scenes' variants (768 / 1024
    # threads) run their batches in order, 14 + 14 + 12 samples (abi.cpp, RT_OPT_BATCH_OVERLAP)
    assert small.stats().n_batches == (6 if scene_id in (5, 6) else 3)
    assert np.array_equal(batched, one)
    serial.set_schedule(rt.RT_SCHED_POOL)
    assert np.array_equal(serial.render(cam, q), one)
    assert serial.stats().n_batches == 3             # 14 + 14 + 12 samples in the whole bound, in order
    serial.close()
    acc = small.accumulator(q)                       # an accumulator batch straddling buffer batches
    acc.add(cam, q, 21)
    acc.add(cam, q, 19)
    ref3 = r.render(cam, rt.Renderer.params(64, 48, 40, 50, bg, 1, spp_chunk=3, out_format=rt.RT_OUT_F64))
    assert np.array_equal(acc.resolve(out_format=rt.RT_OUT_F64), ref3)
    # item pool in buffer batches of whole chunks: 256x192 px x 24 B > 1 MB, one chunk per launch
    q2 = rt.Renderer.params(256, 192, 12, 50, bg, 1, out_format=rt.RT_OUT_F64)
    small.set_schedule(rt.RT_SCHED_ITEMS)
    b2 = small.render(cam, q2)
    assert small.stats().n_batches == 12
    assert np.array_equal(b2, r.render(cam, q2))
    grouped.set_schedule(rt.RT_SCHED_ITEMS)
    assert np.array_equal(grouped.render(cam, q2), b2)
    grouped.upload(world)
    assert np.array_equal(grouped.render(cam, q), one)   # 40 spp: chunks of 3, groups of 3 chunks
    grouped.set_schedule(rt.RT_SCHED_POOL)
    assert np.array_equal(grouped.render(cam, q), one)   # pool blocks of 5 samples across chunks of 3
    grouped.close()
    assert_parity(imgs[2], ob.render(scene_id, W, H, spp, row_begin=1, row_stride=2), f"items scene {scene_id}")


def test_renders_on_two_streams_are_ordered(rt, renderer):
    """a render enqueued on a caller's stream and an immediate render on the
    context's own stream share the context's scratch buffers; the second must be ordered
    after the first (no host sync in between). Both frames must equal separate renders."""
    import torch
    W, H, spp = 320, 240, 32
    world = rt.World(1).build_scene(0)
    cam, bg = rt.scene_camera(0, W, H)
    renderer.upload(world)
    pa = rt.Renderer.params(W, H, spp, 50, bg, 1, out_format=rt.RT_OUT_F32)
    pb = rt.Renderer.params(W, H, 4, 50, bg, 2, out_format=rt.RT_OUT_F32)
    ref_a = renderer.render(cam, pa)
    ref_b = renderer.render(cam, rt.Renderer.params(W, H, 4, 50, bg, 2, out_format=rt.RT_OUT_F32))
    stream = torch.cuda.Stream(torch.device("cuda", 0))
    slab = torch.zeros((H, W, 3), dtype=torch.float32, device="cuda:0")
    renderer.render_device(cam, pa, slab.data_ptr(), stream.cuda_stream)   # enqueued, not waited for
    got_b = renderer.render(cam, pb)                                       # context stream, synchronous
    torch.cuda.synchronize()
    assert np.array_equal(got_b, ref_b)
    assert np.array_equal(slab.cpu().numpy(), ref_a)


@pytest.mark.parametrize("sched", ["AUTO", "POOL", "ITEMS", "CHUNKS"])
def test_empty_shards_render_nothing(rt, renderer, sched):
    """a shard with no tiles (a rank past the frame's tile count) or no rows is
    valid input. rt_render (host and device output, the bench's padded slab), rt_accum_add /
    resolve and rt_render_progressive return RT_OK and write nothing; no division by the shard's
    size. The next non-empty render on the same context is unaffected."""
    import torch
    W, H, spp = 16, 16, 4                        # 2 x 2 = 4 tiles
    world = rt.World(1).build_scene(0)
    cam, bg = rt.scene_camera(0, W, H)
    renderer.upload(world)
    renderer.set_schedule(getattr(rt, "RT_SCHED_" + sched))
    try:
        assert rt.tiles_in_shard(W, H, 5, 8) == 0 and rt.rows_in_shard(H, 17, 4) == 0
        shards = [dict(row_begin=5, row_stride=8, tile_shard=1), dict(row_begin=17, row_stride=4)]
        for sh in shards:
            p = rt.Renderer.params(W, H, spp, 50, bg, 1, out_format=rt.RT_OUT_F64, **sh)
            img = renderer.render(cam, p)
            assert img.size == 0
            st = renderer.stats()
            assert st.samples == 0
            # device output into a non-empty padded slab (bench.py at N > 1): left untouched
            slab = torch.full((8, 16, 3), 7.0, dtype=torch.float64, device="cuda:0")
            stream = torch.cuda.Stream()
            renderer.render_device(cam, p, slab.data_ptr(), stream.cuda_stream)
            stream.synchronize()
            assert bool((slab == 7.0).all())
            acc = renderer.accumulator(p)
            acc.add(cam, p, spp)
            assert acc.samples_done == spp
            assert acc.resolve(out_format=rt.RT_OUT_F64).size == 0
            acc.close()
            assert renderer.render_progressive(cam, p, 2).size == 0
        full = renderer.render(cam, rt.Renderer.params(W, H, spp, 50, bg, 1, out_format=rt.RT_OUT_F64))
        ref = ob.render(0, W, H, spp)
        assert np.abs(full - ref).max() <= 1e-12
    finally:
        renderer.set_schedule(rt.RT_SCHED_AUTO)
