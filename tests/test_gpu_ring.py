"""The per-sample pool's in-kernel reduction (RT_OPT_POOL_RING, csrc/trace_device.hpp
ring_reduce) against the per-sample buffer + reduce_samples it replaces.

A work block is one tile x one chunk of samples and belongs to one wave; its samples wait in
that wave's ring and, when the last one ends, the wave sums every pixel's samples in sample
order from 0.0 — reduce_samples' chunk sum — and writes the chunk partial that reduce_chunks
adds up. Every image must therefore equal the per-sample buffer's bit for bit: ragged tiles,
spp not a multiple of the chunk, chunks of 1..16, row and tile shards, buffer batches,
progressive accumulation, every kernel variant, and the same count_work counters.
"""
import numpy as np
import pytest

from tests import oracle_binding as ob

pytestmark = pytest.mark.gpu

GIB = 1 << 30


def _render(rt, r, scene, W, H, spp, ring, world=None, sched=None, block=0, policy=None, **kw):
    """block: RT_OPT_BLOCK_SAMPLES (the ring runs only when a block is one chunk; small frames'
    blocks are otherwise cut to 4..8 samples, so the tests pass the chunk). policy: an explicit
    RT_OPT_POOL_RING value (default: 2 with ring, else 0)."""
    world = world or rt.World(1).build_scene(scene)
    cam, bg = rt.scene_camera(scene, W, H)
    # 2: whenever blocks allow (1, the default: when the per-sample buffer does not fit the bound)
    r.set_option(rt.RT_OPT_POOL_RING, policy if policy is not None else 2 if ring else 0)
    r.set_option(rt.RT_OPT_BLOCK_SAMPLES, block)
    if sched is not None:
        r.set_schedule(sched)
    r.upload(world)
    try:
        img = r.render(cam, rt.Renderer.params(W, H, spp, kw.pop("depth", 50), bg, 1, out_format=rt.RT_OUT_F64, **kw))
        st = r.stats()
    finally:
        r.set_option(rt.RT_OPT_POOL_RING, 1)
        r.set_option(rt.RT_OPT_BLOCK_SAMPLES, 0)
        r.set_schedule(rt.RT_SCHED_AUTO)
    return img, st


def _same(a, b, label):
    same = a == b
    assert same.all(), f"{label}: {int((~same.all(axis=-1)).sum())} px differ"


@pytest.mark.parametrize("scene,W,H,spp", [(0, 64, 40, 37), (0, 37, 21, 16), (0, 48, 32, 5), (7, 72, 40, 20),
                                           (1, 40, 24, 33), (5, 32, 32, 17), (6, 40, 40, 9), (2, 33, 17, 40)])
def test_ring_equals_per_sample_buffer(rt, renderer, scene, W, H, spp):
    """Both POOL forms on the scene's own variant (random spheres, final, two spheres, Cornell,
    Cornell smoke, Perlin): equal images; the ring form reports its ring and writes partials."""
    c = 4 if spp > 20 else min(16, spp)
    a, sa = _render(rt, renderer, scene, W, H, spp, 1, sched=rt.RT_SCHED_POOL, block=c, spp_chunk=c)
    b, sb = _render(rt, renderer, scene, W, H, spp, 0, sched=rt.RT_SCHED_POOL, block=c, spp_chunk=c)
    assert sa.schedule == sb.schedule == rt.RT_SCHED_POOL
    assert sa.ring_bytes > 0 and sb.ring_bytes == 0 and sa.trace_buf_bytes >= sa.ring_bytes
    _same(a, b, f"scene {scene}")


def test_ring_runs_at_full_blocks_and_is_bit_identical(rt, renderer):
    """A frame large enough that the automatic blocks stay one 16-sample chunk (C2 geometry at
    256 spp: 15,000 tiles x 16 chunks): the ring form runs under AUTO, equal to the per-sample buffer."""
    W, H, spp = 1200, 800, 256
    a, sa = _render(rt, renderer, 0, W, H, spp, 1, depth=8)
    b, sb = _render(rt, renderer, 0, W, H, spp, 0, depth=8)
    assert sa.schedule == rt.RT_SCHED_POOL and sa.ring_bytes > 0 and sb.ring_bytes == 0
    _same(a, b, "C2 rows")


@pytest.mark.parametrize("chunk", [1, 3, 7, 16])
def test_ring_chunk_sizes(rt, renderer, chunk):
    """Chunks of 1..16 samples (blocks of exactly one chunk): the ring sums each, the partials add
    in chunk order; spp 45 leaves a short last chunk."""
    W, H, spp = 512, 256, 45
    a, sa = _render(rt, renderer, 0, W, H, spp, 1, block=chunk, spp_chunk=chunk, depth=8)
    b, _ = _render(rt, renderer, 0, W, H, spp, 0, block=chunk, spp_chunk=chunk, depth=8)
    assert sa.spp_chunk == chunk and sa.ring_bytes > 0
    _same(a, b, f"chunk {chunk}")


def test_ring_shards_and_batches(rt):
    """Row shards, tile shards and a render in many (overlapped) buffer batches under the ring:
    every piece equals the one-launch render."""
    W, H, spp = 400, 240, 48   # chunks of 16 (spp_chunk below): blocks of one chunk, the ring's unit
    r = rt.Renderer(0)
    try:
        world = rt.World(1).build_scene(7)
        full, st = _render(rt, r, 7, W, H, spp, 1, world=world, block=16, spp_chunk=16)
        ref, _ = _render(rt, r, 7, W, H, spp, 0, world=world, block=16, spp_chunk=16)
        _same(full, ref, "whole")
        for rb in range(3):
            part, _ = _render(rt, r, 7, W, H, spp, 1, world=world, block=16, spp_chunk=16, row_begin=rb, row_stride=3)
            _same(part, full[rb::3], f"rows {rb}")
        slabs = [_render(rt, r, 7, W, H, spp, 1, world=world, block=16, spp_chunk=16, row_begin=t, row_stride=4, tile_shard=1)[0]
                 for t in range(4)]
        _same(rt.assemble_tiles(slabs, W, H, 4), full, "tiles")
        r.set_option(rt.RT_OPT_TRACE_BUF_BYTES, st.ring_bytes + (4 << 20))   # the ring + 1 chunk of partials (2.3 MB)
        batched, sb = _render(rt, r, 7, W, H, spp, 1, world=world, block=16, spp_chunk=16)
        assert sb.ring_bytes > 0 and sb.n_batches > 1
        _same(batched, full, "batches")
    finally:
        r.close()


def test_ring_progressive_accumulation(rt, renderer):
    """rt_accum_add in chunk-aligned pieces and rt_render_progressive under the ring: the
    one-launch image."""
    W, H, spp = 256, 160, 64
    world = rt.World(1).build_scene(0)
    cam, bg = rt.scene_camera(0, W, H)
    one, st = _render(rt, renderer, 0, W, H, spp, 0, world=world)   # per-sample buffer, one launch
    renderer.set_option(rt.RT_OPT_BLOCK_SAMPLES, 4)   # spp 64: chunks of 4 (blocks of one chunk: the ring)
    renderer.set_option(rt.RT_OPT_POOL_RING, 2)
    acc = None
    try:
        p = rt.Renderer.params(W, H, spp, 50, bg, 1, out_format=rt.RT_OUT_F64)
        prog = renderer.render_progressive(cam, p, 16)
        assert renderer.stats().ring_bytes > 0
        _same(prog, one, "progressive")
        acc = renderer.accumulator(p)
        for n in (16, 32, 16):
            acc.add(cam, p, n)
        _same(acc.resolve(out_format=rt.RT_OUT_F64), one, "accumulator")
    finally:
        renderer.set_option(rt.RT_OPT_BLOCK_SAMPLES, 0)
        renderer.set_option(rt.RT_OPT_POOL_RING, 1)
        if acc is not None:
            acc.close()


def test_ring_counts_the_same_work(rt, renderer):
    W, H, spp = 256, 128, 16
    a, sa = _render(rt, renderer, 7, W, H, spp, 1, block=16, spp_chunk=16, count_work=1)
    b, sb = _render(rt, renderer, 7, W, H, spp, 0, block=16, spp_chunk=16, count_work=1)
    assert sa.ring_bytes > 0
    assert (sa.casts, sa.node_visits, sa.prim_tests) == (sb.casts, sb.node_visits, sb.prim_tests)
    _same(a, b, "count_work")


def test_ring_against_oracle(rt, renderer):
    """The ring image against the oracle at C4 geometry (rows 72 apart, 24 spp)."""
    W, H, spp, rb, stride = 1920, 1080, 24, 5, 72
    img, st = _render(rt, renderer, 7, W, H, spp, 1, block=2, row_begin=rb, row_stride=stride)
    assert st.ring_bytes > 0 and st.spp_chunk == 2
    ref = ob.render(7, W, H, spp, 50, row_begin=rb, row_stride=stride, threads=16)
    d = np.abs(img - ref)
    assert float(d.max()) <= 1e-3
    assert not (d > 1e-9 * np.maximum(1.0, np.abs(ref))).any()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("scene,W,H,spp", [(0, 1200, 800, 500), (7, 1920, 1080, 1000)])
def test_default_trace_buffer_and_ring_policy(rt, scene, W, H, spp):
    """C2 and C4 at full size under the default bound (64 GiB, round 6): the per-sample buffer in
    one launch (measured as fast as the ring on C2 and 1.4 % faster on C4); under a 4 GiB bound the
    same frame takes the ring in one launch (chunk partials + ring <= 4 GiB); same bits."""
    r = rt.Renderer(0)
    try:
        assert r.get_option(rt.RT_OPT_TRACE_BUF_BYTES) <= 64 * GIB
        img, st = _render(rt, r, scene, W, H, spp, 1, policy=1)
        assert st.schedule == rt.RT_SCHED_POOL and st.ring_bytes == 0
        assert st.n_batches == 1 and st.trace_buf_bytes == W * H * spp * 24   # whole 8x8 tiles here
        r.set_option(rt.RT_OPT_TRACE_BUF_BYTES, 4 * GIB)
        ref, sr = _render(rt, r, scene, W, H, spp, 1, policy=1)
        assert sr.ring_bytes > 0 and sr.n_batches == 1 and sr.trace_buf_bytes <= 4 * GIB
        _same(img, ref, "full frame, buffer vs ring")
    finally:
        r.close()


def test_context_options_round_trip_and_reject_bad_values(rt):
    """rt_ctx_set_option / rt_ctx_get_option: every key round-trips, out-of-range values and
    unknown keys fail with RT_ERR_INVALID (no silent clamping)."""
    r = rt.Renderer(0)
    try:
        assert r.get_option(rt.RT_OPT_POOL_RING) == 1          # default: the ring when needed
        assert r.get_option(rt.RT_OPT_TRACE_BUF_BYTES) <= 64 * GIB
        for key, val in ((rt.RT_OPT_POOL_RING, 2), (rt.RT_OPT_POOL_RING, 0), (rt.RT_OPT_BLOCK_SAMPLES, 8),
                         (rt.RT_OPT_BLOCK_CHUNKS, 3), (rt.RT_OPT_BATCH_OVERLAP, 0),
                         (rt.RT_OPT_TRACE_BUF_BYTES, 64 << 20)):
            r.set_option(key, val)
            assert r.get_option(key) == val, key
        for key, val in ((rt.RT_OPT_POOL_RING, 3), (rt.RT_OPT_POOL_RING, -1), (7, 0), (8, 0), (999, 1)):
            with pytest.raises(rt.RTError):
                r.set_option(key, val)
        with pytest.raises(rt.RTError):
            r.get_option(999)
        # the removed wavefront schedule (ABI v4's 4) is refused as unsupported, not run as AUTO
        with pytest.raises(rt.RTError, match="RT_ERR_UNSUPPORTED"):
            r.set_schedule(4)
        with pytest.raises(rt.RTError, match="RT_ERR_INVALID"):
            r.set_schedule(5)
        r.set_option(rt.RT_OPT_TRACE_BUF_BYTES, 0)               # 0 restores the default
        assert 0 < r.get_option(rt.RT_OPT_TRACE_BUF_BYTES) <= 64 * GIB
    finally:
        r.close()
