"""Tile orders for tile shards (rt_ctx_set_tile_order, rt_last_tile_costs; ABI v4): the
multi-GPU partition of main.rs:497-551 rebalanced by measured tile cost.

A tile order only changes which 8x8 tiles a shard renders (and in which order), never a pixel's
bits: the shards of any order reassemble into the one-launch frame bit for bit, under every
schedule, with the in-kernel reduction ring, across buffer batches and on every variant.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _frame(rt, r, cam, bg, W, H, spp, **kw):
    return r.render(cam, rt.Renderer.params(W, H, spp, 50, bg, 1, out_format=rt.RT_OUT_F64, **kw))


def _shards(rt, r, cam, bg, W, H, spp, world, **kw):
    return [_frame(rt, r, cam, bg, W, H, spp, row_begin=k, row_stride=world, tile_shard=1, **kw) for k in range(world)]


@pytest.mark.parametrize("scene,W,H,spp", [(0, 64, 40, 12), (7, 48, 27, 6), (5, 40, 40, 8), (6, 24, 40, 4)])
def test_tile_order_shards_reassemble_bit_exactly(rt, renderer, scene, W, H, spp):
    """A random permutation and the cost order of a count_work pass: every shard count and
    schedule reassembles into the frame rendered without an order, bit for bit."""
    world_ = rt.World(1).build_scene(scene)
    cam, bg = rt.scene_camera(scene, W, H)
    renderer.upload(world_)
    full = _frame(rt, renderer, cam, bg, W, H, spp)
    tiles = ((W + 7) // 8) * ((H + 7) // 8)
    _frame(rt, renderer, cam, bg, W, H, 2, count_work=1)
    costs = renderer.tile_costs()
    assert len(costs) == tiles and (costs > 0).all()   # every tile's samples took time
    orders = [np.random.default_rng(scene).permutation(tiles), rt.cost_tile_order(costs)]
    try:
        for order in orders:
            renderer.set_tile_order(order)
            for sched in (rt.RT_SCHED_AUTO, rt.RT_SCHED_POOL, rt.RT_SCHED_ITEMS, rt.RT_SCHED_CHUNKS):
                renderer.set_schedule(sched)
                for world in (1, 3, 8):
                    slabs = _shards(rt, renderer, cam, bg, W, H, spp, world)
                    for k, s in enumerate(slabs):
                        assert s.shape == (8, 8 * rt.tiles_in_shard(W, H, k, world), 3)
                    got = rt.assemble_tiles(slabs, W, H, world, order=order)
                    assert np.array_equal(got, full), (scene, sched, world)
            # a full-frame render ignores the order
            assert np.array_equal(_frame(rt, renderer, cam, bg, W, H, spp), full)
    finally:
        renderer.set_tile_order(None)
        renderer.set_schedule(rt.RT_SCHED_AUTO)


def test_tile_order_with_ring_and_batches(rt, renderer):
    """The per-sample pool's in-kernel reduction and overlapped buffer batches under a tile
    order: equal to the one-launch frame."""
    W, H, spp = 200, 120, 48
    world_ = rt.World(1).build_scene(7)
    cam, bg = rt.scene_camera(7, W, H)
    renderer.upload(world_)
    renderer.set_option(rt.RT_OPT_BLOCK_SAMPLES, 16)
    try:
        full = _frame(rt, renderer, cam, bg, W, H, spp, spp_chunk=16)
        _frame(rt, renderer, cam, bg, W, H, 4, count_work=1)
        order = rt.cost_tile_order(renderer.tile_costs())
        renderer.set_tile_order(order)
        renderer.set_option(rt.RT_OPT_POOL_RING, 2)
        slabs = _shards(rt, renderer, cam, bg, W, H, spp, 4, spp_chunk=16)
        assert renderer.stats().ring_bytes > 0
        assert np.array_equal(rt.assemble_tiles(slabs, W, H, 4, order=order), full)
        renderer.set_option(rt.RT_OPT_TRACE_BUF_BYTES, renderer.stats().ring_bytes + 200_000)   # ~1.4 chunks of partials
        slabs = _shards(rt, renderer, cam, bg, W, H, spp, 4, spp_chunk=16)
        assert renderer.stats().n_batches > 1
        assert np.array_equal(rt.assemble_tiles(slabs, W, H, 4, order=order), full)
    finally:
        renderer.set_tile_order(None)
        for key, v in ((rt.RT_OPT_POOL_RING, 1), (rt.RT_OPT_BLOCK_SAMPLES, 0), (rt.RT_OPT_TRACE_BUF_BYTES, 0)):
            renderer.set_option(key, v)


def test_tile_order_is_checked(rt, renderer):
    """Not a permutation, or a permutation of another frame's tiles: RT_ERR_INVALID, nothing
    rendered; tile costs exist only after a count_work render on a pool schedule."""
    W, H = 32, 24   # 12 tiles
    world_ = rt.World(1).build_scene(0)
    cam, bg = rt.scene_camera(0, W, H)
    renderer.upload(world_)
    try:
        for bad in ([0, 1, 1], [0, 5, 1], [3, 1, 2]):
            with pytest.raises(RuntimeError):
                renderer.set_tile_order(np.array(bad))
        renderer.set_tile_order(np.arange(11))                  # 11 tiles: another frame's order
        with pytest.raises(RuntimeError):
            _frame(rt, renderer, cam, bg, W, H, 2, row_begin=0, row_stride=2, tile_shard=1)
        _frame(rt, renderer, cam, bg, W, H, 2)                  # row renders do not use it
        renderer.set_tile_order(None)
        _frame(rt, renderer, cam, bg, W, H, 2)
        assert len(renderer.tile_costs()) == 0                   # no count_work
        renderer.set_schedule(rt.RT_SCHED_CHUNKS)
        _frame(rt, renderer, cam, bg, W, H, 2, count_work=1)
        assert len(renderer.tile_costs()) == 0                   # the chunk schedule counts none
        renderer.set_schedule(rt.RT_SCHED_POOL)
        _frame(rt, renderer, cam, bg, W, H, 2, count_work=1)
        assert len(renderer.tile_costs()) == 12
    finally:
        renderer.set_tile_order(None)
        renderer.set_schedule(rt.RT_SCHED_AUTO)
