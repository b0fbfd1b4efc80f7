"""The N > 1 path on CPU: world_size-2 (and 3) gloo process groups, each rank renders its
interleaved row shard (with the CPU oracle, no GPU here), rank 0 gathers the padded slabs
the way bench.py does over RCCL and re-interleaves them; the frame must equal the
single-process render bit-for-bit (every draw is keyed by pixel and sample). Tile shards
(rt_render_params.tile_shard, bench.py's default for N > 1): the documented slab layout,
gathered and reassembled the same way."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests import oracle_binding as ob

W, H, SPP, SCENE = 24, 19, 3, 7


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank, world, port, out_path):
    import __graft_entry__ as ge
    rt = ge.import_binding()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rows_max = (H + world - 1) // world
    mine = ob.render(SCENE, W, H, SPP, row_begin=rank, row_stride=world, threads=1)
    assert mine.shape[0] == rt.rows_in_shard(H, rank, world) == len(rt.shard_rows(H, rank, world))
    slab = torch.zeros((rows_max, W, 3), dtype=torch.float64)
    slab[: mine.shape[0]] = torch.from_numpy(mine)
    gathered = [torch.empty_like(slab) for _ in range(world)] if rank == 0 else None
    dist.gather(slab, gathered, dst=0)
    if rank == 0:
        frame = rt.assemble_rows([g.numpy() for g in gathered], H, world)
        np.save(out_path, frame)
    dist.barrier()
    dist.destroy_process_group()


def tile_slab(frame, rank, world, order=None):
    """Rank `rank`'s tile shard of a frame in the layout rt_render writes (rt_abi.h tile_shard):
    the tiles at positions t = rank + m*world (raster tile t, or order[t] with a tile order) of
    the 8x8 tile grid side by side in one 8-row slab."""
    H, W = frame.shape[:2]
    tx, ty = (W + 7) // 8, (H + 7) // 8
    pad = np.zeros((ty * 8, tx * 8) + frame.shape[2:], frame.dtype)
    pad[:H, :W] = frame
    ts = list(range(rank, tx * ty, world))
    if order is not None:
        ts = [int(order[t]) for t in ts]
    slab = np.zeros((8, 8 * len(ts)) + frame.shape[2:], frame.dtype)
    for m, t in enumerate(ts):
        y0, x0 = (t // tx) * 8, (t % tx) * 8
        slab[:, 8 * m:8 * m + 8] = pad[y0:y0 + 8, x0:x0 + 8]
    return slab


def _rank_main_tiles(rank, world, port, out_path):
    import __graft_entry__ as ge
    rt = ge.import_binding()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n_max = max(rt.tiles_in_shard(W, H, r, world) for r in range(world))
    mine = tile_slab(ob.render(SCENE, W, H, SPP, threads=1), rank, world)
    assert mine.shape[1] == 8 * rt.tiles_in_shard(W, H, rank, world)
    slab = torch.zeros((8, 8 * n_max, 3), dtype=torch.float64)
    slab[:, : mine.shape[1]] = torch.from_numpy(mine)
    gathered = [torch.empty_like(slab) for _ in range(world)] if rank == 0 else None
    dist.gather(slab, gathered, dst=0)
    if rank == 0:
        np.save(out_path, rt.assemble_tiles(gathered, W, H, world).numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_tile_sharded_gather_equals_single_render(tmp_path, world):
    out = str(tmp_path / "frame.npy")
    mp.start_processes(_rank_main_tiles, args=(world, _free_port(), out), nprocs=world, join=True,
                       start_method="spawn")
    assert np.array_equal(np.load(out), ob.render(SCENE, W, H, SPP, threads=2))


def test_tile_shards_partition_and_assemble():
    """The C ABI's tile count per shard and assemble_tiles (numpy and torch) invert tile_slab."""
    import __graft_entry__ as ge
    rt = ge.import_binding()
    for (h, w) in ((800, 1200), (19, 24), (9, 17), (8, 8)):
        img = np.arange(h * w * 3, dtype=np.float64).reshape(h, w, 3)
        tiles = ((w + 7) // 8) * ((h + 7) // 8)
        for world in (1, 2, 3, 8):
            n = [rt.tiles_in_shard(w, h, r, world) for r in range(world)]
            assert sum(n) == tiles and n == [len(range(r, tiles, world)) for r in range(world)]
            slabs = [tile_slab(img, r, world) for r in range(world)]
            assert np.array_equal(rt.assemble_tiles(slabs, w, h, world), img)
            wide = max(n) * 8   # slabs padded to the largest shard, as gathered
            padded = [torch.from_numpy(np.pad(s, ((0, 0), (0, wide - s.shape[1]), (0, 0)))) for s in slabs]
            assert np.array_equal(rt.assemble_tiles(padded, w, h, world).numpy(), img)
    assert rt.tiles_in_shard(24, 19, 8, 4) == 1 and rt.tiles_in_shard(24, 19, 9, 4) == 0   # 9 tiles


def test_grouped_and_scattered_tile_orders():
    """grouped_tile_order deals runs of consecutive raster tiles round-robin and keeps every
    shard's tile count (rt_tiles_in_shard); scattered_tile_order is a stride permutation."""
    import __graft_entry__ as ge
    rt = ge.import_binding()
    for (n, world, g) in ((32400, 8, 30), (15000, 8, 8), (9, 4, 2), (100, 3, 7), (7, 8, 4), (5, 1, 3)):
        o = rt.grouped_tile_order(n, world, g)
        assert sorted(o.tolist()) == list(range(n))
        for r in range(world):
            assert len(o[r::world]) == len(range(r, n, world))
    o = rt.grouped_tile_order(32400, 8, 30)
    assert o[0::8][:32].tolist() == list(range(30)) + [240, 241]   # runs 0, 8, ...: tiles 0-29, 240-269
    assert rt.scattered_tile_order(10, 3).tolist() == [0, 3, 6, 9, 1, 4, 7, 2, 5, 8]


def test_tile_order_assemble_and_cost_order():
    """assemble_tiles with a tile order (rt_ctx_set_tile_order) inverts the shards that order
    deals, numpy and torch; cost_tile_order sorts most expensive first, ties in raster order,
    and deals shards whose costs differ by at most one tile's."""
    import __graft_entry__ as ge
    rt = ge.import_binding()
    rng = np.random.default_rng(5)
    for (h, w) in ((19, 24), (80, 16), (64, 96)):
        img = np.arange(h * w * 3, dtype=np.float64).reshape(h, w, 3)
        tiles = ((w + 7) // 8) * ((h + 7) // 8)
        for order in (rng.permutation(tiles), np.arange(tiles)[::-1]):
            for world in (1, 3, 8):
                slabs = [tile_slab(img, r, world, order) for r in range(world)]
                assert np.array_equal(rt.assemble_tiles(slabs, w, h, world, order=order), img)
                wide = max(s.shape[1] for s in slabs)
                padded = [torch.from_numpy(np.pad(s, ((0, 0), (0, wide - s.shape[1]), (0, 0)))) for s in slabs]
                assert np.array_equal(rt.assemble_tiles(padded, w, h, world, order=order).numpy(), img)
    with pytest.raises(ValueError):
        rt.assemble_tiles([np.zeros((8, 8, 3))], 16, 16, 1, order=np.arange(3))
    costs = np.array([5, 9, 9, 1, 7, 3, 0, 9], dtype=np.uint64)
    order = rt.cost_tile_order(costs)
    assert order.tolist() == [1, 2, 7, 4, 0, 5, 3, 6] and order.dtype == np.uint32
    heavy = rng.pareto(1.5, 4050 * 8) + 1.0
    o = rt.cost_tile_order(heavy)
    sums = [heavy[o[r::8]].sum() for r in range(8)]
    assert max(sums) - min(sums) <= heavy.max()


def _gathered(slabs, world):
    """Slabs padded to the largest shard's, one row per rank (what the RCCL gather lands on rank 0)."""
    flat = [s.reshape(-1) for s in slabs]
    n = max(f.size for f in flat)
    out = np.zeros((world, n), flat[0].dtype)
    for r, f in enumerate(flat):
        out[r, : f.size] = f
    return out


def test_library_tile_assembly_and_cost_order_match_python():
    """The library's host restatements (ABI v5), which rt_render_gather's reorder kernel and
    rt_comm_tile_order are checked against on the GPU, equal the Python ones: rt_tiles_assemble_host
    inverts every rank's tile slab (raster and permuted orders, f32 and f64, cut edge tiles, more
    ranks than tiles), and rt_cost_tile_order is a stable descending sort (ties in raster order)."""
    import __graft_entry__ as ge
    rt = ge.import_binding()
    rng = np.random.default_rng(11)
    for (h, w) in ((19, 24), (9, 17), (8, 8), (90, 160), (53, 96)):
        tiles = ((w + 7) // 8) * ((h + 7) // 8)
        for dt in (np.float64, np.float32):
            img = rng.standard_normal((h, w, 3)).astype(dt)
            for order in (None, rng.permutation(tiles).astype(np.uint32)):
                for world in (1, 2, 3, 8, tiles + 2):
                    slabs = [tile_slab(img, r, world, order) for r in range(world)]
                    g = _gathered(slabs, world)
                    got = rt.assemble_tiles_host(g, w, h, world, order=order)
                    assert got.dtype == dt and np.array_equal(got, img), (h, w, world, dt)
    with pytest.raises(rt.RTError):   # a slab narrower than the largest shard's
        rt.assemble_tiles_host(np.zeros((2, 10)), 24, 19, 2)
    with pytest.raises(rt.RTError):   # not a permutation
        rt.assemble_tiles_host(np.zeros((1, 9 * 192)), 24, 19, 1, order=np.zeros(9, np.uint32))
    costs = np.array([5, 9, 9, 1, 7, 3, 0, 9], dtype=np.uint64)
    assert rt.cost_tile_order(costs).tolist() == [1, 2, 7, 4, 0, 5, 3, 6]
    for _ in range(5):
        c = rng.integers(0, 50, 4000).astype(np.uint64)   # many ties
        assert np.array_equal(rt.cost_tile_order(c), np.argsort(-c.astype(np.float64), kind="stable"))
    big = np.array([2**62, 2**62 + 1, 7], dtype=np.uint64)   # beyond f64's integers: exact in the library
    assert rt.cost_tile_order(big).tolist() == [1, 0, 2]


@pytest.mark.parametrize("world", [2, 3])
def test_row_sharded_gather_equals_single_render(tmp_path, world):
    out = str(tmp_path / "frame.npy")
    mp.start_processes(_rank_main, args=(world, _free_port(), out), nprocs=world, join=True, start_method="spawn")
    frame = np.load(out)
    full = ob.render(SCENE, W, H, SPP, threads=2)
    assert np.array_equal(frame, full)


def test_assemble_rows_inverse():
    import __graft_entry__ as ge
    rt = ge.import_binding()
    img = np.arange(7 * 2 * 3).reshape(7, 2, 3)
    for world in (1, 2, 3, 8):
        rows_max = (7 + world - 1) // world
        slabs = []
        for r in range(world):
            s = np.zeros((rows_max, 2, 3), img.dtype)
            part = img[r::world]
            s[: len(part)] = part
            slabs.append(s)
        assert np.array_equal(rt.assemble_rows(slabs, 7, world), img)


def test_band_shards_partition_the_frame():
    """bench.py's multi-GPU shards: 8-row bands round-robin. The C ABI's row count, the
    Python row list and assemble_rows agree, and the shards partition every row once."""
    import __graft_entry__ as ge
    rt = ge.import_binding()
    for H in (800, 53, 8, 9):
        img = np.arange(H * 2 * 3).reshape(H, 2, 3)
        for world in (1, 2, 3, 8):
            rows = [rt.shard_rows(H, r, world, 8) for r in range(world)]
            assert sorted(y for rr in rows for y in rr) == list(range(H))
            n = [rt.rows_in_shard(H, r, world, 8) for r in range(world)]
            assert n == [len(rr) for rr in rows], (H, world)
            slabs = []
            for r in range(world):
                s = np.zeros((max(n), 2, 3), img.dtype)
                s[: n[r]] = img[rows[r]]
                slabs.append(s)
            assert np.array_equal(rt.assemble_rows(slabs, H, world, row_block=8), img)
    assert rt.load_library().rt_rows_in_band_shard(800, 0, 8, 6) == 0   # not a power of two
