"""The multi-GPU render behind the C ABI (ABI v5): rt_comm_* and
rt_render_gather — the reference's partition of one frame over workers (main.rs:497-551) and
the merge of their buffers (main.rs:542-547) — on the box's one GPU.

- World size 1 through the library's own RCCL communicator, both constructors
  (rt_comm_init_rank with a unique id, rt_comm_init_all): the tile shard, the RCCL gather, the
  reorder kernel (RT_OPT_COMM_DIRECT 0, or a cost tile order), and the direct render of a world
  of one (the default); frames bit-identical to rt_render's, raster and cost tile order, f64 and
  f32, host and device output.
- The reorder kernel alone (rt_tiles_assemble) with N = 2, 3, 8 shard slabs rendered one after
  the other on the one GPU, in the padded layout the gather lands on rank 0: bit-identical to
  the one-launch frame in raster and cost order, and equal to the host restatement
  (rt_tiles_assemble_host).
RCCL refuses two ranks on one device, so N > 1 communicators are not built here; N > 1 is the
same code with more ranks (tests/test_multirank_cpu.py checks the partition and reassembly on
the CPU, tests/test_gpu_0_multirank.py bench.py's N > 1 branch with rank processes on one GPU)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W, H, SPP = 160, 90, 8   # 20 x 12 tiles; the last tile row is cut (90 = 11 * 8 + 2)


@pytest.fixture(scope="module")
def scene_renderer(rt):
    r = rt.Renderer(0)
    w = rt.World(1).build_scene(0)
    r.upload(w)
    yield r
    r.close()


def _params(rt, bg, fmt, spp=SPP, **kw):
    return rt.Renderer.params(W, H, spp, 50, bg, 1, out_format=fmt, **kw)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("direct", [0, 1])
def test_render_gather_world1_equals_render(rt, scene_renderer, direct):
    """direct 0: the tile shard, the RCCL gather and the reorder kernel, as at any world size;
    direct 1 (RT_OPT_COMM_DIRECT, the default): a world of one in raster order renders straight
    into the frame (no slab, no gather). Under a cost order both take the shard path."""
    cam, bg = rt.scene_camera(0, W, H)
    r = scene_renderer
    comm = rt.Comm(r, 0, 1, rt.Comm.unique_id())
    try:
        assert r.lib.rt_abi_version() == 6
        r.set_option(rt.RT_OPT_COMM_DIRECT, direct)
        assert r.get_option(rt.RT_OPT_COMM_DIRECT) == direct
        for fmt in (rt.RT_OUT_F64, rt.RT_OUT_F32):
            r.set_tile_order(None)
            ref = r.render(cam, _params(rt, bg, fmt))
            got = comm.render_gather(cam, _params(rt, bg, fmt))
            assert got.dtype == ref.dtype and np.array_equal(got, ref), fmt
            st = comm.stats()
            n_tiles = 20 * 12
            slab = 192 * n_tiles * (8 if fmt == rt.RT_OUT_F64 else 4) + 8
            assert st.tiles == n_tiles and st.slab_bytes == (0 if direct else slab)
            assert st.render_ms >= st.kernel_ms > 0 and st.gather_ms >= 0 and st.assemble_ms >= 0
            assert st.peer_failed == 0
            # the cost order (count pass, RCCL all-reduce, the order set): same bits, tiles dealt anew
            comm.tile_order(cam, _params(rt, bg, fmt), 4)
            st = comm.stats()
            assert st.tile_order == 1 and st.cost_pass_ms > 0
            again = comm.render_gather(cam, _params(rt, bg, fmt))
            assert np.array_equal(again, ref), fmt
            assert comm.stats().slab_bytes == slab   # a tile order: the shard path
        r.set_tile_order(None)
    finally:
        comm.close()
        r.set_tile_order(None)
        r.set_option(rt.RT_OPT_COMM_DIRECT, 1)


@pytest.mark.timeout(300)
def test_render_gather_device_output_on_a_torch_stream(rt, scene_renderer):
    """out_on_device: rank 0's frame lands in a torch tensor, the work enqueued on a torch stream."""
    import torch
    cam, bg = rt.scene_camera(0, W, H)
    r = scene_renderer
    r.set_tile_order(None)
    ref = r.render(cam, _params(rt, bg, rt.RT_OUT_F64))
    comm = rt.Comm(r, 0, 1, rt.Comm.unique_id())
    try:
        dev = torch.device("cuda", 0)
        frame = torch.full((H, W, 3), float("nan"), dtype=torch.float64, device=dev)
        stream = torch.cuda.Stream(dev)
        stream.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(stream):
            comm.render_gather_device(cam, _params(rt, bg, rt.RT_OUT_F64), frame.data_ptr(), stream.cuda_stream)
        stream.synchronize()
        assert np.array_equal(frame.cpu().numpy(), ref)
    finally:
        comm.close()


@pytest.mark.timeout(300)
def test_render_gather_all_one_process(rt):
    """rt_comm_init_all / rt_comm_tile_order_all / rt_render_gather_all (one process driving its
    GPUs from one thread through RCCL group calls) over the box's one device; the final scene."""
    r = rt.Renderer(0)
    try:
        r.upload(rt.World(1).build_scene(7))
        cam, bg = rt.scene_camera(7, W, H)
        ref = r.render(cam, _params(rt, bg, rt.RT_OUT_F64))
        comms = rt.Comm.init_all([r])
        try:
            assert comms[0].rank == 0 and comms[0].world == 1
            got = rt.render_gather_all(comms, cam, _params(rt, bg, rt.RT_OUT_F64))
            assert np.array_equal(got, ref)
            rt.tile_order_all(comms, cam, _params(rt, bg, rt.RT_OUT_F64), 4)
            assert comms[0].stats().tile_order == 1
            got = rt.render_gather_all(comms, cam, _params(rt, bg, rt.RT_OUT_F64))
            assert np.array_equal(got, ref)
        finally:
            for c in comms:
                c.close()
    finally:
        r.close()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("order", ["raster", "cost"])
def test_reorder_kernel_reassembles_shards(rt, scene_renderer, world, order):
    """N shard slabs rendered on the one GPU into the padded layout RCCL's gather lands on rank 0
    ([rank][slab of the largest shard]), then rt_tiles_assemble: the one-launch frame bit for bit.
    The cost order comes from the library's own pass (rt_last_tile_costs -> rt_cost_tile_order)."""
    import torch
    cam, bg = rt.scene_camera(0, W, H)
    r = scene_renderer
    r.set_tile_order(None)
    ref = r.render(cam, _params(rt, bg, rt.RT_OUT_F64))
    try:
        tile_order = None
        if order == "cost":
            r.render(cam, _params(rt, bg, rt.RT_OUT_F32, spp=4, count_work=1))
            tile_order = rt.cost_tile_order(r.tile_costs())
            assert not np.array_equal(tile_order, np.arange(len(tile_order)))
            r.set_tile_order(tile_order)
        n_max = rt.tiles_in_shard(W, H, 0, world)
        slab_elems = 192 * n_max
        dev = torch.device("cuda", 0)
        gathered = torch.full((world, slab_elems), float("nan"), dtype=torch.float64, device=dev)
        stream = torch.cuda.Stream(dev)
        stream.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(stream):
            for q in range(world):
                p = _params(rt, bg, rt.RT_OUT_F64, row_begin=q, row_stride=world, tile_shard=1)
                r.render_device(cam, p, gathered[q].data_ptr(), stream.cuda_stream)
            frame = torch.full((H, W, 3), float("nan"), dtype=torch.float64, device=dev)
            r.assemble_device(gathered.data_ptr(), slab_elems, world, _params(rt, bg, rt.RT_OUT_F64),
                              frame.data_ptr(), stream.cuda_stream)
        stream.synchronize()
        got = frame.cpu().numpy()
        assert np.array_equal(got, ref), (world, order)
        host = rt.assemble_tiles_host(gathered.cpu().numpy(), W, H, world, order=tile_order)
        assert np.array_equal(host, ref)
    finally:
        r.set_tile_order(None)
