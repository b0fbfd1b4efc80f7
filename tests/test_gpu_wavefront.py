"""The wavefront schedule (RT_SCHED_WAVEFRONT, csrc/trace_wavefront.hip) against the
megakernel's per-sample pool and the oracle.

Per (pixel, sample) the wavefront kernels run the megakernel's arithmetic in the same order
(the same walk order per ray, the deferred instance BLAS after the top-level walk, the same
draws), and the per-sample records are reduced by the same kernel, so every image must equal
the pool's bit for bit — at ragged sizes, with a path pool far smaller than the frame (slots
reused thousands of times), in row and tile shards and in buffer batches — and the work
counters (casts, node visits, primitive tests) must be equal too.
"""
import numpy as np
import pytest

from tests import oracle_binding as ob

pytestmark = pytest.mark.gpu

LINF = 1e-3
REL = 1e-9


def _render(rt, r, world, W, H, spp, sched, paths=0, **kw):
    cam, bg = rt.scene_camera(7, W, H)
    r.set_schedule(sched)
    r.set_option(rt.RT_OPT_WF_PATHS, paths)
    r.upload(world)
    try:
        img = r.render(cam, rt.Renderer.params(W, H, spp, 50, bg, 1, out_format=rt.RT_OUT_F64, **kw))
        st = r.stats()
    finally:
        r.set_schedule(rt.RT_SCHED_AUTO)
        r.set_option(rt.RT_OPT_WF_PATHS, 0)
    return img, st


@pytest.fixture(scope="module")
def final_world(rt):
    return rt.World(1).build_scene(7)


@pytest.mark.parametrize("W,H,spp,paths", [(64, 36, 8, 0), (64, 36, 8, 2048), (96, 54, 16, 4096), (37, 21, 5, 2048)])
def test_wavefront_equals_pool_bit_for_bit(rt, renderer, final_world, W, H, spp, paths):
    pool, sp = _render(rt, renderer, final_world, W, H, spp, rt.RT_SCHED_POOL)
    wf, sw = _render(rt, renderer, final_world, W, H, spp, rt.RT_SCHED_WAVEFRONT, paths)
    assert sp.schedule == rt.RT_SCHED_POOL and sw.schedule == rt.RT_SCHED_WAVEFRONT
    assert sw.wf_iterations > 0 and sw.samples == W * H * spp
    same = wf == pool
    assert same.all(), f"{int((~same.all(axis=2)).sum())} px differ"


@pytest.mark.timeout(300)
def test_wavefront_whole_c4_frame_equals_pool(rt, renderer, final_world):
    """C4's whole 1920x1080 frame (8 spp: 16.6 M samples, every tile, depth-50 tails) under the
    default path pool and a 256 K-slot pool: the pool's image bit for bit."""
    W, H, spp = 1920, 1080, 8
    pool, _ = _render(rt, renderer, final_world, W, H, spp, rt.RT_SCHED_POOL)
    for paths in (0, 1 << 18):
        wf, st = _render(rt, renderer, final_world, W, H, spp, rt.RT_SCHED_WAVEFRONT, paths)
        assert st.schedule == rt.RT_SCHED_WAVEFRONT
        same = wf == pool
        assert same.all(), f"paths {paths}: {int((~same.all(axis=2)).sum())} px differ"


def test_wavefront_counts_the_same_work(rt, renderer, final_world):
    """count_work: the same casts, node visits and primitive tests as the pool (the walks are the
    pool's, ray for ray), and the same image."""
    W, H, spp = 96, 54, 8
    a, sa = _render(rt, renderer, final_world, W, H, spp, rt.RT_SCHED_POOL, count_work=1)
    b, sb = _render(rt, renderer, final_world, W, H, spp, rt.RT_SCHED_WAVEFRONT, count_work=1)
    assert sb.schedule == rt.RT_SCHED_WAVEFRONT
    assert (sa.casts, sa.node_visits, sa.prim_tests) == (sb.casts, sb.node_visits, sb.prim_tests)
    assert np.array_equal(a, b)


def test_wavefront_against_oracle_at_c4_geometry(rt, renderer, final_world):
    W, H, spp, rb, stride = 1920, 1080, 24, 5, 72
    img, st = _render(rt, renderer, final_world, W, H, spp, rt.RT_SCHED_WAVEFRONT, row_begin=rb, row_stride=stride)
    assert st.schedule == rt.RT_SCHED_WAVEFRONT
    ref = ob.render(7, W, H, spp, 50, row_begin=rb, row_stride=stride, threads=16)
    d = np.abs(img - ref)
    assert float(d.max()) <= LINF
    assert not (d > REL * np.maximum(1.0, np.abs(ref))).any()


def test_wavefront_shards_and_batches_reassemble(rt, final_world):
    """Row shards and tile shards of the frame, and a render split into buffer batches by a small
    trace-output bound: every piece equals the one-launch pool render's pixels."""
    W, H, spp = 80, 48, 24
    r = rt.Renderer(0)
    try:
        full, _ = _render(rt, r, final_world, W, H, spp, rt.RT_SCHED_POOL)
        for rb in range(3):
            part, st = _render(rt, r, final_world, W, H, spp, rt.RT_SCHED_WAVEFRONT, 2048, row_begin=rb, row_stride=3)
            assert st.schedule == rt.RT_SCHED_WAVEFRONT
            assert np.array_equal(part, full[rb::3])
        slabs = [_render(rt, r, final_world, W, H, spp, rt.RT_SCHED_WAVEFRONT, 2048, row_begin=t, row_stride=4,
                         tile_shard=1)[0] for t in range(4)]
        assert np.array_equal(rt.assemble_tiles(slabs, W, H, 4), full)
        r.set_option(rt.RT_OPT_TRACE_BUF_BYTES, 1 << 20)   # 11 samples of 60 tiles x 64 px per batch
        batched, st = _render(rt, r, final_world, W, H, spp, rt.RT_SCHED_WAVEFRONT)
        assert st.schedule == rt.RT_SCHED_WAVEFRONT and st.n_batches > 1
        assert np.array_equal(batched, full)
    finally:
        r.close()


def test_wavefront_outside_its_feature_set_runs_auto(rt, renderer):
    """The random scene (spheres variant) and the Cornell box are not the wavefront kernels'
    feature set: the request runs AUTO's schedule, with the same image."""
    for scene_id, (W, H) in ((0, (48, 32)), (5, (32, 32))):
        world = rt.World(1).build_scene(scene_id)
        cam, bg = rt.scene_camera(scene_id, W, H)
        renderer.upload(world)
        p = rt.Renderer.params(W, H, 4, 50, bg, 1, out_format=rt.RT_OUT_F64)
        auto = renderer.render(cam, p)
        renderer.set_schedule(rt.RT_SCHED_WAVEFRONT)
        try:
            img = renderer.render(cam, p)
            assert renderer.stats().schedule in (rt.RT_SCHED_POOL, rt.RT_SCHED_ITEMS)
        finally:
            renderer.set_schedule(rt.RT_SCHED_AUTO)
        assert np.array_equal(img, auto)
