"""The f32 fast mode (RT_PREC_F32) against the f64 path.

The f32 mode draws and rounds differently, so its paths are not the f64 paths: parity is
statistical. Per scene, 8x8-pixel block means of the f32 image and of an f64 image agree
within their standard error, estimated from the spread of further f64 seeds (t-statistics,
as tests/test_gpu_fullsize.py::test_independent_seeds_agree_statistically does for two f64
seeds), and the image means agree to well under 1 %. The f64 images are themselves the
oracle-pinned path (tests/test_gpu_parity.py).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _render(rt, renderer, scene_id, W, H, spp, seed, precision):
    renderer.set_precision(precision)
    try:
        img, st = rt.render_scene(scene_id, W, H, spp, 50, render_seed=seed, out_format=rt.RT_OUT_F64,
                                  renderer=renderer)
    finally:
        renderer.set_precision(rt.RT_PREC_F64)
    assert st.precision == precision
    return img


@pytest.mark.parametrize("scene_id,W,H,spp,mean_tol", [
    (0, 64, 48, 64, 0.01),     # random spheres (C1/C2/C5): r = 1000 ground sphere, glass, metal
    (5, 48, 48, 128, 0.02),    # Cornell box (C3): rects, instanced boxes, light
    (7, 64, 32, 96, 0.03),     # final scene (C4): BVH, media, Perlin, image, motion blur
])
def test_f32_mode_agrees_statistically(rt, renderer, scene_id, W, H, spp, mean_tol):
    f64 = [_render(rt, renderer, scene_id, W, H, spp, s, rt.RT_PREC_F64) for s in range(1, 9)]
    f32 = _render(rt, renderer, scene_id, W, H, spp, 1, rt.RT_PREC_F32)
    assert np.all(np.isfinite(f32)) and f32.min() >= 0.0
    assert not np.array_equal(f32, f64[0])      # its own paths, not the f64 bits

    def blocks(x):
        return x.reshape(H // 8, 8, W // 8, 8, 3).mean(axis=(1, 3))

    bm = np.stack([blocks(x) for x in f64])
    sd = bm[1:].std(axis=0, ddof=1)
    se = np.sqrt(2.0) * np.maximum(sd, 1e-6)
    t = np.abs(blocks(f32) - bm[0]) / se
    assert float(np.mean(t)) < 1.5, float(np.mean(t))         # E|t_6| ~ 0.85
    assert int(np.sum(t > 6.0)) <= 2, int(np.sum(t > 6.0))   # P(|t_6| > 6) ~ 1e-3 per block
    ref = float(np.mean(f64))
    assert abs(float(f32.mean()) / ref - 1.0) < mean_tol, (float(f32.mean()), ref)


def test_f32_mode_all_scenes_and_schedules(rt, renderer):
    """Every reference scene renders in f32 (finite, non-negative, within a few % of the f64
    image mean). The f32 mode's draws are keyed per (pixel, sample) like the f64 mode's, so a
    row shard gives the bits of the whole frame; its translation units contract FMAs (round 6,
    DESIGN.md §5.6), so the kernels of different schedules (CHUNKS / POOL / ITEMS: each compiles
    the path code on its own) round differently in the last bits and agree statistically."""
    for scene_id in range(8):   # (128 spp: at 32 the Cornell box's small light leaves ~10 % noise in the mean)
        a = _render(rt, renderer, scene_id, 32, 24, 128, 3, rt.RT_PREC_F32)
        b = _render(rt, renderer, scene_id, 32, 24, 128, 3, rt.RT_PREC_F64)
        assert np.all(np.isfinite(a)) and a.min() >= 0.0, scene_id
        assert abs(float(a.mean()) / max(float(b.mean()), 1e-12) - 1.0) < 0.1, scene_id
    world = rt.World(1).build_scene(7)
    cam, bg = rt.scene_camera(7, 40, 30)
    renderer.upload(world)
    renderer.set_precision(rt.RT_PREC_F32)
    try:
        imgs = []
        for sched in (rt.RT_SCHED_CHUNKS, rt.RT_SCHED_POOL, rt.RT_SCHED_ITEMS):
            renderer.set_schedule(sched)
            imgs.append(renderer.render(cam, rt.Renderer.params(40, 30, 8, 50, bg, 1, out_format=rt.RT_OUT_F64)))
        shard = renderer.render(cam, rt.Renderer.params(40, 30, 8, 50, bg, 1, row_begin=1, row_stride=3,
                                                        out_format=rt.RT_OUT_F64))
        # count_work in the f32 mode: the final-scene (and spheres) variants have one
        renderer.render(cam, rt.Renderer.params(40, 30, 8, 50, bg, 1, count_work=1, out_format=rt.RT_OUT_F64))
        st = renderer.stats()
        assert st.casts >= 40 * 30 * 8 and st.node_visits > 0 and st.prim_tests > 0
        assert renderer.counters()[21] > 0   # phase timers ran
        cornell = rt.World(1).build_scene(5)
        renderer.upload(cornell)
        with pytest.raises(rt.RTError, match="UNSUPPORTED"):
            renderer.render(cam, rt.Renderer.params(40, 30, 8, 50, bg, 1, count_work=1, out_format=rt.RT_OUT_F64))
        renderer.upload(world)
    finally:
        renderer.set_precision(rt.RT_PREC_F64)
        renderer.set_schedule(rt.RT_SCHED_AUTO)
    for im in imgs[1:]:
        assert abs(float(im.mean()) / float(imgs[0].mean()) - 1.0) < 0.03
    assert np.array_equal(shard, imgs[2][1::3])   # ITEMS, the last schedule set: the same kernel
