"""GPU checks at BASELINE.json's full frame sizes, through properties that do not need
the oracle to render the whole frame:

- every BASELINE geometry against the oracle on a bounded row subset (C2/C5 scene at
  1200x800, Cornell at 800x800, the final scene at 1920x1080);
- the full C2 frame (1200x800, 500 spp, depth 50): finite, deterministic (two renders are
  bit-identical), and equal to the sum of its progressive batches;
- statistical parity across independent seeds: with another render seed the image
  changes pixel by pixel, but block means agree within their Monte Carlo error.
"""
import numpy as np
import pytest

from tests import oracle_binding as ob

pytestmark = pytest.mark.gpu

LINF = 1e-3          # north_star tolerance
REL = 1e-9           # path identity (f64 output)


def _parity(got, ref, label):
    diff = np.abs(got - ref)
    assert float(diff.max()) <= LINF, f"{label}: L_inf {float(diff.max())}"
    bad = diff > REL * np.maximum(1.0, np.abs(ref))
    assert not bad.any(), f"{label}: {int(bad.sum())} px differ"


@pytest.mark.parametrize("scene_id,W,H,stride", [(0, 1200, 800, 97), (5, 800, 800, 61), (7, 1920, 1080, 181)])
def test_baseline_geometries_on_row_subsets(rt, renderer, scene_id, W, H, stride):
    img, _ = rt.render_scene(scene_id, W, H, 2, 50, row_begin=3, row_stride=stride, out_format=rt.RT_OUT_F64,
                             renderer=renderer)
    ref = ob.render(scene_id, W, H, 2, row_begin=3, row_stride=stride)
    _parity(img, ref, f"scene {scene_id} {W}x{H}")


def test_full_c2_frame_deterministic_and_batch_additive(rt, renderer):
    W, H, spp = 1200, 800, 500
    world = rt.World(1).build_scene(0)
    cam, bg = rt.scene_camera(0, W, H)
    renderer.upload(world)
    p = rt.Renderer.params(W, H, spp, 50, bg, 1, out_format=rt.RT_OUT_F64)
    a = renderer.render(cam, p)
    b = renderer.render(cam, p)
    assert np.all(np.isfinite(a)) and a.min() >= 0.0
    assert np.array_equal(a, b)
    # the same frame as progressive batches on chunk boundaries (rt_accum_*): same bits
    chunk = renderer.stats().spp_chunk
    acc = renderer.accumulator(rt.Renderer.params(W, H, spp, 50, bg, 1, spp_chunk=chunk))
    done = 0
    while done < spp:
        n = min(3 * chunk, spp - done)
        acc.add(cam, rt.Renderer.params(W, H, spp, 50, bg, 1, spp_chunk=chunk), n)
        done += n
    assert acc.samples_done == spp
    c = acc.resolve(divisor=spp, out_format=rt.RT_OUT_F64)
    acc.close()
    assert np.array_equal(a, c)


def test_independent_seeds_agree_statistically(rt, renderer):
    """seeds 1 and 2 give different paths (pixels differ) but the same
    expected image: 8x8-pixel block means agree within their standard error, estimated
    from the spread of eight further seeds (t-statistics with 7 degrees of freedom)."""
    W, H, spp = 64, 48, 64
    imgs = [rt.render_scene(0, W, H, spp, 50, render_seed=s, out_format=rt.RT_OUT_F64, renderer=renderer)[0]
            for s in range(1, 11)]
    assert not np.array_equal(imgs[0], imgs[1])

    def blocks(x):
        return x.reshape(H // 8, 8, W // 8, 8, 3).mean(axis=(1, 3))

    bm = np.stack([blocks(x) for x in imgs])
    sd = bm[2:].std(axis=0, ddof=1)
    se = np.sqrt(2.0) * np.maximum(sd, 1e-6)
    t = np.abs(bm[0] - bm[1]) / se
    assert float(np.mean(t)) < 1.5, float(np.mean(t))          # E|t_7| ~ 0.85
    assert int(np.sum(t > 6.0)) <= 2, int(np.sum(t > 6.0))    # P(|t_7| > 6) ~ 5e-4 per block
    # and the global mean agrees to well within 1 %
    assert abs(float(imgs[0].mean()) / float(np.mean(imgs[2:])) - 1.0) < 0.01


def test_device_output_on_a_torch_stream_matches_host_render(rt, renderer):
    """bench.py's step: render_device into a torch tensor on a torch stream, then a torch
    copy on that stream, must see the finished frame (same bits as the host-output render)."""
    import torch
    W, H, spp = 96, 64, 8
    world = rt.World(1).build_scene(0)
    cam, bg = rt.scene_camera(0, W, H)
    renderer.upload(world)
    stream = torch.cuda.Stream(torch.device("cuda", 0))
    slab = torch.zeros((H, W, 3), dtype=torch.float32, device="cuda:0")
    with torch.cuda.stream(stream):
        renderer.render_device(cam, rt.Renderer.params(W, H, spp, 50, bg, 1, out_format=rt.RT_OUT_F32),
                               slab.data_ptr(), stream.cuda_stream)
        frame = slab.clone()
    torch.cuda.synchronize()
    host = renderer.render(cam, rt.Renderer.params(W, H, spp, 50, bg, 1, out_format=rt.RT_OUT_F32))
    assert np.array_equal(frame.cpu().numpy(), host)
