"""GPU checks at BASELINE.json's full frame sizes, through properties that do not need
the oracle to render the whole frame:

- every BASELINE config against the oracle at its FULL sample count and depth (VERDICT r02
  item 2): C1's whole 1200x800x10 frame, C2 500 spp and C3 1000 spp on two rows, C4 1000 spp
  on one row, C5 4096 spp on one 4096-pixel row of the 4096x4096 frame in many buffer
  batches (both schedules), so the highest sample indices and the depth-50 tails are checked;
- every BASELINE config against the oracle on a bounded row subset at its own geometry
  and depth: C1 (1200x800, 10 spp, depth 8), C2 (1200x800, depth 50, 64 spp), C3 (Cornell
  800x800, 64 spp), C4 (final scene 1920x1080, 48 spp) and C5 (4096x4096: pixel keys up to
  16.7 M, rendered in many buffer batches through the carry kernels);
- the kernel variants (conservative f32 slabs vs f64 slabs, LDS vs scratch stack, TLAS in
  LDS or not) and the accel modes render the FULL C2 / C3 / C4 frames bit-identically;
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


# BASELINE.json configs at their own geometry, depth and a real sample depth, on row subsets
# the oracle renders in about a second (C1 full spp; C2/C3/C4 at 48-64 spp, i.e. 3-4 chunks
# of 16 and sample indices far past the first few)
@pytest.mark.parametrize("cfg,scene_id,W,H,spp,depth,row_begin,stride", [
    ("C1", 0, 1200, 800, 10, 8, 2, 5),
    ("C2", 0, 1200, 800, 64, 50, 11, 50),
    ("C3", 5, 800, 800, 64, 50, 7, 10),
    ("C4", 7, 1920, 1080, 48, 50, 5, 36),
])
def test_baseline_configs_against_oracle(rt, renderer, cfg, scene_id, W, H, spp, depth, row_begin, stride):
    img, st = rt.render_scene(scene_id, W, H, spp, depth, row_begin=row_begin, row_stride=stride,
                              out_format=rt.RT_OUT_F64, renderer=renderer)
    ref = ob.render(scene_id, W, H, spp, depth, row_begin=row_begin, row_stride=stride, threads=16)
    assert img.shape == (len(range(row_begin, H, stride)), W, 3)
    _parity(img, ref, cfg)


# BASELINE.json configs at their FULL spp and depth: rows chosen so the
# oracle (16 threads, reference-faithful linear scans) finishes in seconds
FULL = {   # cfg: scene, W, H, spp, depth, row_begin, row_stride
    "C1": (0, 1200, 800, 10, 8, 0, 1),          # the whole frame, 9.6 M samples
    "C2": (0, 1200, 800, 500, 50, 330, 235),    # rows 330, 565: 1.2 M samples
    "C3": (5, 800, 800, 1000, 50, 200, 320),    # rows 200, 520: 1.6 M samples
    "C4": (7, 1920, 1080, 1000, 50, 540, 1080),  # row 540: 1.9 M samples
}


@pytest.mark.parametrize("cfg", sorted(FULL))
@pytest.mark.timeout(300)
def test_baseline_configs_full_spp_against_oracle(rt, renderer, cfg):
    scene_id, W, H, spp, depth, row_begin, stride = FULL[cfg]
    img, st = rt.render_scene(scene_id, W, H, spp, depth, row_begin=row_begin, row_stride=stride,
                              out_format=rt.RT_OUT_F64, renderer=renderer)
    assert st.samples == img.shape[0] * W * spp
    ref = _full_ref(cfg)
    assert img.shape == ref.shape == (len(range(row_begin, H, stride)), W, 3)
    _parity(img, ref, cfg + " full spp")


_FULL_REF = {}


def _full_ref(cfg):
    if cfg not in _FULL_REF:
        scene_id, W, H, spp, depth, row_begin, stride = FULL[cfg]
        _FULL_REF[cfg] = ob.render(scene_id, W, H, spp, depth, row_begin=row_begin, row_stride=stride, threads=16)
    return _FULL_REF[cfg]


@pytest.mark.timeout(300)
def test_c1_whole_frame_ppm_bytes_equal_oracle(rt, renderer, tmp_path):
    """VERDICT r03 item 1 (a22/f1): the product's PPM of C1's whole 1200x800x10 frame (depth 8)
    is byte-identical to the oracle's write_color (math.rs:119-132, main.rs:472,591-596) of the
    product's own f64 means AND to the oracle's PPM of the oracle's own render of the frame. The
    frame is rendered through rt_render with RT_OUT_F64 (sum * (1/spp) in f64, the reference's
    `self.x * scale`) and written by rt_write_ppm_f64."""
    scene_id, W, H, spp, depth, _, _ = FULL["C1"]
    img, _ = rt.render_scene(scene_id, W, H, spp, depth, out_format=rt.RT_OUT_F64, renderer=renderer)
    assert img.shape == (H, W, 3) and img.dtype == np.float64
    mine, own, ref = tmp_path / "product.ppm", tmp_path / "oracle_of_product.ppm", tmp_path / "oracle.ppm"
    rt.write_ppm(img, str(mine))
    ob.write_ppm(img, str(own))
    ob.write_ppm(_full_ref("C1"), str(ref))
    b = mine.read_bytes()
    assert b.startswith(b"P3\n1200 800\n255\n\n") and b.count(b"\n") == 4 + W * H
    assert b == own.read_bytes(), "product write_color != oracle write_color of the same means"
    assert b == ref.read_bytes(), "product PPM != oracle PPM of the oracle's render"
    # and channel by channel (a mismatch would name its pixel)
    assert np.array_equal(rt.write_color(img), ob.write_color(_full_ref("C1")))


_C5_REF = {}


@pytest.mark.parametrize("sched", ["POOL", "ITEMS"])
@pytest.mark.timeout(300)
def test_c5_full_spp_row_against_oracle(rt, sched):
    """C5 at its full 4096 spp and depth 50 on row 2100 of the 4096x4096 frame (16.8 M
    samples; pixel keys ~8.6 M), under a 16 MB trace-output bound: the per-sample pool runs
    in ~26 batches whose chunk sums are carried across batches (samples up to 4095), the item
    pool in 2."""
    W = H = 4096
    spp, rows = 4096, dict(row_begin=2100, row_stride=4096)
    r = rt.Renderer(0)
    r.set_option(rt.RT_OPT_TRACE_BUF_BYTES, 16 << 20)
    try:
        r.set_schedule(getattr(rt, "RT_SCHED_" + sched))
        world = rt.World(1).build_scene(0)
        cam, bg = rt.scene_camera(0, W, H)
        r.upload(world)
        img = r.render(cam, rt.Renderer.params(W, H, spp, 50, bg, 1, out_format=rt.RT_OUT_F64, **rows))
        st = r.stats()
        assert st.n_batches >= (20 if sched == "POOL" else 2), st.n_batches
    finally:
        r.close()
    if "ref" not in _C5_REF:
        _C5_REF["ref"] = ob.render(0, W, H, spp, 50, threads=16, **rows)
    assert img.shape == (1, W, 3)
    _parity(img, _C5_REF["ref"], f"C5 full spp ({sched})")


@pytest.mark.parametrize("sched", ["POOL", "ITEMS", "RING"])
def test_c5_geometry_many_buffer_batches(rt, sched):
    """C5's 4096x4096 frame (pixel keys y*4096 + x up to 16.7 M) on 8 full-width rows incl.
    the top one, 40 spp (chunks of 3), with a 1 MB trace-output bound so the render runs
    in many buffer batches: per-sample pool 1 sample per batch, chunks straddling batches
    (reduce_samples_carry); item pool 1 chunk per batch (accumulate_chunks); RING, the per-sample
    pool reducing in the kernel, 1 chunk of partials per batch beside its two rings."""
    W = H = 4096
    spp, rows = 40, dict(row_begin=511, row_stride=512)
    r = rt.Renderer(0)
    r.set_option(rt.RT_OPT_TRACE_BUF_BYTES, 1 << 20)
    r.set_option(rt.RT_OPT_POOL_RING, 2 if sched == "RING" else 0)
    r.set_schedule(rt.RT_SCHED_ITEMS if sched == "ITEMS" else rt.RT_SCHED_POOL)
    world = rt.World(1).build_scene(0)
    cam, bg = rt.scene_camera(0, W, H)
    r.upload(world)
    img = r.render(cam, rt.Renderer.params(W, H, spp, 50, bg, 1, out_format=rt.RT_OUT_F64, **rows))
    st = r.stats()
    assert st.n_batches == (40 if sched == "POOL" else 14), st.n_batches
    assert (st.ring_bytes > 0) == (sched == "RING")
    r.close()
    ref = ob.render(0, W, H, spp, 50, threads=16, **rows)
    assert img.shape == (8, W, 3)
    _parity(img, ref, f"C5 geometry ({sched})")


@pytest.mark.parametrize("scene_id,W,H,spp", [(0, 1200, 800, 16), (5, 800, 800, 16), (7, 1920, 1080, 8)])
def test_variants_bit_identical_at_full_size(rt, renderer, scene_id, W, H, spp):
    """The conservative f32 slab test (boxes padded on the host, flatten.cpp to_f32_box) is a
    claim about rare rays; check it where they occur: whole C2 / C3 / C4 frames (7.7 M to
    16.6 M samples) with f32 vs f64 slabs, LDS vs scratch stack, TLAS in LDS vs L2 — every
    pixel bit for bit."""
    world = rt.World(1).build_scene(scene_id)
    cam, bg = rt.scene_camera(scene_id, W, H)
    renderer.upload(world)
    p = rt.Renderer.params(W, H, spp, 50, bg, 1, out_format=rt.RT_OUT_F64)
    ref = None
    try:
        for v in [(1, 1, 1), (0, 1, 1), (1, 0, 1), (1, 1, 0), (0, 0, 0)]:
            renderer.set_variant(*v)
            img = renderer.render(cam, p)
            st = renderer.stats()
            # a scene without BVH nodes (Cornell) tests no slab: it runs the f64-slab kernel
            assert st.slab32 == (v[0] if scene_id != 5 else 0)
            if ref is None:
                ref = img
            else:
                same = img == ref
                assert same.all(), f"variant {v}: {int((~same.all(axis=2)).sum())} px differ"
    finally:
        renderer.set_variant(1, 1, 1)


def test_accel_modes_bit_identical_at_full_c2_size(rt, renderer):
    """SURVEY §8 f3 at the headline geometry: the reference's list scan (LINEAR) and the SAH
    BVH give the same C2 frame bit for bit (closest hit does not depend on the hierarchy)."""
    W, H, spp = 1200, 800, 4
    world = rt.World(1).build_scene(0)
    cam, bg = rt.scene_camera(0, W, H)
    p = rt.Renderer.params(W, H, spp, 50, bg, 1, out_format=rt.RT_OUT_F64)
    out = {}
    for accel in (rt.RT_ACCEL_SAH, rt.RT_ACCEL_LINEAR):
        renderer.upload(world, accel)
        out[accel] = renderer.render(cam, p)
    renderer.upload(world)
    assert np.array_equal(out[rt.RT_ACCEL_SAH], out[rt.RT_ACCEL_LINEAR])


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


@pytest.mark.parametrize("sched", ["POOL", "ITEMS", "RING"])
def test_overlapped_buffer_batches_at_c2_size(rt, renderer, sched):
    """the trace-output buffer is bounded (default 4 GB); a render larger than
    the bound runs in batches traced on two streams into the bound's two halves while the
    render's stream reduces the previous batch. The whole C2 frame at 48 spp under a 256 MB bound
    (per-sample pool: 5 samples per half, 10 batches; item pool: chunks of 3, 5 chunks per half,
    4 batches) equals the one-batch render bit for bit, and so does the same bound without
    overlap (RT_OPT_BATCH_OVERLAP 0: 11 samples or chunks per batch, 5 and 2 batches). Batches
    overlap only for kernels of 256-thread workgroups (abi.cpp): the overlapped runs take the
    random scene's partial-TLAS instantiation (lds_nodes 0: 256 threads); the default one (768-
    thread workgroups, 6 waves per SIMD) runs its batches in order, as with the option at 0."""
    W, H, spp = 1200, 800, 48
    world = rt.World(1).build_scene(0)
    cam, bg = rt.scene_camera(0, W, H)
    p = rt.Renderer.params(W, H, spp, 50, bg, 1, out_format=rt.RT_OUT_F64)
    renderer.upload(world)
    renderer.set_schedule(rt.RT_SCHED_ITEMS)   # the reference image: one launch
    try:
        one = renderer.render(cam, p)
        assert renderer.stats().n_batches == 1
    finally:
        renderer.set_schedule(rt.RT_SCHED_AUTO)
    for overlap, lds_nodes in (("1", 0), ("0", 0), ("1", 1)):
        r = rt.Renderer(0)
        r.set_option(rt.RT_OPT_TRACE_BUF_BYTES, 256 << 20)
        r.set_option(rt.RT_OPT_BATCH_OVERLAP, int(overlap))
        r.set_option(rt.RT_OPT_POOL_RING, 2 if sched == "RING" else 0)
        r.set_variant(1, 1, lds_nodes)
        try:
            r.set_schedule(rt.RT_SCHED_ITEMS if sched == "ITEMS" else rt.RT_SCHED_POOL)
            r.upload(world)
            img = r.render(cam, p)
            st = r.stats()
        finally:
            r.close()
        # RING: the ring (two when overlapped) leaves the 256 MB bound less than one 23 MB chunk of
        # partials per batch, so batches of one chunk (the bound's floor)
        expect = {("POOL", "1", 0): 10, ("POOL", "0", 0): 5, ("POOL", "1", 1): 5, ("ITEMS", "1", 0): 4,
                  ("ITEMS", "0", 0): 2, ("ITEMS", "1", 1): 2}.get((sched, overlap, lds_nodes), 16)
        assert st.n_batches == expect, (overlap, lds_nodes, st.n_batches)
        same = img == one
        assert same.all(), f"overlap {overlap} lds_nodes {lds_nodes}: {int((~same.all(axis=2)).sum())} px differ"
