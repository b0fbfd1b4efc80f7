"""General Hittable nesting (hittable.rs:30-41: Translate / RotateY wrap any Hittable, a
ConstantMedium's boundary is any Hittable) on the GPU against the oracle.

Each world is built twice by the same constructor calls — in the product (rt_world_*) and
in the oracle (orc_world_*, tests/oracle_binding.py TwinWorld) — and rendered by both. The
product lowers the nesting by pushing Translate/RotateY chains down (flatten.cpp
lower_instance); the oracle evaluates the reference's recursion as written. Bar as in
tests/test_gpu_parity.py: L_inf <= 1e-3 and path identity (relative 1e-9).
"""
import numpy as np
import pytest

from tests import oracle_binding as ob
from tests.test_gpu_parity import assert_parity

pytestmark = pytest.mark.gpu


def _cam24(cam):
    v = []
    for f in ("origin", "lower_left_corner", "horizontal", "vertical", "u", "v", "w"):
        v += list(getattr(cam, f))
    return np.array(v + [cam.lens_radius, cam.time0, cam.time1])


def _render_both(rt, renderer, tw, W, H, spp, look_from, look_at, bg, vfov=40.0, accel=None):
    cam = rt.camera_new(look_from, look_at, (0.0, 1.0, 0.0), vfov, W / H, 0.1, 10.0, 0.0, 1.0)
    renderer.upload(tw.product, rt.RT_ACCEL_SAH if accel is None else accel)
    got = renderer.render(cam, rt.Renderer.params(W, H, spp, 50, bg, 1, out_format=rt.RT_OUT_F64))
    ref = tw.oracle.render(_cam24(cam), bg, W, H, spp)
    return got, ref


def _nested_world(rt):
    """Instances over instances, an instance over a BVH holding instances, a medium and
    spheres, a medium under two instances whose boundary is itself an instanced box, a bare
    BVH as a medium boundary, and a light."""
    tw = ob.TwinWorld(rt, 5)
    white = tw.lambertian(tw.solid(0.73, 0.73, 0.73))
    red = tw.lambertian(tw.checker((0.65, 0.05, 0.05), (0.9, 0.9, 0.9)))
    metal = tw.metal((0.8, 0.8, 0.9), 0.1)
    glass = tw.dielectric(1.5)
    light = tw.diffuse_light(tw.solid(6.0, 6.0, 6.0))
    phase = tw.isotropic(tw.solid(0.8, 0.8, 0.9))
    tw.push(tw.sphere(white, (0.0, -1000.0, 0.0), 1000.0))
    tw.push(tw.xz_rect(light, -2.0, 2.0, -2.0, 2.0, 6.0))
    # Translate(RotateY(BVH[RotateY(Translate(box)), medium(sphere), spheres]))
    inner = tw.rotate_y(tw.translate(tw.box((0.0, 0.0, 0.0), (0.8, 1.6, 0.8), red), (0.3, 0.0, 0.0)), 25.0)
    fog = tw.constant_medium(tw.sphere(white, (-1.2, 0.7, 0.0), 0.7), 0.9, phase)
    group = tw.bvh([inner, fog, tw.sphere(metal, (1.4, 0.5, 0.3), 0.5), tw.sphere(glass, (0.2, 0.4, 1.3), 0.4)])
    tw.push(tw.translate(tw.rotate_y(group, -30.0), (0.0, 0.0, -1.0)))
    # Translate(RotateY(medium(Translate(RotateY(box))))): a medium under instances with an
    # instanced boundary, like cornell_smoke's boxes one level further down
    smoke = tw.constant_medium(tw.translate(tw.rotate_y(tw.box((0.0, 0.0, 0.0), (1.0, 1.0, 1.0), white), 15.0),
                                            (-0.5, 0.0, -0.5)), 1.5, phase)
    tw.push(tw.translate(tw.rotate_y(smoke, 40.0), (-2.5, 0.0, 1.5)))
    # a medium bounded by a bare BVH of two spheres
    tw.push(tw.constant_medium(tw.bvh([tw.sphere(white, (2.6, 0.6, 1.8), 0.6), tw.sphere(white, (3.3, 0.6, 1.8), 0.6)]),
                               1.2, phase))
    # an instance over an instance over a BVH of spheres (a chain of 3 ops)
    balls = tw.bvh([tw.sphere(white, (0.4 * i, 0.25, 0.0), 0.2) for i in range(6)])
    tw.push(tw.translate(tw.rotate_y(tw.translate(balls, (-1.0, 0.0, 0.0)), 70.0), (1.5, 0.0, -3.0)))
    return tw


def test_nested_world_matches_oracle(rt, renderer):
    tw = _nested_world(rt)
    soa = tw.product.flatten()
    assert soa.n_media == 3 and soa.n_instances >= 5
    got, ref = _render_both(rt, renderer, tw, 48, 32, 6, (7.0, 4.0, 9.0), (0.0, 0.7, 0.0), (0.5, 0.6, 0.8))
    assert renderer.stats().variant_features == 4095          # media under instances: the all-features variant
    assert float(ref.max()) > 0.0
    assert_parity(got, ref, "nested world")


def test_nested_world_accel_modes_and_f32(rt, renderer):
    """The same world through the LINEAR and MEDIAN lowerings gives the same bits; the f32
    mode renders it too (finite, mean within 10 % of the f64 image)."""
    tw = _nested_world(rt)
    imgs = [_render_both(rt, renderer, tw, 32, 24, 4, (7.0, 4.0, 9.0), (0.0, 0.7, 0.0), (0.5, 0.6, 0.8), accel=a)[0]
            for a in (rt.RT_ACCEL_SAH, rt.RT_ACCEL_LINEAR, rt.RT_ACCEL_MEDIAN)]
    for im in imgs[1:]:
        assert np.array_equal(im, imgs[0])
    renderer.set_precision(rt.RT_PREC_F32)
    try:
        f32 = _render_both(rt, renderer, tw, 32, 24, 32, (7.0, 4.0, 9.0), (0.0, 0.7, 0.0), (0.5, 0.6, 0.8))[0]
    finally:
        renderer.set_precision(rt.RT_PREC_F64)
    f64 = _render_both(rt, renderer, tw, 32, 24, 32, (7.0, 4.0, 9.0), (0.0, 0.7, 0.0), (0.5, 0.6, 0.8))[0]
    assert np.all(np.isfinite(f32)) and abs(float(f32.mean()) / float(f64.mean()) - 1.0) < 0.1


def _moving_world(rt, t0, t1):
    tw = ob.TwinWorld(rt, 3)
    white = tw.lambertian(tw.checker((0.2, 0.3, 0.1), (0.9, 0.9, 0.9)))
    red = tw.lambertian(tw.solid(0.7, 0.1, 0.1))
    metal = tw.metal((0.8, 0.8, 0.9), 0.2)
    tw.push(tw.sphere(white, (0.0, -1000.0, 0.0), 1000.0))
    for i in range(5):
        c0 = (-2.0 + i, 0.3, 0.2 * i)
        tw.push(tw.moving_sphere(red if i % 2 else metal, c0, (c0[0], c0[1] + 0.4, c0[2]), t0, t1, 0.3))
    tw.push(tw.moving_sphere(red, (0.5, 1.2, -1.0), (0.9, 1.2, -1.0), 0.0, 1.0, 0.4))
    return tw


@pytest.mark.parametrize("t0,t1,feat", [(0.0, 1.0, 0), (0.25, 0.75, 4095), (-1.0, 2.0, 4095)])
def test_moving_sphere_shutters_match_oracle(rt, renderer, t0, t1, feat):
    """MovingSphere::center (hittable.rs:556-558) for any shutter: [0, 1] shutters (every
    reference scene) take the spheres variant, which loads no per-primitive shutter flag;
    another shutter selects FEAT_SHUTTER (the all-features variant) and its division."""
    tw = _moving_world(rt, t0, t1)
    got, ref = _render_both(rt, renderer, tw, 40, 24, 6, (6.0, 2.0, 5.0), (0.0, 0.5, 0.0), (0.7, 0.8, 1.0))
    assert renderer.stats().variant_features == feat
    assert_parity(got, ref, f"moving spheres, shutter [{t0}, {t1}]")


@pytest.mark.parametrize("moving", [False, True])
def test_instanced_spheres_static_or_moving_match_oracle(rt, renderer, moving):
    """Spheres under an instance (Translate(RotateY(BVH)), the final scene's cluster shape):
    all static -> the final-scene variant, whose nested sphere tests load no velocity
    (FEAT_STATIC); one moving sphere among them (FEAT_NEST_MOVING) -> the all-features
    variant with the moving centre (hittable.rs:556-558). Both against the oracle."""
    from tests.oracle_binding import TwinWorld
    tw = TwinWorld(rt)
    white = tw.lambertian(tw.solid(0.73, 0.73, 0.73))
    red = tw.lambertian(tw.solid(0.65, 0.05, 0.05))
    ids = [tw.sphere(white, (0.5 * i - 1.0, 0.3 + 0.1 * (i % 3), 0.2 * (i % 2)), 0.25) for i in range(6)]
    if moving:
        ids.append(tw.moving_sphere(red, (0.0, 1.0, 0.0), (0.3, 1.2, 0.0), 0.0, 1.0, 0.3))
    tw.push(tw.translate(tw.rotate_y(tw.bvh(ids), 25.0), (0.2, 0.0, -0.5)))
    tw.push(tw.sphere(white, (0.0, -100.0, 0.0), 100.0))
    got, ref = _render_both(rt, renderer, tw, 40, 24, 6, (5.0, 2.0, 6.0), (0.0, 0.5, 0.0), (0.7, 0.8, 1.0))
    assert renderer.stats().variant_features == (4095 if moving else 287)
    assert_parity(got, ref, f"instanced spheres (moving={moving})")


@pytest.mark.parametrize("n_spheres", [3, 40])
def test_shared_blas_under_two_instances_matches_oracle(rt, renderer, n_spheres):
    """Two instances over one BVH (a single-leaf BVH of 3 spheres, or a 40-sphere tree): the
    upload rewrites a BLAS's leaf codes relative to its first slot once, keeps the base in the
    device instance record for both instances (16-bit stack entries in the final-scene
    variant), and both copies must render as the oracle does."""
    tw = ob.TwinWorld(rt)
    white = tw.lambertian(tw.solid(0.73, 0.73, 0.73))
    glass = tw.dielectric(1.5)
    ids = [tw.sphere(glass if i % 3 == 0 else white, (0.3 * (i % 8) - 1.0, 0.25 + 0.3 * (i // 8), 0.1 * (i % 2)), 0.14)
           for i in range(n_spheres)]
    balls = tw.bvh(ids)
    tw.push(tw.translate(tw.rotate_y(balls, 30.0), (-0.8, 0.0, 0.0)))
    tw.push(tw.translate(balls, (1.0, 0.0, -0.6)))
    tw.push(tw.sphere(white, (0.0, -100.0, 0.0), 100.0))
    got, ref = _render_both(rt, renderer, tw, 48, 32, 6, (3.0, 2.0, 6.0), (0.0, 0.6, 0.0), (0.7, 0.8, 1.0))
    assert renderer.stats().variant_features == 287
    assert_parity(got, ref, f"shared BLAS ({n_spheres} spheres)")


def _sphere_field(rt, n):
    """A spheres-only world of n small spheres on a grid plus the ground (the spheres variant)."""
    tw = ob.TwinWorld(rt, 4)
    ground = tw.lambertian(tw.checker((0.2, 0.3, 0.1), (0.9, 0.9, 0.9)))
    mats = [tw.lambertian(tw.solid(0.7, 0.2, 0.1)), tw.metal((0.8, 0.8, 0.9), 0.1), tw.dielectric(1.5)]
    tw.push(tw.sphere(ground, (0.0, -1000.0, 0.0), 1000.0))
    side = int(np.ceil(np.sqrt(n)))
    for i in range(n):
        x, z = i % side, i // side
        tw.push(tw.sphere(mats[i % 3], (-6.0 + 12.0 * x / side, 0.12, -6.0 + 12.0 * z / side), 0.1))
    return tw


@pytest.mark.parametrize("n", [300, 1100])
def test_sphere_fields_both_stack_widths_match_oracle(rt, renderer, n):
    """The spheres variant keeps 16-bit LDS stack entries when its TLAS node records lie
    below 32 KB of LDS and its leaf codes fit (SceneDev.stack16_ok: <= 408 TLAS nodes, <= 1023
    leaf slots); 1100 spheres exceed that and take the partial-TLAS instantiation with
    32-bit entries. Both against the oracle."""
    tw = _sphere_field(rt, n)
    got, ref = _render_both(rt, renderer, tw, 32, 20, 3, (7.0, 2.0, 6.0), (0.0, 0.0, 0.0), (0.7, 0.8, 1.0))
    assert renderer.stats().variant_features == 0
    assert_parity(got, ref, f"sphere field of {n}")


def _box_world(rt):
    """Top-level boxes that stress the box test's edge cases (box_t's six sides under f32 slab
    padding): a grid of unit boxes on integer coordinates (shared edge planes, exact ties at edges), boxes
    of thickness 0, 1e-12, 1e-7 and 1e-3 (thinner than their padding: both sides of an axis are
    candidates), boxes near the scene extent, a box the camera's rays start inside (exit sides
    win), metal and glass boxes (rays leave from and re-enter box faces) and a light."""
    tw = ob.TwinWorld(rt, 9)
    white = tw.lambertian(tw.solid(0.73, 0.73, 0.73))
    red = tw.lambertian(tw.checker((0.65, 0.05, 0.05), (0.9, 0.9, 0.9)))
    metal = tw.metal((0.8, 0.8, 0.9), 0.05)
    glass = tw.dielectric(1.5)
    light = tw.diffuse_light(tw.solid(5.0, 5.0, 5.0))
    for i in range(-5, 5):
        for j in range(-5, 5):
            h = 1.0 + ((i * 7 + j * 3) % 4)
            tw.push(tw.box((float(i), 0.0, float(j)), (float(i + 1), h, float(j + 1)),
                           (white, red, metal)[(i + j) % 3]))
    for k, th in enumerate((0.0, 1e-12, 1e-7, 1e-3)):
        tw.push(tw.box((-6.0 + 3.0 * k, 5.0, -7.0), (-4.0 + 3.0 * k, 5.0 + th, -5.0), white))
        tw.push(tw.box((6.5, 1.0 + 1.5 * k, -3.0 + 2.0 * k), (6.5 + th, 2.0 + 1.5 * k, -1.5 + 2.0 * k), red))
    tw.push(tw.box((-2.0, 5.5, -2.0), (2.0, 6.0, 2.0), glass))
    tw.push(tw.box((990.0, -10.0, -10.0), (1000.0, 300.0, 10.0), white))     # near the extent
    tw.push(tw.box((-30.0, -1.0, -30.0), (30.0, 40.0, 30.0), white))         # encloses everything
    tw.push(tw.xz_rect(light, -3.0, 3.0, -3.0, 3.0, 12.0))
    return tw


@pytest.mark.parametrize("look_from,look_at", [((13.0, 9.0, 11.0), (0.0, 1.0, 0.0)), ((0.5, 3.0, 0.5), (0.7, 0.0, 0.2)),
                                               ((-8.0, 5.0, -6.0), (6.5, 2.5, -2.0))])
def test_box_world_on_final_variant_matches_oracle(rt, look_from, look_at):
    """Boxes on the final-scene variant (the one C4's 400 ground boxes run on;
    RT_OPT_EXTRA_FEATURES adds the noise bit so a world of boxes selects it): grid-aligned
    edges, boxes thinner than their f32 padding, rays starting inside a box, against the
    oracle to the parity bar. (The candidate-side box test this once compared against is a
    rejected experiment, scripts/experiments/r05_rejected_experiments.patch.)"""
    tw = _box_world(rt)
    W, H, spp = 64, 40, 6
    cam = rt.camera_new(look_from, look_at, (0.0, 1.0, 0.0), 50.0, W / H, 0.1, 10.0, 0.0, 1.0)
    bg = (0.3, 0.35, 0.4)
    p = rt.Renderer.params(W, H, spp, 50, bg, 1, out_format=rt.RT_OUT_F64)
    r = rt.Renderer(0)
    r.set_option(rt.RT_OPT_EXTRA_FEATURES, 8)
    try:
        r.upload(tw.product)
        img = r.render(cam, p)
        assert r.stats().variant_features == 287 and r.stats().slab32 == 1
    finally:
        r.close()
    ref = tw.oracle.render(_cam24(cam), bg, W, H, spp)
    assert float(ref.max()) > 0.0
    assert_parity(img, ref, "box world")


@pytest.mark.parametrize("world", ["instanced", "shared", "nested"])
def test_instanced_bvh_worlds_match_oracle(rt, renderer, world):
    """Instances over BVHs of simple primitives (a deferred nested walk per cast): one instanced
    cluster, one BLAS shared by two instances, and the general nesting world, against the
    oracle's recursive list walk."""
    if world == "instanced":
        tw = ob.TwinWorld(rt)
        white = tw.lambertian(tw.solid(0.73, 0.73, 0.73))
        glass = tw.dielectric(1.5)
        ids = [tw.sphere(glass if i % 4 == 0 else white, (0.5 * i - 1.0, 0.3 + 0.1 * (i % 3), 0.2 * (i % 2)), 0.25)
               for i in range(12)]
        tw.push(tw.translate(tw.rotate_y(tw.bvh(ids), 25.0), (0.2, 0.0, -0.5)))
        tw.push(tw.sphere(white, (0.0, -100.0, 0.0), 100.0))
        view = ((5.0, 2.0, 6.0), (0.0, 0.5, 0.0))
    elif world == "shared":
        tw = ob.TwinWorld(rt)
        white = tw.lambertian(tw.solid(0.73, 0.73, 0.73))
        balls = tw.bvh([tw.sphere(white, (0.3 * (i % 8) - 1.0, 0.25 + 0.3 * (i // 8), 0.1 * (i % 2)), 0.14)
                        for i in range(40)])
        tw.push(tw.translate(tw.rotate_y(balls, 30.0), (-0.8, 0.0, 0.0)))
        tw.push(tw.translate(balls, (1.0, 0.0, -0.6)))
        tw.push(tw.sphere(white, (0.0, -100.0, 0.0), 100.0))
        view = ((3.0, 2.0, 6.0), (0.0, 0.6, 0.0))
    else:
        tw = _nested_world(rt)
        view = ((7.0, 4.0, 9.0), (0.0, 0.7, 0.0))
    W, H, spp, bg = 48, 32, 6, (0.7, 0.8, 1.0)
    cam = rt.camera_new(view[0], view[1], (0.0, 1.0, 0.0), 40.0, W / H, 0.1, 10.0, 0.0, 1.0)
    p = rt.Renderer.params(W, H, spp, 50, bg, 1, out_format=rt.RT_OUT_F64)
    renderer.upload(tw.product)
    img = renderer.render(cam, p)
    ref = tw.oracle.render(_cam24(cam), bg, W, H, spp)
    assert_parity(img, ref, f"instanced BVHs ({world})")
