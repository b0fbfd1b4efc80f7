"""CPU-side checks of the product library: it loads, exports every symbol the header
declares, and its host scene model reproduces the oracle's scenes and cameras exactly
(no GPU needed — no compute calls)."""
import ctypes
import os
import re

import numpy as np
import pytest

from tests import oracle_binding as ob

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "rt", "rt_abi.h")


def header_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_header_symbol(rt):
    lib = rt.load_library()
    declared = header_symbols()
    assert len(declared) >= 30
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing
    assert sorted(declared) == sorted(rt.EXPORTED)
    assert lib.rt_abi_version() == 6


@pytest.mark.parametrize("scene_id", range(8))
def test_scene_builders_match_oracle(rt, scene_id):
    """Same draw order as the reference builders (main.rs:52-289, incl. BVH axis draws and Perlin tables)."""
    w = rt.World(7).build_scene(scene_id)
    info = w.info()
    o = ob.scene_info(scene_id, 7)
    assert info.n_hittables == o["n_hittables"]
    assert info.n_materials == o["n_materials"]
    assert info.n_leaf_prims == o["n_leaf_prims"]
    assert info.checksum == o["checksum"]


def test_random_scene_composition(rt):
    """main.rs:254-287: 1 ground + kept small spheres + 3 big; ~485 objects."""
    counts = [rt.World(s).build_scene(0).info().n_hittables for s in range(1, 21)]
    assert all(470 <= c <= 489 for c in counts)
    assert len(set(counts)) > 1          # the layout really depends on the seed


@pytest.mark.parametrize("scene_id", range(8))
def test_flatten_all_scenes(rt, scene_id):
    w = rt.World(1).build_scene(scene_id)
    soa = w.flatten()
    assert soa.n_prims >= 1 and soa.n_materials == w.info().n_materials
    if scene_id == 7:
        assert soa.n_instances == 1 and soa.n_media == 2 and soa.image_bytes == 1024 * 512 * 3
    if scene_id == 6:
        assert soa.n_media == 2 and soa.n_instances == 2


def test_build_options_change_the_tree_not_the_scene(rt):
    """rt_world_set_build_option (the SAH knobs, no environment variable): forcing every set of
    two into one leaf and disabling the Box-pair rule builds a different final-scene tree from
    the same primitives; the tables stay valid; an unknown key or a NaN is refused."""
    a = rt.SceneSoA.from_buffer_copy(rt.World(1).build_scene(7).flatten())
    w = rt.World(1).build_scene(7)
    w.set_build_option(rt.RT_BUILD_SPLIT_BOX_PAIRS, 0).set_build_option(rt.RT_BUILD_SPLIT_BLAS_PAIRS, 0)
    b = rt.SceneSoA.from_buffer_copy(w.flatten())
    assert a.n_prims == b.n_prims and a.n_prim_refs == b.n_prim_refs
    assert a.n_nodes != b.n_nodes
    rt.validate_soa(b)
    w.set_build_option(rt.RT_BUILD_SPLIT_BOX_PAIRS, -1).set_build_option(rt.RT_BUILD_SPLIT_BLAS_PAIRS, -1)
    c = rt.SceneSoA.from_buffer_copy(w.flatten())
    assert c.n_nodes == a.n_nodes   # defaults restored
    with pytest.raises(rt.RTError):
        w.set_build_option(99, 1.0)
    with pytest.raises(rt.RTError):
        w.set_build_option(rt.RT_BUILD_C_ISECT, float("nan"))


def test_library_build_identity_matches_sources(rt):
    """the loaded library carries the source hash it was compiled from
    (rt_build_info); it must be the hash of the tree it sits in, or profiles keyed by that hash
    would describe another build."""
    import __graft_entry__ as ge
    assert rt.build_info() == ge.source_hash(), (rt.build_info(), ge.source_hash())


NODE_DT = np.dtype([("lo0", "<f4", 3), ("hi0", "<f4", 3), ("lo1", "<f4", 3), ("hi1", "<f4", 3),
                    ("child", "<i4", 2), ("pad", "<i4", 2)])


def soa_tables(soa):
    def arr(ptr, dtype, n):
        if n == 0:
            return np.zeros(0, dtype)
        buf = (ctypes.c_char * (n * np.dtype(dtype).itemsize)).from_address(ptr)
        return np.frombuffer(bytes(buf), dtype=dtype)
    prims = arr(soa.prims, np.dtype((np.void, 96)), soa.n_prims)
    refs = arr(soa.prim_refs, "<i4", soa.n_prim_refs)
    nodes = arr(soa.nodes, NODE_DT, soa.n_nodes)
    inst = arr(soa.instances, np.dtype([("n_ops", "<i4"), ("kind", "<i4"), ("child", "<i4"), ("rest", "V116")]),
               soa.n_instances)
    return prims, refs, nodes, inst


def leaf_prims(code, refs):
    code = ~code
    return refs[(code >> 5):(code >> 5) + (code & 31)].tolist()


def reachable(root, refs, nodes):
    """Multiset of the primitives a full walk from a root reference tests."""
    out, todo = [], [root]
    while todo:
        r = todo.pop()
        if r < 0:
            out.extend(leaf_prims(r, refs))
        else:
            todo.extend(nodes[r]["child"].tolist())
    return out


@pytest.mark.parametrize("scene_id", range(8))
def test_accel_modes_cover_the_same_primitives(rt, scene_id):
    """LINEAR (hit_hittables' scan) and MEDIAN (the reference BvhNodes) lower the
    same primitive table as SAH; every primitive is reachable in every mode; LINEAR is a chain
    of unbounded nodes whose leaves come in list order; the recorded stack needs fit."""
    tabs, walks = {}, {}
    world = rt.World(1).build_scene(scene_id)      # owns the tables until the next flatten
    for accel in (rt.RT_ACCEL_SAH, rt.RT_ACCEL_LINEAR, rt.RT_ACCEL_MEDIAN):
        soa = rt.SceneSoA.from_buffer_copy(world.flatten(accel))   # the view is reused by the next flatten
        assert soa.accel == accel
        prims, refs, nodes, inst = soa_tables(soa)
        tabs[accel] = (prims, refs, nodes, soa)
        walk = reachable(soa.tlas_root, refs, nodes)
        for i in inst:
            if i["kind"] == 1:
                walk += reachable(int(i["child"]), refs, nodes)
        walks[accel] = walk
        assert 1 <= soa.tlas_depth <= 32 and 0 <= soa.blas_depth <= 32
    p0 = tabs[rt.RT_ACCEL_SAH][0]
    for accel in (rt.RT_ACCEL_LINEAR, rt.RT_ACCEL_MEDIAN):
        assert np.array_equal(tabs[accel][0], p0)            # identical primitive table
        assert set(walks[accel]) == set(walks[rt.RT_ACCEL_SAH])
    assert sorted(walks[rt.RT_ACCEL_LINEAR]) == sorted(walks[rt.RT_ACCEL_SAH])   # each exactly once
    _, refs, nodes, soa = tabs[rt.RT_ACCEL_LINEAR]
    if soa.n_nodes:
        assert np.all(np.isinf(nodes["lo0"])) and np.all(np.isinf(nodes["hi1"]))
        assert soa.tlas_depth == 2                           # a chain needs one stack entry
    order, r = [], soa.tlas_root                             # child 0 first = list order
    while r >= 0:
        c0, r = nodes[r]["child"].tolist()
        order += leaf_prims(c0, refs)
    order += leaf_prims(r, refs)
    assert order == sorted(order)


@pytest.mark.parametrize("scene_id,w,h", [(0, 1200, 800), (5, 800, 800), (7, 1920, 1080), (4, 64, 36)])
def test_camera_matches_oracle_bitwise(rt, scene_id, w, h):
    cam, _ = rt.scene_camera(scene_id, w, h)
    mine = np.array(list(cam.origin) + list(cam.lower_left_corner) + list(cam.horizontal) + list(cam.vertical) +
                    list(cam.u) + list(cam.v) + list(cam.w) + [cam.lens_radius, cam.time0, cam.time1])
    assert np.array_equal(mine, ob.camera(scene_id, w, h))


def test_camera_new_book_values(rt):
    cam = rt.camera_new((13, 2, 3), (0, 0, 0), (0, 1, 0), 20.0, 1.5, 0.1, 10.0, 0.0, 1.0)
    assert cam.lens_radius == 0.05
    w = np.array(cam.w)
    assert np.allclose(w, np.array([13, 2, 3]) / np.linalg.norm([13, 2, 3]))
    # viewport height 2*tan(10deg)*focus, width = aspect * height
    assert np.linalg.norm(cam.vertical) == pytest.approx(20 * np.tan(np.radians(10)), rel=1e-14)
    assert np.linalg.norm(cam.horizontal) == pytest.approx(1.5 * 20 * np.tan(np.radians(10)), rel=1e-14)


def test_presets_match_reference_table(rt):
    p = rt.scene_preset(7)   # main.rs:442-459
    assert tuple(p.look_from) == (478.0, 278.0, -600.0) and p.vfov == 40.0
    assert p.default_width == 800 and p.default_spp == 2000 and p.aperture == 0.1 and p.focus_dist == 10.0
    p0 = rt.scene_preset(0)  # main.rs:316-333
    assert tuple(p0.background) == (0.7, 0.8, 1.0) and p0.default_spp == 100
    with pytest.raises(rt.RTError):
        rt.scene_preset(8)   # main.rs:461-463 panics


def test_errors_do_not_abort(rt):
    w = rt.World(1)
    with pytest.raises(rt.RTError):
        w.sphere(1, (0, 0, 0), 1.0)         # no material 1 yet
    m = w.lambertian(w.solid(0.5, 0.5, 0.5))
    assert m == 1                            # 1-based handles (main.rs:46-49)
    with pytest.raises(rt.RTError):
        w.push(12345)
    with pytest.raises(rt.RTError):
        w.build_scene(42)
    lib = rt.load_library()
    assert lib.rt_ctx_create(0, None) == -1
    assert lib.rt_render(None, None, None, None) == -1
    assert lib.rt_rows_in_shard(800, 3, 8) == 100
    assert lib.rt_rows_in_shard(7, 3, 8) == 1
    assert lib.rt_rows_in_shard(7, 7, 8) == 0
    # progressive accumulation entry points reject null handles before touching a device
    assert lib.rt_accum_create(None, None, None) == -1
    assert lib.rt_accum_add(None, None, None, None, 4) == -1
    assert lib.rt_accum_get(None, None, None) == -1
    assert lib.rt_accum_set(None, None, 0) == -1
    assert lib.rt_accum_resolve(None, None, 0.0, 0, 0, None) == -1
    assert lib.rt_render_progressive(None, None, None, 1, rt.PROGRESS_FN(), None, None) == -1
    lib.rt_accum_destroy(None)
    # multi-GPU entry points (ABI v5) check their arguments before loading RCCL or touching a device
    assert lib.rt_comm_init_rank(None, 0, 1, None, None) == -1
    assert lib.rt_comm_init_all(None, 0, None) == -1
    assert lib.rt_comm_tile_order(None, None, None, 8) == -1
    assert lib.rt_render_gather(None, None, None, None) == -1
    assert lib.rt_render_gather_all(None, 0, None, None, None) == -1
    assert lib.rt_comm_last_stats(None, None) == -1
    assert lib.rt_tiles_assemble(None, None, 0, 1, None, None) == -1
    assert lib.rt_comm_rank(None, None, None) == -1
    lib.rt_comm_destroy(None)
    with pytest.raises(rt.RTError):
        w.flatten(7)                         # unknown accel mode


def test_unsupported_nesting_reported(rt):
    """What the lowering still refuses: chains of more than 4 Translate/RotateY ops, and a
    medium boundary that holds a medium."""
    w = rt.World(1)
    m = w.lambertian(w.solid(1, 1, 1))
    x = w.sphere(m, (0, 0, 0), 1.0)
    for i in range(5):
        x = w.translate(x, (1, 0, 0))
    w.push(x)
    with pytest.raises(rt.RTError, match="UNSUPPORTED"):
        w.flatten()
    w = rt.World(1)
    m = w.lambertian(w.solid(1, 1, 1))
    phase = w.isotropic(w.solid(1, 1, 1))
    inner = w.constant_medium(w.sphere(m, (0, 0, 0), 1.0), 0.5, phase)
    boundary = w.translate(w.bvh([inner, w.sphere(m, (3, 0, 0), 1.0)]), (0, 1, 0))
    w.push(w.constant_medium(boundary, 0.1, phase))
    with pytest.raises(rt.RTError, match="UNSUPPORTED"):
        w.flatten()


def test_nested_instances_and_media_flatten(rt):
    """hittable.rs:30-41 composes freely: instances over instances, instances over BVHs of
    instances and media, media under instances, a bare BVH as a medium boundary. The lowering
    pushes Translate/RotateY chains down (flatten.cpp lower_instance): every instance ends on
    one primitive, one medium or a BLAS of primitives, and validation accepts the tables."""
    w = rt.World(2)
    m = w.lambertian(w.solid(0.5, 0.5, 0.5))
    phase = w.isotropic(w.solid(0.8, 0.8, 0.8))
    inner = w.rotate_y(w.translate(w.box((0, 0, 0), (1, 2, 1), m), (0.5, 0, 0)), 20.0)
    fog = w.constant_medium(w.sphere(m, (0, 1, 0), 0.8), 0.7, phase)
    group = w.bvh([inner, fog, w.sphere(m, (2, 0.5, 0), 0.5), w.sphere(m, (-2, 0.5, 0), 0.5)])
    w.push(w.translate(w.rotate_y(group, -30.0), (0, 0, 3)))
    w.push(w.constant_medium(w.bvh([w.sphere(m, (5, 1, 0), 1.0), w.sphere(m, (6, 1, 0), 1.0)]), 0.3, phase))
    soa = w.flatten()
    assert soa.n_media == 2 and soa.n_instances == 4   # box chain, fog, the spheres' BLAS, the bare-BVH boundary
    assert rt.validate_soa(rt.SceneSoA.from_buffer_copy(soa)) == (soa.tlas_depth, soa.blas_depth)


def test_custom_world_flattens(rt):
    """The reference's constructor surface composes: BVH over boxes, instances, media."""
    w = rt.World(3)
    white = w.lambertian(w.solid(0.73, 0.73, 0.73))
    boxes = [w.box((i, 0, 0), (i + 0.5, 1, 1), white) for i in range(10)]
    w.push(w.bvh(boxes))
    inst = w.translate(w.rotate_y(w.bvh([w.sphere(white, (0, j, 0), 0.3) for j in range(5)]), 30.0), (0, 0, 5))
    w.push(inst)
    w.push(w.constant_medium(w.sphere(white, (0, 0, 0), 50.0), 0.01, w.isotropic(w.solid(1, 1, 1))))
    w.push(w.xy_rect(w.diffuse_light(w.solid(4, 4, 4)), 0, 1, 0, 1, -2))
    soa = w.flatten()
    assert soa.n_instances == 1 and soa.n_media == 1
    assert w.info().n_leaf_prims == 10 + 5 + 1 + 1


def test_ppm_writer_reference_format(rt, tmp_path):
    """math.rs:119-132 + main.rs:472,591-596: P3, blank line after 255, rows top to bottom, NaN -> 0."""
    img = np.zeros((2, 3, 3), np.float32)
    img[1, 0] = [1.0, 0.25, 0.0]    # top-left pixel (row 1 = top since y = 0 is the bottom)
    img[0, 2] = [np.nan, 4.0, 0.5]  # bottom-right
    path = tmp_path / "x.ppm"
    rt.write_ppm(img, str(path))
    lines = path.read_text().split("\n")
    assert lines[:4] == ["P3", "3 2", "255", ""]
    assert lines[4] == "255 128 0"           # (int)(256 * clamp(sqrt(x), 0, .999))
    assert lines[4 + 5] == "0 255 181"       # NaN -> 0, clamp to .999 -> 255, sqrt(.5)*256 = 181.02
    assert len([l for l in lines[4:] if l]) == 6


def _boundary_values():
    """Channel values within a few ulp of every write_color rounding boundary: 256*sqrt(m) = k
    at m = k^2/65536 (k = 1..255), the clamp's 0.999^2, plus the special cases (0, -0, tiny,
    negative, NaN, +-inf, huge)."""
    ms = []
    for k in range(0, 257):
        b = k * k / 65536.0
        v = b
        for _ in range(4):
            v = np.nextafter(v, -np.inf)
            ms.append(v)
        v = b
        ms.append(v)
        for _ in range(4):
            v = np.nextafter(v, np.inf)
            ms.append(v)
    c = 0.999 * 0.999
    ms += [np.nextafter(c, -np.inf), c, np.nextafter(c, np.inf), 0.0, -0.0, 5e-324, -1e-300, -1.0,
           np.nan, np.inf, -np.inf, 1e308, 0.5, 1.0, 2.0]
    return np.array(ms, dtype=np.float64)


def _py_write_color(x, spp):
    """An independent Python restatement of write_color (math.rs:119-132) for one channel."""
    import math
    scale = 1.0 / spp
    y = x * scale
    r = math.sqrt(y) if y >= 0 else float("nan")
    c = 0.0 if r < 0.0 else 0.999 if r > 0.999 else r
    v = 256.0 * c
    return 0 if v != v else int(v)


def test_write_color_f64_at_rounding_boundaries(rt):
    """rt_write_color (the product's f64 write_color) equals the oracle's restatement and an
    independent Python one on means placed within 4 ulp of every k^2/65536 boundary, and on sums
    over spp = 10 / 500 / 1000 / 4096 samples built near the same boundaries (sum * (1/spp) lands
    on either side of them): VERDICT r03 item 1."""
    from tests import oracle_binding as ob
    m = _boundary_values()
    for spp in (1, 10, 500, 1000, 4096):
        with np.errstate(over="ignore"):   # 1e308 * spp -> inf: one more special case
            x = m * spp if spp > 1 else m
        if spp > 1:   # the sums' own neighbours too, so x * (1/spp) straddles each boundary
            x = np.concatenate([x, np.nextafter(x, np.inf), np.nextafter(x, -np.inf)])
        x = x[: len(x) // 3 * 3].reshape(-1, 1, 3)
        got = rt.write_color(x, spp)
        want = ob.write_color(x, spp)
        assert np.array_equal(got, want), spp
        py = np.array([_py_write_color(float(v), spp) for v in x.reshape(-1)], np.int32).reshape(x.shape)
        assert np.array_equal(got, py), spp


def test_ppm_f64_file_equals_oracle_bytes(rt, tmp_path):
    """rt_write_ppm_f64 writes the oracle's orc_write_ppm bytes (header, row order, values) on a
    frame of boundary means, and on the same frame as sums over 500 samples."""
    from tests import oracle_binding as ob
    m = _boundary_values()
    n = len(m) // 3 // 7 * 7 * 3
    img = m[:n].reshape(-1, 7, 3)          # rows x 7 x 3
    for spp, data in ((1, img), (500, img * 500)):
        a, b = tmp_path / f"p{spp}.ppm", tmp_path / f"o{spp}.ppm"
        rt.write_ppm(data, str(a), samples_per_pixel=spp)
        ob.write_ppm(data, str(b), samples_per_pixel=spp)
        assert a.read_bytes() == b.read_bytes()
        assert a.read_bytes().startswith(b"P3\n7 %d\n255\n\n" % img.shape[0])


def test_f32_frame_writer_can_differ_at_boundaries(rt):
    """Why the f64 writer exists: rounding the mean to f32 first (rt_write_ppm, the f32 frame)
    moves some boundary means across k^2/65536."""
    m = _boundary_values()
    m = m[np.isfinite(m) & (m > 0) & (m < 1)]
    f64 = np.array([_py_write_color(float(v), 1) for v in m])
    f32 = np.array([_py_write_color(float(np.float32(v)), 1) for v in m])
    assert (f64 != f32).sum() > 0


# ---- rt_scene_validate (a foreign SoA must not overrun the traversal stack or
# make the persistent kernel walk a cycle; the depth fields are not trusted)

def _soa_with_nodes(rt, world, accel=0):
    soa = rt.SceneSoA.from_buffer_copy(world.flatten(accel))
    _, _, nodes, _ = soa_tables(soa)
    nodes = nodes.copy()
    soa.nodes = nodes.ctypes.data
    return soa, nodes


@pytest.mark.parametrize("scene_id", range(8))
def test_validate_recomputes_flatten_depths(rt, scene_id):
    world = rt.World(1).build_scene(scene_id)
    for accel in (rt.RT_ACCEL_SAH, rt.RT_ACCEL_LINEAR, rt.RT_ACCEL_MEDIAN):
        soa = rt.SceneSoA.from_buffer_copy(world.flatten(accel))
        assert rt.validate_soa(soa) == (soa.tlas_depth, soa.blas_depth), accel


def test_validate_ignores_understated_depths(rt):
    world = rt.World(1).build_scene(7)
    soa = rt.SceneSoA.from_buffer_copy(world.flatten())
    true = (soa.tlas_depth, soa.blas_depth)
    assert true[0] > 2 and true[1] > 1
    soa.tlas_depth, soa.blas_depth = 1, 0           # a foreign host that under-reports
    assert rt.validate_soa(soa) == true


def test_validate_rejects_cycles_and_bad_refs(rt):
    world = rt.World(1).build_scene(0)
    soa, nodes = _soa_with_nodes(rt, world)
    assert soa.n_nodes > 4
    inner = [i for i in range(soa.n_nodes) if nodes[i]["child"][0] >= 0]
    i = inner[-1]
    nodes[i]["child"][1] = soa.tlas_root            # back edge to the root: a cycle
    with pytest.raises(rt.RTError, match="cycle"):
        rt.validate_soa(soa)
    soa, nodes = _soa_with_nodes(rt, world)
    nodes[0]["child"][0] = soa.n_nodes              # node index out of range
    with pytest.raises(rt.RTError, match="bad node"):
        rt.validate_soa(soa)
    soa, nodes = _soa_with_nodes(rt, world)
    nodes[0]["child"][0] = ~((soa.n_prim_refs << 5) | 3)   # leaf range past the prim refs
    with pytest.raises(rt.RTError, match="bad node"):
        rt.validate_soa(soa)
    soa, nodes = _soa_with_nodes(rt, world)
    nodes[0]["child"][1] = nodes[0]["child"][0]     # a DAG (shared child) is legal
    rt.validate_soa(soa)


def test_validate_rejects_a_chain_deeper_than_the_stack(rt):
    """A node chain whose walk needs more than 32 stack entries is refused (the kernel's
    scratch stack holds 32 TLAS + 32 BLAS entries)."""
    w = rt.World(1)
    m = w.lambertian(w.solid(0.5, 0.5, 0.5))
    for i in range(40):
        w.push(w.sphere(m, (float(i), 0.0, 0.0), 0.4))
    soa, nodes = _soa_with_nodes(rt, w)
    n = 40
    deep = np.zeros(n, dtype=NODE_DT)               # a left-deep chain: node k -> (node k+1, leaf k)
    for k in range(n):
        deep[k]["lo0"] = deep[k]["lo1"] = (-1e3, -1e3, -1e3)
        deep[k]["hi0"] = (1e3, 1e3, 1e3)
        deep[k]["hi1"] = (2e3, 1e3, 1e3)            # different boxes: either side may go first
        deep[k]["child"] = (k + 1 if k + 1 < n else ~((0 << 5) | 1), ~((k % soa.n_prim_refs << 5) | 1))
    soa.nodes, soa.n_nodes, soa.tlas_root, soa.n_tlas_nodes = deep.ctypes.data, n, 0, n
    with pytest.raises(rt.RTError, match="UNSUPPORTED"):
        rt.validate_soa(soa)


def test_ctypes_structs_match_the_c_header(rt, tmp_path):
    """The Python binding's ctypes mirrors of the ABI's structs (rt_stats, rt_render_params,
    rt_camera, rt_scene_preset, rt_world_info, rt_scene_soa) have the C header's size and field
    offsets (compiled here with gcc against include/rt/rt_abi.h)."""
    import subprocess
    import ctypes
    structs = {"rt_stats": rt.Stats, "rt_render_params": rt.RenderParams, "rt_camera": rt.Camera,
               "rt_scene_preset": rt.ScenePreset, "rt_world_info": rt.WorldInfo, "rt_scene_soa": rt.SceneSoA,
               "rt_comm_stats": rt.CommStats}
    src = ['#include <stdio.h>', '#include <stddef.h>', '#include "rt/rt_abi.h"', "int main(void) {"]
    for cname, py in structs.items():
        src.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            if not f.startswith("pad"):
                src.append(f'printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    src.append("return 0; }")
    c = tmp_path / "layout.c"
    c.write_text("\n".join(src))
    exe = tmp_path / "layout"
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    subprocess.run(["gcc", "-I" + inc, str(c), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    for line in out:
        if not line:
            continue
        cname, field, val = line.split()
        py = structs[cname]
        got = ctypes.sizeof(py) if field == "size" else getattr(py, field).offset
        assert got == int(val), (cname, field, got, int(val))
