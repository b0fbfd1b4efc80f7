"""rtiow_amd — Python host binding over the C ABI (include/rt/rt_abi.h).

This mirrors the reference's host surface (themeshpotato/rust-ray-tracing-in-a-weekend):
``World`` + ``register_material`` (main.rs:40-50), the Hittable / Material / Texture
constructors (hittable.rs:77-207, material.rs:6-12, texture.rs:4-22), the scene
builders (main.rs:52-289), ``Camera::new`` (camera.rs:18-56) and the render loop
(main.rs:497-551, ray_color main.rs:19-38), which here runs as the HIP megakernel in
``lib/librtiow_amd.so``.

There is no CPU fallback: if the shared library is missing or no GPU is visible,
``Renderer`` raises. (The CPU oracle under oracle/ is test infrastructure only.)
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RT_LIB_PATH", os.path.join(HERE, "lib", "librtiow_amd.so"))
REPO = os.path.dirname(HERE)
EARTH_JPG = os.path.join(REPO, "assets", "earthmap.jpg")

RT_OK = 0
ERRORS = {-1: "RT_ERR_INVALID", -2: "RT_ERR_HIP", -3: "RT_ERR_UNSUPPORTED", -4: "RT_ERR_OOM",
          -5: "RT_ERR_NO_DEVICE", -6: "RT_ERR_NO_SCENE", -7: "RT_ERR_COMM", -8: "RT_ERR_PEER"}
RT_COMM_ID_BYTES = 128

SCENES = {"random": 0, "two_spheres": 1, "two_perlin": 2, "earth": 3, "simple_light": 4,
          "cornell": 5, "cornell_smoke": 6, "final": 7}
SCENES_NEEDING_IMAGE = (3, 7)

RT_OUT_F32, RT_OUT_F64 = 0, 1
RT_SCHED_CHUNKS = 0
RT_SCHED_POOL = 1
RT_SCHED_ITEMS = 2
RT_SCHED_AUTO = 3
RT_PREC_F64 = 0
RT_PREC_F32 = 1
RT_ACCEL_SAH = 0
RT_ACCEL_LINEAR = 1     # hit_hittables linear scan (hittable.rs:31-41)
RT_ACCEL_MEDIAN = 2     # the reference BvhNode hierarchy (hittable.rs:77-130)
# context options (rt_ctx_set_option)
RT_OPT_TRACE_BUF_BYTES = 1
RT_OPT_BATCH_OVERLAP = 2
RT_OPT_BLOCK_SAMPLES = 3
RT_OPT_BLOCK_CHUNKS = 4
RT_OPT_EXTRA_FEATURES = 5
RT_OPT_HOIST = 6
RT_OPT_POOL_RING = 9
RT_OPT_COMM_DIRECT = 10
# SAH builder options (rt_world_set_build_option)
RT_BUILD_C_ISECT = 1
RT_BUILD_MAX_LEAF = 2
RT_BUILD_FORCE_LEAF = 3
RT_BUILD_ROOT_LEAF = 4
RT_BUILD_SPLIT_BOX_PAIRS = 5
RT_BUILD_SPLIT_BLAS_PAIRS = 6

# every symbol include/rt/rt_abi.h declares
EXPORTED = [
    "rt_abi_version", "rt_last_error", "rt_device_count", "rt_ctx_create", "rt_ctx_destroy",
    "rt_world_create", "rt_world_destroy", "rt_world_texture_solid", "rt_world_texture_checker",
    "rt_world_texture_noise", "rt_world_texture_image", "rt_world_material_lambertian",
    "rt_world_material_metal", "rt_world_material_dielectric", "rt_world_material_diffuse_light",
    "rt_world_material_isotropic", "rt_world_sphere", "rt_world_moving_sphere", "rt_world_rect",
    "rt_world_box", "rt_world_translate", "rt_world_rotate_y", "rt_world_constant_medium",
    "rt_world_bvh", "rt_world_push", "rt_world_build_scene", "rt_world_info_get", "rt_camera_new",
    "rt_scene_preset_get", "rt_scene_camera", "rt_world_flatten", "rt_ctx_upload_soa",
    "rt_ctx_upload_world", "rt_render", "rt_rows_in_shard", "rt_rows_in_band_shard", "rt_tiles_in_shard", "rt_last_stats", "rt_last_counters", "rt_write_ppm",
    "rt_write_ppm_f64", "rt_write_color",
    "rt_ctx_set_variant", "rt_device_eval", "rt_accum_create", "rt_accum_destroy", "rt_accum_add",
    "rt_accum_get", "rt_accum_set", "rt_accum_resolve", "rt_render_progressive", "rt_ctx_set_schedule", "rt_ctx_set_precision",
    "rt_scene_validate", "rt_build_info", "rt_ctx_set_option", "rt_ctx_get_option", "rt_world_set_build_option",
    "rt_last_tile_costs", "rt_ctx_set_tile_order",
    "rt_comm_unique_id", "rt_comm_init_rank", "rt_comm_init_all", "rt_comm_destroy", "rt_comm_rank",
    "rt_comm_tile_order", "rt_comm_tile_order_all", "rt_render_gather", "rt_render_gather_all",
    "rt_comm_last_stats", "rt_tiles_assemble", "rt_tiles_assemble_host", "rt_cost_tile_order",
]

# int (*rt_progress_fn)(void* user, int64_t samples_done, int64_t samples_total)
PROGRESS_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64)


class RTError(RuntimeError):
    pass


class Camera(ctypes.Structure):
    """rt_camera == the reference's Camera struct (camera.rs:4-15)."""
    _fields_ = [("origin", ctypes.c_double * 3), ("lower_left_corner", ctypes.c_double * 3),
                ("horizontal", ctypes.c_double * 3), ("vertical", ctypes.c_double * 3),
                ("u", ctypes.c_double * 3), ("v", ctypes.c_double * 3), ("w", ctypes.c_double * 3),
                ("lens_radius", ctypes.c_double), ("time0", ctypes.c_double), ("time1", ctypes.c_double)]


class ScenePreset(ctypes.Structure):
    _fields_ = [("look_from", ctypes.c_double * 3), ("look_at", ctypes.c_double * 3),
                ("background", ctypes.c_double * 3), ("vfov", ctypes.c_double),
                ("aperture", ctypes.c_double), ("focus_dist", ctypes.c_double),
                ("time0", ctypes.c_double), ("time1", ctypes.c_double),
                ("default_width", ctypes.c_int32), ("default_spp", ctypes.c_int32),
                ("default_aspect", ctypes.c_double)]


class WorldInfo(ctypes.Structure):
    _fields_ = [("n_hittables", ctypes.c_int32), ("n_materials", ctypes.c_int32),
                ("n_leaf_prims", ctypes.c_int32), ("n_media", ctypes.c_int32), ("checksum", ctypes.c_double)]


class SceneSoA(ctypes.Structure):
    _fields_ = [("n_prims", ctypes.c_int32), ("n_prim_refs", ctypes.c_int32), ("n_nodes", ctypes.c_int32),
                ("n_instances", ctypes.c_int32), ("n_materials", ctypes.c_int32), ("n_textures", ctypes.c_int32),
                ("n_perlin", ctypes.c_int32), ("n_media", ctypes.c_int32), ("tlas_root", ctypes.c_int32),
                ("accel", ctypes.c_int32), ("image_bytes", ctypes.c_int64), ("pad_extent", ctypes.c_double),
                ("tlas_depth", ctypes.c_int32), ("blas_depth", ctypes.c_int32),
                ("n_tlas_nodes", ctypes.c_int32), ("pad0", ctypes.c_int32),
                ("prims", ctypes.c_void_p), ("prim_refs", ctypes.c_void_p), ("nodes", ctypes.c_void_p),
                ("instances", ctypes.c_void_p), ("materials", ctypes.c_void_p), ("textures", ctypes.c_void_p),
                ("perlin_ranvec", ctypes.c_void_p), ("perlin_perm", ctypes.c_void_p),
                ("image_data", ctypes.c_void_p)]


class RenderParams(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("spp", ctypes.c_int32),
                ("max_depth", ctypes.c_int32), ("spp_chunk", ctypes.c_int32), ("row_begin", ctypes.c_int32),
                ("row_stride", ctypes.c_int32), ("out_format", ctypes.c_int32),
                ("out_on_device", ctypes.c_int32), ("count_work", ctypes.c_int32),
                ("background", ctypes.c_double * 3), ("render_seed", ctypes.c_uint64),
                ("stream", ctypes.c_void_p), ("row_block", ctypes.c_int32), ("tile_shard", ctypes.c_int32)]


class Stats(ctypes.Structure):
    _fields_ = [("kernel_ms", ctypes.c_double), ("reduce_ms", ctypes.c_double), ("samples", ctypes.c_uint64),
                ("casts", ctypes.c_uint64), ("node_visits", ctypes.c_uint64), ("prim_tests", ctypes.c_uint64),
                ("n_items", ctypes.c_uint64), ("n_chunks", ctypes.c_int32), ("spp_chunk", ctypes.c_int32),
                ("scene_bytes", ctypes.c_int64), ("node_bytes", ctypes.c_int32), ("prim_bytes", ctypes.c_int32),
                ("material_bytes", ctypes.c_int32), ("variant_features", ctypes.c_int32),
                ("slab32", ctypes.c_int32), ("lds_stack", ctypes.c_int32), ("lds_nodes", ctypes.c_int32),
                ("cycles_camera", ctypes.c_uint64),
                ("cycles_trace", ctypes.c_uint64), ("cycles_shade", ctypes.c_uint64),
                ("wave_steps", ctypes.c_uint64), ("wave_node_steps", ctypes.c_uint64),
                ("cycles_nodes", ctypes.c_uint64), ("cycles_leaves", ctypes.c_uint64),
                ("schedule", ctypes.c_int32), ("n_batches", ctypes.c_int32),
                ("wave_leaf_steps", ctypes.c_uint64), ("camera_lanes", ctypes.c_uint64),
                ("camera_steps", ctypes.c_uint64), ("shade_lanes", ctypes.c_uint64),
                ("shade_steps", ctypes.c_uint64), ("precision", ctypes.c_int32), ("waves_per_simd", ctypes.c_int32),
                ("trace_buf_bytes", ctypes.c_int64), ("overlapped", ctypes.c_int32), ("reserved0", ctypes.c_int32),
                ("ring_bytes", ctypes.c_int64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class CommStats(ctypes.Structure):
    """rt_comm_stats: the last rt_render_gather / rt_comm_tile_order of one rank."""
    _fields_ = [("render_ms", ctypes.c_double), ("gather_ms", ctypes.c_double), ("assemble_ms", ctypes.c_double),
                ("kernel_ms", ctypes.c_double), ("slab_bytes", ctypes.c_int64), ("tiles", ctypes.c_int32),
                ("tile_order", ctypes.c_int32), ("cost_pass_ms", ctypes.c_double), ("peer_failed", ctypes.c_int32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib = None


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Loads lib/librtiow_amd.so (built by __graft_entry__.build()); raises if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RTError(f"HIP library not built: {path} (run __graft_entry__.build())")
    lib = ctypes.CDLL(path)
    P, I, D, U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_uint64
    PI = ctypes.POINTER(ctypes.c_int)
    PD = ctypes.POINTER(ctypes.c_double)
    sigs = {
        "rt_abi_version": ([], I), "rt_last_error": ([], ctypes.c_char_p), "rt_build_info": ([], ctypes.c_char_p),
        "rt_ctx_set_option": ([P, I, ctypes.c_int64], I),
        "rt_ctx_get_option": ([P, I, ctypes.POINTER(ctypes.c_int64)], I),
        "rt_world_set_build_option": ([P, I, D], I),
        "rt_device_count": ([PI], I), "rt_ctx_create": ([I, ctypes.POINTER(P)], I),
        "rt_ctx_destroy": ([P], None), "rt_world_create": ([U64, ctypes.POINTER(P)], I),
        "rt_world_destroy": ([P], None), "rt_world_texture_solid": ([P, D, D, D, PI], I),
        "rt_world_texture_checker": ([P, PD, PD, PI], I), "rt_world_texture_noise": ([P, D, PI], I),
        "rt_world_texture_image": ([P, P, I, I, PI], I),
        "rt_world_material_lambertian": ([P, I, PI], I), "rt_world_material_metal": ([P, PD, D, PI], I),
        "rt_world_material_dielectric": ([P, D, PI], I), "rt_world_material_diffuse_light": ([P, I, PI], I),
        "rt_world_material_isotropic": ([P, I, PI], I), "rt_world_sphere": ([P, I, PD, D, PI], I),
        "rt_world_moving_sphere": ([P, I, PD, PD, D, D, D, PI], I),
        "rt_world_rect": ([P, I, I, D, D, D, D, D, PI], I), "rt_world_box": ([P, PD, PD, I, PI], I),
        "rt_world_translate": ([P, I, PD, PI], I), "rt_world_rotate_y": ([P, I, D, PI], I),
        "rt_world_constant_medium": ([P, I, D, I, PI], I), "rt_world_bvh": ([P, PI, I, D, D, PI], I),
        "rt_world_push": ([P, I], I), "rt_world_build_scene": ([P, I, P, I, I], I),
        "rt_world_info_get": ([P, ctypes.POINTER(WorldInfo)], I),
        "rt_camera_new": ([PD, PD, PD, D, D, D, D, D, D, ctypes.POINTER(Camera)], I),
        "rt_scene_preset_get": ([I, ctypes.POINTER(ScenePreset)], I),
        "rt_scene_camera": ([I, I, I, ctypes.POINTER(Camera), PD], I),
        "rt_world_flatten": ([P, I, ctypes.POINTER(ctypes.POINTER(SceneSoA))], I),
        "rt_ctx_upload_soa": ([P, ctypes.POINTER(SceneSoA)], I),
        "rt_scene_validate": ([ctypes.POINTER(SceneSoA), ctypes.POINTER(ctypes.c_int32),
                               ctypes.POINTER(ctypes.c_int32)], I), "rt_ctx_upload_world": ([P, P, I], I),
        "rt_render": ([P, ctypes.POINTER(Camera), ctypes.POINTER(RenderParams), P], I),
        "rt_rows_in_shard": ([I, I, I], I), "rt_rows_in_band_shard": ([I, I, I, I], I),
        "rt_tiles_in_shard": ([I, I, I, I], I), "rt_last_stats": ([P, ctypes.POINTER(Stats)], I),
        "rt_last_counters": ([P, P, I], I),
        "rt_last_tile_costs": ([P, P, ctypes.c_int64], I), "rt_ctx_set_tile_order": ([P, P, ctypes.c_int64], I),
        "rt_write_ppm": ([P, I, I, ctypes.c_char_p], I),
        "rt_write_ppm_f64": ([P, I, I, I, ctypes.c_char_p], I),
        "rt_write_color": ([P, I, ctypes.c_int64, P], I),
        "rt_device_eval": ([P, I, P, P, P, P, I], I), "rt_ctx_set_variant": ([P, I, I, I], I),
        "rt_accum_create": ([P, ctypes.POINTER(RenderParams), ctypes.POINTER(P)], I),
        "rt_ctx_set_schedule": ([P, I], I),
        "rt_ctx_set_precision": ([P, I], I),
        "rt_accum_destroy": ([P], None),
        "rt_accum_add": ([P, P, ctypes.POINTER(Camera), ctypes.POINTER(RenderParams), I], I),
        "rt_accum_get": ([P, P, ctypes.POINTER(ctypes.c_int64)], I),
        "rt_accum_set": ([P, P, ctypes.c_int64], I),
        "rt_accum_resolve": ([P, P, D, I, I, P], I),
        "rt_render_progressive": ([P, ctypes.POINTER(Camera), ctypes.POINTER(RenderParams), I, PROGRESS_FN, P,
                                   P], I),
        "rt_comm_unique_id": ([P], I), "rt_comm_init_rank": ([P, I, I, P, ctypes.POINTER(P)], I),
        "rt_comm_init_all": ([P, I, P], I), "rt_comm_destroy": ([P], None), "rt_comm_rank": ([P, PI, PI], I),
        "rt_comm_tile_order": ([P, ctypes.POINTER(Camera), ctypes.POINTER(RenderParams), I], I),
        "rt_comm_tile_order_all": ([P, I, ctypes.POINTER(Camera), ctypes.POINTER(RenderParams), I], I),
        "rt_render_gather": ([P, ctypes.POINTER(Camera), ctypes.POINTER(RenderParams), P], I),
        "rt_render_gather_all": ([P, I, ctypes.POINTER(Camera), ctypes.POINTER(RenderParams), P], I),
        "rt_comm_last_stats": ([P, ctypes.POINTER(CommStats)], I),
        "rt_tiles_assemble": ([P, P, ctypes.c_int64, I, ctypes.POINTER(RenderParams), P], I),
        "rt_tiles_assemble_host": ([P, ctypes.c_int64, I, I, I, I, P, P], I),
        "rt_cost_tile_order": ([P, ctypes.c_int64, P], I),
    }
    for name, (args, res) in sigs.items():
        fn = getattr(lib, name, None)
        if fn is None:   # an older build (A/B runs); build() and tests/test_abi.py check every export
            continue
        fn.argtypes = args
        fn.restype = res
    _lib = lib
    return lib


def build_info() -> str:
    """rt_build_info: the source hash the loaded library was compiled from."""
    return load_library().rt_build_info().decode()


def _check(rc: int, what: str) -> None:
    if rc != RT_OK:
        msg = _lib.rt_last_error().decode() if _lib is not None else ""
        raise RTError(f"{what} failed: {ERRORS.get(rc, rc)} {msg}")


def _d3(v: Sequence[float]):
    return (ctypes.c_double * 3)(*[float(x) for x in v])


def load_earth_texture(path: str = EARTH_JPG) -> np.ndarray:
    """RGB8 texels of textures/earthmap.jpg (texture.rs:12-22; decoded with PIL instead of stb_image)."""
    from PIL import Image
    return np.ascontiguousarray(np.asarray(Image.open(path).convert("RGB"), dtype=np.uint8))


class World:
    """The reference's World (main.rs:40-50) with its Hittable / Material / Texture constructors."""

    def __init__(self, scene_seed: int = 1):
        self.lib = load_library()
        h = ctypes.c_void_p()
        _check(self.lib.rt_world_create(ctypes.c_uint64(scene_seed), ctypes.byref(h)), "rt_world_create")
        self.h = h
        self._keep = []

    def close(self):
        if self.h:
            self.lib.rt_world_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _id(self, fn, *args) -> int:
        out = ctypes.c_int()
        _check(fn(self.h, *args, ctypes.byref(out)), fn.__name__)
        return out.value

    # textures (texture.rs:4-22)
    def solid(self, r, g, b): return self._id(self.lib.rt_world_texture_solid, r, g, b)
    def checker(self, even, odd): return self._id(self.lib.rt_world_texture_checker, _d3(even), _d3(odd))
    def noise(self, scale): return self._id(self.lib.rt_world_texture_noise, scale)

    def image(self, rgb: np.ndarray):
        rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
        return self._id(self.lib.rt_world_texture_image, rgb.ctypes.data, rgb.shape[1], rgb.shape[0])

    # materials (material.rs:6-12) -> 1-based handles
    def lambertian(self, tex): return self._id(self.lib.rt_world_material_lambertian, tex)
    def metal(self, albedo, fuzz): return self._id(self.lib.rt_world_material_metal, _d3(albedo), fuzz)
    def dielectric(self, ir): return self._id(self.lib.rt_world_material_dielectric, ir)
    def diffuse_light(self, tex): return self._id(self.lib.rt_world_material_diffuse_light, tex)
    def isotropic(self, tex): return self._id(self.lib.rt_world_material_isotropic, tex)

    # hittables (hittable.rs:30-41)
    def sphere(self, mat, center, radius): return self._id(self.lib.rt_world_sphere, mat, _d3(center), radius)

    def moving_sphere(self, mat, c0, c1, t0, t1, radius):
        return self._id(self.lib.rt_world_moving_sphere, mat, _d3(c0), _d3(c1), t0, t1, radius)

    def xy_rect(self, mat, x0, x1, y0, y1, k): return self._id(self.lib.rt_world_rect, 0, mat, x0, x1, y0, y1, k)
    def xz_rect(self, mat, x0, x1, z0, z1, k): return self._id(self.lib.rt_world_rect, 1, mat, x0, x1, z0, z1, k)
    def yz_rect(self, mat, y0, y1, z0, z1, k): return self._id(self.lib.rt_world_rect, 2, mat, y0, y1, z0, z1, k)
    def box(self, mn, mx, mat): return self._id(self.lib.rt_world_box, _d3(mn), _d3(mx), mat)
    def translate(self, child, offset): return self._id(self.lib.rt_world_translate, child, _d3(offset))
    def rotate_y(self, child, angle): return self._id(self.lib.rt_world_rotate_y, child, angle)

    def constant_medium(self, boundary, density, phase):
        return self._id(self.lib.rt_world_constant_medium, boundary, density, phase)

    def bvh(self, ids, t0=0.0, t1=1.0):
        arr = (ctypes.c_int * len(ids))(*ids)
        return self._id(self.lib.rt_world_bvh, arr, len(ids), t0, t1)

    def push(self, hid):
        _check(self.lib.rt_world_push(self.h, hid), "rt_world_push")

    def set_build_option(self, key: int, value: float):
        """rt_world_set_build_option: an SAH builder option of this world's flatten (RT_BUILD_*)."""
        _check(self.lib.rt_world_set_build_option(self.h, key, float(value)), "rt_world_set_build_option")
        return self

    def build_scene(self, scene_id: int, image: Optional[np.ndarray] = None):
        """The reference's scene builders (main.rs:52-289)."""
        if scene_id in SCENES_NEEDING_IMAGE and image is None:
            image = load_earth_texture()
        if image is not None:
            image = np.ascontiguousarray(image, dtype=np.uint8)
            self._keep.append(image)
            ptr, w, h = image.ctypes.data, image.shape[1], image.shape[0]
        else:
            ptr, w, h = None, 0, 0
        _check(self.lib.rt_world_build_scene(self.h, scene_id, ptr, w, h), "rt_world_build_scene")
        return self

    def info(self) -> WorldInfo:
        out = WorldInfo()
        _check(self.lib.rt_world_info_get(self.h, ctypes.byref(out)), "rt_world_info_get")
        return out

    def flatten(self, accel: int = RT_ACCEL_SAH) -> SceneSoA:
        p = ctypes.POINTER(SceneSoA)()
        _check(self.lib.rt_world_flatten(self.h, accel, ctypes.byref(p)), "rt_world_flatten")
        return p.contents


def validate_soa(soa: SceneSoA):
    """rt_scene_validate: (tlas_depth, blas_depth) the kernel's walks need; raises RTError on a
    malformed table (out-of-range index, cycle, too deep)."""
    lib = load_library()
    t, b = ctypes.c_int32(), ctypes.c_int32()
    _check(lib.rt_scene_validate(ctypes.byref(soa), ctypes.byref(t), ctypes.byref(b)), "rt_scene_validate")
    return t.value, b.value


def camera_new(look_from, look_at, vup, vfov, aspect_ratio, aperture, focus_dist, time0, time1) -> Camera:
    lib = load_library()
    cam = Camera()
    _check(lib.rt_camera_new(_d3(look_from), _d3(look_at), _d3(vup), vfov, aspect_ratio, aperture, focus_dist,
                             time0, time1, ctypes.byref(cam)), "rt_camera_new")
    return cam


def scene_preset(scene_id: int) -> ScenePreset:
    lib = load_library()
    out = ScenePreset()
    _check(lib.rt_scene_preset_get(scene_id, ctypes.byref(out)), "rt_scene_preset_get")
    return out


def scene_camera(scene_id: int, width: int, height: int):
    """(Camera, background) of a preset scene at width x height (aspect = width/height)."""
    lib = load_library()
    cam = Camera()
    bg = (ctypes.c_double * 3)()
    _check(lib.rt_scene_camera(scene_id, width, height, ctypes.byref(cam), bg), "rt_scene_camera")
    return cam, tuple(bg)


def rows_in_shard(height: int, row_begin: int, row_stride: int, row_block: int = 1) -> int:
    if row_block > 1:
        return load_library().rt_rows_in_band_shard(height, row_begin, row_stride, row_block)
    return load_library().rt_rows_in_shard(height, row_begin, row_stride)


def shard_shape(params) -> tuple:
    """(rows, width) of a render's output: its rows of the image, or a tile shard's slab."""
    if params.tile_shard:
        n = tiles_in_shard(params.width, params.height, params.row_begin, params.row_stride)
        return (8 if n else 0), 8 * n
    return rows_in_shard(params.height, params.row_begin, params.row_stride, params.row_block), params.width


def shard_rows(height: int, rank: int, world: int, row_block: int = 1):
    """Image rows of rank `rank` in the N-way partition, in the shard's order: single rows
    y = rank + k*world, or bands of row_block rows interleaved the same way."""
    if row_block <= 1:
        return list(range(rank, height, world))
    return [y for band in range(rank, (height + row_block - 1) // row_block, world)
            for y in range(band * row_block, min(height, (band + 1) * row_block))]


def tiles_in_shard(width: int, height: int, tile_begin: int, tile_stride: int) -> int:
    """8x8 tiles of a tile shard (rt_render_params.tile_shard = 1)."""
    return load_library().rt_tiles_in_shard(width, height, tile_begin, tile_stride)


def _perm(a, axes):
    return a.permute(*axes) if hasattr(a, "permute") else a.transpose(axes)


def cost_tile_order(costs) -> np.ndarray:
    """rt_ctx_set_tile_order's order from per-tile costs (rt_last_tile_costs): the raster tiles
    by cost, most expensive first (ties in raster order). Dealt round-robin, every shard gets
    every N-th tile of the sorted list, so the shards' costs differ by at most about one
    tile's, and each shard renders its expensive tiles first. Integer costs go through the
    library's rt_cost_tile_order (what rt_comm_tile_order sets); others are sorted here."""
    c = np.asarray(costs)
    if c.dtype.kind in "ui" and (c.size == 0 or c.min() >= 0):
        c = np.ascontiguousarray(c, dtype=np.uint64)
        out = np.empty(c.size, dtype=np.uint32)
        _check(load_library().rt_cost_tile_order(c.ctypes.data, c.size, out.ctypes.data), "rt_cost_tile_order")
        return out
    return np.argsort(-np.asarray(c, dtype=np.float64), kind="stable").astype(np.uint32)


def assemble_tiles_host(slabs: np.ndarray, width: int, height: int, world: int, order=None) -> np.ndarray:
    """rt_tiles_assemble_host: slabs is world x slab_elems (f32 or f64; rank r's tile slab, padded
    to the largest shard's, at row r) -> the height x width x 3 frame."""
    a = np.ascontiguousarray(slabs)
    if a.dtype not in (np.float32, np.float64) or a.ndim < 2 or a.shape[0] != world:
        raise RTError("slabs: world x slab_elems of f32 / f64")
    a = a.reshape(world, -1)
    o = None if order is None else np.ascontiguousarray(order, dtype=np.uint32)
    out = np.zeros((height, width, 3), dtype=a.dtype)
    _check(load_library().rt_tiles_assemble_host(a.ctypes.data, a.shape[1], world, width, height, a.dtype.itemsize,
                                                 None if o is None else o.ctypes.data, out.ctypes.data),
           "rt_tiles_assemble_host")
    return out


def scattered_tile_order(n_tiles: int, stride: int) -> np.ndarray:
    """Every stride-th raster tile first (0, s, 2s, ...), then 1, 1 + s, ...: one GPU's frame
    spread over the image as an s-way round-robin shard is (scripts/tile_locality.py)."""
    return np.concatenate([np.arange(k, n_tiles, stride) for k in range(stride)]).astype(np.uint32)


def grouped_tile_order(n_tiles: int, world: int, group: int) -> np.ndarray:
    """A tile order that deals runs of `group` consecutive raster tiles round-robin over `world`
    tile shards (run j to shard j mod world), instead of single tiles: each shard's waves then work
    on neighbouring tiles. Shard r holds positions r, r + world, ... (rt_tiles_in_shard tiles);
    a run that does not fit its shard's remaining count continues on the next shard with room."""
    cap = [len(range(r, n_tiles, world)) for r in range(world)]
    lists = [[] for _ in range(world)]
    for j, t0 in enumerate(range(0, n_tiles, group)):
        k = j % world
        for t in range(t0, min(t0 + group, n_tiles)):
            while cap[k] == 0:
                k = (k + 1) % world
            lists[k].append(t)
            cap[k] -= 1
    order = np.empty(n_tiles, dtype=np.uint32)
    for r in range(world):
        order[r::world] = lists[r]
    return order


def assemble_tiles(slabs, width: int, height: int, world: int, out=None, order=None):
    """Inverse of the tile partition: slabs[r] is rank r's 8 x (8 * n_r) x 3 tile slab (the
    tiles at positions t = r + m*world side by side: raster tiles, or order[t] with a tile order
    set on the renderers, rt_ctx_set_tile_order; wider padding is ignored). Works on numpy
    arrays and torch tensors alike; returns the height x width x 3 frame."""
    tx, ty = (width + 7) // 8, (height + 7) // 8
    like = slabs[0]
    if hasattr(like, "new_empty"):
        tiles = like.new_empty((ty * tx, 8, 8, like.shape[-1]))
        if order is not None:
            import torch as _torch
            order = _torch.as_tensor(np.ascontiguousarray(order, dtype=np.int64), device=like.device)
    else:
        import numpy as _np
        tiles = _np.empty((ty * tx, 8, 8, like.shape[-1]), dtype=like.dtype)
        if order is not None:
            order = _np.asarray(order, dtype=_np.int64)
    if order is not None and len(order) != tx * ty:
        raise ValueError(f"tile order of {len(order)} tiles for a frame of {tx * ty}")
    for r in range(world):
        n = len(range(r, ty * tx, world))
        if n:
            dst = slice(r, None, world) if order is None else order[r::world]
            tiles[dst] = _perm(slabs[r][:, :8 * n].reshape(8, n, 8, like.shape[-1]), (1, 0, 2, 3))
    frame = _perm(tiles.reshape(ty, tx, 8, 8, like.shape[-1]), (0, 2, 1, 3, 4)).reshape(ty * 8, tx * 8, like.shape[-1])
    if out is None:
        return frame[:height, :width]
    out[...] = frame[:height, :width]
    return out


def assemble_rows(slabs, height: int, world: int, out=None, row_block: int = 1):
    """Inverse of the row partition: slabs[r] holds rank r's rows (padded to the largest
    shard). Works on numpy arrays and torch tensors alike."""
    if out is None:
        import numpy as _np
        out = _np.empty((height,) + tuple(slabs[0].shape[1:]), dtype=slabs[0].dtype)
    for r in range(world):
        if row_block <= 1:
            n = len(range(r, height, world))
            out[r::world] = slabs[r][:n]
            continue
        k = 0
        for band in range(r, (height + row_block - 1) // row_block, world):
            y0, y1 = band * row_block, min(height, (band + 1) * row_block)
            out[y0:y1] = slabs[r][k:k + (y1 - y0)]
            k += y1 - y0
    return out


def write_ppm(rgb: np.ndarray, path: str, samples_per_pixel: int = 1) -> None:
    """P3 writer of the reference (write_color, math.rs:119-132; main.rs:472, 591-596):
    height x width x 3, row 0 = bottom. An f64 array takes rt_write_ppm_f64 — the reference's
    bytes exactly: pass rt_render's RT_OUT_F64 mean with samples_per_pixel=1, or per-pixel sums
    (Accumulator.get) with their spp. An f32 array (the f32 frame) takes rt_write_ppm, whose
    f32-rounded mean can move a channel at a rounding boundary by one."""
    lib = load_library()
    if np.asarray(rgb).dtype == np.float64:
        a = np.ascontiguousarray(rgb, dtype=np.float64)
        _check(lib.rt_write_ppm_f64(a.ctypes.data, samples_per_pixel, a.shape[1], a.shape[0], str(path).encode()),
               "rt_write_ppm_f64")
        return
    if samples_per_pixel != 1:
        raise RTError("an f32 frame is a mean: samples_per_pixel must be 1")
    a = np.ascontiguousarray(rgb, dtype=np.float32)
    _check(lib.rt_write_ppm(a.ctypes.data, a.shape[1], a.shape[0], str(path).encode()), "rt_write_ppm")


def write_color(rgb: np.ndarray, samples_per_pixel: int = 1) -> np.ndarray:
    """The reference's write_color channel values (int32, same shape) of f64 sums / means."""
    lib = load_library()
    a = np.ascontiguousarray(rgb, dtype=np.float64)
    out = np.empty(a.shape, dtype=np.int32)
    _check(lib.rt_write_color(a.ctypes.data, samples_per_pixel, a.size // 3, out.ctypes.data), "rt_write_color")
    return out


class Renderer:
    """One device context: upload a world, render row shards through the megakernel."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        n = ctypes.c_int()
        _check(self.lib.rt_device_count(ctypes.byref(n)), "rt_device_count")
        if n.value <= 0:
            raise RTError("no HIP device visible")
        h = ctypes.c_void_p()
        _check(self.lib.rt_ctx_create(device, ctypes.byref(h)), "rt_ctx_create")
        self.h = h

    def close(self):
        if self.h:
            self.lib.rt_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload(self, world: World, accel: int = RT_ACCEL_SAH):
        _check(self.lib.rt_ctx_upload_world(self.h, world.h, accel), "rt_ctx_upload_world")

    @staticmethod
    def params(width, height, spp, max_depth=50, background=(0.0, 0.0, 0.0), render_seed=1, row_begin=0,
               row_stride=1, spp_chunk=0, out_format=RT_OUT_F32, out_on_device=0, count_work=0, stream=None,
               row_block=1, tile_shard=0):
        p = RenderParams()
        p.row_block = row_block
        p.tile_shard = tile_shard
        p.width, p.height, p.spp, p.max_depth = width, height, spp, max_depth
        p.spp_chunk, p.row_begin, p.row_stride = spp_chunk, row_begin, row_stride
        p.out_format, p.out_on_device, p.count_work = out_format, out_on_device, count_work
        p.background = _d3(background)
        p.render_seed = render_seed
        p.stream = stream
        return p

    def render(self, camera: Camera, params: RenderParams, out=None) -> np.ndarray:
        """Host-output render: returns rows_local x width x 3 mean radiance (row k = k-th selected
        row), or for a tile shard its 8 x (8 * tiles_local) x 3 slab."""
        n_rows, width = shard_shape(params)
        dt = np.float64 if params.out_format == RT_OUT_F64 else np.float32
        if out is None:
            out = np.empty((n_rows, width, 3), dtype=dt)
        if out.dtype != dt or out.size < n_rows * width * 3 or not out.flags.c_contiguous:
            raise RTError(f"output buffer too small or of the wrong type for {n_rows} x {width} x 3 {dt}")
        params.out_on_device = 0
        _check(self.lib.rt_render(self.h, ctypes.byref(camera), ctypes.byref(params), out.ctypes.data), "rt_render")
        return out

    def render_device(self, camera: Camera, params: RenderParams, dev_ptr: int, stream: Optional[int] = None):
        """Enqueues a render into a device buffer (e.g. a torch tensor's data_ptr()) on `stream`."""
        params.out_on_device = 1
        params.stream = stream
        _check(self.lib.rt_render(self.h, ctypes.byref(camera), ctypes.byref(params), ctypes.c_void_p(dev_ptr)),
               "rt_render")

    def render_progressive(self, camera: Camera, params: RenderParams, batch_spp: int, progress=None) -> np.ndarray:
        """rt_render in sample batches; progress(samples_done, samples_total) -> truthy stops early."""
        n_rows, width = shard_shape(params)
        dt = np.float64 if params.out_format == RT_OUT_F64 else np.float32
        out = np.empty((n_rows, width, 3), dtype=dt)
        params.out_on_device = 0
        cb = PROGRESS_FN(lambda _u, done, total: int(bool(progress(done, total)))) if progress else PROGRESS_FN()
        _check(self.lib.rt_render_progressive(self.h, ctypes.byref(camera), ctypes.byref(params), batch_spp, cb,
                                              None, out.ctypes.data), "rt_render_progressive")
        return out

    def accumulator(self, params: RenderParams) -> "Accumulator":
        return Accumulator(self, params)

    def set_schedule(self, schedule: int):
        _check(self.lib.rt_ctx_set_schedule(self.h, schedule), "rt_ctx_set_schedule")

    def set_precision(self, precision: int):
        """RT_PREC_F64 (default: path-identical to the oracle, last-ulp summation differences) or
        RT_PREC_F32 (fast mode, statistical parity)."""
        _check(self.lib.rt_ctx_set_precision(self.h, precision), "rt_ctx_set_precision")

    def set_option(self, key: int, value: int):
        """rt_ctx_set_option (RT_OPT_*): buffer bound, batch overlap, block sizes, extra features, ..."""
        _check(self.lib.rt_ctx_set_option(self.h, key, int(value)), "rt_ctx_set_option")

    def get_option(self, key: int) -> int:
        v = ctypes.c_int64()
        _check(self.lib.rt_ctx_get_option(self.h, key, ctypes.byref(v)), "rt_ctx_get_option")
        return v.value

    def set_variant(self, slab32: int = 1, lds_stack: int = 1, lds_nodes: int = 1):
        _check(self.lib.rt_ctx_set_variant(self.h, slab32, lds_stack, lds_nodes), "rt_ctx_set_variant")

    def counters(self, n: int = 32) -> np.ndarray:
        """The last count_work render's raw counters (rt_last_counters: phase wave-cycles etc.)."""
        out = np.zeros(n, dtype=np.uint64)
        rc = self.lib.rt_last_counters(self.h, out.ctypes.data, n)
        if rc < 0:
            _check(rc, "rt_last_counters")
        return out[:rc]

    def tile_costs(self) -> np.ndarray:
        """Lane-cycles per raster 8x8 tile of the last count_work render on a pool schedule
        (rt_last_tile_costs); empty if it counted none."""
        n = self.lib.rt_last_tile_costs(self.h, None, 0)
        if n < 0:
            _check(n, "rt_last_tile_costs")
        out = np.zeros(n, dtype=np.uint64)
        if n:
            _check(min(0, self.lib.rt_last_tile_costs(self.h, out.ctypes.data, n)), "rt_last_tile_costs")
        return out

    def set_tile_order(self, order=None):
        """rt_ctx_set_tile_order: tile shards take the frame's tiles in this order (a permutation
        of its raster tiles, e.g. cost_tile_order(tile_costs())); None: raster order."""
        if order is None:
            _check(self.lib.rt_ctx_set_tile_order(self.h, None, 0), "rt_ctx_set_tile_order")
            return
        o = np.ascontiguousarray(np.asarray(order), dtype=np.uint32)
        _check(self.lib.rt_ctx_set_tile_order(self.h, o.ctypes.data, len(o)), "rt_ctx_set_tile_order")

    def stats(self) -> Stats:
        s = Stats()
        _check(self.lib.rt_last_stats(self.h, ctypes.byref(s)), "rt_last_stats")
        return s

    def assemble_device(self, slabs_ptr: int, slab_elems: int, world: int, params: RenderParams, frame_ptr: int,
                        stream: Optional[int] = None):
        """rt_tiles_assemble: gathered tile slabs (device) -> frame (device), in this context's tile order."""
        params.stream = stream
        _check(self.lib.rt_tiles_assemble(self.h, ctypes.c_void_p(slabs_ptr), slab_elems, world, ctypes.byref(params),
                                          ctypes.c_void_p(frame_ptr)), "rt_tiles_assemble")

    def device_eval(self, fn: int, x, y=None, z=None) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.ascontiguousarray(x if y is None else y, dtype=np.float64)
        z = np.ascontiguousarray(x if z is None else z, dtype=np.float64)
        out = np.empty_like(x)
        _check(self.lib.rt_device_eval(self.h, fn, x.ctypes.data, y.ctypes.data, z.ctypes.data, out.ctypes.data,
                                       x.size), "rt_device_eval")
        return out


class Comm:
    """One rank of a multi-GPU render (rt_comm_*): binds a Renderer (its device) to rank `rank` of
    `world`. One process per GPU: rank 0 makes the id (Comm.unique_id()) and sends it to the others
    (any channel), every rank then builds Comm(renderer, rank, world, uid). One process over several
    GPUs: Comm.init_all(renderers)."""

    def __init__(self, renderer: Renderer, rank: int, world: int, uid: bytes, _handle=None):
        self.r, self.lib = renderer, renderer.lib
        self.rank, self.world = rank, world
        if _handle is not None:
            self.h = _handle
            return
        if len(uid) != RT_COMM_ID_BYTES:
            raise RTError("unique id must be %d bytes" % RT_COMM_ID_BYTES)
        h = ctypes.c_void_p()
        buf = (ctypes.c_uint8 * RT_COMM_ID_BYTES).from_buffer_copy(uid)
        _check(self.lib.rt_comm_init_rank(renderer.h, rank, world, buf, ctypes.byref(h)), "rt_comm_init_rank")
        self.h = h

    @staticmethod
    def unique_id() -> bytes:
        buf = (ctypes.c_uint8 * RT_COMM_ID_BYTES)()
        _check(load_library().rt_comm_unique_id(buf), "rt_comm_unique_id")
        return bytes(buf)

    @staticmethod
    def init_all(renderers) -> list:
        n = len(renderers)
        ctxs = (ctypes.c_void_p * n)(*[r.h.value if isinstance(r.h, ctypes.c_void_p) else r.h for r in renderers])
        hs = (ctypes.c_void_p * n)()
        _check(load_library().rt_comm_init_all(ctxs, n, hs), "rt_comm_init_all")
        return [Comm(r, i, n, b"", _handle=ctypes.c_void_p(hs[i])) for i, r in enumerate(renderers)]

    def close(self):
        if self.h:
            self.lib.rt_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def tile_order(self, camera: Camera, params: RenderParams, cost_spp: int = 8):
        """Collective rt_comm_tile_order: every rank counts its raster shard, one all-reduce, the
        cost order set on every rank's context."""
        params.stream = params.stream if params.stream else None
        _check(self.lib.rt_comm_tile_order(self.h, ctypes.byref(camera), ctypes.byref(params), cost_spp),
               "rt_comm_tile_order")

    def render_gather(self, camera: Camera, params: RenderParams, out=None):
        """Collective rt_render_gather into host memory: rank 0 returns the height x width x 3 frame
        (or fills `out`), the other ranks None."""
        params.out_on_device = 0
        if self.rank != 0:
            _check(self.lib.rt_render_gather(self.h, ctypes.byref(camera), ctypes.byref(params), None),
                   "rt_render_gather")
            return None
        dt = np.float64 if params.out_format == RT_OUT_F64 else np.float32
        if out is None:
            out = np.empty((params.height, params.width, 3), dtype=dt)
        if out.dtype != dt or out.size != params.height * params.width * 3 or not out.flags.c_contiguous:
            raise RTError("frame buffer of the wrong shape or type")
        _check(self.lib.rt_render_gather(self.h, ctypes.byref(camera), ctypes.byref(params), out.ctypes.data),
               "rt_render_gather")
        return out

    def render_gather_device(self, camera: Camera, params: RenderParams, dev_ptr: Optional[int],
                             stream: Optional[int] = None):
        """Collective rt_render_gather, enqueued on `stream`: rank 0's frame into a device buffer."""
        params.out_on_device = 1
        params.stream = stream
        _check(self.lib.rt_render_gather(self.h, ctypes.byref(camera), ctypes.byref(params),
                                         ctypes.c_void_p(dev_ptr) if dev_ptr else None), "rt_render_gather")

    def stats(self) -> CommStats:
        s = CommStats()
        _check(self.lib.rt_comm_last_stats(self.h, ctypes.byref(s)), "rt_comm_last_stats")
        return s


def _comm_array(comms):
    return (ctypes.c_void_p * len(comms))(*[c.h.value for c in comms])


def tile_order_all(comms, camera: Camera, params: RenderParams, cost_spp: int = 8):
    """rt_comm_tile_order_all over the ranks of one process (Comm.init_all)."""
    params.stream = None
    _check(load_library().rt_comm_tile_order_all(_comm_array(comms), len(comms), ctypes.byref(camera),
                                                 ctypes.byref(params), cost_spp), "rt_comm_tile_order_all")


def render_gather_all(comms, camera: Camera, params: RenderParams) -> np.ndarray:
    """rt_render_gather_all over the ranks of one process: the frame in host memory."""
    params.out_on_device = 0
    params.stream = None
    dt = np.float64 if params.out_format == RT_OUT_F64 else np.float32
    out = np.empty((params.height, params.width, 3), dtype=dt)
    _check(load_library().rt_render_gather_all(_comm_array(comms), len(comms), ctypes.byref(camera),
                                               ctypes.byref(params), out.ctypes.data), "rt_render_gather_all")
    return out


class Accumulator:
    """Progressive / resumable accumulation over one row shard (rt_accum_*)."""

    def __init__(self, renderer: Renderer, params: RenderParams):
        self.r, self.lib = renderer, renderer.lib
        self.rows, self.width = shard_shape(params)
        h = ctypes.c_void_p()
        _check(self.lib.rt_accum_create(renderer.h, ctypes.byref(params), ctypes.byref(h)), "rt_accum_create")
        self.h = h

    def close(self):
        if self.h:
            self.lib.rt_accum_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add(self, camera: Camera, params: RenderParams, sample_count: int):
        _check(self.lib.rt_accum_add(self.r.h, self.h, ctypes.byref(camera), ctypes.byref(params), sample_count),
               "rt_accum_add")

    @property
    def samples_done(self) -> int:
        n = ctypes.c_int64()
        _check(self.lib.rt_accum_get(self.h, None, ctypes.byref(n)), "rt_accum_get")
        return n.value

    def checkpoint(self):
        """(sums rows x width x 3 f64, samples done) — what rt_accum_set restores."""
        sums = np.empty((self.rows, self.width, 3), dtype=np.float64)
        n = ctypes.c_int64()
        _check(self.lib.rt_accum_get(self.h, sums.ctypes.data, ctypes.byref(n)), "rt_accum_get")
        return sums, n.value

    def restore(self, sums: np.ndarray, samples_done: int):
        sums = np.ascontiguousarray(sums, dtype=np.float64)
        assert sums.shape == (self.rows, self.width, 3)
        _check(self.lib.rt_accum_set(self.h, sums.ctypes.data, samples_done), "rt_accum_set")

    def resolve(self, divisor: float = 0.0, out_format: int = RT_OUT_F32) -> np.ndarray:
        dt = np.float64 if out_format == RT_OUT_F64 else np.float32
        out = np.empty((self.rows, self.width, 3), dtype=dt)
        _check(self.lib.rt_accum_resolve(self.r.h, self.h, divisor, out_format, 0, out.ctypes.data),
               "rt_accum_resolve")
        return out


def render_scene(scene_id: int, width: int, height: int, spp: int, max_depth: int = 50, scene_seed: int = 1,
                 render_seed: int = 1, row_begin: int = 0, row_stride: int = 1, out_format: int = RT_OUT_F32,
                 spp_chunk: int = 0, device: int = 0, renderer: Optional[Renderer] = None,
                 image: Optional[np.ndarray] = None, accel: int = RT_ACCEL_SAH):
    """One-call path: build the preset scene, upload, render the row shard. Returns (image, stats)."""
    world = World(scene_seed).build_scene(scene_id, image)
    cam, bg = scene_camera(scene_id, width, height)
    r = renderer or Renderer(device)
    r.upload(world, accel)
    p = Renderer.params(width, height, spp, max_depth, bg, render_seed, row_begin, row_stride, spp_chunk,
                        out_format)
    img = r.render(cam, p)
    return img, r.stats()
