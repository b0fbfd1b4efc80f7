"""ctypes binding of the CPU oracle (oracle/liboracle.so) — TEST INFRASTRUCTURE ONLY.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
checker / CPU baseline; never by the product path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from functools import lru_cache

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
# RT_ORACLE_LIB: another build of the same source (the sanitizer run, tests/test_sanitizers.py)
ORACLE_LIB = os.environ.get("RT_ORACLE_LIB", os.path.join(ORACLE_DIR, "build", "liboracle.so"))
EARTH_JPG = os.path.join(REPO, "assets", "earthmap.jpg")

SPLIT_ROWS, SPLIT_SAMPLES = 0, 1


class Params(ctypes.Structure):
    _fields_ = [("scene_id", ctypes.c_int), ("scene_seed", ctypes.c_uint64), ("render_seed", ctypes.c_uint64),
                ("width", ctypes.c_int), ("height", ctypes.c_int), ("spp", ctypes.c_int),
                ("max_depth", ctypes.c_int), ("spp_chunk", ctypes.c_int), ("row_begin", ctypes.c_int),
                ("row_stride", ctypes.c_int), ("threads", ctypes.c_int), ("split", ctypes.c_int),
                ("image_rgb", ctypes.c_void_p), ("image_w", ctypes.c_int), ("image_h", ctypes.c_int)]


class Stats(ctypes.Structure):
    _fields_ = [("casts", ctypes.c_uint64), ("samples", ctypes.c_uint64), ("seconds", ctypes.c_double)]


@lru_cache(maxsize=1)
def lib() -> ctypes.CDLL:
    src = os.path.join(ORACLE_DIR, "oracle.c")
    if not os.path.exists(ORACLE_LIB) or (os.path.exists(src) and
                                          os.path.getmtime(src) > os.path.getmtime(ORACLE_LIB)):
        subprocess.run(["make", "-C", ORACLE_DIR, "-s"], check=True)
    l = ctypes.CDLL(ORACLE_LIB)
    l.orc_render.argtypes = [ctypes.POINTER(Params), ctypes.c_void_p, ctypes.POINTER(Stats)]
    l.orc_render.restype = ctypes.c_int
    l.orc_scene_info.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                 ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                 ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_double)]
    l.orc_scene_info.restype = ctypes.c_int
    l.orc_eval.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_int]
    l.orc_eval.restype = ctypes.c_int
    l.orc_philox.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    l.orc_philox.restype = None
    l.orc_pstream.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]
    l.orc_pstream.restype = None
    l.orc_camera.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    l.orc_camera.restype = ctypes.c_int
    return l


@lru_cache(maxsize=1)
def earth_texture() -> np.ndarray:
    from PIL import Image
    return np.ascontiguousarray(np.asarray(Image.open(EARTH_JPG).convert("RGB"), dtype=np.uint8))


def render(scene_id: int, width: int, height: int, spp: int, max_depth: int = 50, scene_seed: int = 1,
           render_seed: int = 1, row_begin: int = 0, row_stride: int = 1, threads: int = 0,
           split: int = SPLIT_ROWS, spp_chunk: int = 0, return_stats: bool = False):
    """Mean radiance of the selected rows, shape (rows, width, 3) f64 (row k = row_begin + k*row_stride)."""
    img = earth_texture() if scene_id in (3, 7) else np.zeros((1, 1, 3), np.uint8)
    if threads <= 0:
        threads = min(8, os.cpu_count() or 1)
    n_rows = 0 if row_begin >= height else (height - row_begin + row_stride - 1) // row_stride
    if spp_chunk <= 0:
        spp_chunk = min(16, max(1, (spp + 15) // 16))   # the product's automatic chunking (abi.cpp auto_chunk)
    p = Params(scene_id, scene_seed, render_seed, width, height, spp, max_depth, spp_chunk, row_begin, row_stride,
               threads, split, img.ctypes.data, img.shape[1], img.shape[0])
    out = np.zeros((n_rows, width, 3), dtype=np.float64)
    st = Stats()
    rc = lib().orc_render(ctypes.byref(p), out.ctypes.data, ctypes.byref(st))
    if rc != 0:
        raise RuntimeError(f"orc_render failed: {rc}")
    return (out, st) if return_stats else out


def scene_info(scene_id: int, scene_seed: int = 1):
    img = earth_texture()
    n_h, n_m, n_l = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    cs = ctypes.c_double()
    rc = lib().orc_scene_info(scene_id, scene_seed, img.ctypes.data, img.shape[1], img.shape[0],
                              ctypes.byref(n_h), ctypes.byref(n_m), ctypes.byref(n_l), ctypes.byref(cs))
    if rc != 0:
        raise RuntimeError("orc_scene_info failed")
    return {"n_hittables": n_h.value, "n_materials": n_m.value, "n_leaf_prims": n_l.value, "checksum": cs.value}


def evaluate(fn: int, x, y=None, z=None) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(x if y is None else y, dtype=np.float64)
    z = np.ascontiguousarray(x if z is None else z, dtype=np.float64)
    out = np.empty_like(x)
    if lib().orc_eval(fn, x.ctypes.data, y.ctypes.data, z.ctypes.data, out.ctypes.data, x.size) != 0:
        raise ValueError(fn)
    return out


def philox(ctr, key) -> np.ndarray:
    c = np.ascontiguousarray(ctr, dtype=np.uint32)
    k = np.ascontiguousarray(key, dtype=np.uint32)
    out = np.zeros(4, dtype=np.uint32)
    lib().orc_philox(c.ctypes.data, k.ctypes.data, out.ctypes.data)
    return out


def camera(scene_id: int, width: int, height: int) -> np.ndarray:
    out = np.zeros(24, dtype=np.float64)
    if lib().orc_camera(scene_id, width, height, out.ctypes.data) != 0:
        raise ValueError(scene_id)
    return out


def pstream(seed: int, pixel: int, sample: int, n: int) -> np.ndarray:
    out = np.zeros(n, np.uint64)
    lib().orc_pstream(seed, pixel, sample, n, out.ctypes.data)
    return out
