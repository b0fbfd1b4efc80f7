"""Shared numeric core (include/rt/rt_numerics.h) on the host, through the oracle library.

Pins: Philox4x32-10 against Random123's published KATs and ROCm rocrand's host engine
(tests/golden/philox_kat.txt, tests/golden/make_philox_kat.cpp); the only golden data
the reference holds — the sphere_uv table of math.rs:292-294; and the fdlibm-style
sin/cos/log/atan2/acos against numpy (glibc) within a few ulp.
"""
import os

import numpy as np
import pytest

from tests import oracle_binding as ob

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _ulp_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    spacing = np.spacing(np.maximum(np.abs(a), np.abs(b)))
    return np.abs(a - b) / np.maximum(spacing, np.finfo(np.float64).tiny)


def test_philox_kat():
    lines = open(os.path.join(GOLDEN, "philox_kat.txt")).read().split("\n")
    n = 0
    for line in lines:
        if not line.strip():
            continue
        lhs, rhs = line.split("->")
        w = [int(t, 16) for t in lhs.split()]
        want = [int(t, 16) for t in rhs.split()]
        got = ob.philox(w[:4], w[4:6])
        assert list(got) == want, line
        n += 1
    assert n >= 11


def test_philox_random123_published():
    # Random123 kat_vectors, philox4x32 R=10
    assert list(ob.philox([0, 0, 0, 0], [0, 0])) == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    assert list(ob.philox([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0])) == \
        [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]


def _xoshiro128pp(state, n):
    """xoshiro128++ as published (Blackman & Vigna, prng.di.unimi.it/xoshiro128plusplus.c)."""
    M = 0xFFFFFFFF
    rotl = lambda x, k: ((x << k) | (x >> (32 - k))) & M  # noqa: E731
    s = list(state)
    out = []
    for _ in range(n):
        out.append((rotl((s[0] + s[3]) & M, 7) + s[0]) & M)
        t = (s[1] << 9) & M
        s[2] ^= s[0]
        s[3] ^= s[1]
        s[1] ^= s[2]
        s[0] ^= s[3]
        s[2] ^= t
        s[3] = rotl(s[3], 11)
    return out


@pytest.mark.parametrize("seed,pixel,sample", [(1, 0, 0), (1, 959999, 499), (0xDEADBEEF12345678, 17, 3)])
def test_path_stream_is_philox_seeded_xoshiro128pp(seed, pixel, sample):
    """rt_pstream: state = Philox4x32-10((pixel, sample, 0, RT_STREAM_PATH), seed); each u64
    draw = (xoshiro128++ output << 32) | next output."""
    state = ob.philox([pixel, sample, 0, 0x9A750000], [seed & 0xFFFFFFFF, seed >> 32])
    words = _xoshiro128pp([int(v) for v in state], 40)
    want = [(words[2 * i] << 32) | words[2 * i + 1] for i in range(20)]
    assert [int(v) for v in ob.pstream(seed, pixel, sample, 20)] == want


@pytest.mark.parametrize("p,uv", [
    ((1, 0, 0), (0.5, 0.5)), ((-1, 0, 0), (0.0, 0.5)), ((0, 1, 0), (0.5, 1.0)),
    ((0, -1, 0), (0.5, 0.0)), ((0, 0, 1), (0.25, 0.5)), ((0, 0, -1), (0.75, 0.5)),
])
def test_sphere_uv_reference_table(p, uv):
    """math.rs:292-294 — the reference's only embedded known-answer table."""
    x, y, z = (np.array([c], np.float64) for c in p)
    u = ob.evaluate(5, x, y, z)[0]
    v = ob.evaluate(6, x, y, z)[0]
    assert u == pytest.approx(uv[0], abs=1e-15)
    assert v == pytest.approx(uv[1], abs=1e-15)


def test_sin_cos_accuracy():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(-4, 4, 20000), rng.uniform(-2e4, 2e4, 20000), rng.uniform(-1e5, 1e5, 5000),
                        np.array([0.0, -0.0, 1e-300, np.pi / 4, np.pi / 2, np.pi, 1e-9])])
    assert np.max(_ulp_err(ob.evaluate(0, x), np.sin(x))) <= 2.0
    assert np.max(_ulp_err(ob.evaluate(1, x), np.cos(x))) <= 2.0


def test_sin_special_values():
    s = ob.evaluate(0, np.array([np.inf, -np.inf, np.nan]))
    assert np.all(np.isnan(s))
    z = ob.evaluate(0, np.array([0.0, -0.0]))
    assert z[0] == 0.0 and np.signbit(z[1])


def test_log_accuracy():
    rng = np.random.default_rng(1)
    x = np.concatenate([rng.uniform(0, 1, 50000), 2.0 ** -rng.uniform(0, 53, 20000), np.array([2.0 ** -53, 1.0, 5e-324])])
    assert np.max(_ulp_err(ob.evaluate(2, x), np.log(x))) <= 1.5
    sp = ob.evaluate(2, np.array([0.0, -1.0, np.inf]))
    assert sp[0] == -np.inf and np.isnan(sp[1]) and sp[2] == np.inf


def test_atan2_acos_accuracy():
    rng = np.random.default_rng(2)
    y = rng.normal(size=30000)
    x = rng.normal(size=30000)
    assert np.max(_ulp_err(ob.evaluate(3, y, x), np.arctan2(y, x))) <= 2.0
    c = np.concatenate([rng.uniform(-1, 1, 30000), np.array([-1.0, 1.0, 0.0, 0.5, -0.5, 1 - 1e-16])])
    assert np.max(_ulp_err(ob.evaluate(4, c), np.arccos(c))) <= 2.0
    assert np.isnan(ob.evaluate(4, np.array([1.0000000000000002]))[0])   # like Rust's acos > 1


def test_pow5_close_to_libm():
    x = np.random.default_rng(3).uniform(0, 1, 20000)
    assert np.max(_ulp_err(ob.evaluate(7, x), np.power(x, 5.0))) <= 3.0


def test_rand_float_mappings():
    """rand 0.8: Standard f64 = (u64 >> 11) * 2^-53; gen_range(-1..=1) via UniformFloat::new_inclusive."""
    bits = np.array([0, 1 << 11, (1 << 64) - 1, 1 << 63, 0x123456789abcdef0], dtype=np.uint64)
    x = bits.view(np.float64)
    u = ob.evaluate(10, x)
    expect = (bits >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
    assert np.array_equal(u, expect)
    assert u.max() < 1.0 and u.min() == 0.0
    r = ob.evaluate(11, x)
    assert r.min() >= -1.0 and r.max() <= 1.0
    assert r[0] == -1.0
    # value0_1 = (u64 >> 12 as mantissa in [1,2)) - 1; scale s.t. max_rand*scale + low <= high
    top = ob.evaluate(11, np.array([(1 << 64) - 1], dtype=np.uint64).view(np.float64))[0]
    assert top <= 1.0 and top > 1.0 - 1e-15


def test_sin_sign_matches_sin():
    """rt_sin_sign (the checker texture's fast path, texture.rs:35-41) against the sign of
    rt_sin itself, incl. arguments next to multiples of pi/2, tiny, zero, inf and NaN; and the
    checker decision (product of three sines < 0) it feeds."""
    rng = np.random.default_rng(5)
    k = rng.integers(-4000, 4000, 20000).astype(np.float64)
    near = k * (np.pi / 2)
    near = np.concatenate([near, np.nextafter(near, np.inf), np.nextafter(near, -np.inf)])
    x = np.concatenate([rng.uniform(-200, 200, 50000), near, 10.0 * rng.uniform(-15, 15, 20000),
                        2.0 ** -rng.uniform(0, 1070, 2000) * rng.choice([-1, 1], 2000),
                        [0.0, -0.0, np.inf, -np.inf, np.nan, 5e-324, -5e-324]])
    s = ob.evaluate(0, x)
    sg = ob.evaluate(12, x)
    exact = np.where(np.isnan(s) | (s == 0), 0, np.sign(s))
    known = sg != 2
    assert np.all(sg[known] == exact[known])
    assert np.all(np.abs(s[~known]) < 2.0 ** -300)        # "tiny" only where |sin| really is
    a, b, c = (x[rng.permutation(x.size)] for _ in range(3))
    sa, sb, sc = (ob.evaluate(0, v) for v in (a, b, c))
    ga, gb, gc = (ob.evaluate(12, v) for v in (a, b, c))
    full = sa * sb * sc < 0.0
    ok = (ga != 2) & (gb != 2) & (gc != 2)
    assert np.array_equal(full[ok], (ga * gb * gc)[ok] < 0)
