"""CPU: the product's exact hash (mahout_amd/csrc/cms_hash.h: key reduction,
2^63 == 25 folding, Barrett mod w) compiled for the host and compared with the
oracle's signed 128-bit BigInteger restatement on millions of keys."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "cpp", "hash_host_shim.hip")
OUT = os.path.join(HERE, "cpp", "_build", "libhash_host_shim.so")


@pytest.fixture(scope="module")
def shim():
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    if not os.path.exists(OUT) or os.path.getmtime(OUT) < max(os.path.getmtime(SRC), os.path.getmtime(
            os.path.join(HERE, "..", "mahout_amd", "csrc", "cms_hash.h"))):
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-fPIC", "-shared", SRC, "-o",
                               OUT])
    lib = ctypes.CDLL(OUT)
    lib.host_buckets.restype = None
    return lib


def _host(shim, a, b, width, keys):
    keys = np.ascontiguousarray(keys, np.int64)
    out = np.zeros((keys.size, len(a)), np.int32)
    vp = ctypes.c_void_p
    shim.host_buckets(a.ctypes.data_as(vp), b.ctypes.data_as(vp), len(a), width, keys.ctypes.data_as(vp),
                      ctypes.c_int64(keys.size), out.ctypes.data_as(vp))
    return out


@pytest.mark.parametrize("seed", [42, 0, 7])
@pytest.mark.parametrize("width", [1, 3, 39, 40, 1000, 1024, 4096, 8192, 32768, 30011])
def test_product_hash_matches_oracle(shim, oracle, seed, width):
    rng = np.random.Generator(np.random.PCG64(seed * 1000 + width))
    keys = np.concatenate([
        rng.integers(-2 ** 63, 2 ** 63 - 1, size=200000, dtype=np.int64),
        np.arange(-5000, 5000, dtype=np.int64),
        np.array([2 ** 63 - 1, -2 ** 63, 9223372036854775783, 9223372036854775782, -9223372036854775783,
                  -9223372036854775784, 2 ** 62, -2 ** 62], np.int64),
    ])
    a, b = oracle.hash_params(seed, 6)
    np.testing.assert_array_equal(_host(shim, a, b, width, keys), oracle.hash_keys(a, b, width, keys))


def test_extreme_hash_params(shim, oracle):
    """a = Long.MIN_VALUE (Math.abs leaves it negative) and a, b >= p."""
    keys = np.random.Generator(np.random.PCG64(1)).integers(-2 ** 63, 2 ** 63 - 1, size=50000, dtype=np.int64)
    a = np.array([-2 ** 63, 2 ** 63 - 1, 9223372036854775783, 9223372036854775790, 0, 1], np.int64)
    b = np.array([2 ** 63 - 1, -2 ** 63, 9223372036854775800, 0, 9223372036854775783, 5], np.int64)
    for w in [1024, 1000]:
        np.testing.assert_array_equal(_host(shim, a, b, w, keys), oracle.hash_keys(a, b, w, keys))


def _modes(shim, a, b, width, keys):
    keys = np.ascontiguousarray(keys, np.int64)
    d = len(a)
    each = np.zeros((keys.size, d), np.int32)
    exact = np.zeros((keys.size, d), np.int32)
    fb = np.zeros(1, np.int64)
    vp = ctypes.c_void_p
    shim.host_buckets_modes(a.ctypes.data_as(vp), b.ctypes.data_as(vp), d, width, keys.ctypes.data_as(vp),
                            ctypes.c_int64(keys.size), each.ctypes.data_as(vp), exact.ctypes.data_as(vp),
                            fb.ctypes.data_as(vp))
    return each, exact, int(fb[0])


@pytest.mark.parametrize("depth", [4, 5, 6, 7])
@pytest.mark.parametrize("width", [1, 2, 1024, 4096, 8192, 1 << 20, 1 << 24, 1 << 25])
def test_quotient_route_small_keys(shim, oracle, depth, width):
    """bucket_q (the fp64-quotient route for keys below 2^32 at power-of-two
    widths) and each_bucket's unrolled rows equal the folding route and the
    oracle, margin fallbacks included (about 1 hash in 30,000 takes one)."""
    rng = np.random.Generator(np.random.PCG64(width * 10 + depth))
    keys = np.concatenate([
        rng.integers(0, 2 ** 32, size=400000, dtype=np.int64),
        rng.integers(0, 10_000_000, size=100000, dtype=np.int64),
        np.arange(0, 20000, dtype=np.int64),
        np.array([2 ** 32 - 1, 2 ** 32, 2 ** 31, 2 ** 31 - 1, -1, 0], np.int64),
    ])
    a, b = oracle.hash_params(depth * 7 + 1, depth)
    each, exact, fb = _modes(shim, a, b, width, keys)
    np.testing.assert_array_equal(each, exact)
    np.testing.assert_array_equal(each, oracle.hash_keys(a, b, width, keys))
    if 1 < width <= (1 << 24):
        assert fb > 0  # the margin route ran (and agreed)


def test_quotient_route_margin_cases(shim, oracle):
    """Keys whose quotient (a'k + b') / p lies within 2^-16 of an integer for
    some row: the fp64 floor alone is unreliable there, so the residue check
    decides.  Found by exact search over a key range per row."""
    a, b = oracle.hash_params(42, 5)
    p = 2 ** 63 - 25
    picked = []
    ks = np.arange(0, 3_000_000, dtype=np.int64)
    for r in range(5):
        ar, br = int(a[r]) % p, int(b[r]) % p
        # fractional part of (ar k + br) / p in units of p, vectorised with
        # Python ints over a strided subset (exact)
        sub = ks[r::7]
        fr = np.array([((ar * int(k) + br) % p) for k in sub], dtype=object)
        near = [int(k) for k, f in zip(sub, fr) if f < p >> 17 or f > p - (p >> 17)]
        picked += near[:200]
    keys = np.array(sorted(set(picked)), np.int64)
    assert keys.size > 20
    for w in [1024, 8192, 1 << 20]:
        each, exact, fb = _modes(shim, a, b, w, keys)
        assert fb >= keys.size  # every picked key took the margin route in its row
        np.testing.assert_array_equal(each, oracle.hash_keys(a, b, w, keys))


@pytest.mark.parametrize("width", [1, 2, 7, 24, 39, 1000, 2047, 30011, 2440690, (1 << 31) - 1])
def test_wbq_route_equals_barrett_route(shim, oracle, width):
    """bucket_wbq (per-owner shapes: fp64 quotient + wrapping residue, then
    Barrett) equals bucket_wb and the oracle for every width, keys below and
    above 2^32 and the margin keys of test_quotient_route_margin_cases."""
    rng = np.random.Generator(np.random.PCG64(width))
    keys = np.concatenate([rng.integers(0, 2 ** 32, size=300000, dtype=np.int64),
                           rng.integers(-2 ** 63, 2 ** 63 - 1, size=20000, dtype=np.int64),
                           np.arange(0, 5000, dtype=np.int64), np.array([2 ** 32 - 1, 2 ** 32, -1], np.int64)])
    a, b = oracle.hash_params(width % 1000 + 3, 24)
    q = np.zeros((keys.size, 24), np.int32)
    w = np.zeros((keys.size, 24), np.int32)
    vp = ctypes.c_void_p
    shim.host_buckets_wb(a.ctypes.data_as(vp), b.ctypes.data_as(vp), 24, width, keys.ctypes.data_as(vp),
                         ctypes.c_int64(keys.size), q.ctypes.data_as(vp), w.ctypes.data_as(vp))
    np.testing.assert_array_equal(q, w)
    np.testing.assert_array_equal(q[:, :6], oracle.hash_keys(a[:6], b[:6], width, keys))


def test_per_owner_barrett_low_word_remainder():
    """k_po_wide_bound's po_mod_w (cms_profiles.hip): s mod w for s < 2^63 and
    w < 2^30 from the Barrett estimate qq = (s * floor((2^64-1)/w)) >> 64 with
    only the low 32 bits of s - qq * w and two conditional subtractions --
    sound because qq is q - 2 .. q, so the true remainder s - qq * w < 3w <
    2^32.  Checked in exact integers at random and at the edges (s near
    multiples of w, s = 2^63 - 26, widths 1, 2, powers of two, 2^30 - 1)."""
    import random
    rng = random.Random(11)
    widths = [1, 2, 3, 7, 1025, 2049, 4096, 65537, 2440690, (1 << 30) - 1, 1 << 29]
    widths += [rng.randrange(1, 1 << 30) for _ in range(200)]
    for w in widths:
        m = ((1 << 64) - 1) // w
        ss = [0, 1, w - 1, w, w + 1, (1 << 63) - 26, (1 << 63) - 26 - ((1 << 63) - 26) % w]
        ss += [rng.randrange(0, (1 << 63) - 25) for _ in range(200)]
        ss += [k * w + d for k in (rng.randrange(0, ((1 << 63) - 26) // w) for _ in range(20)) for d in (0, w - 1)]
        for s in ss:
            qq = (s * m) >> 64
            assert s // w - 2 <= qq <= s // w
            rem = (s - qq * w) & 0xFFFFFFFF
            rem = rem - w if rem >= w else rem
            rem = rem - w if rem >= w else rem
            assert rem == s % w, (s, w)


@pytest.mark.parametrize("width", [1024, 8192, 1 << 24, 1000, 30011, 2440690])
def test_quotient_routes_at_two_to_the_32(shim, oracle, width):
    """a', b' within ~2^10 of p make a'/p and b'/p round to 1.0, so for
    k' = 2^32 - 1 the fp64 quotient y = fma(a'/p, k', b'/p) rounds up to
    exactly 2^32 while the true quotient is 2^32 - 1: the estimate needs 33
    bits. bucket_q (power-of-two widths) and bucket_wbq (any
    width) must still equal the folding route and the oracle."""
    p = 2 ** 63 - 25
    a = np.array([p - 1, p - 2, p - 1000, -2 ** 63, p - 1, 2 ** 63 - 1], np.int64)
    b = np.array([p - 1, p - 1, p - 3, 2 ** 63 - 1, p - 700, p - 1], np.int64)
    keys = np.array([2 ** 32 - 1, 2 ** 32 - 2, 2 ** 32 - 3, 2 ** 32 - 1000, 2 ** 32, 2 ** 31, 0, 1], np.int64)
    ref = oracle.hash_keys(a, b, width, keys)
    if width & (width - 1) == 0:
        each, exact, _ = _modes(shim, a, b, width, keys)
        np.testing.assert_array_equal(exact, ref)
        np.testing.assert_array_equal(each, ref)
    q = np.zeros((keys.size, a.size), np.int32)
    w = np.zeros((keys.size, a.size), np.int32)
    vp = ctypes.c_void_p
    shim.host_buckets_wb(a.ctypes.data_as(vp), b.ctypes.data_as(vp), a.size, width, keys.ctypes.data_as(vp),
                         ctypes.c_int64(keys.size), q.ctypes.data_as(vp), w.ctypes.data_as(vp))
    np.testing.assert_array_equal(w, ref)
    np.testing.assert_array_equal(q, ref)
