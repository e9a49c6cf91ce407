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
