"""GPU edge cases of the sketch path against the oracle: empty and ragged
inputs, single owners, the extreme shapes the ABI allows (depth 32, width 1,
width 32768), duplicate pairs, all-zero sketches (NaN similarities) and the
u32 overflow guard."""
import numpy as np
import pytest

from mahout_amd import SketchTable
from mahout_amd._lib import CmsError, CMS_E_OVERFLOW, CMS_E_PARAM, CMS_E_STATE
from mahout_amd.synth import zipf_stream, to_csr

pytestmark = pytest.mark.gpu


def same(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return a.shape == b.shape and bool(np.all((a == b) | (np.isnan(a) & np.isnan(b))))


def otable(oracle, n, d, w, rows, keys, vals=None):
    a, b = oracle.hash_params(42, d)
    return oracle.build_table(n, d, w, a, b, rows, keys, vals)


def row_sims(oracle, t, q):
    r = oracle.similarities_row(t, q)
    r[q] = oracle.cosine_cm(t[q], t[q])
    return r


def test_empty_table_and_empty_batches(oracle):
    """No data: every counter zero, every similarity NaN (den == 0 on every
    row, DoubleCountMinSketch.java:139-147), empty top-k lists."""
    with SketchTable(5, depth=3, width=64) as t:
        t.ingest(np.zeros(0, np.int64), np.zeros(0, np.int64))
        t.ingest_csr(np.zeros(6, np.int64), np.zeros(0, np.int64))
        t.finalize()
        assert not t.read_counters().any()
        assert np.isnan(t.similarities(0, np.arange(5))).all()
        ids, sc = t.most_similar(0, 3)
        assert ids.size == 0
        _, _, cnt = t.top_k_all(3)
        assert (cnt == 0).all()


def test_ragged_csr_with_empty_owners(oracle):
    n, d, w = 9, 4, 128
    off = np.array([0, 0, 3, 3, 3, 10, 10, 11, 11, 20], np.int64)
    keys = np.array([5, 5, 6, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 1], np.int64)
    rows = np.repeat(np.arange(n), np.diff(off))
    exp = otable(oracle, n, d, w, rows, keys)
    with SketchTable(n, depth=d, width=w) as t:
        t.ingest_csr(off, keys)
        t.finalize()
        assert same(t.read_counters(), exp)
        for q in range(n):
            assert same(t.similarities(q, np.arange(n)), row_sims(oracle, exp, q))


def test_single_owner_and_duplicates(oracle):
    """One owner; duplicate (owner, key) pairs add, as repeated update() calls do."""
    keys = np.array([3, 3, 3, -1, 2 ** 62, 3], np.int64)
    rows = np.zeros(keys.size, np.int64)
    exp = otable(oracle, 1, 5, 256, rows, keys)
    with SketchTable(1, depth=5, width=256) as t:
        t.ingest(rows, keys)
        t.finalize()
        assert same(t.read_counters(), exp)
        assert t.similarity(0, 0) == oracle.cosine_cm(exp[0], exp[0])
        assert t.most_similar(0, 5)[0].size == 0  # only itself, which is excluded


@pytest.mark.parametrize("d,w", [(32, 16), (1, 1), (2, 32768), (3, 1000)])
def test_extreme_shapes(oracle, d, w):
    n = 40
    items, users = zipf_stream(3000, n, 20_000, seed=d * 1000 + w)
    exp = otable(oracle, n, d, w, items, users)
    with SketchTable(n, depth=d, width=w) as t:
        t.ingest(items, users)
        t.finalize()
        assert same(t.read_counters(), exp)
        for q in [0, n - 1]:
            assert same(t.similarities(q, np.arange(n)), row_sims(oracle, exp, q))
        ids, _ = t.most_similar(0, 7)
        eids, _ = oracle.top_users(np.arange(n), oracle.similarities_row(exp, 0), 7)
        assert ids.tolist() == eids.tolist()


@pytest.mark.parametrize("d,w", [(32, 16), (2, 48), (4, 96), (1, 1024)])
def test_bulk_csr_build_odd_widths(oracle, d, w):
    """The LDS row build (CSR ingest) at widths whose sketch rows are not
    whole 16-B words of 4-bit counters (d*w % 32 == 0 but w % 32 != 0) keeps
    u16 rows; w % 32 == 0 takes the narrow forms -- all equal the oracle."""
    n = 300
    items, users = zipf_stream(5000, n, 60_000, seed=d + w)
    off, keys, _ = to_csr(items, users, n)
    exp = otable(oracle, n, d, w, items, users)
    with SketchTable(n, depth=d, width=w) as t:
        t.ingest_csr(off, keys)
        t.finalize()
        assert same(t.read_counters(), exp)
        for q in [0, 7, n - 1]:
            assert same(t.similarities(q, np.arange(n)), row_sims(oracle, exp, q))
        st = t.stats()
        narrow = st["nibble_rows"] + st["crumb_rows"] + st["bit_rows"] + st["u8_rows"] + st["list_rows"]
        assert (narrow > 0) == (w % 32 == 0), st


def test_bulk_build_of_width_32768_owner_rows(oracle):
    """The LDS row build at the largest width (128 KiB rows) with hot rows."""
    n, d, w = 30, 2, 32768
    items, users = zipf_stream(200_000, n, 300_000, seed=3)
    off, keys, _ = to_csr(items, users, n)
    exp = otable(oracle, n, d, w, items, users)
    with SketchTable(n, depth=d, width=w) as t:
        t.ingest_csr(off, keys)
        t.finalize()
        assert same(t.read_counters(), exp)


def test_overflow_guard_and_bad_params():
    with pytest.raises(CmsError) as e:
        SketchTable(4, depth=33, width=64)
    assert e.value.code == CMS_E_PARAM
    with pytest.raises(CmsError) as e:
        SketchTable(4, depth=3, width=40000)
    assert e.value.code == CMS_E_PARAM
    with SketchTable(2, depth=2, width=16) as t:
        big = np.full(3, 2.0 ** 31, np.float32)  # row mass reaches 2^32 (> u32)
        with pytest.raises(CmsError) as e:
            t.ingest(np.zeros(3, np.int64), np.arange(3, dtype=np.int64), big)
        assert e.value.code == CMS_E_OVERFLOW
    with SketchTable(2, depth=2, width=16) as t:
        with pytest.raises(CmsError) as e:
            t.similarity(0, 1)  # before finalize
        assert e.value.code == CMS_E_STATE


def test_device_csr_offsets_checked_before_the_build():
    """cms_ingest_csr_device checks offsets[0] == 0 and non-decreasing on the
    device before any counter is touched (the build would otherwise read keys
    outside the caller's buffer); the table stays as it was."""
    import torch
    from mahout_amd._lib import CMS_E_PARAM, CmsError
    with SketchTable(4, depth=2, width=64) as t:
        keys = torch.arange(10, dtype=torch.int64, device="cuda")
        good = torch.tensor([0, 3, 6, 8, 10], dtype=torch.int64, device="cuda")
        t.ingest_csr_device(good, keys)
        t.finalize()
        before = t.read_counters()
        for bad in ([0, 3, 2, 8, 10], [1, 3, 6, 8, 10]):
            with pytest.raises(CmsError) as ei:
                t.ingest_csr_device(torch.tensor(bad, dtype=torch.int64, device="cuda"), keys)
            assert ei.value.code == CMS_E_PARAM
        t.finalize()
        assert np.array_equal(t.read_counters(), before)
