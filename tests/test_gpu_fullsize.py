"""Config 2 at full size (BASELINE.json configs[1]: Zipf 1M users x 100K items,
50M pairs, d=5, w=4096) through the device COO path the bench times.

The oracle cannot rebuild 50M pairs in seconds, so the whole table is checked
through size-independent properties of DoubleCountMinSketch.update
(`T/impl/common/DoubleCountMinSketch.java:72-80`): every update adds its
increment once to each of the d rows, so with unit increments each row of an
owner's sketch sums to that owner's pair count (a checksum per owner per row,
all 100K owners); the table does not depend on stream order (a shuffled copy
of the stream builds the identical table); and the owners the hot-row paths
handle (the hottest ones) plus a random sample are rebuilt by the oracle from
their own pairs and compared bit for bit.
"""
import numpy as np
import pytest

from mahout_amd import SketchTable
from mahout_amd.synth import zipf_stream_torch

pytestmark = pytest.mark.gpu

N_USERS, N_ITEMS, N_PAIRS, D, W, SEED = 1_000_000, 100_000, 50_000_000, 5, 4096, 42
CHUNK = 2500  # owners per read-back: 2500 x 5 x 4096 fp64 = 410 MB of host memory


def _build(items, users):
    t = SketchTable(N_ITEMS, depth=D, width=W, seed=SEED)
    t.ingest_device_rows(items, users, None, items.numel())
    t.finalize()
    t.synchronize()
    return t


def test_config2_full_size_properties(oracle):
    import torch

    items, users = zipf_stream_torch(N_USERS, N_ITEMS, N_PAIRS, device="cuda")
    counts = torch.bincount(items, minlength=N_ITEMS).cpu().numpy()
    assert int(counts.sum()) == N_PAIRS

    perm = torch.randperm(N_PAIRS, device="cuda", generator=torch.Generator(device="cuda").manual_seed(7))
    t1 = _build(items, users)
    t2 = _build(items[perm], users[perm])
    del perm
    try:
        # checksum of checksums: every row of every owner sums to its pair count
        for o in range(0, N_ITEMS, CHUNK):
            c1 = t1.read_counters(o, CHUNK)
            sums = c1.sum(axis=2)
            np.testing.assert_array_equal(sums, np.repeat(counts[o:o + CHUNK, None], D, axis=1).astype(np.float64))
            if (o // CHUNK) % 8 == 0:  # order independence, 1 chunk in 8 (the read-back dominates the test)
                np.testing.assert_array_equal(t2.read_counters(o, CHUNK), c1)
            del c1

        # bit-exact owners: the 4 hottest (the 8192-key slice / hot-row path) and 12 random ones
        rng = np.random.default_rng(2026)
        hot = np.argsort(counts)[-4:]
        sample = np.concatenate([hot, rng.choice(np.flatnonzero(counts), 12, replace=False)])
        a, b = oracle.hash_params(SEED, D)
        for owner in sample.tolist():
            mask = items == owner
            keys = users[mask].cpu().numpy()
            assert keys.size == counts[owner]
            want = oracle.build_table(1, D, W, a, b, np.zeros(keys.size, np.int64), keys)
            np.testing.assert_array_equal(t1.read_counters(owner, 1), want)
    finally:
        t1.close()
        t2.close()


def test_config2_full_size_csr_equals_coo():
    """The DataModel layout (per-owner CSR, `GenericDataModel.java:91`) and the
    unordered COO stream build the same config-2 table."""
    import torch

    items, users = zipf_stream_torch(N_USERS, N_ITEMS, N_PAIRS, seed=11, device="cuda")
    order = torch.sort(items, stable=True).indices
    offsets = torch.zeros(N_ITEMS + 1, dtype=torch.int64, device="cuda")
    offsets[1:] = torch.cumsum(torch.bincount(items, minlength=N_ITEMS), 0)
    csr_keys = users[order].contiguous()
    del order
    t1 = _build(items, users)
    t2 = SketchTable(N_ITEMS, depth=D, width=W, seed=SEED)
    try:
        t2.ingest_csr_device(offsets, csr_keys)
        t2.finalize()
        t2.synchronize()
        for o in range(0, N_ITEMS, 4 * CHUNK):  # 1 chunk in 4, the hottest owners are spread by the permutation
            np.testing.assert_array_equal(t2.read_counters(o, CHUNK), t1.read_counters(o, CHUNK))
        hot = int(torch.argmax(offsets[1:] - offsets[:-1]))
        np.testing.assert_array_equal(t2.read_counters(hot, 1), t1.read_counters(hot, 1))
    finally:
        t1.close()
        t2.close()


def test_config2_full_size_top_k_all(oracle):
    """All-pairs top-100 over the whole config-2 table: the
    symmetric streaming pass (`cms_top_k_all`) equals the per-row slab path on
    sampled row blocks, every list is full and ordered (score desc, ID asc,
    `SimilarUser.java:62-78`), and sampled scores equal the oracle's
    `CosineCM` on the owners' fp64 sketches."""
    import torch

    k = 100
    items, users = zipf_stream_torch(N_USERS, N_ITEMS, N_PAIRS, device="cuda")
    t = _build(items, users)
    del items, users
    try:
        ids, sc, cnt = t.top_k_all(k)
        assert (cnt == k).mean() > 0.99  # only owners with (almost) no pairs can have short lists
        valid = np.arange(k)[None, :] < cnt[:, None]
        assert not np.isnan(sc[valid]).any()
        pair = valid[:, 1:]
        assert (np.diff(sc, axis=1)[pair] <= 0).all()
        tie = pair & (np.diff(sc, axis=1) == 0)
        assert (np.diff(ids, axis=1)[tie] > 0).all()
        assert (ids != np.arange(N_ITEMS)[:, None])[valid].all()  # self is NaN, never listed
        for begin in (0, 41_000, N_ITEMS - 512):
            ri, rs, rc = t.top_k_rows(begin, 512, k)
            np.testing.assert_array_equal(rc, cnt[begin:begin + 512])
            np.testing.assert_array_equal(ri, ids[begin:begin + 512])
            np.testing.assert_array_equal(rs, sc[begin:begin + 512])
        rng = np.random.default_rng(5)
        for row in rng.choice(np.flatnonzero(cnt == k), 3, replace=False).tolist():
            sa = t.read_counters(row, 1)[0]
            for j in (0, 1, k // 2, k - 1):
                want = oracle.cosine_cm(sa, t.read_counters(int(ids[row, j]), 1)[0])
                assert sc[row, j] == want
    finally:
        t.close()
