"""GPU: the incremental all-pairs top-k refresh (cms_top_k_refresh, config 5's
periodic refresh) equals the whole job (cms_top_k_all) on the same table, bit
for bit, after every batch.

The reference recomputes nothing incrementally: a Refreshable
(`T/common/Refreshable.java:51`) re-reads its DataModel and the precomputed
similarities are rebuilt whole (`ItemSimilarityJob.java:101`, one
`TopItems.getTopUsers` per owner, `TopItems.java:91-136`).  The refresh must
therefore give exactly that whole result; cms_top_k_all is itself checked
against the oracle's TopItems restatement in test_gpu_parity.py.
"""
import numpy as np
import pytest

from mahout_amd import SketchTable
from mahout_amd.synth import zipf_stream

pytestmark = pytest.mark.gpu


def _same_lists(a, b):
    """Bit equality of two (ids, scores, counts) answers, padding included:
    past counts[r] every ID is -1 and every score NaN (include/mahout_cms.h,
    cms_top_k_all)."""
    ids, sc, cnt = a
    rids, rsc, rcnt = b
    if not np.array_equal(cnt, rcnt):
        return "counts differ at rows %s" % np.nonzero(cnt != rcnt)[0][:10].tolist()
    n, k = ids.shape
    pad = np.arange(k)[None, :] >= cnt[:, None]
    for x_ids, x_sc in ((ids, sc), (rids, rsc)):
        if not (x_ids[pad] == -1).all() or not np.isnan(x_sc[pad]).all():
            return "padding past a row's count is not (-1, NaN)"
    if not np.array_equal(ids, rids):
        return "ids differ at rows %s" % np.nonzero((ids != rids).any(1))[0][:10].tolist()
    eq = (sc == rsc) | (np.isnan(sc) & np.isnan(rsc))
    if not eq.all():
        return "scores differ at rows %s" % np.nonzero(~eq.all(1))[0][:10].tolist()
    return None


def _oracle_rows(O, table, lists, rows, k, weighted=False):
    """The refreshed lists of `rows` against the oracle's TopItems.getTopUsers
    loop (TopItems.java:91-136) over that row's exact similarities
    (DoubleCountMinSketch.cosine via CosineCM, oracle/cms_oracle.c)."""
    ids, sc, cnt = lists
    n = table.shape[0]
    for row in rows:
        exp = O.similarities_row(table, int(row), weighted)
        eids, esc = O.top_users(np.arange(n, dtype=np.int64), exp, k)
        if ids[row, :cnt[row]].tolist() != eids.tolist():
            return "row %d: ids differ from the oracle" % row
        if not np.array_equal(sc[row, :cnt[row]], esc, equal_nan=True):
            return "row %d: scores differ from the oracle" % row
    return None


def _batch(rng, n, frac, size, vmax, n_keys):
    """A COO batch whose owners are a random `frac` of all owners (Zipf-weighted
    inside that subset) -- the touched set of one streaming interval."""
    touched = rng.choice(n, size=max(1, int(frac * n)), replace=False)
    p = 1.0 / np.arange(1, touched.size + 1) ** 1.1
    rows = touched[rng.choice(touched.size, size=size, p=p / p.sum())].astype(np.int64)
    keys = rng.integers(0, n_keys, size=size).astype(np.int64)
    vals = rng.integers(1, vmax + 1, size=size).astype(np.float32)
    return rows, keys, vals


@pytest.mark.parametrize("n,d,w,vmax,k,weighted,seed", [
    (12000, 4, 256, 2, 25, False, 56),    # fp4 blocks beside int8 blocks, multi-wave bands
    (11776, 3, 128, 2, 20, False, 55),    # no fp4 image (w % 256): int8 waves only
    (3000, 5, 8192, 3, 100, False, 58),   # the config-4 shape: fp4, int8 and multi-limb owners
    (1800, 3, 256, 1, 64, True, 53),      # weighted: not on the symmetric kernel (all pairs recomputed)
    (700, 5, 512, 2, 5, False, 54),       # fewer than one block pair per wave
])
def test_refresh_equals_whole_job(n, d, w, vmax, k, weighted, seed, oracle):
    rng = np.random.Generator(np.random.PCG64(seed))
    items, users = zipf_stream(4000, n, 400_000, seed=seed)
    vals = rng.integers(1, vmax + 1, size=items.size).astype(np.float32)
    # at the config-4 shape the refreshed lists are also checked against the
    # oracle after every batch: touched and untouched sampled rows
    check_oracle = w == 8192
    stream = [(items.astype(np.int64), users.astype(np.int64), vals)]
    a, b = oracle.hash_params(42, d)
    with SketchTable(n, depth=d, width=w, seed=42, weighted=weighted) as t:
        t.ingest(items, users, vals)
        t.finalize()
        first = t.top_k_refresh(k)
        assert t.refresh_stats()[2] == 1
        err = _same_lists(first, t.top_k_all(k))
        assert err is None, err
        # batches touching 1% .. 30% of the owners; sizes through both the
        # plain-atomic and the owner-grouped incremental paths
        for step, (frac, size) in enumerate([(0.01, 2000), (0.05, 40_000), (0.15, 20_000), (0.3, 60_000),
                                             (0.002, 50)]):
            rows, keys, v = _batch(rng, n, frac, size, vmax, 4000)
            t.ingest(rows, keys, v)
            stream.append((rows, keys, v))
            t.finalize()
            got = t.top_k_refresh(k)
            touched, redone, full = t.refresh_stats()
            assert full == 1, "an incremental refresh fell back to a whole job"
            assert touched == np.unique(rows).size
            exp = t.top_k_all(k)
            err = _same_lists(got, exp)
            assert err is None, (step, frac, err, (touched, redone))
            if check_oracle:
                table = oracle.build_table(n, d, w, a, b, *[np.concatenate(c) for c in zip(*stream)])
                tr = np.unique(rows)
                untouched = np.setdiff1d(np.arange(n), tr)
                sample = np.concatenate([rng.choice(tr, min(3, tr.size), replace=False),
                                         rng.choice(untouched, 3, replace=False)])
                err = _oracle_rows(oracle, table, got, sample, k, weighted)
                assert err is None, (step, frac, err)
                del table
        # no batch since: the kept lists are returned as they are
        again = t.top_k_refresh(k)
        assert t.refresh_stats()[0] == 0
        assert _same_lists(again, exp) is None


def test_refresh_owner_ids_and_invalidation():
    """Owner IDs (not rows) in the output; a CSR ingest invalidates the kept
    lists (the next refresh is a whole job) and a different k starts over."""
    n, d, w, k = 4000, 4, 256, 30
    ids_of = np.arange(n, dtype=np.int64) * 7 + 1000
    items, users = zipf_stream(3000, n, 200_000, seed=9)
    with SketchTable(n, depth=d, width=w, seed=42, owner_ids=ids_of) as t:
        t.ingest(ids_of[items], users)
        t.finalize()
        t.top_k_refresh(k)
        rng = np.random.Generator(np.random.PCG64(3))
        rows, keys, v = _batch(rng, n, 0.1, 30_000, 1, 3000)
        t.ingest(ids_of[rows], keys, v)
        t.finalize()
        got = t.top_k_refresh(k)
        assert t.refresh_stats()[2] == 1
        assert _same_lists(got, t.top_k_all(k)) is None
        valid = np.arange(k)[None, :] < got[2][:, None]
        listed = got[0][valid]
        assert listed.size > 0 and set(np.unique(listed).tolist()) <= set(ids_of.tolist())
        assert (got[0][~valid] == -1).all() and np.isnan(got[1][~valid]).all()  # defined padding
        # another k: whole job again
        got = t.top_k_refresh(k + 5)
        assert t.refresh_stats()[2] == 2
        assert _same_lists(got, t.top_k_all(k + 5)) is None
        # a CSR batch does not mark owners: the next refresh is a whole job
        off = np.zeros(n + 1, np.int64)
        off[11:] = 3  # owner row 10 gets three keys
        t.ingest_csr(off, np.array([5, 6, 7], np.int64))
        t.finalize()
        got = t.top_k_refresh(k + 5)
        assert t.refresh_stats()[2] == 3
        assert _same_lists(got, t.top_k_all(k + 5)) is None


def test_refresh_lists_feed_generic_item_similarity():
    """The refreshed lists as Taste's precomputed similarities
    (GenericItemSimilarity(Iterable<ItemItemSimilarity>),
    GenericItemSimilarity.java:71-95): every listed pair answers with the
    GPU's own pair similarity, an unlisted pair with NaN."""
    from mahout_amd.taste import GenericItemSimilarity, similarities_from_top_k
    n, d, w, k = 600, 4, 256, 8
    items, users = zipf_stream(2000, n, 60_000, seed=12)
    with SketchTable(n, depth=d, width=w, seed=42) as t:
        t.ingest(items, users)
        t.finalize()
        t.top_k_refresh(k)
        rng = np.random.Generator(np.random.PCG64(5))
        rows, keys, v = _batch(rng, n, 0.1, 5000, 1, 2000)
        t.ingest(rows, keys, v)
        t.finalize()
        ids, sc, cnt = t.top_k_refresh(k)
        g = GenericItemSimilarity(similarities_from_top_k(ids, sc, cnt))
        listed = set()
        for r in range(0, n, 37):
            sims = t.similarities(r, np.arange(n))
            for i in range(cnt[r]):
                p = int(ids[r, i])
                listed.add((min(r, p), max(r, p)))
                assert g.itemSimilarity(r, p) == sims[p] == g.itemSimilarity(p, r)
        a, b = next((a, b) for a in range(n) for b in range(a + 1, n) if (a, b) not in listed
                    and b not in ids[a, :cnt[a]] and a not in ids[b, :cnt[b]])
        assert np.isnan(g.itemSimilarity(a, b))


def test_refresh_after_release_scratch(oracle):
    """cms_release_scratch frees the kept lists: a COO ingest after it must not
    mark into them, and the next refresh is a whole job equal to the whole
    all-pairs answer (and to the oracle's TopItems lists)."""
    n, d, w, k = 3000, 4, 256, 16
    items, users = zipf_stream(3000, n, 200_000, seed=21)
    rng = np.random.Generator(np.random.PCG64(21))
    with SketchTable(n, depth=d, width=w, seed=42) as t:
        t.ingest(items, users)
        t.finalize()
        t.top_k_refresh(k)
        t.release_scratch()
        rows, keys, v = _batch(rng, n, 0.1, 20_000, 1, 3000)
        t.ingest(rows, keys, v)
        t.finalize()
        got = t.top_k_refresh(k)
        assert t.refresh_stats()[2] == 2  # whole job: the kept lists were released
        assert _same_lists(got, t.top_k_all(k)) is None
        a, b = oracle.hash_params(42, d)
        table = oracle.build_table(n, d, w, a, b, np.concatenate([items, rows]), np.concatenate([users, keys]),
                                   np.concatenate([np.ones(items.size, np.float32), v]))
        assert _oracle_rows(oracle, table, got, [0, int(rows[0]), n // 3, n - 1], k) is None
        # and the incremental path works again from the new kept lists
        rows, keys, v = _batch(rng, n, 0.05, 5_000, 1, 3000)
        t.ingest(rows, keys, v)
        t.finalize()
        got = t.top_k_refresh(k)
        assert t.refresh_stats()[2] == 2
        assert _same_lists(got, t.top_k_all(k)) is None


def test_device_outputs_equal_host_outputs():
    """cms_top_k_all_device / cms_top_k_refresh_device write the same lists,
    padding included, into caller device buffers."""
    import torch
    n, d, w, k = 2500, 4, 256, 12
    items, users = zipf_stream(3000, n, 150_000, seed=31)
    with SketchTable(n, depth=d, width=w, seed=42) as t:
        t.ingest(items, users)
        t.finalize()
        host = t.top_k_all(k)
        dev = t.top_k_all_device(k)
        assert all(isinstance(x, torch.Tensor) and x.is_cuda for x in dev)
        assert _same_lists(tuple(x.cpu().numpy() for x in dev), host) is None
        t.top_k_refresh(k)
        rng = np.random.Generator(np.random.PCG64(31))
        rows, keys, v = _batch(rng, n, 0.1, 10_000, 1, 3000)
        t.ingest(rows, keys, v)
        t.finalize()
        dev = t.top_k_refresh_device(k)
        assert _same_lists(tuple(x.cpu().numpy() for x in dev), t.top_k_all(k)) is None


def test_noop_refresh_reports_no_touched_classes():
    """Two refreshes with no ingest between them: the second recomputes
    nothing, and cms_refresh_classes says so (it used to repeat
    the previous refresh's touched counts, which the bench prices)."""
    n, d, w, k = 2500, 4, 256, 12
    items, users = zipf_stream(3000, n, 150_000, seed=41)
    rng = np.random.Generator(np.random.PCG64(41))
    with SketchTable(n, depth=d, width=w, seed=42) as t:
        t.ingest(items, users)
        t.finalize()
        t.top_k_refresh(k)
        rows, keys, v = _batch(rng, n, 0.1, 10_000, 1, 3000)
        t.ingest(rows, keys, v)
        t.finalize()
        first = t.top_k_refresh(k)
        assert t.refresh_stats()[0] > 0
        assert sum(c[1] for c in t.refresh_classes().values()) > 0
        again = t.top_k_refresh(k)
        assert t.refresh_stats()[0] == 0
        cls = t.refresh_classes()
        assert all(c[1] == 0 for c in cls.values()), cls
        assert sum(c[0] for c in cls.values()) == n
        assert _same_lists(again, first) is None


def test_stats_struct_size_contract():
    """cms_get_stats writes only the fields a caller's (possibly older,
    shorter) cms_stats has room for, and refuses a missing struct_size."""
    import ctypes
    from mahout_amd import _lib
    lib = _lib.load()
    items, users = zipf_stream(1000, 500, 20_000, seed=5)
    with SketchTable(500, depth=4, width=256, seed=42) as t:
        t.ingest(items, users)
        t.finalize()
        full = t.stats()
        assert full["struct_size"] == ctypes.sizeof(_lib.CmsStats) and full["num_owners"] == 500
        buf = (ctypes.c_uint8 * ctypes.sizeof(_lib.CmsStats))(*([0xAB] * ctypes.sizeof(_lib.CmsStats)))
        s = _lib.CmsStats.from_buffer(buf)
        short = _lib.CmsStats.num_owners.offset + 8  # an old caller's struct ending at num_owners
        s.struct_size = short
        assert lib.cms_get_stats(t._h, ctypes.byref(s)) == 0
        assert s.struct_size == short and s.pairs_ingested == full["pairs_ingested"] and s.num_owners == 500
        assert all(b == 0xAB for b in bytes(buf)[short:])  # nothing past the caller's struct
        s.struct_size = 0
        assert lib.cms_get_stats(t._h, ctypes.byref(s)) != 0
