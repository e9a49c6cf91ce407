"""Configs 3 + 4 at full size on one GPU (BASELINE.json configs[2], configs[3]):
a 500M-pair Zipf stream (10M users x 1M items) into the d=5, w=8192 table --
163.8 GB as u32, 82 GB as this build's u16 narrow rows -- then the all-pairs
top-100 of every one of the 1M items through cms_top_k_all.

The oracle cannot hold a 1M x 40960 fp64 table, so the check is split the way
the domain allows:
  * checksum of checksums -- every update adds its increment once to each of
    the d rows (`T/impl/common/DoubleCountMinSketch.java:72-80`), so each row
    of every one of the 1M sketches sums to that owner's pair count (read on
    the device, cms_read_counters_device, compared with an independent
    torch.bincount of the stream);
  * the 16 hottest owners (the 8192-key slice / u32 hot-row path) and 32
    random ones rebuilt by the oracle from their own pairs, bit for bit;
  * all-pairs top-100 (`TopItems.java:91-136`, `SimilarUser.java:62-78`):
    ordering rules on every list and no overflow redo; for sampled rows whose
    lists come from fp4 x fp4 blocks, int8 blocks and multi-limb owners, the
    oracle computes the row's similarity to ALL 1M owners from the stream
    itself (each owner's sketch rows rebuilt from its own keys,
    orc_cosine_queries_csr), the exact pair kernel must equal all 1M of them,
    and the list must equal the oracle's TopItems loop over the oracle's
    similarities;
  * config 5: one streaming batch, then cms_top_k_refresh equals cms_top_k_all
    on the updated table for all 1M lists.
"""
import numpy as np
import pytest

from mahout_amd import SketchTable
from mahout_amd.synth import zipf_stream_torch

pytestmark = pytest.mark.gpu

N_USERS, N_ITEMS, N_PAIRS, D, W, SEED, K = 10_000_000, 1_000_000, 500_000_000, 5, 8192, 42, 100
CHUNK = 16384  # owners per device read-back: 16384 x 40960 u32 = 2.7 GB


def _same(a, b):
    return bool(np.all((a == b) | (np.isnan(a) & np.isnan(b))))


@pytest.mark.timeout(900)
def test_config34_full_size(oracle):
    import torch

    items, users = zipf_stream_torch(N_USERS, N_ITEMS, N_PAIRS, seed=20261016, device="cuda")
    counts_d = torch.bincount(items, minlength=N_ITEMS)
    counts = counts_d.cpu().numpy()
    assert int(counts.sum()) == N_PAIRS
    t = SketchTable(N_ITEMS, depth=D, width=W, seed=SEED)
    try:
        t.ingest_device_rows(items, users, None, N_PAIRS)
        t.finalize()
        t.synchronize()

        # 1. checksum of checksums over all 1M owners, and each owner's largest counter
        rowmax = torch.empty(N_ITEMS, dtype=torch.int64, device="cuda")
        buf = torch.empty((CHUNK, D, W), dtype=torch.int32, device="cuda")
        for o in range(0, N_ITEMS, CHUNK):
            c = min(CHUNK, N_ITEMS - o)
            v = t.read_counters_device(o, c, buf[:c])
            sums = v.sum(dim=2, dtype=torch.int64)
            want = counts_d[o:o + c, None].expand(c, D)
            assert torch.equal(sums, want), o
            rowmax[o:o + c] = v.view(c, -1).amax(dim=1).to(torch.int64)
        del buf, v, sums
        rowmax = rowmax.cpu().numpy()

        # the whole stream grouped by owner on the host (the oracle's CSR; a
        # stable sort keeps each owner's keys in stream order)
        order = torch.sort(items, stable=True)[1]
        su_all = users[order].cpu().numpy()
        del order, items, users, counts_d
        off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        a, b = oracle.hash_params(SEED, D)

        def oracle_sketch(owner):
            lo, hi = int(off[owner]), int(off[owner + 1])
            return oracle.build_table(1, D, W, a, b, np.zeros(hi - lo, np.int64), su_all[lo:hi])

        # 2. the hottest 16 and 32 random owners bit for bit against the oracle
        rng = np.random.default_rng(2027)
        hot = np.argsort(counts)[-16:]
        sample = np.unique(np.concatenate([hot, rng.choice(np.flatnonzero(counts), 32, replace=False)]))
        for owner in sample.tolist():
            np.testing.assert_array_equal(t.read_counters(owner, 1), oracle_sketch(owner), err_msg=str(owner))
        torch.cuda.empty_cache()
        t.release_scratch()

        # 3. all-pairs top-100 of every owner
        ids, sc, cnt = t.top_k_all(K)
        st = t.stats()
        assert st["topk_redo"] == 0
        assert st["fp4_owners"] > 0 and st["multi_limb_owners"] > 0
        assert (cnt == K).mean() > 0.99
        valid = np.arange(K)[None, :] < cnt[:, None]
        assert not np.isnan(sc[valid]).any()
        pair = valid[:, 1:]
        dsc = np.diff(sc, axis=1)
        assert (dsc[pair] <= 0).all()
        assert (np.diff(ids, axis=1)[pair & (dsc == 0)] > 0).all()  # ties by ID ascending
        assert (ids != np.arange(N_ITEMS)[:, None])[valid].all()  # self never listed

        # 4. sampled rows from every operand class against the oracle: each
        # row's similarity to ALL 1M owners, the owners' sketch rows rebuilt
        # by the oracle from their own keys (orc_cosine_queries_csr), and the
        # oracle's TopItems loop over those similarities
        fp4 = np.flatnonzero((rowmax <= 4) & (counts > 0))
        i8 = np.flatnonzero((rowmax > 4) & (rowmax < 128))
        ml = np.flatnonzero(rowmax >= 128)
        rows = np.concatenate([rng.choice(fp4, 2, replace=False), rng.choice(i8, 2, replace=False),
                               rng.choice(ml, 2, replace=False)])
        qsk = np.stack([oracle_sketch(r).reshape(-1) for r in rows.tolist()])
        osims = oracle.cosine_queries_csr(qsk, off, su_all, None, D, W, a, b, threads=16)
        all_ids = np.arange(N_ITEMS, dtype=np.int64)
        for qi, row in enumerate(rows.tolist()):
            want = osims[qi].copy()
            want[row] = np.nan  # MostSimilarEstimator: the owner itself is NaN
            sims = t.similarities(row, all_ids)  # exact pair kernel over all 1M owners
            sims[row] = np.nan
            same = (sims == want) | (np.isnan(sims) & np.isnan(want))
            assert same.all(), (row, np.flatnonzero(~same)[:8])
            eids, esc = oracle.top_users(all_ids, want, K)
            assert ids[row, :cnt[row]].tolist() == eids.tolist(), row
            assert _same(sc[row, :cnt[row]], esc), row
        del su_all

        # 5. config 5 at this size: the incremental refresh after one 1.25M-pair
        # Zipf batch equals the whole job on the updated table, every list
        def same_lists(a_, b_):
            i1, s1, c1 = a_
            i2, s2, c2 = b_
            if not np.array_equal(c1, c2):
                return False
            pad = np.arange(K)[None, :] >= c1[:, None]
            if not ((i1[pad] == -1).all() and np.isnan(s1[pad]).all()):  # defined padding
                return False
            return bool(np.array_equal(i1, i2)) and _same(s1, s2)

        assert same_lists(t.top_k_refresh(K), (ids, sc, cnt))  # whole job; keeps the 2k-deep lists
        bi, bu = zipf_stream_torch(N_USERS, N_ITEMS, 1_250_000, seed=777_000, device="cuda")
        t.ingest_device_rows(bi.contiguous(), bu.contiguous(), None, int(bi.numel()))
        t.finalize()
        redo0 = t.stats()["topk_redo"]
        got = t.top_k_refresh(K)
        touched, redone, full = t.refresh_stats()
        assert full == 1 and 0 < touched < N_ITEMS // 2
        # the refresh's lists keep their room (seeded thresholds): no whole-row recomputes
        assert redone == 0 and t.stats()["topk_redo"] == redo0
        cls = t.refresh_classes()
        assert sum(c[0] for c in cls.values()) == N_ITEMS and sum(c[1] for c in cls.values()) == touched, cls
        assert same_lists(got, t.top_k_all(K))
        # refreshed lists of 2 touched and 2 untouched owners against the
        # oracle's TopItems loop over the updated table's exact similarities
        tb = np.unique(bi.cpu().numpy())
        untouched = np.setdiff1d(np.flatnonzero(counts), tb)
        gi, gs, gc = got
        for row in np.concatenate([rng.choice(tb, 2, replace=False), rng.choice(untouched, 2, replace=False)]).tolist():
            sims = t.similarities(row, all_ids)
            sims[row] = np.nan
            eids, esc = oracle.top_users(all_ids, sims, K)
            assert gi[row, :gc[row]].tolist() == eids.tolist(), row
            assert _same(gs[row, :gc[row]], esc), row
            sa = t.read_counters(row, 1)[0]
            for p in np.concatenate([gi[row, :gc[row]][:20], rng.choice(N_ITEMS, 20, replace=False)]).tolist():
                if p != row:
                    assert _same(np.array([sims[p]]), np.array([oracle.cosine_cm(sa, t.read_counters(p, 1)[0])])), (row, p)
    finally:
        t.close()
        torch.cuda.empty_cache()
