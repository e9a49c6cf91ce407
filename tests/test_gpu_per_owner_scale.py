"""GPU: the reference's native per-owner-shape CosineCM (CountMinSketchConfig
shapes, userSimilarity(u1, u2) hashing u1 at u2's shape: CosineCM.java:83-96,
CountMinSketchConfig.java:120-158) at the scale bench.py times it: the
config-2 DataModel (the bench's 50M-pair Zipf stream, seed 20261015, as 100K
items keyed by 1M users), CountMinSketchConfig(q=1) for every item, and the
WHOLE pruned all-pairs top-100 (cms_top_k_all: grouped narrow classes,
big-query class sketches, the row-0 bound for wide candidates, exact
survivors).

Eight query rows -- the two smallest queries of more than 4096 preferences
(the k_po_bigq path), the two smallest wide owners (w > 2048), two of the
widest narrow part (w 1025..2048) and two random rows -- are checked against
the oracle's restatement over ALL 100K candidates (oracle.per_owner_rows_csr:
u1's sketch at each candidate's shape against the candidate's own sketch,
bit for bit), and each of their all-pairs lists against the oracle's
TopItems.getTopUsers loop on those values.  The query rows' shapes are
checked against the oracle's computeConfig search.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N_USERS, N_ITEMS, PAIRS, SEED_STREAM, K = 1_000_000, 100_000, 50_000_000, 20261015, 100


def _same(x, y):
    x, y = np.asarray(x), np.asarray(y)
    return x.shape == y.shape and bool(np.all((x == y) | (np.isnan(x) & np.isnan(y))))


def test_config2_per_owner_all_pairs_rows_equal_oracle(oracle):
    import torch
    from mahout_amd import SketchTable
    from mahout_amd.synth import zipf_stream_torch
    items, users = zipf_stream_torch(N_USERS, N_ITEMS, PAIRS, seed=SEED_STREAM, device="cuda")
    order = torch.argsort(items, stable=True)  # bench.csr_on_device: the DataModel's per-item key order
    ckeys = users[order].contiguous()
    del order
    off_d = torch.zeros(N_ITEMS + 1, dtype=torch.int64, device="cuda")
    off_d[1:] = torch.cumsum(torch.bincount(items, minlength=N_ITEMS), 0)
    del items, users
    n = N_ITEMS
    with SketchTable.per_owner_shapes(n, seed=42) as t:
        t.ingest_csr_device(off_d, ckeys)
        t.configure_owner_shapes(1.0, N_USERS)
        t.finalize()
        ids, sc, cnt = t.top_k_all(K)
        st = t.stats()
        assert st["po_wide_pairs"] > 0 and st["po_wide_exact"] < st["po_wide_pairs"]  # the pruned path ran
        _, _, ws, ds = t.owner_shapes()
        off = off_d.cpu().numpy()
        keys = ckeys.cpu().numpy()
        nnz = np.diff(off)
        rng = np.random.default_rng(20261015)

        def smallest(mask, k):
            cand = np.flatnonzero(mask)
            return cand[np.argsort(nnz[cand], kind="stable")[:k]].tolist()

        big = smallest(nnz > 4096, 2)
        wide = smallest(ws > 2048, 2)
        part2 = np.flatnonzero((ws > 1024) & (ws <= 2048) & (nnz <= 20000))
        narrow_wide = rng.choice(part2, 2, replace=False).tolist()
        rand = rng.choice(n, 2, replace=False).tolist()
        rows = big + wide + narrow_wide + rand
        assert len(set(rows)) == 8, rows
        allids = np.arange(n, dtype=np.int64)
        got = np.stack([t.similarities(q, allids) for q in rows])
    a, b = oracle.hash_params(42, 32)
    for q in rows:  # CountMinSketchConfig.computeConfig for the queries' own shapes
        w_o, d_o, _, _ = oracle.compute_config(int(nnz[q]), N_USERS, 1.0)
        assert (int(ws[q]), int(ds[q])) == (w_o, d_o), q
    want = oracle.per_owner_rows_csr(off, keys, (ws, ds), a, b, np.array(rows, np.int64),
                                     threads=oracle.max_threads())
    for i, q in enumerate(rows):
        assert _same(got[i], want[i]), (q, int(np.sum(~((got[i] == want[i]) | (np.isnan(got[i]) & np.isnan(want[i]))))))
        row = want[i].copy()
        row[q] = np.nan  # mostSimilar never offers the owner itself
        eids, esc = oracle.top_users(allids, row, K)
        assert ids[q, :cnt[q]].tolist() == eids.tolist(), q
        assert _same(sc[q, :cnt[q]], esc), q
