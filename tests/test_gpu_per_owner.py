"""GPU parity of the per-owner-shape mode (CosineCM with its CountMinSketchConfig).

The reference's native CosineCM sizes each user's sketch from
CountMinSketchConfig (T/impl/common/CountMinSketchConfig.java:120-158) and
compares u1's sketch built with u2's (delta, epsilon) against u2's own
(T/impl/similarity/CosineCM.java:83-96).  Every value below is checked bit for
bit against the oracle's restatement (oracle/oracle.py per_owner_*), which
rebuilds both sketches per pair exactly as exportProfile does.

Parity note: the Fmeasure search evaluates Math.pow; the GPU uses the device
libm and the oracle glibc.  Their last-ulp differences could only flip an
argmax whose top two scores agree to ~1e-16 relative; the gaps on these data
are ~1e-8, so the chosen shapes must match exactly (asserted).
"""
import numpy as np
import pytest

from mahout_amd import SketchTable
from mahout_amd._lib import CmsError, CMS_E_SKETCH, CMS_E_STATE, CMS_E_NO_SUCH_ID
from mahout_amd.synth import movielens_like, to_csr

pytestmark = pytest.mark.gpu

SEED = 42


def same(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return a.shape == b.shape and bool(np.all((a == b) | (np.isnan(a) & np.isnan(b))))


def small_model(n_users=120, n_items=400, n_ratings=6000, seed=5):
    """A GenericDataModel-shaped CSR: users own sketches keyed by item ID,
    integer ratings 1..5, each user's preferences in item-ID order."""
    users, items, ratings = movielens_like(n_users, n_items, n_ratings, seed=seed, min_per_user=5)
    uid = np.unique(users)
    rows = np.searchsorted(uid, users)
    order = np.lexsort((items, rows))
    rows, items, ratings = rows[order], items[order], ratings[order]
    off, keys, vals = to_csr(rows, items, uid.size, ratings)
    return uid, off, keys, vals, n_items


def make(uid, off, keys, vals, weighted=False):
    t = SketchTable.per_owner_shapes(uid.size, seed=SEED, weighted=weighted, owner_ids=uid)
    t.ingest_csr(off, keys, vals)
    return t


@pytest.mark.parametrize("q", [0.5, 1.0, 2.0])
def test_configure_matches_countminsketchconfig(oracle, q):
    uid, off, keys, vals, u = small_model()
    with make(uid, off, keys, vals) as t:
        t.configure_owner_shapes(q, u)
        de, ep, w, d = t.owner_shapes()
    ode, oep = oracle.owner_config(off, u, q)
    assert np.array_equal(de, ode) and np.array_equal(ep, oep)
    ow, od = oracle.owner_shapes(ode, oep)
    assert np.array_equal(w, ow) and np.array_equal(d, od)
    assert (w > 0).all() and len(set(zip(w.tolist(), d.tolist()))) > 10  # genuinely heterogeneous


@pytest.mark.parametrize("weighted", [False, True])
def test_similarities_asymmetric_bit_exact(oracle, weighted):
    uid, off, keys, vals, u = small_model()
    a, b = oracle.hash_params(SEED, 32)
    with make(uid, off, keys, vals, weighted) as t:
        t.configure_owner_shapes(1.0, u)
        t.finalize()
        shapes = t.owner_shapes()[2:]
        for q in [0, 1, 17, uid.size - 1]:
            got = t.similarities(int(uid[q]), uid)
            exp = np.array([oracle.per_owner_similarity(off, keys, vals, shapes, a, b, q, c, weighted)
                            for c in range(uid.size)])
            assert same(got, exp)
        # userSimilarity(u1, u2) != userSimilarity(u2, u1) in general (u2's shape decides)
        s12, s21 = t.similarity(int(uid[0]), int(uid[1])), t.similarity(int(uid[1]), int(uid[0]))
        assert s12 == oracle.per_owner_similarity(off, keys, vals, shapes, a, b, 0, 1, weighted)
        assert s21 == oracle.per_owner_similarity(off, keys, vals, shapes, a, b, 1, 0, weighted)


def test_own_sketches_point_query_and_top_k(oracle):
    uid, off, keys, vals, u = small_model()
    a, b = oracle.hash_params(SEED, 32)
    with make(uid, off, keys, vals) as t:
        t.configure_owner_shapes(1.0, u)
        t.finalize()
        w, d = t.owner_shapes()[2:]
        for r in [0, 5, uid.size - 1]:
            own = oracle.export_profile(off, keys, vals, r, int(w[r]), int(d[r]), a, b)
            assert same(t.read_owner_sketch(int(uid[r])), own)
            for key in [int(keys[off[r]]), 7, -3, 10 ** 12]:
                assert t.point_query(int(uid[r]), key) == oracle.sketch_get(own, a, b, key)
        for q in [0, 3, 50]:
            row = np.array([oracle.per_owner_similarity(off, keys, vals, (w, d), a, b, q, c)
                            for c in range(uid.size)])
            row[q] = np.nan  # MostSimilarEstimator skips the user itself
            eids, escs = oracle.top_users(uid, row, 10)
            ids, scs = t.most_similar(int(uid[q]), 10)
            assert ids.tolist() == eids.tolist() and same(scs, escs)
        ids, scs, cnt = t.top_k_all(5)
        for q in [0, 3, 50]:
            assert ids[q, :cnt[q]].tolist() == t.most_similar(int(uid[q]), 5)[0].tolist()


def test_estimate_preferences_per_owner(oracle):
    uid, off, keys, vals, u = small_model()
    a, b = oracle.hash_params(SEED, 32)
    with make(uid, off, keys, vals) as t:
        t.configure_owner_shapes(1.0, u)
        t.finalize()
        w, d = t.owner_shapes()[2:]
        user = 4
        nb = [7, 4, 11, 30, 2, 90]
        items = np.unique(keys)[:64]
        got = t.estimate_preferences(int(uid[user]), uid[nb], items, capper=(1.0, 5.0))
        exp = []
        for it in items:
            pref_sum = tot = 0.0
            cnt = 0
            for r in nb:
                if r == user:
                    continue
                own = oracle.export_profile(off, keys, vals, r, int(w[r]), int(d[r]), a, b)
                p = np.float32(oracle.sketch_get(own, a, b, int(it)))
                if p == 0:
                    continue
                s = oracle.per_owner_similarity(off, keys, vals, (w, d), a, b, user, r)
                if np.isnan(s):
                    continue
                pref_sum += s * float(p)
                tot += s
                cnt += 1
            e = np.float32(pref_sum / tot) if cnt > 1 else np.float32(np.nan)
            exp.append(np.float32(min(max(e, 1.0), 5.0)) if cnt > 1 else e)
        assert same(got, np.array(exp, np.float32))


def test_wide_shapes_global_scratch_and_inexact_regime(oracle):
    """Caller-supplied (delta, epsilon): widths beyond the LDS row (global
    scratch path) and counters large enough that valueA leaves the exact fp64
    regime (sequential reference-order sums)."""
    n = 6
    off = np.array([0, 3, 7, 9, 12, 14, 20], np.int64)
    keys = np.array([1, 2, 3, 1, 5, 9, 11, 2, 3, 4, 5, 6, 100, 200, 1, 2, 3, 4, 5, 6], np.int64)
    vals = np.array([1, 2, 3, 4, 5, 1, 1, 2 ** 26, 2 ** 26, 3, 3, 3, 1, 2, 1, 1, 1, 1, 1, 1], np.float32)
    widths = np.array([5000, 9000, 3, 4097, 1, 40], np.float64)
    depths = np.array([2, 3, 5, 1, 32, 4], np.float64)
    de, ep = np.exp(-depths), np.exp(1.0) / widths
    uid = np.arange(n, dtype=np.int64) * 10
    a, b = oracle.hash_params(SEED, 32)
    with make(uid, off, keys, vals) as t:
        t.set_owner_delta_epsilon(de, ep)
        t.finalize()
        shapes = t.owner_shapes()[2:]
        assert np.array_equal(shapes[0], oracle.owner_shapes(de, ep)[0])
        for q in range(n):
            exp = np.array([oracle.per_owner_similarity(off, keys, vals, shapes, a, b, q, c) for c in range(n)])
            assert same(t.similarities(int(uid[q]), uid), exp)
        # the all-pairs slabs: narrow classes on the grouped kernel, the wide
        # owners (5000, 9000, 4097) on k_po_pairs, and owner 2's pairs (norms
        # past 2^53) replayed through the sequential path
        ids, sc, cnt = t.top_k_all(4)
        for q in range(n):
            row = np.array([oracle.per_owner_similarity(off, keys, vals, shapes, a, b, q, c) for c in range(n)])
            row[q] = np.nan
            eids, esc = oracle.top_users(uid, row, 4)
            assert ids[q, :cnt[q]].tolist() == eids.tolist() and same(sc[q, :cnt[q]], esc), q


def test_grouped_all_pairs_many_classes(oracle):
    """The all-pairs top-k over a model whose owners share shape classes
    (groups of up to 16 candidates per workgroup, classes split over several
    groups): equal to the per-row similarities (k_po_pairs) and to the
    oracle's TopItems loop on sampled rows."""
    users, items, ratings = movielens_like(1500, 300, 45_000, seed=21, min_per_user=3)
    uid = np.unique(users)
    rows = np.searchsorted(uid, users)
    order = np.lexsort((items, rows))
    off, keys, vals = to_csr(rows[order], items[order], uid.size, ratings[order])
    n, k = uid.size, 20
    a, b = oracle.hash_params(SEED, 32)
    with make(uid, off, keys, vals) as t:
        t.configure_owner_shapes(1.0, 300)
        t.finalize()
        w, d = t.owner_shapes()[2:]
        classes = {}
        for r in range(n):
            classes.setdefault((int(w[r]), int(d[r])), []).append(r)
        assert max(len(v) for v in classes.values()) > 16  # a class spans several groups
        ids, sc, cnt = t.top_k_all(k)
        for q in [0, 1, n // 3, n // 2, n - 1]:
            row = t.similarities(int(uid[q]), uid)  # per-pair kernel
            row[q] = np.nan
            eids, esc = oracle.top_users(uid, row, k)
            assert ids[q, :cnt[q]].tolist() == eids.tolist() and same(sc[q, :cnt[q]], esc), q
        for q in [0, n - 1]:
            row = np.array([oracle.per_owner_similarity(off, keys, vals, (w, d), a, b, q, c) for c in range(n)])
            row[q] = np.nan
            eids, esc = oracle.top_users(uid, row, k)
            assert ids[q, :cnt[q]].tolist() == eids.tolist() and same(sc[q, :cnt[q]], esc), q


def test_errors_like_the_reference(oracle):
    uid, off, keys, vals, u = small_model(n_users=30, n_items=100, n_ratings=600)
    with make(uid, off, keys, vals) as t:
        with pytest.raises(CmsError) as e:  # getDelta before configure -> TasteException
            t.finalize()
        assert e.value.code == CMS_E_STATE
        de, ep = oracle.owner_config(off, u, 1.0)
        de[3] = 0.0  # trove's 0.0 for a missing owner -> CMException on use
        ep[3] = 0.0
        t.set_owner_delta_epsilon(de, ep)
        t.finalize()
        t.similarity(int(uid[3]), int(uid[4]))  # u1's own config is never read
        with pytest.raises(CmsError) as e:
            t.similarity(int(uid[4]), int(uid[3]))
        assert e.value.code == CMS_E_SKETCH
        with pytest.raises(CmsError) as e:
            t.similarity(int(uid[0]), 123456789)
        assert e.value.code == CMS_E_NO_SUCH_ID
        with pytest.raises(CmsError) as e:
            t.ingest(np.array([uid[0]]), np.array([1]))
        assert e.value.code == CMS_E_STATE
        with pytest.raises(CmsError) as e:
            t.read_counters()
        assert e.value.code == CMS_E_STATE


def test_taste_mirror_cosinecm_with_countminsketchconfig(oracle):
    """taste.CosineCM(model, CountMinSketchConfig(q), HashFunctionBuilder(seed)):
    the reference's constructor shape, per-owner sizing searched on the GPU."""
    from mahout_amd.datamodel import GenericDataModel
    from mahout_amd.taste import CosineCM, CountMinSketchConfig, HashFunctionBuilder, TasteException
    uid, off, keys, vals, _ = small_model(n_users=60, n_items=200, n_ratings=2000, seed=11)
    model = GenericDataModel.from_csr(uid, off, keys, vals)
    conf = CountMinSketchConfig(1.0)
    with pytest.raises(TasteException):
        conf.getDelta(int(uid[0]))  # configure first (CountMinSketchConfig.java:230-240)
    sim = CosineCM(model, conf, HashFunctionBuilder(SEED))
    de, ep = oracle.owner_config(off, model.getNumItems(), 1.0)
    assert conf.getDelta(int(uid[7])) == de[7] and conf.getEpsilon(int(uid[7])) == ep[7]
    assert conf.getDelta(-12345) == 0.0  # trove default for a missing owner
    shapes = oracle.owner_shapes(de, ep)
    a, b = oracle.hash_params(SEED, 32)
    for u1, u2 in [(0, 1), (1, 0), (5, 59), (59, 5), (3, 3)]:
        exp = oracle.per_owner_similarity(off, keys, vals, shapes, a, b, u1, u2)
        assert same(sim.userSimilarity(int(uid[u1]), int(uid[u2])), exp)
    sim.close()


def test_big_queries_and_full_classes(oracle):
    """Owners with more than 4096 preferences (k_po_bigq: u1 hashed once per
    shape class, dense dots against the transposed member image) and classes
    of more than 64 members (several 64-member groups, the dense and the
    sparse dot path): the all-pairs top-k equals the per-pair kernel's rows,
    a handle without the big-query kernel (CMS_PO_NO_BIGQ=1), a handle
    without the wide owners' row-0 bound (CMS_PO_NO_PRUNE=1), and the
    oracle's TopItems loop on sampled big and small rows."""
    import os
    from mahout_amd.synth import zipf_stream
    items, users = zipf_stream(50_000, 3000, 300_000, seed=33)
    off, keys, _ = to_csr(items, users, 3000)
    nnz = np.diff(off)
    assert (nnz > 4096).sum() >= 3 and (nnz <= 64).sum() > 1000
    uid = np.arange(3000, dtype=np.int64) * 7 + 3
    n, k = uid.size, 25
    a, b = oracle.hash_params(SEED, 32)

    def run(env):
        old = {kk: os.environ.get(kk) for kk in env}
        os.environ.update(env)
        try:
            with make(uid, off, keys, None) as t:
                t.configure_owner_shapes(1.0, 50_000)
                t.finalize()
                shapes = t.owner_shapes()[2:]
                lists = t.top_k_all(k)
                big = np.flatnonzero(nnz > 4096)[:3].tolist()
                rows = {q: t.similarities(int(uid[q]), uid) for q in big + [0, n // 2, n - 1]}
                st = t.stats()
                run.pruned = (st["po_wide_pairs"], st["po_wide_exact"])
                return shapes, lists, rows
        finally:
            for kk, v in old.items():
                if v is None:
                    os.environ.pop(kk, None)
                else:
                    os.environ[kk] = v

    shapes, (ids, sc, cnt), rows = run({})
    w, d = shapes
    cls = {}
    for r in range(n):
        cls.setdefault((int(w[r]), int(d[r])), []).append(r)
    assert max(len(v) for v in cls.values()) > 64
    wide_pairs, wide_exact = run.pruned
    assert wide_pairs > 0 and wide_exact < wide_pairs  # the row-0 bound ruled wide pairs out
    _, (ids2, sc2, cnt2), _ = run({"CMS_PO_NO_BIGQ": "1"})
    assert np.array_equal(cnt, cnt2) and np.array_equal(ids, ids2) and same(sc, sc2)
    # every (query, wide owner) pair computed exactly: the same lists
    _, (ids3, sc3, cnt3), _ = run({"CMS_PO_NO_PRUNE": "1"})
    assert run.pruned == (0, 0)
    assert np.array_equal(cnt, cnt3) and np.array_equal(ids, ids3) and same(sc, sc3)
    for q, row in rows.items():
        row = row.copy()
        row[q] = np.nan
        eids, esc = oracle.top_users(uid, row, k)
        assert ids[q, :cnt[q]].tolist() == eids.tolist() and same(sc[q, :cnt[q]], esc), q
    # the per-pair kernel's rows against the oracle (a big and a small query;
    # the candidates of their lists plus a random sample: the oracle rebuilds
    # both sketches per pair)
    rng = np.random.default_rng(4)
    for q in [list(rows)[0], n - 1]:
        cols = np.unique(np.concatenate([np.searchsorted(uid, ids[q, :cnt[q]]), rng.choice(n, 60, replace=False)]))
        cols = cols[cols != q]
        exp = np.array([oracle.per_owner_similarity(off, keys, None, shapes, a, b, q, int(c)) for c in cols])
        assert same(rows[q][cols], exp), q
