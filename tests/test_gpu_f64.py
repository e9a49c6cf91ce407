"""GPU parity of the fp64-counter mode (CMS_COUNTER_F64): DoubleCountMinSketch's
own counter type for float preferences the exact u32 mode cannot hold --
non-dyadic values with realistic per-owner masses, and negative values.

The reference adds `(double) float pref` into fp64 counters in the owner's
PreferenceArray order (`T/impl/common/DoubleCountMinSketch.java:72-80`) and
sums valueA / valueB / valueAB sequentially in j order (`:114-149`); the
oracle restates exactly that arithmetic, so the bar is bit equality (NaN ==
NaN) for counters, similarities, point queries, estimates and top-k lists.
"""
import numpy as np
import pytest

from mahout_amd import SketchTable
from mahout_amd._lib import CMS_E_PARAM, CMS_E_STATE, CmsError
from mahout_amd.synth import to_csr, zipf_stream

pytestmark = pytest.mark.gpu


def same(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return a.shape == b.shape and bool(np.all((a == b) | (np.isnan(a) & np.isnan(b))))


def _stream(n, npairs, seed, kind):
    items, users = zipf_stream(3000, n, npairs, seed=seed)
    rng = np.random.Generator(np.random.PCG64(seed))
    if kind == "ratings":  # ordinary float ratings (non-dyadic), owner masses in the thousands
        vals = np.round(rng.uniform(0.5, 5.0, items.size), 1).astype(np.float32)
    elif kind == "signed":  # centred / negative preferences
        vals = rng.normal(0.0, 1.7, items.size).astype(np.float32)
    else:  # TasteTestCase-like 0.1 .. 0.8
        vals = rng.choice(np.array([0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8], np.float32), items.size)
    return items, users, vals


@pytest.mark.parametrize("kind,n,d,w", [("ratings", 400, 4, 1024), ("signed", 300, 5, 512), ("taste", 200, 3, 100)])
@pytest.mark.parametrize("weighted", [False, True])
def test_f64_counters_similarities_topk_bit_exact(oracle, kind, n, d, w, weighted):
    items, users, vals = _stream(n, 120_000, 11 + n, kind)
    a, b = oracle.hash_params(42, d)
    exp = oracle.build_table(n, d, w, a, b, items, users, vals)
    with SketchTable(n, depth=d, width=w, seed=42, weighted=weighted, counters="f64") as t:
        t.ingest(items, users, vals)  # host COO: grouped by owner, stream order kept
        t.finalize()
        assert same(t.read_counters(), exp)
        for q in (0, 7, n // 2, n - 1):
            ref = oracle.similarities_row(exp, q, weighted)
            ref[q] = oracle.cosine_cm(exp[q], exp[q], weighted)
            assert same(t.similarities(q, np.arange(n)), ref), q
        for key in [int(users[0]), int(users[1]), 5, -9, 2 ** 40]:
            assert t.point_query(3, key) == oracle.sketch_get(exp[3], a, b, key)
        k = 25
        ids, sc, cnt = t.top_k_all(k)
        for q in range(0, n, max(1, n // 13)):
            eids, esc = oracle.top_users(np.arange(n), oracle.similarities_row(exp, q, weighted), k)
            assert ids[q, :cnt[q]].tolist() == eids.tolist(), q
            assert same(sc[q, :cnt[q]], esc), q
        nb = ids[5, :10]
        nb = np.concatenate([nb, [5]])
        its = np.unique(users)[:300]
        got = t.estimate_preferences(5, nb, its, (0.5, 5.0))
        ref = np.array([oracle.estimate_preference(exp, a, b, 5, nb, int(k_), weighted, (0.5, 5.0)) for k_ in its],
                       np.float32)
        assert same(got, ref)


def test_f64_csr_equals_coo_and_accumulates_in_order(oracle):
    """The DataModel layout (CSR, the order CosineCM.exportProfile iterates)
    and a second batch into the live table: each counter receives its
    increments batch after batch, as repeated update() calls do."""
    n, d, w = 300, 4, 256
    items, users, vals = _stream(n, 90_000, 5, "ratings")
    a, b = oracle.hash_params(42, d)
    exp = oracle.build_table(n, d, w, a, b, items, users, vals)
    half = items.size // 2
    with SketchTable(n, depth=d, width=w, seed=42, counters="f64") as t:
        for lo, hi in ((0, half), (half, items.size)):
            off, keys, v = to_csr(items[lo:hi], users[lo:hi], n, vals[lo:hi])
            t.ingest_csr(off, keys, v)
        t.finalize()
        assert same(t.read_counters(), exp)
        assert same(t.similarities(3, np.arange(n)), np.where(np.arange(n) == 3, oracle.cosine_cm(exp[3], exp[3]),
                                                              oracle.similarities_row(exp, 3)))


def test_f64_values_u32_cannot_hold(oracle):
    """The case the u32 mode rejects: 0.1-granular ratings need 27 fractional
    bits, so an owner's mass overflows 2^32 at 32 preference units; fp64
    counters take it as the reference does."""
    n, d, w = 50, 4, 128
    rows = np.repeat(np.arange(n), 400)
    keys = np.tile(np.arange(400), n)
    vals = np.full(rows.size, 4.1, np.float32)
    a, b = oracle.hash_params(42, d)
    with pytest.raises(CmsError):
        with SketchTable(n, depth=d, width=w, seed=42, frac_bits=27) as t:
            t.ingest(rows, keys, vals)
            t.finalize()
    exp = oracle.build_table(n, d, w, a, b, rows, keys, vals)
    with SketchTable(n, depth=d, width=w, seed=42, counters="f64") as t:
        t.ingest(rows, keys, vals)
        t.finalize()
        assert same(t.read_counters(), exp)
        assert same(t.similarities(0, np.arange(n)), np.where(np.arange(n) == 0, oracle.cosine_cm(exp[0], exp[0]),
                                                              oracle.similarities_row(exp, 0)))


def test_f64_mode_boundaries():
    import torch
    with SketchTable(10, depth=2, width=64, counters="f64") as t:
        rows = torch.tensor([0, 1], dtype=torch.int64, device="cuda")
        with pytest.raises(CmsError) as ei:
            t.ingest_device_rows(rows, rows, None, 2)
        assert ei.value.code == CMS_E_STATE
    with pytest.raises(CmsError) as ei:  # past the fp64 mode's 2^20 counters per sketch row
        SketchTable(10, depth=2, width=(1 << 20) + 1, counters="f64")
    assert ei.value.code == CMS_E_PARAM
    with pytest.raises(CmsError) as ei:  # u32 counters: LDS-staged rows up to 32768
        SketchTable(10, depth=2, width=32769)
    assert ei.value.code == CMS_E_PARAM


@pytest.mark.parametrize("kind", ["ratings", "signed"])
def test_f64_per_owner_shapes_bit_exact(oracle, kind):
    """CosineCM with its CountMinSketchConfig (per-owner shapes) on fp64
    counters: u1's sketch built at u2's shape in preference order against u2's
    own (`CosineCM.java:41-96`), point queries of own sketches, top-k."""
    from mahout_amd.synth import movielens_like
    users, items, _ = movielens_like(120, 400, 6000, seed=5, min_per_user=5)
    uid = np.unique(users)
    rows = np.searchsorted(uid, users)
    order = np.lexsort((items, rows))
    rows, items = rows[order], items[order]
    rng = np.random.Generator(np.random.PCG64(8))
    vals = (np.round(rng.uniform(0.5, 5.0, rows.size), 1) if kind == "ratings" else rng.normal(0, 2, rows.size))
    vals = vals.astype(np.float32)
    off, keys, v = to_csr(rows, items, uid.size, vals)
    a, b = oracle.hash_params(42, 32)
    with SketchTable(uid.size, seed=42, owner_ids=uid, per_owner=True, counters="f64") as t:
        t.ingest_csr(off, keys, v)
        t.configure_owner_shapes(1.0, 400)
        t.finalize()
        w, d = t.owner_shapes()[2:]
        for q in [0, 17, uid.size - 1]:
            got = t.similarities(int(uid[q]), uid)
            exp = np.array([oracle.per_owner_similarity(off, keys, v, (w, d), a, b, q, c) for c in range(uid.size)])
            assert same(got, exp), q
        for r in [0, 5]:
            own = oracle.export_profile(off, keys, v, r, int(w[r]), int(d[r]), a, b)
            assert same(t.read_owner_sketch(int(uid[r])), own)
            for key in [int(keys[off[r]]), 7, -3]:
                assert t.point_query(int(uid[r]), key) == oracle.sketch_get(own, a, b, key)
        row = np.array([oracle.per_owner_similarity(off, keys, v, (w, d), a, b, 3, c) for c in range(uid.size)])
        row[3] = np.nan
        eids, escs = oracle.top_users(uid, row, 10)
        ids, scs = t.most_similar(int(uid[3]), 10)
        assert ids.tolist() == eids.tolist() and same(scs, escs)


@pytest.mark.parametrize("per_owner", [False, True])
def test_taste_mirror_float_datamodel(oracle, per_owner):
    """taste.CosineCM over a float-rated DataModel whose preferences the u32
    counters cannot hold (0.1-granular values, owner masses past 2^32 units of
    2^-27): the mirror picks fp64 counters and matches the reference, where
    round 1 raised TasteException (CMS_E_OVERFLOW)."""
    from mahout_amd.datamodel import GenericDataModel
    from mahout_amd.synth import movielens_like
    from mahout_amd.taste import CosineCM, CountMinSketchConfig, FixedShapeConfig, HashFunctionBuilder, counter_units
    users, items, _ = movielens_like(80, 300, 5000, seed=12, min_per_user=20)
    uid = np.unique(users)
    rows = np.searchsorted(uid, users)
    order = np.lexsort((items, rows))
    rows, items = rows[order], items[order]
    vals = np.round(np.random.Generator(np.random.PCG64(12)).uniform(1.0, 5.0, rows.size), 1).astype(np.float32)
    off, keys, v = to_csr(rows, items, uid.size, vals)
    assert counter_units(off, v) == (0, "f64")
    model = GenericDataModel.from_csr(uid, off, keys, v)
    a, b = oracle.hash_params(42, 32)
    if per_owner:
        sim = CosineCM(model, CountMinSketchConfig(1.0), HashFunctionBuilder(42))
        de, ep = oracle.owner_config(off, model.getNumItems(), 1.0)
        shapes = oracle.owner_shapes(de, ep)
        pairs = [(0, 1), (1, 0), (7, 70), (3, 3)]
        for u1, u2 in pairs:
            exp = oracle.per_owner_similarity(off, keys, v, shapes, a, b, u1, u2)
            assert same(sim.userSimilarity(int(uid[u1]), int(uid[u2])), exp)
    else:
        sim = CosineCM(model, FixedShapeConfig(4, 256), HashFunctionBuilder(42))
        exp = oracle.build_table(uid.size, 4, 256, a, b, rows, items, vals)
        for u1, u2 in [(0, 1), (7, 70), (3, 3)]:
            assert same(sim.userSimilarity(int(uid[u1]), int(uid[u2])), oracle.cosine_cm(exp[u1], exp[u2]))
    assert sim.table.counters == "f64"
    sim.close()


@pytest.mark.parametrize("w", [16385, 65536])
def test_f64_wide_rows_built_in_place(oracle, w):
    """fp64 counters wider than an LDS row (DoubleCountMinSketch(width, depth,
    ...) has no width limit, `T/impl/common/DoubleCountMinSketch.java:32-36`):
    the build updates the table rows in place, each bucket by one thread in
    key order, so counters and similarities stay bit-exact."""
    n, d = 60, 2
    items, users, vals = _stream(n, 40_000, 5 + w, "ratings")
    a, b = oracle.hash_params(42, d)
    exp = oracle.build_table(n, d, w, a, b, items, users, vals)
    with SketchTable(n, depth=d, width=w, seed=42, counters="f64") as t:
        t.ingest(items, users, vals)
        t.finalize()
        assert same(t.read_counters(), exp)
        for q in (0, n - 1):
            ref = oracle.similarities_row(exp, q)
            ref[q] = oracle.cosine_cm(exp[q], exp[q])
            assert same(t.similarities(q, np.arange(n)), ref), q
        assert t.point_query(1, int(users[0])) == oracle.sketch_get(exp[1], a, b, int(users[0]))
