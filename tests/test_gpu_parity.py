"""GPU parity: libmahout_cms.so (gfx950) against the CPU restatement oracle.

Bar: bit-exact hash indices and counters; cosine/similarity values compared
bit for bit (the exact-integer + IEEE fp64 epilogue reproduces the
reference's arithmetic; the north-star tolerance of 1e-5 relative is the
ceiling, asserted separately as a floor check).
"""
import math

import numpy as np
import pytest

from mahout_amd import SketchTable
from mahout_amd._lib import CmsError, CMS_E_NO_SUCH_ID, CMS_E_VALUE, CMS_E_STATE, CMS_E_PARAM
from mahout_amd.synth import zipf_stream, to_csr

pytestmark = pytest.mark.gpu

EDGE = np.array([0, 1, -1, 2 ** 63 - 1, -2 ** 63, 9223372036854775783, 9223372036854775782, -9223372036854775783,
                 -9223372036854775784, 2 ** 62, -2 ** 62, 943, 1682], np.int64)


def same(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return a.shape == b.shape and bool(np.all((a == b) | (np.isnan(a) & np.isnan(b))))


def oracle_table(oracle, n, d, w, seed, rows, keys, vals=None):
    a, b = oracle.hash_params(seed, d)
    return oracle.build_table(n, d, w, a, b, rows, keys, vals)


@pytest.mark.parametrize("width", [1024, 4096, 8192, 1000, 39, 1])
def test_hash_keys_bit_exact(oracle, width):
    rng = np.random.Generator(np.random.PCG64(width))
    keys = np.concatenate([EDGE, rng.integers(-2 ** 63, 2 ** 63 - 1, size=100000, dtype=np.int64)])
    with SketchTable(4, depth=5, width=width, seed=42) as t:
        a, b = t.hash_params()
        oa, ob = oracle.hash_params(42, 5)
        assert a.tolist() == oa.tolist() and b.tolist() == ob.tolist()
        np.testing.assert_array_equal(t.hash_keys(keys), oracle.hash_keys(oa, ob, width, keys))


def test_ingest_small_atomic_path(oracle):
    rows = np.array([0, 1, 1, 2, 3, 3, 3, 0], np.int64)
    keys = np.array([5, -7, 5, 2 ** 62, 1, 1, 99, -2 ** 63], np.int64)
    with SketchTable(4, depth=4, width=64, seed=42) as t:
        t.ingest(rows, keys)
        t.finalize()
        assert same(t.read_counters(), oracle_table(oracle, 4, 4, 64, 42, rows, keys))


@pytest.mark.parametrize("n,d,w,npairs", [(3000, 4, 256, 400_000), (700, 5, 1024, 300_000), (50, 3, 100, 270_000)])
def test_ingest_partition_path_with_hot_rows(oracle, n, d, w, npairs):
    items, users = zipf_stream(20000, n, npairs, seed=n)
    with SketchTable(n, depth=d, width=w, seed=7) as t:
        t.ingest(items, users)
        t.finalize()
        got = t.read_counters()
    exp = oracle_table(oracle, n, d, w, 7, items, users)
    assert same(got, exp)
    assert np.bincount(items, minlength=n).max() > 32768  # a hot row was split into several slices


@pytest.mark.parametrize("shape", ["u32_max", "one_wide", "negative", "edge", "all_wide"])
def test_partition_key_width_modes(oracle, shape):
    """Keys at the u32 boundary, a single key past it, negative keys, the
    int64 edge values and a stream whose every key is wide, through the COO
    partition (and a second batch through the same partition workspace), give
    the oracle's table bit for bit.  The partition carries keys as u32 tokens:
    keys in [0, 2^31) as themselves, all others as their index in the batch
    (escapes), so every case but the plain one exercises the escape path."""
    n, d, w = 900, 5, 512
    items, users = zipf_stream(30000, n, 400_000, seed=17)
    keys = users.astype(np.int64).copy()
    if shape == "u32_max":
        keys[::7] = 2 ** 32 - 1 - keys[::7]  # still narrow, top of the u32 range
    elif shape == "one_wide":
        keys[len(keys) // 2] = 2 ** 32  # a single key needs the 8-byte path
    elif shape == "negative":
        keys[-1] = -1
    elif shape == "all_wide":
        keys = keys * 977 + 2 ** 40
    else:
        keys[: len(EDGE)] = EDGE
    with SketchTable(n, depth=d, width=w, seed=7) as t:
        t.ingest(items, keys)
        t.finalize()
        got = t.read_counters()
        assert same(got, oracle_table(oracle, n, d, w, 7, items, keys))
        # a second batch through the same partition workspace (live-table path)
        t.ingest(items, users)
        t.finalize()
        got2 = t.read_counters()
    both_i = np.concatenate([items, items])
    both_k = np.concatenate([keys, users.astype(np.int64)])
    assert same(got2, oracle_table(oracle, n, d, w, 7, both_i, both_k))


@pytest.mark.parametrize("n,npairs,vals", [(20000, 3_000_000, False), (20000, 1_500_000, True), (1_000_000, 2_000_000, False)])
def test_partition_hot_routing_equals_two_pass(oracle, n, npairs, vals, monkeypatch):
    """Bulk COO builds route the sampled hottest owners straight to their
    final place in pass 1 (partition_to_spans); the table equals the plain
    two-pass partition's and the oracle's bit for bit, with and without
    preference values, and at 1M owners (pass-1 fan-out 977 coarse + 1024 hot
    bins)."""
    d, w = 3, 256
    items, users = zipf_stream(200_000, n, npairs, seed=n + npairs)
    v = None
    if vals:
        v = np.random.Generator(np.random.PCG64(2)).integers(1, 6, size=items.size).astype(np.float32)
    import torch
    cnt = np.bincount(items, minlength=n)
    # the 16 hottest owners and 2000 random ones are checked against the oracle
    sel = np.unique(np.concatenate([np.argsort(-cnt, kind="stable")[:16],
                                    np.random.Generator(np.random.PCG64(4)).integers(0, n, 2000)]))
    got = {}
    for mode in ("hot", "two_pass"):
        if mode == "two_pass":
            monkeypatch.setenv("CMS_NO_HOT_ROUTING", "1")
        with SketchTable(n, depth=d, width=w, seed=11) as t:
            t.ingest(items, users, v)
            t.finalize()
            got[mode] = t.read_counters_device().cpu()
            torch.cuda.synchronize()
    assert torch.equal(got["hot"], got["two_pass"])
    remap = np.full(n, -1, np.int64)
    remap[sel] = np.arange(sel.size)
    m = remap[items] >= 0
    exp = oracle_table(oracle, sel.size, d, w, 11, remap[items[m]], users[m], None if v is None else v[m])
    assert same(got["hot"].numpy()[sel].astype(np.float64), exp)


def test_reserved_hot_slots_then_late_promotion(oracle):
    """A fresh build reserves hot slots for every owner its bound allows (here
    all of a tiny universe) and claims them on the device; a later batch that
    lifts a still-narrow row past 2^16 promotes it into a slot beyond the
    reservation.  Counters stay exact."""
    n, d, w = 8, 2, 64
    rng = np.random.Generator(np.random.PCG64(5))
    rows1 = np.concatenate([np.zeros(200_000, np.int64), rng.integers(1, 8, 100_000).astype(np.int64)])
    keys1 = rng.integers(0, 1000, rows1.size).astype(np.int64)
    rows2 = np.full(300_000, 7, np.int64)
    keys2 = rng.integers(0, 1000, rows2.size).astype(np.int64)
    with SketchTable(n, depth=d, width=w, seed=42) as t:
        t.ingest(rows1, keys1)
        t.finalize()
        assert same(t.read_counters(), oracle_table(oracle, n, d, w, 42, rows1, keys1))
        t.ingest(rows2, keys2)
        t.finalize()
        got = t.read_counters()
        assert t.stats()["table_bytes"] > 2 * n * d * w  # rows 0 and 7 hold u32 slots
    assert same(got, oracle_table(oracle, n, d, w, 42, np.concatenate([rows1, rows2]), np.concatenate([keys1, keys2])))


def test_ingest_csr_matches_coo(oracle):
    n, d, w = 2000, 5, 512
    items, users = zipf_stream(50000, n, 500_000, seed=3)
    off, keys, _ = to_csr(items, users, n)
    with SketchTable(n, depth=d, width=w, seed=42) as t:
        t.ingest_csr(off, keys)
        t.finalize()
        got = t.read_counters()
    assert same(got, oracle_table(oracle, n, d, w, 42, items, users))


def test_integer_values_and_bad_value(oracle):
    n = 300
    items, users = zipf_stream(5000, n, 300_000, seed=9)
    vals = np.random.Generator(np.random.PCG64(1)).integers(1, 6, size=items.size).astype(np.float32)
    with SketchTable(n, depth=4, width=1024, seed=42) as t:
        t.ingest(items, users, vals)
        t.finalize()
        assert same(t.read_counters(), oracle_table(oracle, n, 4, 1024, 42, items, users, vals))
    with SketchTable(n, depth=4, width=1024, seed=42) as t:
        bad = vals.copy()
        bad[12345] = 0.5
        with pytest.raises(CmsError) as ei:
            t.ingest(items, users, bad)
        assert ei.value.code == CMS_E_VALUE


@pytest.mark.parametrize("path", ["coo", "csr"])
def test_fractional_preferences_scaled_counters(oracle, path):
    """Half-star ratings (frac_bits 1) through both build paths and the atomic
    path: counters read back in preference units, similarities, point queries
    and estimates bit-exact against the oracle's plain fp64 accumulation."""
    n, d, w = 400, 4, 512
    items, users = zipf_stream(6000, n, 200_000, seed=21)
    vals = (np.random.Generator(np.random.PCG64(2)).integers(1, 11, size=items.size) / 2.0).astype(np.float32)
    exp = oracle_table(oracle, n, d, w, 42, items, users, vals)
    with SketchTable(n, depth=d, width=w, seed=42, frac_bits=1) as t:
        if path == "coo":
            t.ingest(items, users, vals)
        else:
            off, keys, v2 = to_csr(items, users, n, vals)
            t.ingest_csr(off, keys, v2)
        t.ingest(items[:1000], users[:1000], vals[:1000])  # small batch: the atomic path on a live table
        t.finalize()
        exp = oracle_table(oracle, n, d, w, 42, np.concatenate([items, items[:1000]]),
                           np.concatenate([users, users[:1000]]), np.concatenate([vals, vals[:1000]]))
        assert same(t.read_counters(), exp)
        for q in [0, 7, 123]:
            ref = _oracle_row_sims(oracle, exp, q)
            ref[q] = oracle.cosine_cm(exp[q], exp[q])
            assert same(t.similarities(q, np.arange(n)), ref)
        a, b = oracle.hash_params(42, d)
        for key in [int(users[0]), 5, -9]:
            assert t.point_query(3, key) == oracle.sketch_get(exp[3], a, b, key)
        nb, its = [5, 9, 3, 77], users[:40]
        got = t.estimate_preferences(3, nb, its)
        ref = np.array([oracle.estimate_preference(exp, a, b, 3, nb, int(k)) for k in its], np.float32)
        assert same(got, ref)
    with SketchTable(n, depth=d, width=w, seed=42, frac_bits=1) as t:
        bad = vals.copy()
        bad[77] = 0.25
        with pytest.raises(CmsError) as ei:
            t.ingest(items, users, bad)
        assert ei.value.code == CMS_E_VALUE


def test_float_preferences_like_tastetestcase(oracle):
    """Arbitrary float preferences (0.1 .. 0.8, TasteTestCase's values): the
    smallest exact scale frac_bits_for picks, similarities bit-exact."""
    from mahout_amd.sketch import frac_bits_for
    n, d, w = 50, 3, 64
    rng = np.random.Generator(np.random.PCG64(4))
    items = rng.integers(0, n, 600).astype(np.int64)
    users = rng.integers(0, 40, 600).astype(np.int64)
    vals = rng.choice(np.array([0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8], np.float32), 600)
    fb = frac_bits_for(vals)
    assert fb > 20
    exp = oracle_table(oracle, n, d, w, 42, items, users, vals)
    with SketchTable(n, depth=d, width=w, seed=42, frac_bits=fb) as t:
        t.ingest(items, users, vals)
        t.finalize()
        assert same(t.read_counters(), exp)
        for q in range(0, n, 7):
            ref = _oracle_row_sims(oracle, exp, q)
            ref[q] = oracle.cosine_cm(exp[q], exp[q])
            assert same(t.similarities(q, np.arange(n)), ref)


@pytest.mark.parametrize("frac_bits", [0, 2])
def test_narrow_and_hot_rows_at_the_u16_boundary(oracle, frac_bits):
    """Rows whose mass stays below 2^16 are stored as u16, the others in u32
    slots.  Row 0 ends the bulk build at counter 65535 (narrow), row 1 at
    65540 (hot); small batches then push row 0 to 2^16 (promotion on the atomic
    path), keep row 2 narrow, and a big accumulate batch promotes row 3."""
    n, d, w = 6, 2, 64
    sc = 2.0 ** -frac_bits
    rows = np.concatenate([np.zeros(13107, np.int64), np.ones(13108, np.int64), np.full(500, 2, np.int64),
                           np.full(5000, 3, np.int64)])
    keys = np.concatenate([np.full(13107, 7, np.int64), np.full(13108, 9, np.int64), np.arange(500, dtype=np.int64),
                           np.arange(5000, dtype=np.int64) % 50])
    vals = np.concatenate([np.full(13107, 5, np.float32), np.full(13108, 5, np.float32), np.ones(500, np.float32),
                           np.ones(5000, np.float32)]) * np.float32(sc)
    batches = [(rows, keys, vals)]
    with SketchTable(n, depth=d, width=w, seed=42, frac_bits=frac_bits) as t:
        off, ck, cv = to_csr(rows, keys, n, vals)
        t.ingest_csr(off, ck, cv)  # the LDS row build (bulk path)
        t.finalize()
        assert same(t.read_counters(), oracle_table(oracle, n, d, w, 42, rows, keys, vals))
        assert t.stats()["table_bytes"] < n * d * w * 4  # mostly narrow
        b2 = (np.array([0, 2, 2], np.int64), np.array([7, 1, 2], np.int64), np.full(3, sc, np.float32))
        t.ingest(*b2)  # atomic path: row 0 reaches 65536 in counter units
        batches.append(b2)
        big_r = np.concatenate([np.full(300_000, 3, np.int64), np.full(1000, 5, np.int64)])
        big_k = np.concatenate([np.arange(300_000, dtype=np.int64) % 97, np.arange(1000, dtype=np.int64)])
        big_v = np.full(big_r.size, sc, np.float32)
        t.ingest(big_r, big_k, big_v)  # accumulate build (or sorted atomics): row 3 becomes hot
        batches.append((big_r, big_k, big_v))
        t.finalize()
        exp = oracle_table(oracle, n, d, w, 42, np.concatenate([b[0] for b in batches]),
                           np.concatenate([b[1] for b in batches]), np.concatenate([b[2] for b in batches]))
        assert same(t.read_counters(), exp)
        assert exp[0].max() == 65536 * sc and exp[1].max() == 65540 * sc
        for q in range(n):
            ref = _oracle_row_sims(oracle, exp, q)
            ref[q] = oracle.cosine_cm(exp[q], exp[q])
            assert same(t.similarities(q, np.arange(n)), ref)
        a, b = oracle.hash_params(42, d)
        for r in range(n):
            assert t.point_query(r, 7) == oracle.sketch_get(exp[r], a, b, 7)


def test_owner_ids_and_errors(oracle):
    ids = np.array([-50, 3, 10, 11, 1000], np.int64)
    with SketchTable(5, depth=4, width=128, seed=42, owner_ids=ids) as t:
        with pytest.raises(CmsError) as ei:
            t.similarity(3, 10)
        assert ei.value.code == CMS_E_STATE
        t.ingest(np.array([3, 3, 1000, -50, 10], np.int64), np.array([1, 2, 1, 1, 2], np.int64))
        t.finalize()
        with pytest.raises(CmsError) as ei:
            t.similarity(3, 4)
        assert ei.value.code == CMS_E_NO_SUCH_ID
        with pytest.raises(CmsError) as ei:
            t.ingest(np.array([7], np.int64), np.array([1], np.int64))
        assert ei.value.code == CMS_E_NO_SUCH_ID
        # owner 11 never ingested: zero sketch -> every row denominator 0 -> NaN
        assert math.isnan(t.similarity(3, 11))
        assert abs(t.similarity(3, 3) - 1.0) < 1e-15


@pytest.mark.parametrize("weighted", [False, True])
def test_accumulate_equals_single_batch(oracle, weighted):
    """Split (hot) rows' slices add into their slot rows with global atomics:
    unit streams through k_build_slices (all d sketch rows of a 65535-key
    slice in one u16 LDS image, one key pass), valued streams through
    k_build_rows' slices (a key pass per pair of sketch rows); both
    bit-exact, fresh and accumulating."""
    n, d, w = 1500, 4, 512
    items, users = zipf_stream(30000, n, 800_000, seed=21)
    vals = np.random.Generator(np.random.PCG64(21)).integers(1, 4, items.size).astype(np.float32) if weighted else None
    part = (lambda lo, hi: None) if vals is None else (lambda lo, hi: vals[lo:hi])
    with SketchTable(n, depth=d, width=w, seed=42) as t:
        t.ingest(items[:400_000], users[:400_000], part(0, 400_000))  # partition build into an empty table
        t.ingest(items[400_000:700_000], users[400_000:700_000], part(400_000, 700_000))  # accumulate build
        t.ingest(items[700_000:], users[700_000:], part(700_000, items.size))  # atomic path (small batch)
        t.finalize()
        got = t.read_counters()
        exp = oracle_table(oracle, n, d, w, 42, items, users, vals)
        assert same(got, exp)
        # the hottest owners were split into slices in both builds (their slot
        # rows summed from the slices, old counters included the second time):
        # their norms show in every similarity of their rows
        cnt = np.bincount(items[:400_000], minlength=n)
        assert cnt.max() > 2 * 8192
        for q in np.argsort(cnt)[-3:]:
            e = oracle.similarities_row(exp, int(q))
            e[q] = oracle.cosine_cm(exp[q], exp[q])
            assert same(t.similarities(int(q), np.arange(n)), e), q


def _oracle_row_sims(oracle, table, q, weighted=False):
    return oracle.similarities_row(table, q, weighted)


@pytest.mark.parametrize("weighted", [False, True])
def test_similarities_bit_exact(oracle, weighted):
    n, d, w = 400, 5, 1024
    items, users = zipf_stream(8000, n, 300_000, seed=5)
    vals = np.random.Generator(np.random.PCG64(2)).integers(1, 6, size=items.size).astype(np.float32)
    ot = oracle_table(oracle, n, d, w, 42, items, users, vals)
    with SketchTable(n, depth=d, width=w, seed=42, weighted=weighted) as t:
        t.ingest(items, users, vals)
        t.finalize()
        assert t.stats()["exact_norms"] == 1
        for q in [0, 1, 17, 399]:
            got = t.similarities(q, np.arange(n))
            exp = _oracle_row_sims(oracle, ot, q, weighted)
            exp[q] = oracle.cosine_cm(ot[q], ot[q], weighted)
            assert same(got, exp), q
            assert t.similarity(q, (q + 1) % n) == exp[(q + 1) % n] or (
                math.isnan(exp[(q + 1) % n]) and math.isnan(t.similarity(q, (q + 1) % n)))


def test_inexact_norm_regime_matches_sequential_reference(oracle):
    """Counters large enough that sum(c^2) >= 2^53: the reference's fp64 sums
    round; the GPU switches to the reference's sequential order."""
    n, d, w = 6, 3, 64
    rng = np.random.Generator(np.random.PCG64(4))
    rows = np.repeat(np.arange(n), 40)
    keys = rng.integers(0, 1000, size=rows.size).astype(np.int64)
    vals = rng.integers(2 ** 22, 2 ** 24, size=rows.size).astype(np.float32)
    ot = oracle_table(oracle, n, d, w, 42, rows, keys, vals)
    with SketchTable(n, depth=d, width=w, seed=42) as t:
        t.ingest(rows, keys, vals)
        t.finalize()
        assert t.stats()["exact_norms"] == 0
        assert same(t.read_counters(), ot)
        for q in range(n):
            exp = _oracle_row_sims(oracle, ot, q)
            exp[q] = oracle.cosine_cm(ot[q], ot[q])
            assert same(t.similarities(q, np.arange(n)), exp)


def _collision_free_seed(oracle, keys, depth, width):
    for seed in range(1, 10000):
        a, b = oracle.hash_params(seed, depth)
        h = oracle.hash_keys(a, b, width, np.array(keys, np.int64))
        if all(len(set(h[:, r].tolist())) == len(keys) for r in range(depth)):
            return seed
    raise AssertionError


def test_reference_kats_on_gpu(oracle):
    """VectorSimilarityMeasuresTest (0.769846046 +- 1e-6) and ItemSimilarityJobTest
    (0.45, 0.89 +- 0.01) through collision-free sketches on the GPU."""
    va = [0, 2, 0, 0, 8, 3, 0, 6, 0, 1, 2, 2, 0]
    vb = [3, 0, 0, 0, 7, 0, 2, 2, 1, 3, 2, 1, 1]
    seed = _collision_free_seed(oracle, list(range(13)), 4, 1024)
    with SketchTable(2, depth=4, width=1024, seed=seed) as t:
        t.ingest(np.array([0] * 13 + [1] * 13), np.array(list(range(13)) * 2), np.array(va + vb, np.float32))
        t.finalize()
        assert abs(t.similarity(0, 1) - 0.769846046) < 1e-6
    lines = ["2,1,1", "1,2,1", "3,4,1", "1,3,2", "2,3,1"]
    users, items, prefs = zip(*[map(int, ln.split(",")) for ln in lines])
    seed = _collision_free_seed(oracle, sorted(set(users)), 4, 1024)
    with SketchTable(4, depth=4, width=1024, seed=seed, owner_ids=[1, 2, 3, 4]) as t:
        t.ingest(np.array(items), np.array(users), np.array(prefs, np.float32))
        t.finalize()
        assert abs(t.similarity(1, 3) - 0.45) < 0.01
        assert abs(t.similarity(2, 3) - 0.89) < 0.01
        assert t.similarity(1, 3) == 1 / math.sqrt(5) or abs(t.similarity(1, 3) - 1 / math.sqrt(5)) < 1e-16


def test_point_query(oracle):
    n, d, w = 200, 4, 256
    items, users = zipf_stream(3000, n, 50_000, seed=8)
    ot = oracle_table(oracle, n, d, w, 42, items, users)
    a, b = oracle.hash_params(42, d)
    with SketchTable(n, depth=d, width=w, seed=42) as t:
        t.ingest(items, users)
        t.finalize()
        for owner in [0, 5, 199]:
            for key in [0, 1, int(users[0]), 2999, -4]:
                assert t.point_query(owner, key) == oracle.sketch_get(ot[owner], a, b, key)


def test_most_similar_top_users_semantics(oracle):
    n, d, w = 600, 4, 128
    items, users = zipf_stream(400, n, 60_000, seed=13)  # few users -> many ties / duplicates
    ids = np.arange(n, dtype=np.int64) * 7 + 3
    ot = oracle_table(oracle, n, d, w, 42, items, users)
    with SketchTable(n, depth=d, width=w, seed=42, owner_ids=ids) as t:
        t.ingest(ids[items], users)
        t.finalize()
        for q in [0, 1, 300, 599]:
            for k in [1, 10, 100]:
                sims = _oracle_row_sims(oracle, ot, q)
                eids, esc = oracle.top_users(ids, sims, k)
                gids, gsc = t.most_similar(int(ids[q]), k)
                assert gids.tolist() == eids.tolist(), (q, k)
                assert same(gsc, esc)
        rows, sc, cnt = t.top_k_rows(0, 8, 20)
        for q in range(8):
            eids, _ = oracle.top_users(ids, _oracle_row_sims(oracle, ot, q), 20)
            assert rows[q, :cnt[q]].tolist() == eids.tolist()


def test_movielens_shape_config1(oracle):
    """Config 1 shape: ML-100K stand-in, transposed (item sketches keyed by user),
    d=4, w=1024, integer ratings; all pairs of 64 items + top-10 for 5 items."""
    from mahout_amd.synth import movielens_like
    users, items, ratings = movielens_like()
    item_ids = np.unique(items)
    rows = np.searchsorted(item_ids, items)
    ot = oracle_table(oracle, item_ids.size, 4, 1024, 42, rows, users, ratings)
    with SketchTable(item_ids.size, depth=4, width=1024, seed=42, owner_ids=item_ids) as t:
        t.ingest(items, users, ratings)
        t.finalize()
        assert same(t.read_counters(), ot)
        for q in range(0, 64):
            exp = _oracle_row_sims(oracle, ot, q)
            exp[q] = oracle.cosine_cm(ot[q], ot[q])
            assert same(t.similarities(int(item_ids[q]), item_ids), exp)
        for q in [0, 10, 500, 1000, item_ids.size - 1]:
            eids, _ = oracle.top_users(item_ids, _oracle_row_sims(oracle, ot, q), 10)
            assert t.most_similar(int(item_ids[q]), 10)[0].tolist() == eids.tolist()


def test_device_ingest_orders_against_a_side_stream(oracle):
    """Inputs produced on a non-default torch stream and freed right after the
    (asynchronous) device ingest: event ordering both ways, table exact."""
    import torch
    n, d, w = 300, 4, 256
    items, users = zipf_stream(5000, n, 400_000, seed=41)
    side = torch.cuda.Stream()
    with SketchTable(n, depth=d, width=w, seed=42) as t:
        with torch.cuda.stream(side):
            r = torch.from_numpy(items).to("cuda", non_blocking=True)
            k = torch.from_numpy(users).to("cuda", non_blocking=True)
            r2 = (r * 3 - 2 * r).contiguous()  # produced on the side stream
            k2 = (k + 7 - 7).contiguous()
            t.ingest_device_rows(r2, k2, None, int(r2.numel()))
            del r2, k2
            junk = torch.full((items.size * 4,), -1, dtype=torch.int64, device="cuda")  # may reuse the freed blocks
            del junk
        t.finalize()
        assert same(t.read_counters(), oracle_table(oracle, n, d, w, 42, items, users))


def test_bad_row_index_device_path():
    import torch
    with SketchTable(10, depth=2, width=64) as t:
        rows = torch.tensor([0, 1, 10], dtype=torch.int64, device="cuda")
        keys = torch.tensor([1, 2, 3], dtype=torch.int64, device="cuda")
        # device ingest is asynchronous (stream-ordered against torch's
        # stream, no host wait), so the bad row surfaces from the next
        # synchronising call
        t.ingest_device_rows(rows, keys, None, 3)
        with pytest.raises(CmsError) as ei:
            t.finalize()
        assert ei.value.code == CMS_E_PARAM


@pytest.mark.parametrize("n,d,w,vmax,seed", [(700, 5, 256, 5, 31), (260, 4, 128, 50, 32), (129, 3, 512, 1, 33), (3000, 5, 256, 1, 34),
     (1500, 8, 128, 3, 35), (600, 25, 128, 2, 36),
     (3000, 5, 8192, 3, 37)])  # the config-3/4 shape: d=5, w=8192 (K = 40960), counters <= 4 and > 127
def test_all_pairs_mfma_every_similarity(oracle, n, d, w, vmax, seed):
    """cms_top_k_rows with k = n-1 returns every other owner sorted by
    (similarity desc, ID asc): the whole similarity matrix through the
    int8-limb MFMA kernels (single- and multi-limb tiles), bit for bit."""
    items, users = zipf_stream(3000, n, 300_000, seed=seed)
    vals = np.random.Generator(np.random.PCG64(seed)).integers(1, vmax + 1, size=items.size).astype(np.float32)
    ot = oracle_table(oracle, n, d, w, 42, items, users, vals)
    with SketchTable(n, depth=d, width=w, seed=42) as t:
        t.ingest(items, users, vals)
        t.finalize()
        k = min(n - 1, 1024)
        rows = list(range(0, n, max(1, n // 37))) + [n - 1]
        ids, sc, cnt = t.top_k_rows(5, n - 5, k)  # unaligned query start
        for q in rows:
            if q < 5:
                continue
            sims = _oracle_row_sims(oracle, ot, q)
            eids, esc = oracle.top_users(np.arange(n), sims, k)
            got_ids = ids[q - 5, :cnt[q - 5]]
            assert got_ids.tolist() == eids.tolist(), q
            assert same(sc[q - 5, :cnt[q - 5]], esc), q
    if vmax > 1:
        assert ot.max() > 127  # multi-limb owners were exercised


@pytest.mark.parametrize("k", [1, 10, 100])
def test_top_k_small_k_sampled_threshold(oracle, k):
    """k << n: the one-pass sampled-threshold top-k against TopItems.getTopUsers."""
    n, d, w = 3000, 4, 256
    items, users = zipf_stream(5000, n, 400_000, seed=40 + k)
    ot = oracle_table(oracle, n, d, w, 42, items, users)
    with SketchTable(n, depth=d, width=w, seed=42) as t:
        t.ingest(items, users)
        t.finalize()
        ids, sc, cnt = t.top_k_rows(0, n, k)
        for q in list(range(0, n, 97)) + [n - 1]:
            sims = _oracle_row_sims(oracle, ot, q)
            eids, esc = oracle.top_users(np.arange(n), sims, k)
            assert ids[q, :cnt[q]].tolist() == eids.tolist(), q
            assert same(sc[q, :cnt[q]], esc), q


def test_top_k_heavy_ties(oracle):
    """Many owners with identical sketches: long runs of equal scores, broken
    by owner ID (SimilarUser.compareTo)."""
    n, d, w = 1500, 3, 128
    rng = np.random.Generator(np.random.PCG64(77))
    # owners in groups of 50 share one user profile
    rows, keys = [], []
    for o in range(n):
        g = o // 50
        prof = np.random.Generator(np.random.PCG64(g)).integers(0, 400, size=6)
        rows.append(np.full(prof.size, o))
        keys.append(prof)
    rows = np.concatenate(rows).astype(np.int64)
    keys = np.concatenate(keys).astype(np.int64)
    perm = rng.permutation(rows.size)
    rows, keys = rows[perm], keys[perm]
    ot = oracle_table(oracle, n, d, w, 42, rows, keys)
    with SketchTable(n, depth=d, width=w, seed=42) as t:
        t.ingest(rows, keys)
        t.finalize()
        for k in (5, 60, 300):
            ids, sc, cnt = t.top_k_rows(0, n, k)
            for q in range(0, n, 71):
                sims = _oracle_row_sims(oracle, ot, q)
                eids, esc = oracle.top_users(np.arange(n), sims, k)
                assert ids[q, :cnt[q]].tolist() == eids.tolist(), (k, q)
                assert same(sc[q, :cnt[q]], esc), (k, q)


@pytest.mark.parametrize("n,d,w,vmax,k,weighted,seed", [
    (3000, 5, 256, 3, 10, False, 51),     # multi-limb owners, partial last block
    (2000, 4, 128, 50, 100, False, 52),   # most owners multi-limb: several S x M passes
    (1800, 3, 256, 1, 64, True, 53),      # weighted: every score is +-1, ties by ID everywhere
    (700, 5, 512, 2, 5, False, 54),       # fewer than one 256-row block pair per wave
    (11776, 3, 128, 2, 20, False, 55),    # 46 blocks: multi-wave bands and the half wave
    (12000, 4, 256, 2, 25, False, 56),    # fp4 blocks beside int8 blocks over multi-wave bands
    (5000, 2, 512, 1, 200, False, 57),    # mostly fp4 owners, long lists
    (3000, 5, 8192, 3, 100, False, 58),   # the config-4 shape (d=5, w=8192): fp4, int8 and multi-limb owners
])
def test_top_k_all_streaming_symmetric(oracle, n, d, w, vmax, k, weighted, seed):
    """cms_top_k_all (each unordered pair computed once, streamed into both
    owners' lists) equals the per-row slab path for EVERY owner and the
    oracle's TopItems restatement on a sample of rows, bit for bit."""
    items, users = zipf_stream(4000, n, 400_000, seed=seed)
    vals = np.random.Generator(np.random.PCG64(seed)).integers(1, vmax + 1, size=items.size).astype(np.float32)
    ot = oracle_table(oracle, n, d, w, 42, items, users, vals)
    with SketchTable(n, depth=d, width=w, seed=42, weighted=weighted) as t:
        t.ingest(items, users, vals)
        t.finalize()
        ids, sc, cnt = t.top_k_all(k)
        assert t.stats()["topk_redo"] == 0  # no candidate list overflowed
        rids, rsc, rcnt = t.top_k_rows(0, n, k)
        assert np.array_equal(cnt, rcnt)
        for q in range(n):
            assert ids[q, :cnt[q]].tolist() == rids[q, :rcnt[q]].tolist(), q
            assert same(sc[q, :cnt[q]], rsc[q, :rcnt[q]]), q
        for q in list(range(0, n, max(1, n // 29))) + [n - 1]:
            sims = _oracle_row_sims(oracle, ot, q, weighted)
            eids, esc = oracle.top_users(np.arange(n), sims, k)
            assert ids[q, :cnt[q]].tolist() == eids.tolist(), q
            assert same(sc[q, :cnt[q]], esc), q
        if vmax > 1:
            assert t.stats()["multi_limb_owners"] > 0
        if w % 256 == 0:
            assert t.stats()["fp4_owners"] > 0


@pytest.mark.parametrize("weighted,capper", [(False, None), (False, (1.0, 4.5)), (True, (1.0, 5.0))])
def test_estimate_preferences_point_query_path(oracle, weighted, capper):
    """GenericUserBasedRecommender.doEstimatePreference with the CosineCM
    point query, every item of the universe, bit-exact float estimates."""
    n_users, n_items, d, w = 300, 2000, 4, 512
    # owners are users, keys are items (the non-transposed orientation)
    users, items = zipf_stream(n_items, n_users, 60_000, seed=61)
    vals = np.random.Generator(np.random.PCG64(61)).integers(1, 6, size=items.size).astype(np.float32)
    ot = oracle_table(oracle, n_users, d, w, 42, users, items, vals)
    a, b = oracle.hash_params(42, d)
    with SketchTable(n_users, depth=d, width=w, seed=42, weighted=weighted) as t:
        t.ingest(users, items, vals)
        t.finalize()
        all_items = np.arange(n_items, dtype=np.int64)
        for u in [0, 5, 77, 299]:
            nb, _ = t.most_similar(u, 12)
            nb = np.concatenate([nb, [u]])  # the user's own ID is skipped, as in the reference
            got = t.estimate_preferences(u, nb, all_items, capper)
            exp = np.array([oracle.estimate_preference(ot, a, b, u, nb, it, weighted, capper) for it in all_items],
                           np.float32)
            assert same(got, exp), u
            assert np.isfinite(got).sum() > 0


def test_write_similar_items_csv(oracle, tmp_path):
    """FileSimilarItemsWriter lines for every owner: ascending owner ID, each
    list most similar first, float-narrowed values in Java Double.toString."""
    from mahout_amd.sketch import java_double_to_string
    n, d, w, k = 400, 4, 256, 7
    items, users = zipf_stream(3000, n, 80_000, seed=71)
    ids_universe = np.arange(n, dtype=np.int64) * 3 + 1000
    with SketchTable(n, depth=d, width=w, seed=42, owner_ids=ids_universe) as t:
        t.ingest(ids_universe[items], users)
        t.finalize()
        path = tmp_path / "similar.csv"
        t.write_similar_items(str(path), k)
    lines = path.read_text().splitlines()
    # expected text from the oracle's TopItems lists, not the GPU's own
    ot = oracle_table(oracle, n, d, w, 42, items, users)
    exp = []
    for r in range(n):
        eids, esc = oracle.top_users(np.arange(n), _oracle_row_sims(oracle, ot, r), k)
        for e, v in zip(eids.tolist(), esc.tolist()):
            exp.append(f"{ids_universe[r]},{ids_universe[e]},{java_double_to_string(float(np.float32(v)))}")
    assert lines == exp


def test_write_similarities_other_driver_formats(oracle, tmp_path):
    """ItemSimilarityJob's text result and spark-itemsimilarity's
    TextDelimitedIndexedDatasetWriter lines, from the same all-pairs lists."""
    from mahout_amd.sketch import java_double_to_string as jd
    n, d, w, k = 300, 4, 256, 6
    items, users = zipf_stream(2000, n, 40_000, seed=73)
    ids_universe = np.arange(n, dtype=np.int64) * 7 - 500  # negative IDs included
    with SketchTable(n, depth=d, width=w, seed=42, owner_ids=ids_universe) as t:
        t.ingest(ids_universe[items], users)
        t.finalize()
        p1, p2 = tmp_path / "isj.txt", tmp_path / "spark.tsv"
        t.write_similarities(str(p1), k, "item_similarity_job")
        t.write_similarities(str(p2), k, "spark_itemsimilarity")
    # expected text from the oracle's TopItems lists, not the GPU's own
    ot = oracle_table(oracle, n, d, w, 42, items, users)
    lists = [oracle.top_users(np.arange(n), _oracle_row_sims(oracle, ot, r), k) for r in range(n)]
    pairs = {}
    for r, (eids, esc) in enumerate(lists):
        for e, v in zip(eids.tolist(), esc.tolist()):
            a, b = sorted((int(ids_universe[r]), int(ids_universe[e])))
            pairs.setdefault((a, b), float(v))  # lower ID's list first (rows ascend with IDs)
    exp1 = [f"{a}\t{b}\t{jd(v)}" for (a, b), v in sorted(pairs.items())]
    assert p1.read_text().splitlines() == exp1
    exp2 = []
    for r, (eids, esc) in enumerate(lists):
        el = [f"{ids_universe[e]}:{jd(float(v))}" for e, v in zip(eids.tolist(), esc.tolist()) if v != 0.0]
        exp2.append(f"{ids_universe[r]}\t" + " ".join(el) if el else f"{ids_universe[r]}")
    assert p2.read_text().splitlines() == exp2


@pytest.mark.parametrize("nshards", [2, 3, 8])
def test_top_k_all_shards_merge_exact(oracle, nshards):
    """The multi-GPU decomposition on one GPU: every shard's partial lists
    (pairs split by M rows, S x M chunks and waves), merged, equal the
    single-shard result for every owner."""
    n, d, w, k = 2500, 4, 256, 40
    items, users = zipf_stream(4000, n, 400_000, seed=81)
    vals = np.random.Generator(np.random.PCG64(81)).integers(1, 4, size=items.size).astype(np.float32)
    with SketchTable(n, depth=d, width=w, seed=42) as t:
        t.ingest(items, users, vals)
        t.finalize()
        ids, sc, cnt = t.top_k_all(k)
        parts = [t.top_k_all_partial(k, s, nshards) for s in range(nshards)]
        # each pair in exactly one shard: partial counts never exceed the final lists' candidates
        mi, ms, mc = t.top_k_merge(k, parts)
        assert np.array_equal(mc, cnt)
        for q in range(n):
            assert mi[q, :mc[q]].tolist() == ids[q, :cnt[q]].tolist(), q
            assert same(ms[q, :mc[q]], sc[q, :cnt[q]]), q
        assert t.stats()["multi_limb_owners"] > 0


def test_streaming_refresh_incremental_norms(oracle):
    """Config-5 pattern: a bulk-built table, then small batches through the
    atomic paths (which keep norms and row maxima current incrementally), then a
    refresh.  Counters, pair similarities and all-pairs top-k equal the oracle
    on the whole stream and a table built from it in one batch."""
    n, d, w, k = 2500, 4, 256, 30
    items, users = zipf_stream(4000, n, 600_000, seed=91)
    vals = np.random.Generator(np.random.PCG64(91)).integers(1, 4, size=items.size).astype(np.float32)
    ot = oracle_table(oracle, n, d, w, 42, items, users, vals)
    with SketchTable(n, depth=d, width=w, seed=42) as ref:
        ref.ingest(items, users, vals)
        ref.finalize()
        rids, rsc, rcnt = ref.top_k_all(k)
    with SketchTable(n, depth=d, width=w, seed=42) as t:
        t.ingest(items[:400_000], users[:400_000], vals[:400_000])
        t.finalize()
        t.top_k_all(k)
        # 3 batches through the owner-grouped path (>= 32768 pairs), 5 through plain atomics
        cuts = [400_000, 450_000, 500_000, 550_000] + list(range(560_000, 600_001, 10_000))
        for lo, hi in zip(cuts[:-1], cuts[1:]):
            t.ingest(items[lo:hi], users[lo:hi], vals[lo:hi])
        t.finalize()
        assert same(t.read_counters(), ot)
        for q in [0, 3, 999, n - 1]:
            exp = _oracle_row_sims(oracle, ot, q)
            exp[q] = oracle.cosine_cm(ot[q], ot[q])
            assert same(t.similarities(q, np.arange(n)), exp), q
        ids, sc, cnt = t.top_k_all(k)
        assert np.array_equal(cnt, rcnt)
        for q in range(n):
            assert ids[q, :cnt[q]].tolist() == rids[q, :rcnt[q]].tolist(), q
            assert same(sc[q, :cnt[q]], rsc[q, :rcnt[q]]), q
        assert t.stats()["multi_limb_owners"] > 0


def test_multi_limb_slab_kernel_equals_reference_path(oracle):
    """The multi-limb x single-limb slab block on k_cosine_mls (256 x 192
    tiles, 2- and 4-limb owners) gives the same all-pairs lists as the
    k_cosine_big path (CMS_NO_MLS=1), and the hottest owners' lists equal the
    oracle's TopItems restatement (DoubleCountMinSketch.cosine over the
    sketches, TopItems.getTopUsers)."""
    import os
    n, d, w, k = 3000, 5, 512, 50
    items, users = zipf_stream(5000, n, 500_000, seed=17)
    vals = np.random.Generator(np.random.PCG64(17)).integers(1, 300, size=items.size).astype(np.float32)
    ot = oracle_table(oracle, n, d, w, 42, items, users, vals)
    with SketchTable(n, depth=d, width=w, seed=42) as t:
        t.ingest(items, users, vals)
        t.finalize()
        ids, sc, cnt = t.top_k_all(k)
        st = t.stats()
        assert st["deep_limb_owners"] > 0 and st["multi_limb_owners"] > st["deep_limb_owners"], st
    os.environ["CMS_NO_MLS"] = "1"  # a tunable: read when the handle is created
    try:
        t2 = SketchTable(n, depth=d, width=w, seed=42)
    finally:
        del os.environ["CMS_NO_MLS"]
    with t2:
        t2.ingest(items, users, vals)
        t2.finalize()
        ids2, sc2, cnt2 = t2.top_k_all(k)
        assert np.array_equal(cnt, cnt2)
        for q in range(n):
            assert ids[q, :cnt[q]].tolist() == ids2[q, :cnt2[q]].tolist(), q
            assert same(sc[q, :cnt[q]], sc2[q, :cnt2[q]]), q
        hottest = np.argsort(-ot.max(axis=(1, 2)), kind="stable")[:6]
        for q in hottest.tolist() + [int(np.argsort(-ot.max(axis=(1, 2)))[st["multi_limb_owners"] - 1])]:
            sims = _oracle_row_sims(oracle, ot, q)
            eids, esc = oracle.top_users(np.arange(n), sims, k)
            assert ids[q, :cnt[q]].tolist() == eids.tolist(), q
            assert same(sc[q, :cnt[q]], esc), q


@pytest.mark.parametrize("accumulate", [False, True])
def test_slice_images_reduce_equals_slot_atomics(oracle, accumulate, monkeypatch):
    """k_build_slices with CMS_SLICE_REDUCE=1 writes each 65535-key slice's
    u16 image and k_slice_reduce sums them into the slot rows (stored whole,
    norms and maxima derived in the same pass, for owners of <= 16 slices;
    64-bit atomics plus k_hot_norms for the Zipf head's many-slice owners):
    the table, the norms (through the similarities) and the row maxima equal
    the slot-atomic path's bit for bit, in a fresh build and in an
    accumulating one (a second bulk batch into the live table), and the
    heaviest owners match the oracle."""
    import torch
    n, d, w = 4096, 5, 8192
    rng = np.random.Generator(np.random.PCG64(21))
    # owner 0: 1.3M keys (20 slices: two groups), owner 1: 300K (5 slices),
    # owner 2: 70K (2 slices), owners 3..: a Zipf tail (narrow and mid rows)
    heavy = [np.zeros(1_300_000, np.int64), np.ones(300_000, np.int64), np.full(70_000, 2, np.int64)]
    tail_items, tail_users = zipf_stream(3_000_000, n - 3, 2_000_000, seed=8)
    items = np.concatenate(heavy + [tail_items + 3])
    users = np.concatenate([rng.integers(0, 5_000_000, sum(h.size for h in heavy)), tail_users]).astype(np.int64)
    perm = rng.permutation(items.size)
    items, users = items[perm], users[perm]
    half = items.size // 2
    got = {}
    for mode in ("atomics", "reduce"):
        monkeypatch.setenv("CMS_SLICE_REDUCE", "1" if mode == "reduce" else "0")
        with SketchTable(n, depth=d, width=w, seed=13) as t:
            if accumulate:
                t.ingest(items[:half], users[:half])
                t.ingest(items[half:], users[half:])
            else:
                t.ingest(items, users)
            t.finalize()
            got[mode] = (t.read_counters_device().cpu(),
                         np.stack([t.similarities(q, np.arange(n)) for q in (0, 1, 2, 3, 100)]),
                         t.stats()["hot_rows"])
            torch.cuda.synchronize()
    assert torch.equal(got["atomics"][0], got["reduce"][0])
    assert same(got["atomics"][1], got["reduce"][1])
    assert got["reduce"][2] >= 3
    sel = np.array([0, 1, 2, 3])
    m = np.isin(items, sel)
    exp = oracle_table(oracle, sel.size, d, w, 13, items[m], users[m], None)
    assert same(got["reduce"][0].numpy()[sel].astype(np.float64), exp)


def test_byte_class_rows_once_equal_row_by_row(oracle, monkeypatch):
    """k_build_nibbles with CMS_NIB_ROWS_ONCE=1 (the first key slot's d
    buckets hashed up front, d = 5) builds the same table and forms as the
    row-by-row hashing, on a byte-class-heavy model (list rows, 1-/2-/4-bit
    rows, k_build_bytes escalations, keys past 2^32)."""
    import torch
    n, d, w = 30_000, 5, 8192
    rng = np.random.Generator(np.random.PCG64(41))
    sizes = rng.integers(1, 257, n)
    items = np.repeat(np.arange(n, dtype=np.int64), sizes)
    users = (rng.zipf(1.2, items.size) % 200_000).astype(np.int64)
    users[items % 97 == 0] += 1 << 33
    perm = rng.permutation(items.size)
    items, users = items[perm], users[perm]
    got = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("CMS_NIB_ROWS_ONCE", mode)
        with SketchTable(n, depth=d, width=w, seed=19) as t:
            t.ingest(items, users)
            t.finalize()
            got[mode] = (t.read_counters_device().cpu(), t.owner_forms(),
                         np.stack([t.similarities(q, np.arange(n)) for q in (0, 97, 5000)]))
            torch.cuda.synchronize()
    assert torch.equal(got["0"][0], got["1"][0])
    for a, b in zip(got["0"][1], got["1"][1]):
        assert np.array_equal(np.asarray(a), np.asarray(b))
    assert same(got["0"][2], got["1"][2])
    sel = np.array([0, 97, 5000, 29_999])
    m = np.isin(items, sel)
    remap = np.full(n, -1, np.int64)
    remap[sel] = np.arange(sel.size)
    exp = oracle_table(oracle, sel.size, d, w, 19, remap[items[m]], users[m], None)
    assert same(got["1"][0].numpy()[sel].astype(np.float64), exp)


@pytest.mark.parametrize("variant", ["CMS_MID_WAVES=5", "CMS_MID_THREADS=128"])
def test_mid_waves_equal_mid_workgroups(oracle, monkeypatch, variant):
    """k_build_mid_waves (CMS_MID_WAVES: one wave per mid-class owner, 4-bit
    then u8 rows, list rows for owners of <= 1024 keys; u16 owners and keys
    >= 2^32 handed to k_build_mid) and k_build_mid on 128-thread workgroups
    (CMS_MID_THREADS=128) build the same table, the same row forms and the
    same norms as k_build_mid's 256-thread owners, and sampled mid owners
    match the oracle."""
    var, val = variant.split("=")
    import torch
    n, d, w = 20_000, 5, 8192
    rng = np.random.Generator(np.random.PCG64(31))
    # mid owners of 300..14000 keys with Zipf users (repeats: u8 and u16 rows),
    # a byte-class tail, and one owner whose keys reach past 2^32
    sizes = np.concatenate([rng.integers(300, 1100, 3000), rng.integers(1100, 14000, 1500),
                            rng.integers(1, 200, n - 4500)])
    items = np.repeat(np.arange(n, dtype=np.int64), sizes)
    users = (rng.zipf(1.3, items.size) % 3_000_000).astype(np.int64)
    big = items == 7
    users[big] = users[big] + (1 << 33)
    perm = rng.permutation(items.size)
    items, users = items[perm], users[perm]
    got = {}
    for mode in ("workgroups", "waves"):
        if mode == "waves":
            monkeypatch.setenv(var, val)
        else:
            monkeypatch.delenv(var, raising=False)
        with SketchTable(n, depth=d, width=w, seed=17) as t:
            t.ingest(items, users)
            t.finalize()
            got[mode] = (t.read_counters_device().cpu(), t.owner_forms(),
                         np.stack([t.similarities(q, np.arange(n)) for q in (0, 7, 4000, 9000)]))
            torch.cuda.synchronize()
    assert torch.equal(got["workgroups"][0], got["waves"][0])
    for a, b in zip(got["workgroups"][1], got["waves"][1]):
        assert np.array_equal(np.asarray(a), np.asarray(b))
    assert same(got["workgroups"][2], got["waves"][2])
    sel = np.array([0, 7, 11, 3100, 4000])
    m = np.isin(items, sel)
    remap = np.full(n, -1, np.int64)
    remap[sel] = np.arange(sel.size)
    exp = oracle_table(oracle, sel.size, d, w, 17, remap[items[m]], users[m], None)
    assert same(got["waves"][0].numpy()[sel].astype(np.float64), exp)


@pytest.mark.parametrize("split", ["1024", "4096"])
def test_lower_split_threshold_same_table(oracle, split, monkeypatch):
    """CMS_SPLIT_KEYS moves owners of more than that many keys from the mid
    class to u32 slots built by k_build_slices (single-slice owners of a
    fresh build store their rows whole: no slot zeroing, no atomics): the
    counters and similarities equal the default split's, fresh and after an
    accumulating batch, and sampled owners match the oracle."""
    import torch
    n, d, w = 6000, 5, 8192
    rng = np.random.Generator(np.random.PCG64(51))
    sizes = np.concatenate([rng.integers(1000, 30000, 300), rng.integers(1, 1500, n - 300)])
    items = np.repeat(np.arange(n, dtype=np.int64), sizes)
    users = (rng.zipf(1.3, items.size) % 2_000_000).astype(np.int64)
    perm = rng.permutation(items.size)
    items, users = items[perm], users[perm]
    half = items.size // 2
    got = {}
    for mode in ("default", split):
        if mode == "default":
            monkeypatch.delenv("CMS_SPLIT_KEYS", raising=False)
        else:
            monkeypatch.setenv("CMS_SPLIT_KEYS", mode)
        for acc in (False, True):
            with SketchTable(n, depth=d, width=w, seed=23) as t:
                if acc:
                    t.ingest(items[:half], users[:half])
                    t.ingest(items[half:], users[half:])
                else:
                    t.ingest(items, users)
                t.finalize()
                got[(mode, acc)] = (t.read_counters_device().cpu(),
                                    np.stack([t.similarities(q, np.arange(n)) for q in (0, 150, 3000)]),
                                    t.stats()["hot_rows"])
                torch.cuda.synchronize()
    for acc in (False, True):
        a, b = got[("default", acc)], got[(split, acc)]
        assert torch.equal(a[0], b[0]), acc
        assert same(a[1], b[1]), acc
        assert b[2] > a[2]  # more owners on u32 slots
    sel = np.array([0, 150, 299, 3000])
    m = np.isin(items, sel)
    remap = np.full(n, -1, np.int64)
    remap[sel] = np.arange(sel.size)
    exp = oracle_table(oracle, sel.size, d, w, 23, remap[items[m]], users[m], None)
    assert same(got[(split, False)][0].numpy()[sel].astype(np.float64), exp)


def test_early_slices_same_table(oracle, monkeypatch):
    """CMS_EARLY_SLICES=1: the hot-routed owners of more than the split
    threshold are built beside pass 2 of the partition (k_early_plan,
    k_build_slices on a stream of their own) and the plan skips them: the
    table, the forms, the norms (through the similarities) and the row
    maxima equal the default build's, and the heaviest owners equal the
    oracle."""
    import torch
    n, d, w = 4096, 5, 8192
    rng = np.random.Generator(np.random.PCG64(41))
    # owners 0..2: 1.3M / 300K / 70K keys (many, several, two slices), a Zipf tail
    heavy = [np.zeros(1_300_000, np.int64), np.ones(300_000, np.int64), np.full(70_000, 2, np.int64)]
    tail_items, tail_users = zipf_stream(3_000_000, n - 3, 2_000_000, seed=42)
    items = np.concatenate(heavy + [tail_items + 3])
    users = np.concatenate([rng.integers(0, 5_000_000, sum(h.size for h in heavy)), tail_users]).astype(np.int64)
    perm = rng.permutation(items.size)
    items, users = items[perm], users[perm]
    got = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("CMS_EARLY_SLICES", mode)
        with SketchTable(n, depth=d, width=w, seed=13) as t:
            for _ in range(2):  # twice: the second build reuses the handle's slots and scratch
                t.reset()
                t.ingest(items, users)
                t.finalize()
            got[mode] = (t.read_counters_device().cpu(), t.owner_forms()[0],
                         np.stack([t.similarities(q, np.arange(n)) for q in (0, 1, 2, 3, 100)]),
                         t.stats()["hot_rows"])
            torch.cuda.synchronize()
    assert torch.equal(got["0"][0], got["1"][0])
    assert np.array_equal(got["0"][1], got["1"][1])
    assert same(got["0"][2], got["1"][2])
    assert got["1"][3] >= 3
    sel = np.array([0, 1, 2, 3])
    m = np.isin(items, sel)
    exp = oracle_table(oracle, sel.size, d, w, 13, items[m], users[m], None)
    assert same(got["1"][0].numpy()[sel].astype(np.float64), exp)
