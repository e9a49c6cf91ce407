"""CPU: pin the oracle (oracle/cms_oracle.c) before trusting it as the checker.

- published java.util.Random known answers (the JDK semantics the reference's
  HashFunctionBuilder relies on);
- the C 128-bit hash against an independent big-integer restatement
  (Python ints have java.math.BigInteger semantics for * + and mod);
- the reference's own exact-cosine known answers reproduced through
  collision-free sketches (VectorSimilarityMeasuresTest, ItemSimilarityJobTest);
- the committed golden vectors (tests/golden/golden_cms.json).
"""
import json
import math
import os

import numpy as np
import pytest

from oracle import java_ref as J

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden_cms.json")))


def test_java_random_published_kats():
    kat = GOLDEN["jdk_random"]
    assert J.JavaRandom(0).next_long() == kat["new Random(0).nextLong()"]
    assert J.JavaRandom(42).next_long() == kat["new Random(42).nextLong()"]
    assert J.JavaRandom(42).next_int() == kat["new Random(42).nextInt()"]


def test_java_abs_min_value_stays_negative():
    assert J.java_abs_long(-(2 ** 63)) == -(2 ** 63)
    assert J.java_abs_long(-5) == 5


@pytest.mark.parametrize("seed", [0, 1, 42, -7, 2 ** 40 + 3, 20261015])
def test_hash_params_c_vs_python_vs_golden(oracle, seed):
    a, b = oracle.hash_params(seed, 8)
    pa, pb = J.hash_params(seed, 8)
    assert list(a) == pa and list(b) == pb
    g = GOLDEN["hash_params_depth8"][str(seed)]
    assert list(a) == g["a"] and list(b) == g["b"]


def test_hash_params_survey_values(oracle):
    a, b = oracle.hash_params(42, 5)
    assert list(a) == [5025562857975149833, 5694868678511409995, 6169532649852302182, 6802844026563419272,
                       8552898714322622292]
    assert list(b) == [5843495416241995736, 5111195811822994797, 1782466964123969572, 5086654115216342560,
                       4004755535478349341]


@pytest.mark.parametrize("width", [1, 7, 39, 40, 1000, 1024, 4096, 8192, 32768])
def test_hash_c_vs_bigint(oracle, width):
    rng = np.random.Generator(np.random.PCG64(width))
    keys = np.concatenate([np.array(GOLDEN["hash_indices_seed42_depth5"]["keys"], np.int64),
                           rng.integers(-2 ** 63, 2 ** 63 - 1, size=2000, dtype=np.int64),
                           rng.integers(-3000, 3000, size=500, dtype=np.int64)])
    a, b = oracle.hash_params(42, 5)
    got = oracle.hash_keys(a, b, width, keys)
    for i, k in enumerate(keys.tolist()):
        exp = [J.hash_(int(a[r]), int(b[r]), width, k) for r in range(5)]
        assert list(got[i]) == exp, (width, k)


def test_hash_golden(oracle):
    g = GOLDEN["hash_indices_seed42_depth5"]
    a, b = oracle.hash_params(42, 5)
    keys = np.array(g["keys"], np.int64)
    for w, exp in g["by_width"].items():
        assert oracle.hash_keys(a, b, int(w), keys).tolist() == exp


def _collision_free_seed(oracle, keys, depth, width):
    for seed in range(1, 10000):
        a, b = oracle.hash_params(seed, depth)
        h = oracle.hash_keys(a, b, width, np.array(keys, np.int64))
        if all(len(set(h[:, r].tolist())) == len(keys) for r in range(depth)):
            return seed, a, b
    raise AssertionError("no collision-free seed")


def test_reference_kat_vector_cosine(oracle):
    """VectorSimilarityMeasuresTest.testCosineSimilarity: 0.769846046 +- 1e-6."""
    kat = GOLDEN["reference_kats"]["VectorSimilarityMeasuresTest.testCosineSimilarity"]
    keys = list(range(13))
    seed, a, b = _collision_free_seed(oracle, keys, 4, 1024)
    owners = np.array([0] * 13 + [1] * 13, np.int64)
    k = np.array(keys + keys, np.int64)
    v = np.array(kat["a"] + kat["b"], np.float32)
    t = oracle.build_table(2, 4, 1024, a, b, owners, k, v)
    assert abs(oracle.cosine_cm(t[0], t[1]) - kat["cosine"]) < kat["epsilon"]


def test_reference_kat_item_similarity_job(oracle):
    """ItemSimilarityJobTest.testCompleteJob: items (1,3) -> 0.45, (2,3) -> 0.89 (+- 0.01)
    with item sketches keyed by user (the transposed orientation)."""
    kat = GOLDEN["reference_kats"]["ItemSimilarityJobTest.testCompleteJob"]
    users, items, prefs = zip(*[map(int, ln.split(",")) for ln in kat["lines"]])
    seed, a, b = _collision_free_seed(oracle, sorted(set(users)), 4, 1024)
    item_ids = sorted(set(items))
    rows = np.array([item_ids.index(i) for i in items], np.int64)
    t = oracle.build_table(len(item_ids), 4, 1024, a, b, rows, np.array(users, np.int64),
                           np.array(prefs, np.float32))
    for i1, i2, exp in kat["pairs"]:
        got = oracle.cosine_cm(t[item_ids.index(i1)], t[item_ids.index(i2)])
        assert abs(got - exp) < kat["epsilon"]
    # and the exact values: 1/sqrt(5), 2/sqrt(5)
    assert oracle.cosine_cm(t[0], t[2]) == pytest.approx(1 / math.sqrt(5), abs=1e-15)


def test_sketch_small_golden(oracle):
    g = GOLDEN["sketch_small"]
    a, b = oracle.hash_params(g["seed"], g["depth"])
    t = oracle.build_table(4, g["depth"], g["width"], a, b, np.array(g["owners"], np.int64),
                           np.array(g["keys"], np.int64), np.array(g["vals"], np.float32))
    assert t.astype(np.int64).tolist() == g["counters"]
    for i in range(4):
        for j in range(4):
            exp = g["cosine_cm"][i][j]
            got = oracle.cosine_cm(t[i], t[j])
            assert (exp is None and np.isnan(got)) or got == exp


def test_cosine_nan_and_min_rules(oracle):
    z = np.zeros((3, 8))
    assert np.isnan(oracle.cosine(z, z))  # no row qualifies -> NaN
    a = np.zeros((2, 4))
    b = np.zeros((2, 4))
    a[0, 0] = 1
    b[0, 0] = 1  # row 0 cosine 1
    a[1, 1] = 1
    b[1, 2] = 1  # row 1 cosine 0
    assert oracle.cosine(a, b) == 0.0  # min over rows
    a[1, :] = 0  # row 1 denominator 0 -> skipped
    assert oracle.cosine(a, b) == 1.0


def test_normalize_weight_result_quirks(oracle):
    assert oracle.normalize_weight_result(1.0000000000000002) == 1.0
    assert oracle.normalize_weight_result(-1.5) == -1.0
    # WEIGHTED with count=1, num=0: scaleFactor 0 -> +-1
    assert oracle.normalize_weight_result(0.3, 1, 0, True) == 1.0
    assert oracle.normalize_weight_result(-0.3, 1, 0, True) == -1.0
    assert oracle.normalize_weight_result(0.0, 1, 0, True) == 1.0


def test_top_users_ties_golden(oracle):
    g = GOLDEN["top_users_ties"]
    scores = np.array([np.nan if s is None else s for s in g["scores"]])
    ids, sc = oracle.top_users(np.array(g["ids"], np.int64), scores, g["k"])
    assert ids.tolist() == g["expect_ids"] and sc.tolist() == g["expect_scores"]


def test_top_users_equals_total_order(oracle):
    """getTopUsers over ascending IDs == the first k under (score desc, ID asc)."""
    rng = np.random.Generator(np.random.PCG64(3))
    for trial in range(50):
        n = int(rng.integers(1, 300))
        k = int(rng.integers(1, 40))
        ids = np.arange(n, dtype=np.int64) * 3 - 50
        scores = np.round(rng.random(n) * 4) / 4  # many ties
        scores[rng.random(n) < 0.1] = np.nan
        got, _ = oracle.top_users(ids, scores, k)
        valid = [(-s, i) for s, i in zip(scores, ids) if not np.isnan(s)]
        exp = [i for _, i in sorted(valid)[:k]]
        assert got.tolist() == exp


def test_shape_from_delta_epsilon_quirk(oracle):
    g = GOLDEN["shape_from_delta_epsilon"]
    for w, (ww, dd) in g.items():
        assert oracle.shape_from_delta_epsilon(math.exp(-5.0), math.e / int(w)) == (ww, dd)
    assert g["39"] == [40, 5] and g["1024"] == [1024, 5]
    with pytest.raises(ValueError):
        oracle.shape_from_delta_epsilon(0.0, 0.1)  # missing config entry (trove default 0.0)
    with pytest.raises(ValueError):
        oracle.shape_from_delta_epsilon(0.5, 0.1)  # delta > e^-1


def test_compute_config_ties_go_last(oracle):
    w, d, delta, eps = oracle.compute_config(1, 100, 1.0)
    assert (w, d) == (1, 1) and delta == math.exp(-1.0) and eps == math.e
    w, d, _, _ = oracle.compute_config(50, 1682, 0.5)
    best = max((oracle.fmeasure(ww, dd, 50, 1682, 0.5), dd, ww) for dd in range(1, 25) for ww in range(dd, 51))
    assert oracle.fmeasure(w, d, 50, 1682, 0.5) == best[0]


def test_faithful_pairs_match_prebuilt(oracle):
    """The rebuild-per-call cost model (CosineCM.userSimilarity) equals the
    cosine of prebuilt sketches."""
    from mahout_amd.synth import zipf_stream, to_csr
    items, users = zipf_stream(500, 40, 3000, seed=5)
    off, keys, _ = to_csr(items, users, 40)
    a, b = oracle.hash_params(42, 4)
    t = oracle.build_table(40, 4, 128, a, b, np.repeat(np.arange(40), np.diff(off)), keys)
    pi = np.array([0, 1, 2, 5, 39], np.int64)
    pj = np.array([1, 0, 7, 5, 3], np.int64)
    got = oracle.faithful_pairs(off, keys, None, 40, 4, 128, a, b, pi, pj)
    for p in range(len(pi)):
        exp = oracle.cosine_cm(t[pi[p]], t[pj[p]])
        assert (np.isnan(exp) and np.isnan(got[p])) or got[p] == exp


@pytest.mark.parametrize("vals_kind", ["unit", "float"])
def test_cosine_queries_csr_equals_dense(oracle, vals_kind):
    """The full-size test's all-owners check (orc_cosine_queries_csr: sketch
    rows from each owner's keys, nonzero buckets in ascending order) equals
    the dense CosineCM restatement bit for bit -- colliding keys, empty owners,
    and negative / non-dyadic float preferences included."""
    rng = np.random.default_rng(11)
    n, d, w = 300, 4, 96
    counts = rng.integers(0, 40, n)
    counts[[3, 17]] = 0
    counts[5] = 700  # more keys than buckets
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    owner = np.repeat(np.arange(n), counts).astype(np.int64)
    keys = rng.integers(-2**40, 2**40, off[-1]).astype(np.int64)
    vals = None if vals_kind == "unit" else rng.uniform(-2.5, 5.0, off[-1]).astype(np.float32)
    a, b = oracle.hash_params(7, d)
    table = oracle.build_table(n, d, w, a, b, owner, keys, vals)
    qrows = [0, 5, 17, 42]
    got = oracle.cosine_queries_csr(table[qrows], off, keys, vals, d, w, a, b, threads=4)
    for qi, q in enumerate(qrows):
        want = np.array([oracle.cosine_cm(table[q], table[p]) for p in range(n)])
        same = (got[qi] == want) | (np.isnan(got[qi]) & np.isnan(want))
        assert same.all(), (q, np.flatnonzero(~same)[:5])
