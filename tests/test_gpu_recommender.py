"""GPU: GenericUserBasedRecommender.recommend with NearestNUserNeighborhood
and the CosineCM point-query estimate -- the fork's use case (SURVEY §3-A,
`T/impl/recommender/GenericUserBasedRecommender.java:84-184`,
`T/impl/neighborhood/NearestNUserNeighborhood.java:84-95`) -- on the
ML-100K-shaped stand-in (config 1's data, user-owner orientation).

The GPU answers the neighbourhood (cms_most_similar) and the estimates
(cms_estimate_preferences[_batch]); the candidate set and the final ordering
are the host logic the reference runs (FastIDSet iteration order,
TopItems.getTopItems' PriorityQueue; restated in mahout_amd.taste).  The
oracle recomputes the neighbourhood (similarities + TopItems.getTopUsers) and
every estimate (orc_estimate_preference) from its own fp64 table, and the
recommended lists must be equal item for item, value for value.
"""
import numpy as np
import pytest

from mahout_amd import SketchTable
from mahout_amd import taste
from mahout_amd.datamodel import GenericDataModel
from mahout_amd.synth import movielens_like

pytestmark = pytest.mark.gpu

D, W, SEED, NN, HOW = 4, 1024, 42, 50, 10


def _model():
    users, items, ratings = movielens_like()
    uid = np.unique(users)
    rows = np.searchsorted(uid, users)
    order = np.lexsort((items, rows))  # GenericDataModel: each user's preferences by item ID
    rows, items, ratings = rows[order], items[order], ratings[order]
    off = np.zeros(uid.size + 1, np.int64)
    np.cumsum(np.bincount(rows, minlength=uid.size), out=off[1:])
    return GenericDataModel.from_csr(uid, off, items, ratings), rows, items, ratings


def test_recommend_equals_oracle(oracle):
    model, rows, items, ratings = _model()
    uid = model.getUserIDs()
    a, b = oracle.hash_params(SEED, D)
    table = oracle.build_table(uid.size, D, W, a, b, rows, items, ratings)
    sim = taste.CosineCM(model, taste.FixedShapeConfig(D, W), taste.HashFunctionBuilder(SEED))
    try:
        nbh = taste.NearestNUserNeighborhood(NN, sim, model)
        rec = taste.GenericUserBasedRecommender(model, nbh, sim)
        capper = (model.getMinPreference(), model.getMaxPreference())
        rng = np.random.default_rng(7)
        for u in [int(uid[0]), int(uid[-1])] + rng.choice(uid, 6, replace=False).tolist():
            got = rec.recommend(u, HOW)
            urow = int(np.searchsorted(uid, u))
            sims = oracle.similarities_row(table, urow)
            sims[urow] = np.nan  # NearestNUserNeighborhood's estimator: the user itself is NaN
            nb, _ = oracle.top_users(uid, sims, NN)
            assert nbh.getUserNeighborhood(u).tolist() == nb.tolist(), u
            cand = rec.getAllOtherItems(nb, u).toList()
            nb_rows = np.searchsorted(uid, nb)
            est = np.array([oracle.estimate_preference(table, a, b, urow, nb_rows, it, capper=capper) for it in cand],
                           np.float32)
            gpu_est = rec.doEstimatePreferences(u, nb, cand)
            assert np.array_equal(gpu_est, est, equal_nan=True), u
            want = taste.get_top_items(HOW, cand, est)
            assert [i for i, _ in got] == [i for i, _ in want], u
            assert [float(v) for _, v in got] == [float(v) for _, v in want], u
            assert len(got) == min(HOW, int(np.sum(~np.isnan(est))))
    finally:
        sim.close()


def test_estimate_batch_equals_single_calls(oracle):
    """cms_estimate_preferences_batch (every user's neighbourhood and
    candidates in one call) gives each user's single-call estimates bit for
    bit, NaN for NaN, in u32 and fp64 counter modes."""
    model, rows, items, ratings = _model()
    uid = model.getUserIDs()
    for counter in ("u32", "f64"):
        kw = {"counters": counter}
        with SketchTable(uid.size, depth=D, width=W, seed=SEED, owner_ids=uid, **kw) as t:
            t.ingest(uid[rows], items, ratings)
            t.finalize()
            ids, _, cnt = t.top_k_all(NN)
            users = uid[::3]
            nb_off = np.zeros(users.size + 1, np.int64)
            it_off = np.zeros(users.size + 1, np.int64)
            nbs, its = [], []
            rng = np.random.default_rng(3)
            for j, u in enumerate(users.tolist()):
                r = int(np.searchsorted(uid, u))
                nb = ids[r, :cnt[r]]
                cand = rng.choice(model.getItemIDs(), 40, replace=False)
                nbs.append(nb)
                its.append(cand)
                nb_off[j + 1] = nb_off[j] + nb.size
                it_off[j + 1] = it_off[j] + cand.size
            cap = (1.0, 5.0)
            got = t.estimate_preferences_batch(users, nb_off, np.concatenate(nbs), it_off, np.concatenate(its), cap)
            for j, u in enumerate(users.tolist()):
                one = t.estimate_preferences(u, nbs[j], its[j], cap)
                assert np.array_equal(got[it_off[j]:it_off[j + 1]], one, equal_nan=True), (counter, u)


@pytest.mark.parametrize("counters", ["u32", "f64"])
def test_recommend_all_equals_recommend_for_every_user(counters):
    """GenericUserBasedRecommender.recommend_all (cms_recommend_batch: the
    neighbourhoods from one top-n pass, FastIDSet candidates and
    TopItems.getTopItems in the library, every estimate in one device batch)
    gives, for ALL 943 users, exactly the lists of the per-user recommend()
    path that test_recommend_equals_oracle pins against the oracle: items in
    the same order (ties included) and the same float values. The same path
    is what bench.py's config1.recommender times."""
    model, rows, items, ratings = _model()
    uid = model.getUserIDs()
    if counters == "f64":  # non-dyadic preferences: DoubleCountMinSketch's fp64 counters (taste.counter_units)
        model = GenericDataModel.from_csr(uid, model.offsets, model.keys, model.values * np.float32(0.3))
    sim = taste.CosineCM(model, taste.FixedShapeConfig(D, W), taste.HashFunctionBuilder(SEED))
    assert sim.table.counters == counters
    try:
        nbh = taste.NearestNUserNeighborhood(NN, sim, model)
        rec = taste.GenericUserBasedRecommender(model, nbh, sim)
        users = uid if counters == "u32" else uid[::9]
        got = rec.recommend_all(users, HOW)
        assert len(got) == users.size
        ties = 0
        for u, lst in zip(users.tolist(), got):
            want = rec.recommend(u, HOW)
            assert [i for i, _ in lst] == [i for i, _ in want], u
            assert [float(v) for _, v in lst] == [float(v) for _, v in want], u
            vals = [float(v) for _, v in want]
            ties += len(vals) - len(set(vals))
        assert ties > 0  # capped estimates tie: the tie order was exercised
        # includeKnownItems keeps the user's own items among the candidates
        sub = users[:25]
        got_k = rec.recommend_all(sub, HOW, includeKnownItems=True)
        for u, lst in zip(sub.tolist(), got_k):
            assert lst == rec.recommend(u, HOW, includeKnownItems=True), u
    finally:
        sim.close()
