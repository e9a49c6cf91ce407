"""The row-0 upper bound that prunes per-owner top-k candidates
(k_po_wide_bound, cms_profiles.hip), restated in exact integers and
correctly rounded fp64 on the CPU and checked against the oracle's
CosineCM.userSimilarity (CosineCM.java:83-96: u1 built at u2's shape, the
min over rows of AbstractSimilarity's cosine, oracle/oracle.py
per_owner_similarity) on every ordered pair of a small DataModel:

    userSimilarity(u1, u2) <= normalize(AB_0 / (sqrt(A_lb) * sqrt(B_0))),
    A_lb = max(sum v^2, ceil((sum v)^2 / w)) <= valueA_0.

Test infrastructure only (the oracle is the checker)."""
import math

import numpy as np
import pytest


def _model(rng, n_owners, n_keys):
    offs, keys, vals = [0], [], []
    for _ in range(n_owners):
        m = int(rng.integers(1, 300))
        ks = np.sort(rng.choice(n_keys, m, replace=False))
        keys.append(ks)
        vals.append(rng.integers(1, 6, m).astype(np.float32))
        offs.append(offs[-1] + m)
    return np.array(offs, np.int64), np.concatenate(keys).astype(np.int64), np.concatenate(vals)


@pytest.mark.parametrize("seed", [1, 2])
def test_row0_bound_is_an_upper_bound(oracle, seed):
    rng = np.random.default_rng(seed)
    off, keys, vals = _model(rng, 24, 3000)
    de, ep = oracle.owner_config(off, 3000, 1.0)
    shapes = oracle.owner_shapes(de, ep)
    a, b = oracle.hash_params(42, 32)
    n = off.size - 1
    checked = tight = 0
    for u1 in range(n):
        v = vals[off[u1]:off[u1 + 1]].astype(np.int64)
        s1v, s2v = int((v * v).sum()), int(v.sum())
        for u2 in range(n):
            if u1 == u2 or shapes[0][u2] == 0:
                continue
            w, d = int(shapes[0][u2]), int(shapes[1][u2])
            sim = oracle.per_owner_similarity(off, keys, vals, shapes, a, b, u1, u2)
            s1 = oracle.export_profile(off, keys, vals, u1, w, d, a, b)
            s2 = oracle.export_profile(off, keys, vals, u2, w, d, a, b)
            ab0 = int(round(float(np.dot(s1[0], s2[0]))))  # integer counters: exact
            b0 = int(round(float(np.dot(s2[0], s2[0]))))
            a2 = max(s1v, -(-s2v * s2v // w))
            assert a2 <= int(round(float(np.dot(s1[0], s1[0]))))  # the lower bound on valueA_0
            if b0 == 0 or math.isnan(sim):
                continue
            ub = ab0 / (math.sqrt(a2) * math.sqrt(b0))
            ub = min(1.0, max(-1.0, ub))  # normalize (unweighted: the clamp)
            assert ub >= sim, (u1, u2, ub, sim)
            checked += 1
            tight += ub == sim
    assert checked > 300 and tight > 0  # (collision-free rows make it exact)


def test_sparse_per_owner_rows_equal_dense_oracle(oracle):
    """oracle.per_owner_rows_csr (the sparse, shape-grouped restatement the
    bench-scale per-owner GPU test checks against) equals the dense
    per_owner_similarity bit for bit, including a missing shape (w = 0: NaN)."""
    from mahout_amd.synth import zipf_stream, to_csr
    items, users = zipf_stream(5000, 300, 30000, seed=5)
    off, keys, _ = to_csr(items, users, 300)
    rng = np.random.default_rng(1)
    n = 300
    w = rng.choice([7, 64, 100, 1024, 3001], n).astype(np.int32)
    d = rng.integers(1, 9, n).astype(np.int32)
    w[5] = 0
    a, b = oracle.hash_params(42, 32)
    qs = np.array([0, 3, 150, 299])
    got = oracle.per_owner_rows_csr(off, keys, (w, d), a, b, qs, threads=4)
    for qi, q in enumerate(qs):
        for u2 in range(n):
            if w[u2] == 0:
                assert np.isnan(got[qi, u2])
                continue
            e = oracle.per_owner_similarity(off, keys, None, (w, d), a, b, int(q), u2)
            assert (np.isnan(e) and np.isnan(got[qi, u2])) or e == got[qi, u2], (q, u2)
