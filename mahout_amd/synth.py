"""Synthetic interaction streams of the benchmark shapes.

Zipf item popularity ~ rank^-1.1 and user activity ~ rank^-0.9, truncated to
their ranges by inverse-CDF lookup; rank -> ID through a seeded permutation;
unit increments.  numpy PCG64 on the host (tests, oracle-sized cases) and a
torch generator on the GPU for the full-size bench streams (generation is
outside every timed region).
"""
import numpy as np

ITEM_S = 1.1
USER_S = 0.9


def zipf_cdf(n, s):
    w = np.arange(1, n + 1, dtype=np.float64) ** (-s)
    c = np.cumsum(w)
    return c / c[-1]


def zipf_stream(n_users, n_items, n_pairs, seed=20261015, item_s=ITEM_S, user_s=USER_S):
    """COO stream: (item_ids, user_ids), int64, item orientation (owner=item,
    key=user)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    icdf = zipf_cdf(n_items, item_s)
    ucdf = zipf_cdf(n_users, user_s)
    iperm = rng.permutation(n_items).astype(np.int64)
    uperm = rng.permutation(n_users).astype(np.int64)
    ir = np.minimum(np.searchsorted(icdf, rng.random(n_pairs)), n_items - 1)
    ur = np.minimum(np.searchsorted(ucdf, rng.random(n_pairs)), n_users - 1)
    return iperm[ir], uperm[ur]


def zipf_stream_torch(n_users, n_items, n_pairs, seed=20261015, device="cuda", item_s=ITEM_S, user_s=USER_S):
    """Same distribution, generated on the GPU with torch (bench inputs)."""
    import torch

    g = torch.Generator(device=device)
    g.manual_seed(seed)
    icdf = torch.from_numpy(zipf_cdf(n_items, item_s)).to(device)
    ucdf = torch.from_numpy(zipf_cdf(n_users, user_s)).to(device)
    iperm = torch.randperm(n_items, generator=g, device=device)
    uperm = torch.randperm(n_users, generator=g, device=device)
    items = torch.empty(n_pairs, dtype=torch.int64, device=device)
    users = torch.empty(n_pairs, dtype=torch.int64, device=device)
    step = 1 << 25
    for o in range(0, n_pairs, step):
        m = min(step, n_pairs - o)
        u = torch.rand(m, generator=g, device=device, dtype=torch.float64)
        ir = torch.clamp(torch.searchsorted(icdf, u), max=n_items - 1)
        items[o:o + m] = iperm[ir]
        u = torch.rand(m, generator=g, device=device, dtype=torch.float64)
        ur = torch.clamp(torch.searchsorted(ucdf, u), max=n_users - 1)
        users[o:o + m] = uperm[ur]
    return items, users


def to_csr(owner, key, n_owners, val=None):
    """Group a COO stream by owner (stable), as a DataModel would hold it."""
    order = np.argsort(owner, kind="stable")
    counts = np.bincount(owner, minlength=n_owners)
    off = np.zeros(n_owners + 1, np.int64)
    np.cumsum(counts, out=off[1:])
    v = None if val is None else np.ascontiguousarray(val[order])
    return off, np.ascontiguousarray(key[order]), v


def movielens_like(n_users=943, n_items=1682, n_ratings=100000, seed=20261015, min_per_user=20):
    """ML-100K-shaped stand-in (the real u.data is not available offline):
    943 users x 1682 items x 100,000 integer ratings 1..5 drawn from the
    ML-100K marginal, >= 20 ratings per user, Zipf item popularity, no
    duplicate (user,item) pairs.  Returns (users, items, ratings)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    icdf = zipf_cdf(n_items, 0.8)
    iperm = rng.permutation(n_items) + 1
    # per-user counts: min_per_user + a Zipf-ish share of the rest
    extra = n_ratings - min_per_user * n_users
    w = rng.pareto(1.2, n_users) + 1.0
    cnt = min_per_user + np.floor(extra * w / w.sum()).astype(np.int64)
    cnt[: n_ratings - cnt.sum()] += 1
    cnt = np.minimum(cnt, n_items)
    users, items = [], []
    for u in range(n_users):
        chosen = set()
        while len(chosen) < cnt[u]:
            r = np.minimum(np.searchsorted(icdf, rng.random(cnt[u] * 2)), n_items - 1)
            for x in iperm[r]:
                if len(chosen) < cnt[u]:
                    chosen.add(int(x))
        items.extend(sorted(chosen))
        users.extend([u + 1] * len(chosen))
    users = np.array(users, np.int64)
    items = np.array(items, np.int64)
    ratings = rng.choice(np.arange(1, 6), size=users.size, p=[0.06, 0.11, 0.27, 0.35, 0.21]).astype(np.float32)
    return users, items, ratings
