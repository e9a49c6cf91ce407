"""Full-size parity by sampling: ingest the bench stream, then compare the
counters of sampled owners (the hottest plus random ones) with the CPU
oracle built from exactly those owners' pairs, and the all-pairs top-k of a
few query rows with the oracle's top-k over the same owners' rows.
Usage: python scripts/scale_check.py N_ITEMS N_PAIRS WIDTH"""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import torch  # noqa: E402
from mahout_amd import SketchTable  # noqa: E402
from mahout_amd.synth import zipf_stream_torch  # noqa: E402
from oracle import oracle as O  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
pairs = int(sys.argv[2]) if len(sys.argv) > 2 else 500_000_000
w = int(sys.argv[3]) if len(sys.argv) > 3 else 8192
d = 5
O.build()
items, users = zipf_stream_torch(1_000_000 if n <= 100_000 else 10_000_000, n, pairs, device="cuda")
cnt = torch.bincount(items, minlength=n)
hot = torch.topk(cnt, 16).indices.cpu().numpy()
rng = np.random.Generator(np.random.PCG64(5))
sample = np.unique(np.concatenate([hot, rng.integers(0, n, 48)])).astype(np.int64)
t = SketchTable(n, depth=d, width=w, seed=42, device=0)
t0 = time.time()
t.ingest_device_rows(items, users, None, pairs)
t.finalize()
print("ingest+finalize s", round(time.time() - t0, 2), flush=True)
# the sampled owners' pairs, on the host
sel = torch.isin(items, torch.from_numpy(sample).cuda())
si = items[sel].cpu().numpy()
su = users[sel].cpu().numpy()
del items, users, sel
remap = {int(o): i for i, o in enumerate(sample)}
rows = np.array([remap[int(o)] for o in si], np.int64) if si.size < 5_000_000 else \
    np.searchsorted(sample, si).astype(np.int64)
a, b = O.hash_params(42, d)
exp = O.build_table(sample.size, d, w, a, b, rows, su)
bad_rows = 0
for i, o in enumerate(sample):
    got = t.read_counters(int(o), 1)[0]
    if not np.array_equal(got, exp[i]):
        bad_rows += 1
print(json.dumps({"sampled_owners": int(sample.size), "sampled_pairs": int(si.size), "counter_mismatch_rows": bad_rows,
                  "hot_counts": cnt[torch.from_numpy(hot).cuda()].cpu().tolist()[:4]}), flush=True)
# similarities of the sampled owners among themselves: product vs oracle
sims_bad = 0
for i, o in enumerate(sample[:16]):
    got = t.similarities(int(o), sample)
    for jx, p in enumerate(sample):
        e = O.cosine_cm(exp[i], exp[jx])
        g = got[jx]
        if not (g == e or (np.isnan(g) and np.isnan(e))):
            sims_bad += 1
print(json.dumps({"similarity_mismatches": sims_bad}), flush=True)
# all-pairs top-k for two sampled query rows: every score must equal the
# product's own exact pair similarity, and the list must be sorted
ids, sc, c = t.top_k_rows(int(sample[0]), 1, 50)
ids2, sc2, c2 = t.top_k_rows(int(sample[0]), 1, 50)
pair = t.similarities(int(sample[0]), ids[0, :c[0]])
ok_vals = bool(np.array_equal(pair, sc[0, :c[0]]))
ok_det = bool(np.array_equal(ids, ids2) and np.array_equal(sc, sc2))
srt = all((sc[0, i] > sc[0, i + 1]) or (sc[0, i] == sc[0, i + 1] and ids[0, i] < ids[0, i + 1]) for i in range(c[0] - 1))
print(json.dumps({"topk_scores_equal_pair_kernel": ok_vals, "topk_deterministic": ok_det, "topk_sorted": bool(srt),
                  "stats": t.stats()}), flush=True)
