"""Config 4 on one GPU: mostSimilar top-k for EVERY item of the 1M-item
table through cms_top_k_all, with a spot check against the per-row path."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import torch  # noqa: E402
from mahout_amd import SketchTable  # noqa: E402
from mahout_amd.synth import zipf_stream_torch  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
pairs = int(sys.argv[2]) if len(sys.argv) > 2 else 500_000_000
w = int(sys.argv[3]) if len(sys.argv) > 3 else 8192
k = int(sys.argv[4]) if len(sys.argv) > 4 else 100
d = 5
items, users = zipf_stream_torch(1_000_000 if n <= 100_000 else 10_000_000, n, pairs, seed=20261016, device="cuda")
t = SketchTable(n, depth=d, width=w, seed=42, device=0)
t.ingest_device_rows(items, users, None, pairs)
t.finalize()
del items, users
torch.cuda.empty_cache()
t.release_scratch()
t.set_timing(True)
t.top_k_rows(0, 128, k)  # operands prepared
t.reset_timing()
t0 = time.perf_counter()
ids, sc, cnt = t.top_k_all(k)
wall = time.perf_counter() - t0
tm = {name: t.timing(name)[0] for name in ["topk_all_multi_rows", "topk_all_limbs", "topk_all_waves",
                                           "topk_all_waves_i8", "topk_all_waves_f4", "cand_compact", "cosine_mfma",
                                           "cosine_mfma_limbs", "cosine_mfma_multi", "top_k"]}
st = t.stats()
nm = st["multi_limb_owners"]
ns = n - nm
uniq = n * (n - 1) / 2
ops_waves = ns * (ns - 1) / 2 * 2 * d * w
rows = np.random.Generator(np.random.PCG64(3)).integers(0, n, 48)
ok = True
for r in rows:
    i2, s2, c2 = t.top_k_rows(int(r), 1, k)
    ok &= bool(c2[0] == cnt[r] and np.array_equal(i2[0, :c2[0]], ids[r, :cnt[r]]) and np.array_equal(s2[0, :c2[0]], sc[r, :cnt[r]]))
print(json.dumps({"n": n, "w": w, "k": k, "wall_s": wall, "unique_pairs_per_s": uniq / wall,
                  "timing_ms": tm, "waves_TOPS": ops_waves / (tm["topk_all_waves"] * 1e-3) / 1e12 if tm["topk_all_waves"] else None,
                  "full_lists": int((cnt == k).sum()), "spot_check_rows_equal": ok, "stats": st}))
