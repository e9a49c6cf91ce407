"""Quick MFMA all-pairs timing on the config-2 table (GPU box)."""
import json, sys, time
sys.path.insert(0, ".")
import torch  # noqa
from mahout_amd import SketchTable
from mahout_amd.synth import zipf_stream_torch

n, d, w = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000, 5, int(sys.argv[3]) if len(sys.argv) > 3 else 4096
pairs = int(sys.argv[2]) if len(sys.argv) > 2 else 50_000_000
Q = int(sys.argv[4]) if len(sys.argv) > 4 else 1024
Q0 = int(sys.argv[5]) if len(sys.argv) > 5 else 0
items, users = zipf_stream_torch(1_000_000 if n <= 100_000 else 10_000_000, n, pairs, device="cuda")
t = SketchTable(n, depth=d, width=w, seed=42, device=0)
t.ingest_device_rows(items, users, None, pairs)
t.finalize()
del items, users
t.set_timing(True)
t.top_k_rows(Q0, 128, 100)  # prepare + warm
t.reset_timing()
t0 = time.perf_counter()
ids, sc, cnt = t.top_k_rows(Q0, Q, 100)
dt = time.perf_counter() - t0
ms, nl = t.timing("cosine_mfma")
msm, nm = t.timing("cosine_mfma_multi")
msl, _ = t.timing("cosine_mfma_limbs")
mt, _ = t.timing("top_k")
ops = Q * n * 2 * d * w
print(json.dumps({"n": n, "w": w, "Q": Q, "wall_s": dt, "mfma_ms": ms, "multi_ms": msm, "limbs_ms": msl, "stats": t.stats(), "multi_launches": nm,
                  "topk_ms": mt, "TOPS_fast_kernel": ops / (ms * 1e-3) / 1e12,
                  "TOPS_all": ops / ((ms + msm + msl) * 1e-3) / 1e12, "pairs_per_s": Q * n / dt}))
