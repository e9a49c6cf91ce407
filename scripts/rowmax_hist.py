"""EXPERIMENT: distribution of the largest counter per owner at config 4
(1M items, d=5, w=8192, the 500M-pair config-3 stream) -- which operand
formats could carry each owner class exactly (fp4 e2m1: <= 4, fp6 e2m3:
<= 7, fp8 e4m3: <= 16, int8 limb: <= 127)."""
import json
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402
from mahout_amd import SketchTable  # noqa: E402
from mahout_amd.synth import zipf_stream_torch  # noqa: E402

n, pairs, w, d = 1_000_000, 500_000_000, 8192, 5
chunks, done, it = [], 0, 0
while done < pairs:
    m = min(1 << 26, pairs - done)
    chunks.append(zipf_stream_torch(10_000_000, n, m, seed=20261016 + 7919 * it, device="cuda"))
    done += m
    it += 1
items = torch.cat([c[0] for c in chunks])
users = torch.cat([c[1] for c in chunks])
del chunks
t = SketchTable(n, depth=d, width=w, seed=42, device=0)
t.ingest_device_rows(items, users, None, pairs)
t.finalize()
counts = torch.bincount(items, minlength=n)
del items, users
torch.cuda.empty_cache()
t.release_scratch()
mx = torch.empty(n, dtype=torch.int64, device="cuda")
step = 16384
buf = None
for r0 in range(0, n, step):
    rc = min(step, n - r0)
    buf = t.read_counters_device(r0, rc, out=None)
    mx[r0:r0 + rc] = buf.view(rc, -1).to(torch.int64).amax(dim=1)
edges = [0, 4, 7, 8, 15, 16, 31, 63, 127, 1 << 40]
hist = {}
lo = -1
for e in edges:
    hist[f"({lo},{e}]"] = int(((mx > lo) & (mx <= e)).sum())
    lo = e
# pairs per owner by class
cls = {"<=4": mx <= 4, "5..7": (mx > 4) & (mx <= 7), "8..16": (mx > 7) & (mx <= 16), "17..127": (mx > 16) & (mx <= 127),
       ">=128": mx > 127}
out = {"hist_rowmax": hist,
       "owners": {k: int(v.sum()) for k, v in cls.items()},
       "pairs": {k: int(counts[v].sum()) for k, v in cls.items()},
       "median_pairs": {k: float(counts[v].float().median()) if int(v.sum()) else None for k, v in cls.items()}}
print(json.dumps(out), flush=True)
