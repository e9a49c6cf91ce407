"""Histogram of the owners' largest counter after the config-3 ingest (which
operand class the all-pairs job can give them: fp4 <= 4, fp6 e2m3 <= 7,
int8 single limb < 128, multi-limb)."""
import json
import sys

sys.path.insert(0, ".")
import numpy as np  # noqa: E402
import torch  # noqa: E402
from mahout_amd import SketchTable  # noqa: E402
from mahout_amd.synth import zipf_stream_torch  # noqa: E402

n, d, w, pairs = 1_000_000, 5, 8192, 500_000_000
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
t.synchronize()
del items, users
torch.cuda.empty_cache()
C = 8192
buf = torch.empty((C, d, w), dtype=torch.int32, device="cuda")
mx = np.zeros(n, np.int64)
for o in range(0, n, C):
    c = min(C, n - o)
    v = t.read_counters_device(o, c, buf[:c])
    mx[o:o + c] = v.view(c, -1).amax(dim=1).cpu().numpy()
edges = [0, 1, 5, 8, 16, 128, 1 << 14, 1 << 40]
h = {f"[{a},{b})": int(((mx >= a) & (mx < b)).sum()) for a, b in zip(edges[:-1], edges[1:])}
print(json.dumps({"rowmax_hist": h, "le7": int((mx <= 7).sum()), "le4": int((mx <= 4).sum())}))
