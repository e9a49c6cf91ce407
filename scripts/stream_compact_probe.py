"""Config-5 sustained stream on the headline table, compact rows against
whole slots (CMS_NO_COMPACT=1 in the environment): the bench's 10M-pair Zipf
batches into the resident 1M x 5 x 8192 table built from the 500M-pair
stream; per-batch wall times and the library's timing scopes."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from mahout_amd import SketchTable  # noqa: E402
from mahout_amd.synth import zipf_stream_torch  # noqa: E402

n, d, w = 1_000_000, 5, 8192
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 100
hold_gb = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0  # device memory held beside the table (the bench's config-4 buffers)
t = SketchTable(n, depth=d, width=w, seed=42, device=0)
it_, us = zipf_stream_torch(10_000_000, n, 500_000_000, seed=20261015, device="cuda")
t.ingest_device_rows(it_, us, None, int(it_.numel()))
t.finalize()
del it_, us
held = torch.empty(int(hold_gb * 1e9), dtype=torch.uint8, device="cuda") if hold_gb > 0 else None
torch.cuda.synchronize()
mem0 = torch.cuda.mem_get_info()
t.set_timing(True)
t.reset_timing()
lat = []
for b in range(nb):
    it_, us = zipf_stream_torch(10_000_000, n, 10_000_000, seed=555_000 + b, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    t.ingest_device_rows(it_, us, None, int(it_.numel()))
    torch.cuda.synchronize()
    lat.append((time.perf_counter() - t0) * 1e3)
    del it_, us
    if b % 10 == 0:
        print(f"batch {b}: {lat[-1]:.2f} ms, arena_map {t.timing('arena_map')}", file=sys.stderr, flush=True)
mem1 = torch.cuda.mem_get_info()
scopes = {k: t.timing(k) for k in ("ingest_sorted", "widen_rows", "partition", "build_plan", "arena_map")}
st = t.stats()
slow = sorted(range(nb), key=lambda i: -lat[i])[:3]
print(json.dumps({"batches": nb, "hold_gb": hold_gb, "slowest": [(i, round(lat[i], 2)) for i in slow], "total_ms": sum(lat), "mean_ms": sum(lat) / nb, "max_ms": max(lat),
                  "first5": [round(x, 2) for x in lat[:5]], "median_ms": sorted(lat)[nb // 2],
                  "scopes_ms": scopes, "table_bytes": st["table_bytes"],
                  "forms": {k: st[k] for k in ("hot_rows", "u8_rows", "nibble_rows", "crumb_rows", "bit_rows", "list_rows")},
                  "used_gb_after_build": (mem0[1] - mem0[0]) / 1e9, "used_gb_after_stream": (mem1[1] - mem1[0]) / 1e9}))
