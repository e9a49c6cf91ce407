"""Config-5 incremental ingest rate on a resident 1M x 5 x 8192 table:
Zipf vs uniform batches of 1.25M pairs (owner-grouped atomic path)."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from mahout_amd import SketchTable  # noqa: E402
from mahout_amd.synth import zipf_stream_torch  # noqa: E402

n, d, w = 1_000_000, 5, 8192
t = SketchTable(n, depth=d, width=w, seed=42, device=0)
it_, us = zipf_stream_torch(10_000_000, n, 100_000_000, seed=1, device="cuda")
t.ingest_device_rows(it_, us, None, int(it_.numel()))
t.finalize()
del it_, us
res = {}
for kind in ["zipf", "uniform"]:
    bs = []
    for b in range(16):
        if kind == "zipf":
            bs.append(zipf_stream_torch(10_000_000, n, 1_250_000, seed=100 + b, device="cuda"))
        else:
            g = torch.Generator(device="cuda")
            g.manual_seed(b)
            bs.append((torch.randint(0, n, (1_250_000,), device="cuda", generator=g),
                       torch.randint(0, 10_000_000, (1_250_000,), device="cuda", generator=g)))
    t.ingest_device_rows(bs[0][0], bs[0][1], None, 1_250_000)
    t.synchronize()
    t.set_timing(True)
    t.reset_timing()
    t0 = time.perf_counter()
    for a, b in bs:
        t.ingest_device_rows(a, b, None, 1_250_000)
    t.synchronize()
    dt = time.perf_counter() - t0
    res[kind] = {"updates_per_s": 16 * 1_250_000 / dt, "batch_ms": dt * 1e3 / 16,
                 "timing": {k: t.timing(k) for k in ["partition", "ingest_atomic"]}}
    t.set_timing(False)
t0 = time.perf_counter()
t.finalize()
res["finalize_ms"] = (time.perf_counter() - t0) * 1e3
print(json.dumps(res))
