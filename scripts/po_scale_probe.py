"""Per-owner shapes (CosineCM + CountMinSketchConfig) beyond config 1: the
config-2 stream (1M users x 100K items, 50M pairs) as the transposed
DataModel, CountMinSketchConfig(q=1) for all 100K items, then mostSimilar
top-100 for blocks of query rows over all 100K candidates.

usage: python scripts/po_scale_probe.py [rows_per_block] [whole_job_budget_s] [stream_seed]
(stream_seed 20261015 is bench.py's config-2 stream; the default 20261016 an independent one)

A heartbeat line goes to stderr every 30 s (a profiled run stays visibly alive)."""
import json
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import csr_on_device, per_owner_scale  # noqa: E402
from mahout_amd.synth import zipf_stream_torch  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 64
budget = float(sys.argv[2]) if len(sys.argv) > 2 else 120.0
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 20261016
t0 = time.perf_counter()


def beat():
    while True:
        time.sleep(30)
        print(f"... {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)


threading.Thread(target=beat, daemon=True).start()
items, users = zipf_stream_torch(1_000_000, 100_000, 50_000_000, seed=seed, device="cuda")
print(json.dumps(per_owner_scale(items, users, 100_000, 1_000_000, rows, budget)), flush=True)
print(f"total {time.perf_counter() - t0:.1f} s", file=sys.stderr)
