"""EXPERIMENT: achievable streaming-read rate on the bench's config-2 owner
column (400 MB int64) -- torch reductions and copies timed with events, to
calibrate k_p1_hist's ~3.4 TB/s."""
import json
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402
from mahout_amd.synth import zipf_stream_torch  # noqa: E402

items, users = zipf_stream_torch(1_000_000, 100_000, 50_000_000, seed=20261015, device="cuda")
out = {}


def timed(name, fn, nbytes, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    out[name] = {"ms": ms, "TBps": nbytes / ms / 1e9}


timed("sum_int64_400MB", lambda: items.sum(), 400e6)
timed("max_int64_400MB", lambda: items.max(), 400e6)
buf = torch.empty_like(items)
timed("copy_400MB_read+write", lambda: buf.copy_(items), 800e6)
big = torch.empty(1 << 30, dtype=torch.int64, device="cuda")
big.fill_(1)
timed("sum_int64_8GB", lambda: big.sum(), 8 * (1 << 30), reps=5)
timed("fill_8GB_write", lambda: big.fill_(3), 8 * (1 << 30), reps=5)
print(json.dumps(out))
