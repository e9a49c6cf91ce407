"""HBM write / copy rates on this box (torch fill and copy of a config-2-sized table)."""
import json
import time

import torch

n = 8_192_000_000
x = torch.empty(n, dtype=torch.uint8, device="cuda")
y = torch.empty(n // 8, dtype=torch.uint8, device="cuda")
res = {}
for name, fn, nbytes in [("fill", lambda: x.zero_(), n), ("fill_1gb", lambda: y.zero_(), n // 8),
                         ("copy_1gb", lambda: x[: n // 8].copy_(y), 2 * (n // 8))]:
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 10
    res[name] = {"ms": dt * 1e3, "GBps": nbytes / dt / 1e9}
print(json.dumps(res))
