"""How long device allocations take on this box (the first all-pairs job
allocates ~100 GB of operand images, candidate lists and slab; the bench's
"host_alloc" scope measured ~17 ms per GB through hipMalloc).

Times, per GB: hipMalloc, hipFree, hipMalloc of a size just freed, and
hipMallocAsync + stream sync from the device's default pool (whose freed
blocks stay reserved when the release threshold is raised).  Prints one JSON
line.  Usage: python scripts/alloc_probe.py [GB per allocation] [count]
"""
import ctypes
import json
import sys
import time

gb = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
count = int(sys.argv[2]) if len(sys.argv) > 2 else 4
hip = ctypes.CDLL("libamdhip64.so")
size = ctypes.c_size_t(int(gb * (1 << 30)))


def ok(rc, what):
    if rc != 0:
        raise SystemExit(f"{what}: hip error {rc}")


ok(hip.hipSetDevice(0), "hipSetDevice")
ok(hip.hipDeviceSynchronize(), "sync")
res = {"gb_per_alloc": gb, "count": count}

ptrs = [ctypes.c_void_p() for _ in range(count)]
t0 = time.perf_counter()
for p in ptrs:
    ok(hip.hipMalloc(ctypes.byref(p), size), "hipMalloc")
res["hipMalloc_ms_per_GB"] = (time.perf_counter() - t0) * 1e3 / (gb * count)
t0 = time.perf_counter()
for p in ptrs:
    ok(hip.hipFree(p), "hipFree")
res["hipFree_ms_per_GB"] = (time.perf_counter() - t0) * 1e3 / (gb * count)
t0 = time.perf_counter()
for p in ptrs:
    ok(hip.hipMalloc(ctypes.byref(p), size), "hipMalloc again")
res["hipMalloc_again_ms_per_GB"] = (time.perf_counter() - t0) * 1e3 / (gb * count)
for p in ptrs:
    ok(hip.hipFree(p), "hipFree")

pool = ctypes.c_void_p()
ok(hip.hipDeviceGetDefaultMemPool(ctypes.byref(pool), 0), "default pool")
thr = ctypes.c_uint64(2**64 - 1)
ok(hip.hipMemPoolSetAttribute(pool, 4, ctypes.byref(thr)), "release threshold")  # hipMemPoolAttrReleaseThreshold
stream = ctypes.c_void_p()
ok(hip.hipStreamCreate(ctypes.byref(stream)), "stream")
for rnd in ("first", "reuse"):
    t0 = time.perf_counter()
    for p in ptrs:
        ok(hip.hipMallocAsync(ctypes.byref(p), size, stream), "hipMallocAsync")
    ok(hip.hipStreamSynchronize(stream), "sync")
    res[f"hipMallocAsync_{rnd}_ms_per_GB"] = (time.perf_counter() - t0) * 1e3 / (gb * count)
    for p in ptrs:
        ok(hip.hipFreeAsync(p, stream), "hipFreeAsync")
    ok(hip.hipStreamSynchronize(stream), "sync")
# near capacity: hold most of the device, then time further allocations
free_b = ctypes.c_size_t()
total_b = ctypes.c_size_t()
ok(hip.hipMemGetInfo(ctypes.byref(free_b), ctypes.byref(total_b)), "meminfo")
res["total_GB"] = total_b.value / 1e9
hold = []
while True:
    ok(hip.hipMemGetInfo(ctypes.byref(free_b), ctypes.byref(total_b)), "meminfo")
    if free_b.value < (int(gb * (1 << 30)) + (40 << 30)):
        break
    p = ctypes.c_void_p()
    ok(hip.hipMalloc(ctypes.byref(p), size), "hold")
    hold.append(p)
res["held_GB"] = len(hold) * gb * (1 << 30) / 1e9
near = []
t0 = time.perf_counter()
for _ in range(count):
    ok(hip.hipMemGetInfo(ctypes.byref(free_b), ctypes.byref(total_b)), "meminfo")
    if free_b.value < int(gb * (1 << 30)) + (6 << 30):
        break
    p = ctypes.c_void_p()
    ok(hip.hipMalloc(ctypes.byref(p), size), "near")
    near.append(p)
res["near_full_allocs"] = len(near)
res["hipMalloc_near_full_ms_per_GB"] = (time.perf_counter() - t0) * 1e3 / (gb * max(1, len(near)))
for p in near + hold:
    ok(hip.hipFree(p), "free")
# while the device is busy: ~0.5 s of matmuls queued on torch's stream first
import torch  # noqa: E402
a = torch.randn(8192, 8192, device="cuda")
torch.cuda.synchronize()
for _ in range(40):
    a = a @ a
    a /= a.abs().max()
p = ctypes.c_void_p()
t0 = time.perf_counter()
ok(hip.hipMalloc(ctypes.byref(p), size), "busy")
res["hipMalloc_busy_ms"] = (time.perf_counter() - t0) * 1e3
t0 = time.perf_counter()
torch.cuda.synchronize()
res["queue_left_after_malloc_ms"] = (time.perf_counter() - t0) * 1e3
ok(hip.hipFree(p), "free")
print(json.dumps(res))
