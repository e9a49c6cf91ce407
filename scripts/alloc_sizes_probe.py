"""hipMalloc / hipFree times by size, idle and after other large frees (the
first all-pairs job's 41 GB operand copy allocated slowly in the bench).
Prints one JSON line."""
import ctypes
import json
import time

hip = ctypes.CDLL("libamdhip64.so")
hip.hipSetDevice(0)
hip.hipDeviceSynchronize()
res = {}


def alloc(gb):
    p = ctypes.c_void_p()
    t0 = time.perf_counter()
    rc = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(int(gb * 1e9)))
    if rc:
        raise SystemExit(f"hipMalloc {gb} GB: {rc}")
    return p, (time.perf_counter() - t0) * 1e3


def free(p):
    t0 = time.perf_counter()
    hip.hipFree(p)
    return (time.perf_counter() - t0) * 1e3


for gb in (1, 16, 41):
    p, ms = alloc(gb)
    res[f"idle_{gb}GB_ms"] = round(ms, 2)
    res[f"idle_{gb}GB_free_ms"] = round(free(p), 2)
# the bench's state: ~180 GB held (table, images, stream), ~13 GB of
# scratch in mid-sized buffers freed just before the job's allocations
held = [alloc(8)[0] for _ in range(22)]
scratch = [alloc(1.6)[0] for _ in range(8)]
t0 = time.perf_counter()
for p in scratch:
    free(p)
res["free_scratch_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
for gb in (24.6, 41, 33):
    p, ms = alloc(gb)
    res[f"after_frees_{gb}GB_ms"] = round(ms, 2)
    held.append(p)
for p in held:
    free(p)
print(json.dumps(res))
