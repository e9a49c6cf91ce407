import ctypes, json, time
hip = ctypes.CDLL("libamdhip64.so")
hip.hipSetDevice(0); hip.hipDeviceSynchronize()
res = {}
for gb in (1, 4, 16, 24, 33, 41):
    p = ctypes.c_void_p(); t0 = time.perf_counter()
    rc = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(int(gb * 1e9)))
    res[f"{gb}GB_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
    t0 = time.perf_counter(); hip.hipFree(p); res[f"{gb}GB_free_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
print(json.dumps(res))
