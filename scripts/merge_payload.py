"""Packed-merge payload at bench scale, G ranks simulated on ONE GPU.

G SketchTables (one per rank) each ingest exactly the shard bench.py gives
rank g at world size G (config 2: 50M pairs per rank, 100K items, d=5,
w=4096), then all call cms_finalize_with concurrently from G threads; the
callback sums the G device buffers through host memory (a stand-in for the
RCCL all-reduce).  Reports the packed all-reduce payload per step against the
u32 table and the pack / unpack kernel times -- the parts of the multi-GPU
merge that do not need more than one GPU.

usage: python scripts/merge_payload.py [G ...]
"""
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from mahout_amd import SketchTable  # noqa: E402


def hip_runtime():
    with open("/proc/self/maps") as f:
        for line in f:
            path = line.split()[-1]
            if "libamdhip64.so" in path:
                lib = ctypes.CDLL(path)
                lib.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
                return lib
    raise RuntimeError("libamdhip64 not mapped")


def run(G, args, hip):
    dev = torch.device("cuda:0")
    tables = []
    for g in range(G):
        items, users = bench.rank_stream(args, g, G, dev)
        t = SketchTable(args.n_items, depth=args.depth, width=args.width, seed=42, device=0)
        t.ingest_device_rows(items, users, None, int(items.numel()))
        del items, users
        tables.append(t)
    torch.cuda.synchronize()
    bar = threading.Barrier(G)
    bufs = [None] * G
    calls = []

    def make_cb(g):
        def cb(ptr, count):
            host = np.empty(count, np.uint64)
            hip.hipMemcpy(host.ctypes.data, ptr, count * 8, 2)
            bufs[g] = host
            bar.wait()
            if g == 0:
                tot = bufs[0].copy()
                for x in bufs[1:]:
                    tot += x  # u64 sums, wrap-free by construction
                bufs[0] = tot
                calls.append(count)
            bar.wait()
            hip.hipMemcpy(ptr, bufs[0].ctypes.data, count * 8, 1)
            bar.wait()
        return cb

    for t in tables:
        t.set_timing(True)
    errs = []

    def work(g):
        try:
            tables[g].finalize_with(make_cb(g))
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))
            bar.abort()

    th = [threading.Thread(target=work, args=(g,)) for g in range(G)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    wall = time.perf_counter() - t0
    if errs:
        raise RuntimeError(errs)
    st = tables[0].stats()
    table_bytes = args.n_items * args.depth * args.width * 4
    rec = {"G": G, "pairs_per_rank": args.pairs, "allreduce_bytes": st["merge_words"] * 8,
           "u32_table_bytes": table_bytes, "payload_ratio": st["merge_words"] * 8 / table_bytes,
           "bounds_words": calls[0] if calls else None,
           "pack_ms": tables[0].timing("merge_pack")[0], "unpack_ms": tables[0].timing("merge_unpack")[0],
           "wall_s_host_transport": wall}
    # the merged tables are identical on every simulated rank
    a = tables[0].read_counters(0, 64)
    rec["ranks_agree"] = all(np.array_equal(a, t.read_counters(0, 64)) for t in tables[1:])
    for t in tables:
        t.close()
    torch.cuda.empty_cache()
    return rec


def main():
    class A:
        n_items, n_users, pairs, depth, width = 100_000, 1_000_000, 50_000_000, 5, 4096
    hip = hip_runtime()
    gs = [int(x) for x in sys.argv[1:]] or [2, 4, 8]
    out = [run(G, A, hip) for G in gs]
    for r in out:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
