#!/usr/bin/env python3
"""Benchmark: sketch updates/sec + item-pair cosines/sec @1M items on MI355X
(BASELINE.json metric).

Headline (`value`): config 3's shape, i.e. the metric's "@1M items" -- a
500M-pair Zipf stream (10M users x 1M items), d=5, w=8192.  One step = one
pass of the sketch-update hot path over the stream resident in HBM: reset,
then the rank's unordered COO (item, user) shard -> the finished
[1M][5][8192] sketch table (partition by owner, LDS row build with the zero
fill, norms and row maxima fused), then cms_finalize (with N ranks the packed
RCCL all-reduce of the counters, then the norms).  With N GPUs the same
500M-pair stream is user-hash sharded over the ranks (strong scaling: the
job is fixed, as config 3 states it).

Beside it in the same line: config 4 (all-pairs top-100 of every item on the
headline's table, cosines/s), config 5 (streaming batches + periodic
refresh on that table), config 2 (100K items, weak scaling) as a secondary
ingest line, config 1 (ML-100K shape), and the CPU baselines.

    python bench.py [--gpus N] [--steps K] [--warmup W]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (import before libmahout_cms: one HIP runtime per process)
import torch.distributed as dist  # noqa: E402

METRIC = "sketch updates/sec + item-pair cosines/sec @1M items, 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


_T0 = time.time()


def progress(msg):
    """A progress line on stderr (the JSON line stays the last stdout line):
    a long run keeps writing, so a watchdog can tell it from a hang."""
    print(f"bench-progress: {time.time() - _T0:7.1f} s {msg}", file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    # headline: config 3's shape (the metric's "@1M items")
    ap.add_argument("--n-items", type=int, default=1_000_000)
    ap.add_argument("--n-users", type=int, default=10_000_000)
    ap.add_argument("--pairs", type=int, default=500_000_000, help="pairs of the whole stream (sharded over ranks)")
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--width", type=int, default=8192)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--detail-out", default=None, help="also write the full record (one JSON line) to this file")
    ap.add_argument("--no-extras", action="store_true", help="skip the CSR, host-buffer and query side measurements")
    ap.add_argument("--no-config1", action="store_true")
    ap.add_argument("--no-config2", action="store_true", help="skip the config-2 (100K items) secondary ingest line")
    ap.add_argument("--no-cosine-1m", action="store_true", help="skip configs 4 and 5 on the headline table")
    ap.add_argument("--no-headline", action="store_true",
                    help="profiling aid: run the secondary lines only (no headline value is printed)")
    ap.add_argument("--stream-batches", type=int, default=4, help="config 5: refresh-phase batches (1.25M pairs per rank)")
    ap.add_argument("--stream-pairs", type=float, default=1e9, help="config 5: pairs of the sustained stream (per node)")
    ap.add_argument("--stream-batch", type=float, default=1e7, help="config 5: pairs per sustained-stream batch")
    ap.add_argument("--refresh-every", type=int, default=1,
                    help="config 5: batches between periodic top-k refreshes (cms_top_k_refresh)")
    ap.add_argument("--stream-refresh-multi", action="store_true",
                    help="also run the config-5 streaming phase with a communicator (delta all-gather)")
    return ap.parse_args()


def visible_gpu_count(env=None, kfd_nodes="/sys/class/kfd/kfd/topology/nodes"):
    """GPUs this process may use, WITHOUT initialising HIP (the parent of a
    self-launched multi-rank run must not touch the GPU before its children
    do): the KFD topology's GPU nodes (gpu_id != 0), narrowed by
    HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES when set."""
    env = os.environ if env is None else env
    n = 0
    try:
        for node in os.listdir(kfd_nodes):
            try:
                with open(os.path.join(kfd_nodes, node, "gpu_id")) as f:
                    if int(f.read().strip() or "0") != 0:
                        n += 1
            except (OSError, ValueError):
                continue
    except OSError:
        n = 0
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is not None:
            ids = [x for x in v.split(",") if x.strip() != ""]
            n = min(n, len(ids)) if v.strip() != "" else 0
    return n


def rank_stream(args, rank, world, device):
    """This rank's shard of the user-hash-sharded Zipf stream, on the GPU."""
    from mahout_amd.sketch import shard_of_keys
    from mahout_amd.synth import zipf_stream_torch
    if world == 1:
        return zipf_stream_torch(args.n_users, args.n_items, args.pairs, seed=20261015, device=device)
    shard_tbl = torch.from_numpy(shard_of_keys(np.arange(args.n_users, dtype=np.int64), world)).to(device)
    items_out = torch.empty(args.pairs, dtype=torch.int64, device=device)
    users_out = torch.empty(args.pairs, dtype=torch.int64, device=device)
    got, chunk, it = 0, 1 << 25, 0
    while got < args.pairs:
        it_, us = zipf_stream_torch(args.n_users, args.n_items, chunk, seed=20261015 + 7919 * it, device=device)
        keep = shard_tbl[us] == rank
        it_, us = it_[keep], us[keep]
        m = min(int(it_.numel()), args.pairs - got)
        items_out[got:got + m] = it_[:m]
        users_out[got:got + m] = us[:m]
        got += m
        it += 1
    return items_out, users_out


def csr_on_device(items, users, n):
    """Group the stream by owner on the GPU (setup only, untimed)."""
    order = torch.argsort(items, stable=True)
    ckeys = users[order].contiguous()
    del order
    off = torch.zeros(n + 1, dtype=torch.int64, device=items.device)
    off[1:] = torch.cumsum(torch.bincount(items, minlength=n), 0)
    return off, ckeys


def per_owner_scale(items, users, n, n_users, rows=1024, all_pairs_budget_s=120.0):
    """The reference's native per-owner mode beyond
    config 1: the stream as the transposed DataModel (n items keyed by user),
    CountMinSketchConfig(q=1) shapes for every item (CountMinSketchConfig.java:
    120-158, on the GPU), then mostSimilar top-100 (userSimilarity(u1, u2)
    hashes u1 at u2's shape, CosineCM.java:83-96) for two blocks of `rows`
    query items (rows n/2.. and 0..; the stream permutes item IDs, so both are
    random samples of the items), each over all n candidates, then the whole
    all-pairs top-100 when the pooled block rate predicts it within
    `all_pairs_budget_s`."""
    from mahout_amd import SketchTable
    off, ckeys = csr_on_device(items, users, n)
    po = {"workload": f"{int(items.numel())}-pair DataModel, {n} items x {n_users} users; CountMinSketchConfig(q=1) "
                      f"per item, top-100 of {rows}-item query blocks over all {n} candidates (ordered pairs), "
                      f"then the whole all-pairs top-100 of every item"}
    with SketchTable.per_owner_shapes(n, seed=42) as t:
        t.ingest_csr_device(off, ckeys)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        t.configure_owner_shapes(1.0, n_users)
        po["configure_s"] = time.perf_counter() - t0
        t.finalize()
        _, _, ws, ds = t.owner_shapes()
        po["width_range"] = [int(ws.min()), int(ws.max())]
        po["depth_range"] = [int(ds.min()), int(ds.max())]
        po["sketch_counters"] = int((ws.astype(np.int64) * ds).sum())
        t.top_k_rows(n // 2, 1, 100)  # warm
        for name, r0 in (("median", n // 2), ("head", 0)):
            t0 = time.perf_counter()
            _, _, cnt = t.top_k_rows(r0, rows, 100)
            dt = time.perf_counter() - t0
            st = t.stats()
            po[f"{name}_rows"] = {"first_row": r0, "rows": rows, "s": dt, "ordered_pairs_per_s": rows * n / dt,
                                  "full_lists": int((cnt == 100).sum()),
                                  "wide_pairs_bounded_total": st["po_wide_pairs"],
                                  "wide_pairs_exact_total": st["po_wide_exact"]}
        # the WHOLE all-pairs top-100 (every one of the n*(n-1) ordered pairs),
        # when the block rates predict it finishes within all_pairs_budget_s
        # (zipf_stream_torch permutes the item IDs, so both blocks are random
        # samples of the items: their pooled rate predicts the whole job)
        rate = 2 * rows * n / (po["median_rows"]["s"] + po["head_rows"]["s"])
        po["all_pairs_predicted_s"] = n * n / rate
        if n * n / rate <= all_pairs_budget_s:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            _, _, cnt = t.top_k_all(100)
            dt = time.perf_counter() - t0
            po["all_pairs"] = {"s": dt, "ordered_pairs": n * (n - 1), "ordered_pairs_per_s": n * (n - 1) / dt,
                               "full_lists": int((cnt == 100).sum()),
                               "path": "narrow candidates grouped by (w, d) class (k_po_group_pairs; k_po_bigq for "
                                       "queries of > 4096 preferences); wide owners and the widest narrow part "
                                       "bounded by sketch row 0 against each query's narrow top-k "
                                       "(k_po_wide_bound), the survivors exact (k_po_pairs)",
                               "wide_pairs_bounded_total": t.stats()["po_wide_pairs"],
                               "wide_pairs_exact_total": t.stats()["po_wide_exact"]}
    del off, ckeys
    return po


def host_threads():
    """Threads the CPU baselines may use: the run's OpenMP share (16 on a
    1-GPU box, where nproc reports the whole machine), else the affinity set."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0))


def host_cpu_info():
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)), "threads_used": host_threads(),
            "model": model}


BASELINE_NOTE = ("C restatement of the reference path (oracle/cms_baseline.c), not the JVM (no JDK here): it has no "
                 "BigInteger allocation, no log.debug varargs boxing and no TDoubleArrayList growth, so it is faster "
                 "than the reference it stands in for")


def _timed_blocks(fn, n_rows, block, budget_s):
    """Run fn(lo, hi) over consecutive row blocks (wrapping) until budget_s;
    returns (units done, rows done, seconds)."""
    done, rows, lo = 0, 0, 0
    t0 = time.perf_counter()
    dt = 0.0
    while dt < budget_s:
        hi = min(n_rows, lo + block)
        done += fn(lo, hi)
        rows += hi - lo
        lo = 0 if hi >= n_rows else hi
        dt = time.perf_counter() - t0
    return done, rows, dt


def cpu_baseline(off_d, keys_d, args, budget_s=3.0):
    """Sketch ingest on the host cores, two modes x {1 thread, all threads}
    (oracle/cms_baseline.c):
      faithful  -- the reference cost model: per owner a fresh fp64 sketch
                   (w*d zero fill) and d BigInteger-equivalent (128-bit
                   division) hashes per update;
      efficient -- u32 counters in one shared table, the exact hash by folding
                   2^63 = 25 (mod p).
    Sample: the rank-0 stream's owners in ID order, blocks of owners, about
    budget_s per leg.  `value` is the faithful mode on all threads."""
    from oracle import oracle as O
    off = off_d.cpu().numpy()
    keys = keys_d.cpu().numpy()
    a, b = O.hash_params(42, args.depth)
    n = off.size - 1
    T = host_threads()
    table = np.empty(4096 * args.depth * args.width, np.uint32)
    modes = {}
    for mode in ("faithful", "efficient"):
        for th in (1, T):
            if mode == "faithful":
                fn = lambda lo, hi: O.ingest_faithful(off, keys, None, lo, hi, args.depth, args.width, a, b, th)[0]  # noqa: E731
            else:
                fn = lambda lo, hi: O.ingest_efficient(off, keys, None, lo, hi, args.depth, args.width, a, b, th,  # noqa: E731
                                                       table)[0]
            block = 512 if th == 1 else 4096
            upd, rows, dt = _timed_blocks(fn, n, block, budget_s)
            modes[f"{mode}_{th}t"] = {"updates_per_s": upd / dt, "threads": th, "owners": rows, "updates": upd,
                                      "seconds": round(dt, 2)}
    best = max(modes.values(), key=lambda m: m["updates_per_s"])
    return {"value": modes[f"faithful_{T}t"]["updates_per_s"], "unit": "updates/s", "cores": T, "kind": "port",
            "sample": f"rank-0 config-2 stream, owners in ID order (blocks of 512 / 4096 owners), ~{budget_s:.0f} s per "
                      f"leg; value = faithful mode (fp64 sketch per owner, 128-bit BigInteger-equivalent hash) on "
                      f"{T} threads",
            "modes": modes, "best_updates_per_s": best["updates_per_s"], "host": host_cpu_info(), "note": BASELINE_NOTE}


def query_latency(table, n, calls=2000, threads=8):
    """The drop-in's per-call cost: CosineCM.userSimilarity(u1, u2) as one
    cms_similarity from the host (CosineCMGpu's route), serially and from 8
    threads at once (queries after finalize share the handle: leased streams
    and scratch, MultithreadedBatchItemSimilarities.java:78)."""
    import threading
    rng = np.random.Generator(np.random.PCG64(9))
    a = rng.integers(0, n, calls)
    b = rng.integers(0, n, calls)
    for i in range(50):
        table.similarity(int(a[i]), int(b[i]))
    t0 = time.perf_counter()
    for i in range(calls):
        table.similarity(int(a[i]), int(b[i]))
    serial = (time.perf_counter() - t0) / calls

    def worker(k):
        for i in range(k, calls, threads):
            table.similarity(int(a[i]), int(b[i]))

    ths = [threading.Thread(target=worker, args=(k,)) for k in range(threads)]
    t0 = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    dt = time.perf_counter() - t0
    batch = rng.integers(0, n, 10_000)
    table.similarities(int(a[0]), batch)
    t0 = time.perf_counter()
    for i in range(20):
        table.similarities(int(a[i]), batch)
    bdt = (time.perf_counter() - t0) / 20
    return {"single_pair_us": serial * 1e6, "threads": threads, "threaded_pairs_per_s": calls / dt,
            "batched_10k_pairs_ms": bdt * 1e3, "batched_pairs_per_s": batch.size / bdt,
            "note": "cms_similarity per call from Python ctypes (host round trip + one k_pair_cosine launch); "
                    "itemSimilarities(id, ids[]) as one batched call"}


def cosine_cpu_baseline(items, users, n, d, w, budget_s=3.0, sample_owners=192, seed=5):
    """Config-4 similarity on the host cores, two modes x {1 thread, all
    threads} (oracle/cms_baseline.c):
      faithful  -- the CosineCM cost model: u1's fp64 sketch rebuilt per call
                   (exportProfile), u2's from the cache, min-over-rows cosine;
      efficient -- every sketch prebuilt, per-(owner, row) norms once, one fp64
                   dot per row pair, four partners per sweep.
    Sample: `sample_owners` random items of the config-3/4 stream with all
    their (item, user) pairs; pairs of the sample until the budget."""
    from oracle import oracle as O
    from mahout_amd.synth import to_csr
    rng = np.random.Generator(np.random.PCG64(seed))
    pick = np.sort(rng.choice(n, size=sample_owners, replace=False))
    sel = torch.isin(items, torch.from_numpy(pick).to(items.device))
    it = items[sel].cpu().numpy()
    us = users[sel].cpu().numpy()
    rows = np.searchsorted(pick, it)
    off, keys, _ = to_csr(rows, us, sample_owners)
    a, b = O.hash_params(42, d)
    S = sample_owners
    T = host_threads()
    pi, pj = np.triu_indices(S, 1)
    pi, pj = pi.astype(np.int64), pj.astype(np.int64)
    table = O.build_table(S, d, w, a, b, rows, us)
    modes = {}
    for th in (1, T):
        chunk = 256 * th
        done, _, dt = _timed_blocks(lambda lo, hi: O.faithful_pairs_par(off, keys, None, S, d, w, a, b, pi[lo:hi],
                                                                         pj[lo:hi], th)[0], pi.size, chunk, budget_s)
        modes[f"faithful_{th}t"] = {"pairs_per_s": done / dt, "threads": th, "pairs": done, "seconds": round(dt, 2)}
        rows_per = max(1, 2 * th)
        done, _, dt = _timed_blocks(lambda lo, hi: O.allpairs_efficient(table, lo, hi, th)[0], S, rows_per, budget_s)
        modes[f"efficient_{th}t"] = {"pairs_per_s": done / dt, "threads": th, "pairs": done, "seconds": round(dt, 2)}
    best = max(modes.values(), key=lambda m: m["pairs_per_s"])
    return {"value": modes[f"faithful_{T}t"]["pairs_per_s"], "unit": "item-pair cosines/s", "cores": T, "kind": "port",
            "sample": f"{S} random items of the config-3/4 stream ({int(keys.size)} pairs), d={d} w={w}, unordered "
                      f"pairs of the sample, ~{budget_s:.0f} s per leg; value = faithful CosineCM cost model on {T} threads",
            "modes": modes, "best_pairs_per_s": best["pairs_per_s"], "host": host_cpu_info(), "note": BASELINE_NOTE}


def config1(budget_s=3.0):
    """Config 1 (BASELINE.json configs[0], the JVM-CPU-only case): the
    ML-100K-shaped stand-in through a transposed DataModel (1682 item sketches
    keyed by user, d=4, w=1024, integer ratings), every one of the 1,413,721
    unordered item pairs.  CPU: the efficient mode on all threads is timed over
    ALL pairs; the faithful mode on all threads over all pairs when that fits
    the budget, else over a row prefix (extrapolated, labelled); the 1-thread
    legs over row prefixes (extrapolated).  GPU: the same table ingested and
    the top-100 of every item through cms_top_k_all (every pair computed)."""
    from oracle import oracle as O
    from mahout_amd import SketchTable
    from mahout_amd.synth import movielens_like, to_csr
    users, items, ratings = movielens_like()
    ids = np.unique(items)
    rows = np.searchsorted(ids, items)
    n, d, w = ids.size, 4, 1024
    total = n * (n - 1) // 2
    off, keys, vals = to_csr(rows, users, n, ratings)
    a, b = O.hash_params(42, d)
    table = O.build_table(n, d, w, a, b, rows, users, ratings)
    T = host_threads()
    out = {"workload": f"config 1: ML-100K-shaped stand-in ({users.size} ratings, {n} items x "
                       f"{np.unique(users).size} users), transposed, d={d} w={w}; all {total} unordered item pairs",
           "pairs": total}
    cpu = {}
    for th in (T, 1):
        # efficient: prebuilt sketches
        t0 = time.perf_counter()
        if th == T:
            done, _ = O.allpairs_efficient(table, 0, n, th)
            dt = time.perf_counter() - t0
            cpu[f"efficient_{th}t"] = {"pairs_per_s": done / dt, "seconds": round(dt, 2), "extrapolated": False,
                                       "full_job_s": dt}
        else:
            done, r, dt = _timed_blocks(lambda lo, hi: O.allpairs_efficient(table, lo, hi, 1)[0], n, 8, budget_s)
            cpu[f"efficient_{th}t"] = {"pairs_per_s": done / dt, "seconds": round(dt, 2), "extrapolated": True,
                                       "full_job_s": total / (done / dt)}
        # faithful: u1 rebuilt per call, u2 cached; query rows in order
        pi, pj = np.triu_indices(n, 1)
        pi, pj = pi.astype(np.int64), pj.astype(np.int64)
        done, _, dt = _timed_blocks(lambda lo, hi: O.faithful_pairs_par(off, keys, vals, n, d, w, a, b, pi[lo:hi],
                                                                         pj[lo:hi], th)[0],
                                    total, 65536 * max(1, th // 4), budget_s)
        cpu[f"faithful_{th}t"] = {"pairs_per_s": done / dt, "seconds": round(dt, 2), "extrapolated": done < total,
                                  "full_job_s": total / (done / dt)}
    out["cpu"] = cpu
    out["cpu_threads"] = T
    out["cpu_note"] = BASELINE_NOTE
    with SketchTable(n, depth=d, width=w, seed=42, owner_ids=ids) as t:
        t.ingest(items, users, ratings)
        t.finalize()
        t.top_k_all(100)  # operands prepared, kernels warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _, _, cnt = t.top_k_all(100)
        dt = time.perf_counter() - t0
    out["gpu"] = {"top100_all_items_s": dt, "unique_item_pair_cosines_per_s": total / dt,
                  "full_lists": int((cnt == 100).sum())}
    # the reference's native per-owner mode: CosineCM with
    # CountMinSketchConfig(q=1) -- every item its own (d, w) from the Fmeasure
    # search, u1 hashed at u2's shape; all n*(n-1) ORDERED pairs (asymmetric)
    po = {}
    with SketchTable.per_owner_shapes(n, seed=42, owner_ids=ids) as t:
        t.ingest_csr(off, keys, vals)
        t0 = time.perf_counter()
        t.configure_owner_shapes(1.0, np.unique(users).size)
        po["configure_s"] = time.perf_counter() - t0
        t.finalize()
        _, eps, ws, ds = t.owner_shapes()
        t.top_k_all(100)  # warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _, _, cnt = t.top_k_all(100)
        dt = time.perf_counter() - t0
        po.update({"workload": "CountMinSketchConfig(q=1) shapes per item; top-100 of every item over all ordered "
                               "pairs (userSimilarity(u1, u2) hashes u1 at u2's shape)",
                   "ordered_pairs": n * (n - 1), "top100_all_items_s": dt,
                   "ordered_pairs_per_s": n * (n - 1) / dt, "full_lists": int((cnt == 100).sum()),
                   "width_range": [int(ws.min()), int(ws.max())], "depth_range": [int(ds.min()), int(ds.max())],
                   "sketch_counters": int((ws.astype(np.int64) * ds).sum())})
    out["gpu_per_owner_shapes"] = po
    out["recommender"] = config1_recommender()
    return out


def config1_recommender(nn=50, how_many=10, reps=5):
    """The fork's use case on config 1's data:
    GenericUserBasedRecommender.recommend(user, 10) for ALL 943 users of the
    ML-100K-shaped stand-in (user-owner orientation: sketches keyed by item
    ID, d=4, w=1024), NearestNUserNeighborhood(50) and the CosineCM
    point-query estimate with EstimatedPreferenceCapper
    (GenericUserBasedRecommender.java:84-184, NearestNUserNeighborhood.java:
    84-95).  GPU: the package's mahout_amd.taste.GenericUserBasedRecommender
    .recommend_all -- every neighbourhood from one cms_top_k_all, then
    cms_recommend_batch (FastIDSet candidates and TopItems.getTopItems with
    the JDK heap's tie order in the library, every estimate in one device
    batch); timed end to end over `reps` runs after a warm-up.  The same call
    is checked list for list against per-user recommend() for all 943 users by
    tests/test_gpu_recommender.py::test_recommend_all_equals_recommend_for_every_user.
    CPU beside it: oracle/cms_baseline.c orc_recommend_par (prebuilt fp64
    sketches, the same neighbourhood / candidates / estimates) on all the
    run's threads and on one."""
    from oracle import oracle as O
    from mahout_amd import taste
    from mahout_amd.datamodel import GenericDataModel
    from mahout_amd.synth import movielens_like, to_csr
    users, items, ratings = movielens_like()
    uid, iid = np.unique(users), np.unique(items)
    ur, ir = np.searchsorted(uid, users), np.searchsorted(iid, items)
    nu, ni, d, w = uid.size, iid.size, 4, 1024
    order = np.lexsort((items, ur))  # GenericDataModel: each user's preferences by item ID
    moff = np.zeros(nu + 1, np.int64)
    np.cumsum(np.bincount(ur, minlength=nu), out=moff[1:])
    model = GenericDataModel.from_csr(uid, moff, items[order], ratings[order])
    cap = (float(ratings.min()), float(ratings.max()))
    out = {"workload": f"GenericUserBasedRecommender.recommend(user, {how_many}) for all {nu} users of the "
                       f"ML-100K-shaped stand-in ({users.size} ratings, {ni} items), NearestNUserNeighborhood({nn}), "
                       f"CosineCM d={d} w={w} point-query estimates, EstimatedPreferenceCapper{cap}",
           "users": nu, "path": "mahout_amd.taste.GenericUserBasedRecommender.recommend_all (cms_top_k_all + "
                                "cms_recommend_batch)"}
    sim = taste.CosineCM(model, taste.FixedShapeConfig(d, w), taste.HashFunctionBuilder(42))
    try:
        rec = taste.GenericUserBasedRecommender(model, taste.NearestNUserNeighborhood(nn, sim, model), sim)
        rec.recommend_all(uid, how_many)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            lists = rec.recommend_all(uid, how_many)
        dt = (time.perf_counter() - t0) / reps
    finally:
        sim.close()
    rvals = np.array([float(v) for lst in lists for _, v in lst], np.float64)
    out["gpu"] = {"all_users_s": dt, "users_per_s": nu / dt,
                  "recommended_checksum": float(rvals.sum()),
                  "full_lists": int(sum(len(lst) == how_many for lst in lists))}
    a, b = O.hash_params(42, d)
    table = O.build_table(nu, d, w, a, b, ur, items, ratings)
    off, keys_idx, _ = to_csr(ur, ir, nu, ratings)
    cpu = {}
    T = host_threads()
    for th in (T, 1):
        hi = nu if th == T else max(1, nu // 8)
        t0 = time.perf_counter()
        nest, cs = O.recommend_par(table, a, b, off, keys_idx.astype(np.int32), iid, nn, how_many, 0, hi, th, cap)
        dt = time.perf_counter() - t0
        cpu[f"efficient_{th}t"] = {"users_per_s": hi / dt, "estimates_per_s": nest / dt, "users": int(hi),
                                   "seconds": round(dt, 3), "extrapolated": hi < nu}
        if th == T:
            cpu[f"efficient_{th}t"]["candidate_estimates"] = int(nest)
            cpu[f"efficient_{th}t"]["recommended_checksum"] = cs
    out["cpu"] = cpu
    out["cpu_threads"] = T
    out["cpu_note"] = BASELINE_NOTE
    out["vs_cpu_all_threads"] = out["gpu"]["users_per_s"] / cpu[f"efficient_{T}t"]["users_per_s"]
    # the recommended value multisets agree (tied items may differ only in ID order on the CPU side)
    cs_all = cpu[f"efficient_{T}t"]["recommended_checksum"]  # the all-users leg
    out["checksum_equal"] = bool(abs(out["gpu"]["recommended_checksum"] - cs_all) <= 1e-9 * max(1.0, abs(cs_all)))
    return out


PROFILE_DIR = os.path.join(ROOT, "profiles", "r06")  # this round's committed rocprofv3 summaries


def _pmc_file(name):
    path = os.path.join(PROFILE_DIR, name)
    return path if os.path.exists(path) else None


def _pmc_lookup(summary, kernel):
    """`kernel`'s record; a name with a `*` matches any one template
    argument there (the ring depth of k_cosine_sym is a build constant)."""
    if "*" not in kernel:
        return summary.get(kernel)
    import re
    pat = re.compile(re.escape(kernel).replace(r"\*", r"[^,<>]+") + "$")
    return next((v for k, v in summary.items() if pat.match(k)), None)


def pmc_record(kernel, name):
    """This round's committed PMC summary record of `kernel` (or {})."""
    path = _pmc_file(name)
    if not path:
        return {}
    rec = _pmc_lookup(json.load(open(path)), kernel) or {}
    return {k: v for k, v in rec.items() if k != "counters_avg_per_dispatch"}


def pmc_traffic(kernel, name="pmc_summary.json"):
    """HBM bytes per launch of `kernel` from this round's committed PMC summary
    (profiles/r03/<name>, scripts/profile.sh on the same bench command:
    2 * FETCH_SIZE + WRITE_SIZE, gfx950 FETCH correction); (None, None) when
    that profile is not committed (a stale round's numbers are never used)."""
    path = _pmc_file(name)
    if not path:
        return None, None
    rec = _pmc_lookup(json.load(open(path)), kernel)
    val = (rec.get("hbm_bytes_per_launch") or rec.get("fetch_bytes_per_dispatch")) if rec else None
    return val, os.path.relpath(path, ROOT)


INT8_MFMA_PEAK_TOPS = 5000.0  # dense int8 MFMA (2x the 2.5 PF bf16 dense peak), MI355X_MICROARCH.md
FP4_MFMA_PEAK_TOPS = 10000.0  # dense fp4 (e2m1) MFMA, MI355X_MICROARCH.md (FP6/FP4 ~10 PF dense)


def allpairs_measure(table, row_begin, row_count, k, n, d, w):
    """cms_top_k_rows over [row_begin, row_begin+row_count): every query row
    against all n owners (n^2-shaped slab, no symmetry), HIP-event kernel times.
    Kernels: cosine_mfma = single-limb x single-limb 256x128 tiles (the bulk),
    cosine_mfma_limbs = multi-limb owners as virtual limb rows (M x S, S x M),
    cosine_mfma_multi = multi x multi 128-tiles (int64 folding), top_k."""
    table.set_timing(True)
    table.top_k_rows(row_begin, min(row_count, 128), k)  # operands prepared, kernels warm
    table.reset_timing()
    t0 = time.perf_counter()
    _, _, cnt = table.top_k_rows(row_begin, row_count, k)
    wall = time.perf_counter() - t0
    mf, nf = table.timing("cosine_mfma")
    ml, _ = table.timing("cosine_mfma_limbs")
    mm, nm = table.timing("cosine_mfma_multi")
    tk, _ = table.timing("top_k")
    table.set_timing(False)
    st = table.stats()
    n_multi = max(0, int(st["multi_limb_owners"]))
    pairs = row_count * n
    ops = pairs * 2 * d * w
    ops_ss = row_count * (n - n_multi) * 2 * d * w  # query rows here are single-limb owners
    kern_s = (mf + ml + mm) * 1e-3
    return {
        "query_rows": row_count, "candidates": n, "k": k, "wall_s": wall,
        "ordered_pairs_per_s": pairs / wall,
        "unique_item_pair_cosines_per_s": pairs / 2 / wall,
        "multi_limb_owners": n_multi, "top_k_redo_rows": int(st["topk_redo"]),
        "mfma_ms": mf, "mfma_limb_rows_ms": ml, "mfma_multi_multi_ms": mm, "top_k_ms": tk,
        "single_limb_kernel_TOPS": ops_ss / (mf * 1e-3) / 1e12 if mf else None,
        "single_limb_kernel_frac_int8_peak": ops_ss / (mf * 1e-3) / 1e12 / INT8_MFMA_PEAK_TOPS if mf else None,
        "all_cosine_kernels_TOPS": ops / kern_s / 1e12 if kern_s else None,
        "all_cosine_kernels_frac_int8_peak": ops / kern_s / 1e12 / INT8_MFMA_PEAK_TOPS if kern_s else None,
        "returned_full_lists": int((cnt == k).sum()),
    }


def config3_shard(n_items, n_users, total_pairs, rank, world, device, seed=20261016):
    """This rank's share of the config-3 stream (the same global stream on
    every rank, kept where cms_shard_of_key(user) == rank)."""
    from mahout_amd.sketch import shard_of_keys
    from mahout_amd.synth import zipf_stream_torch
    shard_tbl = None
    if world > 1:
        shard_tbl = torch.from_numpy(shard_of_keys(np.arange(n_users, dtype=np.int64), world)).to(device)
    out_i, out_u = [], []
    chunk, done, it = 1 << 26, 0, 0
    while done < total_pairs:  # the same chunked global stream for every world size
        m = min(chunk, total_pairs - done)
        it_, us = zipf_stream_torch(n_users, n_items, m, seed=seed + 7919 * it, device=device)
        if shard_tbl is not None:
            keep = shard_tbl[us] == rank
            it_, us = it_[keep], us[keep]
        out_i.append(it_)
        out_u.append(us)
        done += m
        it += 1
    return torch.cat(out_i), torch.cat(out_u)


# (the depth-unrolled kernels carry the handle's depth as a template argument)
BUILD_KERNELS = ["void cms::k_build_slices<*>", "void cms::k_build_rows<2>", "void cms::k_build_nibbles<2, *>",
                 "void cms::k_build_mid<2, *, *>", "void cms::k_build_bytes<2>"]


def build_roofline(table, local_pairs, build_ms, build_n, pmc_kernel, pmc_file):
    """Roofline of the row build (the "build_rows" scope: k_build_slices for
    the split owners, k_build_rows for other slot rows, k_build_mid,
    k_build_nibbles, k_build_bytes -- the ingest's dominant phase).

    Algorithmic bytes per launch = what the row build must move for the table
    as it is stored: the grouped key tokens read once (4 B per pair: the COO
    partition hands the build u32 tokens, cms_device.h Keys), the owner spans
    (2 x 8 B per owner) and every counter written once at its stored width
    (4-bit / u8 / u16 narrow rows, u32 hot rows: cms_stats.stored_bytes).  SURVEY 8(d)
    prices every counter at 4 B; that figure is reported beside it as
    `u32_priced_*` -- it exceeds the bytes the kernel has to move, so a
    fraction of it is not a bandwidth fraction and can pass 1.  `traffic` is
    the measured HBM bytes per launch of the same kernel (2 x FETCH_SIZE +
    WRITE_SIZE, gfx950 FETCH correction) from the committed profile."""
    st = table.stats()
    n, d, w = table.num_owners, table.depth, table.width
    stored = int(st["stored_bytes"])
    alg = local_pairs * 4 + n * 16 + stored
    u32_alg = local_pairs * 4 + (n + 1) * 8 + n * d * w * 4
    avg_s = build_ms / build_n * 1e-3 if build_n else None
    # the scope's kernels each run once per build: their measured bytes add up
    kernels = pmc_kernel if isinstance(pmc_kernel, (list, tuple)) else [pmc_kernel]
    parts = [pmc_traffic(kn, pmc_file) for kn in kernels]
    traffic = sum(p[0] for p in parts) if parts and all(p[0] for p in parts) else None
    src = parts[0][1] if parts else None
    out = {"bound": "hbm",
           "kernel": "build_rows scope: " + " + ".join(kn.replace("void cms::", "").replace("cms::", "") for kn in kernels),
           "achieved": alg / avg_s / 1e9 if avg_s else None, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
           "frac": alg / avg_s / 1e9 / HBM_PEAK_GBPS if avg_s else None,
           "traffic": traffic, "traffic_source": src,
           "frac_traffic": traffic / avg_s / 1e9 / HBM_PEAK_GBPS if traffic and avg_s else None,
           "algorithmic_bytes_per_launch": alg,
           "algorithmic_bytes_basis": "key tokens 4 B/pair + spans 16 B/owner + counters at stored width "
                                      f"({int(st['list_rows'])} list rows, {int(st['bit_rows'])} 1-bit rows, "
                                      f"{int(st['crumb_rows'])} 2-bit rows, "
                                      f"{int(st['nibble_rows'])} 4-bit rows, {int(st['u8_rows'])} u8 rows, "
                                      f"{n - int(st['hot_rows']) - int(st['list_rows']) - int(st['bit_rows']) - int(st['crumb_rows']) - int(st['nibble_rows']) - int(st['u8_rows'])} u16 rows, "
                                      f"{int(st['hot_rows'])} u32 rows)",
           "avg_launch_ms": avg_s * 1e3 if avg_s else None,
           "u32_priced_bytes_per_launch": u32_alg,
           "u32_priced_GBps": u32_alg / avg_s / 1e9 if avg_s else None}
    return out


def ingest_steps(table, items, users, npairs, steps, warmup, world, breakdown_names):
    """`warmup` untimed then `steps` timed steps of reset + device COO ingest +
    finalize, bracketed by barrier + synchronize, max over ranks; HIP events
    on the library's stream around k_build_rows only (timing level 1); then a
    separate pass of <= 5 steps with every phase scope timed."""
    def step():
        table.reset()
        table.ingest_device_rows(items, users, None, npairs)
        table.finalize()

    def barrier():
        table.synchronize()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    for _ in range(warmup):
        step()
    table.set_timing(True, level=1)
    table.reset_timing()
    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    build_ms, build_n = table.timing("build_rows")
    ar_ms, ar_n = table.timing("allreduce")
    table.set_timing(True, level=2)
    table.reset_timing()
    bsteps = max(1, min(steps, 5))
    for _ in range(bsteps):
        step()
    table.synchronize()
    breakdown = {}
    for name in breakdown_names:
        ms, n_ = table.timing(name)
        if n_:
            breakdown[name] = round(ms / bsteps, 4)
    table.set_timing(False)
    barrier()
    return {"elapsed_s": elapsed, "ms_per_step": elapsed * 1e3 / steps, "build_ms": build_ms, "build_n": build_n,
            "allreduce_ms_per_step": ar_ms / ar_n if ar_n else None, "breakdown_ms_per_step": breakdown,
            "breakdown_source": f"{bsteps} extra steps after the timed region with every phase scope event-timed"}


BREAKDOWN = ["partition", "build_plan", "build_rows", "hot_norms", "reduce_hot", "norms", "merge_bounds", "merge_pack",
             "allreduce", "merge_unpack"]


def csr_prefix_on_device(items, users, n_owners):
    """CSR of the owners [0, n_owners) of a COO stream (the CPU baseline's
    sample), on the GPU (setup only, untimed)."""
    sel = items < n_owners
    it, us = items[sel], users[sel]
    return csr_on_device(it, us, n_owners)


def hbm_used_gb(device):
    free, total = torch.cuda.mem_get_info(device)
    return (total - free) / 1e9


def cosine_1m(args, t, local, device, rank, world, bar, max_over_ranks):
    """Config 4 on the config-3 table the headline just built: mostSimilar
    top-100 for EVERY one of the 1M items through cms_top_k_all -- each
    unordered pair computed once (fp4 / int8 MFMA, exact fp64 epilogue) and
    streamed into both items' lists; with G ranks the pairs are split G ways
    and the partial lists all-gathered and merged (strong scaling: the job
    is fixed).  Then config 5 (streaming + periodic refresh) on the same
    resident table."""
    n, d, w, k = t.num_owners, t.depth, t.width, 100
    t.set_timing(True)
    t.top_k_rows(0, 128, k)  # limb operands prepared, kernels warm (local work)
    # one untimed job: the blocked operand images and the candidate lists are
    # allocated and written once per table (the timed job is the steady state)
    t.reset_timing()
    first_t0 = time.perf_counter()
    progress("config 4: first all-pairs job")
    t.top_k_all_device(k)
    progress("config 4: steady job")
    first_job_s = time.perf_counter() - first_t0
    # GPU time of the first job's scopes (HIP events); the rest of its wall is
    # host work: the operand images' and candidate lists' first allocations
    first_scopes = {name: t.timing(name)[0] for name in ["limb_prep", "topk_all_multi_rows", "cosine_mfma_limbs",
                                                         "cosine_mfma_multi", "topk_all_waves", "topk_merge",
                                                         "host_alloc", "host_free"]}
    first_scopes["host_alloc_GB"] = t.timing("host_alloc_bytes")[0] / 1e9  # bytes the first job allocated
    mx_ms, mx_bytes = t.timing("host_alloc_max")
    first_scopes["host_alloc_max_ms"] = mx_ms
    first_scopes["host_alloc_max_GB"] = mx_bytes / 1e9
    t.reset_timing()
    bar()
    t0 = time.perf_counter()
    _, _, cnt = t.top_k_all_device(k)  # lists stay in HBM (no 1.6 GB host copy in the timed job)
    bar()
    wall = max_over_ranks(time.perf_counter() - t0)
    used_gb = max_over_ranks(hbm_used_gb(device))  # operand images, slab, candidate lists still held
    cnt = cnt.cpu().numpy()
    tm = {name: t.timing(name)[0] for name in ["topk_all_multi_rows", "topk_all_limbs", "topk_all_waves",
                                               "topk_allgather", "topk_merge"]}
    waves_ms, waves_n = t.timing("topk_all_waves")
    f4_ms, f4_n = t.timing("topk_all_waves_f4")
    i8_ms, i8_n = t.timing("topk_all_waves_i8")
    ml_ms, ml_n = t.timing("cosine_mfma_limbs")  # k_cosine_mls: the multi-limb x single-limb slab blocks
    t.set_timing(False)
    st = t.stats()
    stream = None
    if world == 1 or args.stream_refresh_multi:
        stream = streaming_refresh(t, args, n, k, rank, world, device, bar, max_over_ranks)
    nm = max(0, int(st["multi_limb_owners"]))
    ndeep = max(0, int(st["deep_limb_owners"]))
    ml_hw_ops = (4 * ndeep + 2 * (nm - ndeep)) * (n - nm) * 2 * d * w / world
    uniq = n * (n - 1) / 2
    alg_ops = uniq * 2 * d * w  # F = n(n-1)/2 * 2dw
    ns = n - nm
    nf = max(0, int(st["fp4_owners"]))
    wave_ops = ns * (ns - 1) / 2 * 2 * d * w / world  # this rank's share of the waves
    # the waves feed two datatypes: fp4 x fp4 block pairs (owners whose
    # counters are all <= 4) on the fp4 MFMA, the rest on int8; each share is
    # priced at its own dense peak, so `peak` is the mix's ideal rate
    f4_ops = nf * (nf - 1) / 2 * 2 * d * w / world
    i8_ops = wave_ops - f4_ops
    wave_peak = wave_ops / (f4_ops / FP4_MFMA_PEAK_TOPS + i8_ops / INT8_MFMA_PEAK_TOPS) if wave_ops else None
    job_f4 = nf * (nf - 1) / 2 * 2 * d * w
    job_peak = alg_ops / (job_f4 / FP4_MFMA_PEAK_TOPS + (alg_ops - job_f4) / INT8_MFMA_PEAK_TOPS)
    wave_ach = wave_ops / (waves_ms * 1e-3) / 1e12 if waves_ms else None
    cos_traffic = pmc_traffic("void cms::k_cosine_sym<*, 64, 1, 8>", "cosine_pmc_summary.json")
    cos_pmc = pmc_record("void cms::k_cosine_sym<*, 64, 1, 8>", "cosine_pmc_summary.json")
    cos_pmc8 = pmc_record("void cms::k_cosine_sym<*, 64, 0, 8>", "cosine_pmc_summary.json")
    cos_pmcm = pmc_record("void cms::k_cosine_mls<2>", "cosine_pmc_summary.json")
    return {
        "workload": f"config 4: top-{k} most similar items for every one of the {n} items of the config-3 table "
                    f"(d={d} w={w}; {world} GPU(s), pairs split over the ranks, partial lists all-gathered)",
        "n_gpus": world, "scaling": "strong",
        "unique_item_pair_cosines_per_s": uniq / wall,
        "wall_s": wall,
        "first_job_s": first_job_s,
        "first_job_scopes_ms": {k_: round(v_, 2) for k_, v_ in first_scopes.items() if v_},
        "hbm_used_gb": used_gb,
        "algorithmic_TOPS": alg_ops / wall / 1e12,
        "frac_int8_peak_per_gpu": alg_ops / wall / 1e12 / INT8_MFMA_PEAK_TOPS / world,
        "mixed_peak_TOPS": job_peak,
        "frac_mixed_peak_per_gpu": alg_ops / wall / 1e12 / job_peak / world,
        # dominant kernel: the fp4 symmetric waves (k_cosine_sym<NS,64,1>, the
        # largest share of the job); its avg launch matches rocprofv3's for that name
        "roofline": {"bound": "mfma", "kernel": "k_cosine_sym<NS,64,1> (fp4 symmetric waves)",
                     "achieved": f4_ops / (f4_ms * 1e-3) / 1e12 if f4_ms else None,
                     "peak": FP4_MFMA_PEAK_TOPS, "unit": "TOP/s",
                     "frac": f4_ops / (f4_ms * 1e-3) / 1e12 / FP4_MFMA_PEAK_TOPS if f4_ms else None,
                     "avg_launch_ms": f4_ms / f4_n if f4_n else None,
                     "algorithmic_ops_per_launch": f4_ops / f4_n if f4_n else None,
                     "traffic": cos_traffic[0], "traffic_unit": "bytes per launch (2 x FETCH_SIZE)",
                     "traffic_source": cos_traffic[1],
                     "pmc_mfma_busy_frac": cos_pmc.get("mfma_busy_frac"), "pmc_l2_hit": cos_pmc.get("l2_hit")},
        "roofline_int8_waves": {"bound": "mfma", "kernel": "k_cosine_sym<NS,64,0> (int8 symmetric waves)",
                                "pmc_mfma_busy_frac": cos_pmc8.get("mfma_busy_frac"),
                                "achieved": i8_ops / (i8_ms * 1e-3) / 1e12 if i8_ms else None,
                                "peak": INT8_MFMA_PEAK_TOPS, "unit": "TOP/s",
                                "frac": i8_ops / (i8_ms * 1e-3) / 1e12 / INT8_MFMA_PEAK_TOPS if i8_ms else None,
                                "avg_launch_ms": i8_ms / i8_n if i8_n else None},
        "roofline_all_waves": {"achieved": wave_ach, "peak": wave_peak, "unit": "TOP/s",
                               "peak_basis": f"fp4 {FP4_MFMA_PEAK_TOPS:.0f} TOP/s for the fp4 x fp4 pairs, int8 "
                                             f"{INT8_MFMA_PEAK_TOPS:.0f} TOP/s for the rest, weighted by their ops",
                               "frac": wave_ach / wave_peak if wave_ach and wave_peak else None,
                               "ms": waves_ms, "launches": waves_n},
        "multi_limb_block": {"kernel": "k_cosine_mls<LS> (multi-limb x single-limb slab blocks, 256 x 192 tiles)",
                             "ms": ml_ms, "launches": ml_n,
                             "hw_int8_ops": ml_hw_ops,
                             "hw_frac_int8_peak": ml_hw_ops / (ml_ms * 1e-3) / 1e12 / INT8_MFMA_PEAK_TOPS if ml_ms else None,
                             "hw_ops_basis": "limb slots x single-limb owners x 2dw (each limb is an int8 pass)",
                             "pmc_mfma_busy_frac": cos_pmcm.get("mfma_busy_frac"), "pmc_l2_hit": cos_pmcm.get("l2_hit")},
        "fp4_owners": nf,
        "timing_ms_rank0": tm,
        "multi_limb_owners": nm, "full_lists": int((cnt == k).sum()), "topk_redo_rows": int(st["topk_redo"]),
        "config5_streaming": stream,
    }


def streaming_refresh(t, args, n, k, rank, world, device, bar, max_over_ranks):
    """Config 5 on the resident 1M-item table (BASELINE configs[4]: a 1B-pair
    stream at 10M pairs/s, incremental sketch + periodic top-k refresh).

    Sustained ingest: the whole 1B-pair stream (per node; user-hash sharded
    over the ranks) in batches of 10M pairs -- one second of the stream each --
    through the incremental path (grouped by owner, k_ingest_sorted: exact
    atomics that keep norms and row maxima current), each batch generated
    outside the timed region; one finalize at the end (with G ranks: the delta
    logs all-gathered and applied).  Periodic refresh: after the stream, short
    batches of 1.25M pairs (an eighth of a second of the stream) each followed
    by finalize + cms_top_k_refresh_device, against the whole job that builds
    the kept lists."""
    from mahout_amd.sketch import shard_of_keys
    from mahout_amd.synth import zipf_stream_torch
    shard_tbl = None
    if world > 1:
        shard_tbl = torch.from_numpy(shard_of_keys(np.arange(10_000_000, dtype=np.int64), world)).to(device)

    def batch(seed, size):
        it_, us = zipf_stream_torch(10_000_000, n, size, seed=seed, device=device)
        if shard_tbl is not None:
            keep = shard_tbl[us] == rank
            it_, us = it_[keep], us[keep]
        return it_.contiguous(), us.contiguous()

    # ---- sustained ingest of the 1B-pair stream ----
    progress("config 5: stream")
    t.set_timing(True)
    t.reset_timing()
    total = int(args.stream_pairs)
    bsize = int(args.stream_batch)
    nbatch = (total + bsize - 1) // bsize
    ingest_s, local, worst, worst_b = 0.0, 0, 0.0, -1
    lat = []
    for b in range(nbatch):
        it_, us = batch(555_000 + b, min(bsize, total - b * bsize))
        bar()
        t0 = time.perf_counter()
        t.ingest_device_rows(it_, us, None, int(it_.numel()))
        bar()
        dt = max_over_ranks(time.perf_counter() - t0)
        ingest_s += dt
        lat.append(dt)
        if dt > worst:
            worst, worst_b = dt, b
        local += int(it_.numel())
        del it_, us
    t0 = time.perf_counter()
    t.finalize()
    bar()
    fin_s = max_over_ranks(time.perf_counter() - t0)
    sorted_ms, sorted_n = t.timing("ingest_sorted")
    atomic_ms, atomic_n = t.timing("ingest_atomic")
    kern = "k_ingest_sorted" if sorted_n else "k_ingest_atomic"
    kern_ms, kern_n = (sorted_ms, sorted_n) if sorted_n else (atomic_ms, atomic_n)
    alg = local * (16 + 2 * 5 * 4)
    sustained = {
        "stream_pairs": total, "batch_pairs": bsize, "batches": nbatch,
        "ingest_s": ingest_s, "finalize_s": fin_s,
        "sustained_updates_per_s": total / ingest_s,
        "x_realtime": (total / ingest_s) / 10e6,  # the stream arrives at 10M pairs/s
        "batch_latency_ms": ingest_s * 1e3 / nbatch, "batch_latency_max_ms": worst * 1e3, "slowest_batch": worst_b,
        "widen_ms": t.timing("widen_rows")[0], "arena_map_ms": t.timing("arena_map"),
        "arena_map_parts_ms": {k: t.timing("arena_map_" + k)[0] for k in ("create", "map", "access")},
        # the first batches move the touched compact rows to slots of their
        # own, mapping arena memory (host time in arena_map_ms, box-dependent);
        # the rate over the later batches is the table's steady state
        "steady_updates_per_s": (bsize * len(lat[10:]) / sum(lat[10:])) if len(lat) > 10 else None,
        "path": f"{kern} (batches of >= 32768 pairs into a live table are grouped by owner first and take "
                "k_ingest_sorted: exact u32 global atomics, norm / row-max / mass deltas reduced per owner inside the "
                "wave; smaller batches take k_ingest_atomic)",
        "roofline": {"bound": "hbm", "kernel": kern, "algorithmic_bytes_per_update": 56,
                     "note": "SURVEY 8(d) prices an incremental update at 56 B of streaming traffic; the kernel's d "
                             "counter updates per pair are scattered single-dword atomics (one 64-B sector RMW each), "
                             "whose measured ceiling is far below the streaming rate (DESIGN 4.1)",
                     "achieved": alg / (kern_ms * 1e-3) / 1e9 if kern_n else None, "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": alg / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS if kern_n else None,
                     "avg_launch_ms": kern_ms / kern_n if kern_n else None},
    }

    # ---- periodic refresh ----
    per_batch = 1_250_000
    nb = max(1, args.stream_batches)
    batches = [batch(777_000 + b, per_batch * world) for b in range(nb)]
    # owners the batches touch: the refresh recomputes every pair with a
    # touched owner, i.e. 1 - (1 - f)^2 of the pairs for a touched fraction f
    touched_all = torch.unique(torch.cat([b[0] for b in batches])).numel() / n
    touched_one = sum(torch.unique(b[0]).numel() for b in batches) / (n * nb)
    every = max(1, args.refresh_every)
    # the periodic refresh keeps 2k-deep lists: one whole job builds them
    scope_names = ["limb_prep", "topk_all_multi_rows", "cosine_mfma_limbs", "cosine_mfma_multi", "topk_all_waves_f4",
                   "topk_all_waves_i8", "topk_merge", "top_k", "cosine_mfma", "host_alloc", "host_free"]

    def scopes():  # GPU time of the job's phases (HIP events, this rank)
        return {nm: round(t.timing(nm)[0], 1) for nm in scope_names if t.timing(nm)[0]}

    t.set_timing(True)
    t.reset_timing()
    bar()
    t0 = time.perf_counter()
    t.top_k_refresh_device(k)
    bar()
    keep_s = max_over_ranks(time.perf_counter() - t0)
    keep_scopes = scopes()
    periods = []
    cnt = None
    for bi, (it_, us) in enumerate(batches):
        bar()
        t.ingest_device_rows(it_, us, None, int(it_.numel()))
        bar()
        if (bi + 1) % every == 0 or bi == nb - 1:
            t0 = time.perf_counter()
            t.finalize()  # with G ranks: the delta logs all-gathered and applied
            bar()
            fs = max_over_ranks(time.perf_counter() - t0)
            t.reset_timing()
            t0 = time.perf_counter()
            _, _, cnt = t.top_k_refresh_device(k)  # lists stay in HBM (Refreshable consumers read them there)
            bar()
            rs = max_over_ranks(time.perf_counter() - t0)
            touched, redone, full = t.refresh_stats()
            periods.append({"after_batch": bi + 1, "finalize_s": round(fs, 5), "refresh_s": round(rs, 4),
                            "touched_owner_frac": touched / n, "lists_redone": redone, "whole_jobs": full,
                            "classes": t.refresh_classes(), "scopes_ms": scopes()})
    cnt = cnt.cpu().numpy()
    t.set_timing(False)
    del batches
    lat = [p["finalize_s"] + p["refresh_s"] for p in periods]
    all_pairs = n * (n - 1) / 2
    recomputed_rate = sum((1 - (1 - p["touched_owner_frac"]) ** 2) * all_pairs / p["refresh_s"]
                          for p in periods) / len(periods)
    whole_rate = all_pairs / keep_s

    def class_work(p):
        # The pairs a refresh must redo, per operand class, priced at the whole
        # job's own per-pair time for that class: multi-limb rows (every pair
        # with a multi-limb owner), int8 waves (int8 x int8 and int8 x fp4) and
        # fp4 waves.  Touched owners are the frequent ones, so they sit in the
        # costly classes: this is the refresh's time at the whole job's per-pair
        # cost, class by class.
        c = p["classes"]
        (m, tm), (i8, ti), (f4, tf) = c["multi"], c["int8"], c["fp4"]
        um, ui, uf = m - tm, i8 - ti, f4 - tf

        def tri(x):
            return x * (x - 1) / 2
        frac = {"multi": 1 - (um * (ui + uf) + tri(um)) / max(1, m * (i8 + f4) + tri(m)),
                "i8": 1 - (ui * uf + tri(ui)) / max(1, i8 * f4 + tri(i8)),
                "f4": 1 - tri(uf) / max(1, tri(f4))}
        scope = {"multi": "topk_all_multi_rows", "i8": "topk_all_waves_i8", "f4": "topk_all_waves_f4"}
        whole_ms = {k: keep_scopes.get(v, 0.0) for k, v in scope.items()}
        return frac, sum(whole_ms[k] * frac[k] for k in frac) / 1e3

    class_fracs, expect = zip(*[class_work(p) for p in periods])
    return {
        "workload": f"config 5: a {total}-pair Zipf stream (10M pairs/s) into the resident {n}-item table in "
                    f"{bsize}-pair batches; then {nb} batches of {per_batch} pairs per GPU, every {every} batch(es) "
                    f"finalize + incremental top-{k} refresh of every item (cms_top_k_refresh)",
        "sustained": sustained,
        "sustained_updates_per_s": sustained["sustained_updates_per_s"],
        "steady_updates_per_s": sustained["steady_updates_per_s"],
        "path": sustained["path"],
        "roofline": sustained["roofline"],
        "refresh_batches": nb, "pairs_per_batch_per_gpu": per_batch,
        "refresh_every_batches": every,
        "keep_lists_whole_job_s": keep_s,
        "keep_lists_whole_job_scopes_ms": keep_scopes,
        "refresh_latency_s": sum(lat) / len(lat),
        "refresh_latency_max_s": max(lat),
        # unique pairs with a touched owner (the ones a refresh recomputes) per second
        "refresh_recomputed_pairs_per_s": recomputed_rate,
        # ... against the whole job's unique pairs per second (1.0: a refresh is as efficient per pair)
        "refresh_pair_rate_vs_whole_job": recomputed_rate / whole_rate,
        "refresh_vs_whole_job": keep_s / (sum(lat) / len(lat)),
        # per class: the fraction of the class's pairs a refresh must redo, and the refresh time those pairs
        # would take at the whole job's per-pair time for their class (1.0: the refresh redoes them as fast)
        "refresh_class_pair_fracs": [{k: round(v, 4) for k, v in f.items()} for f in class_fracs],
        "refresh_s_at_whole_job_class_rates": sum(expect) / len(expect),
        "refresh_class_weighted_rate_vs_whole_job": (sum(expect) / len(expect)) / (sum(p["refresh_s"] for p in periods)
                                                                                 / len(periods)),
        # the refresh latency in arrival intervals: one interval = the time one refresh batch (all ranks)
        # takes to arrive at 10M pairs/s (0.125 s per 1.25M-pair batch on one GPU, 1 s on eight)
        "batch_interval_s": per_batch * world / 10e6,
        "refresh_latency_in_batch_intervals": (sum(lat) / len(lat)) / (per_batch * world / 10e6),
        "refresh_periods": periods,
        "full_lists": int((cnt == k).sum()),
        "touched_owner_frac": {"all_batches": touched_all, "per_batch": touched_one,
                               "pairs_to_recompute_all_batches": 1 - (1 - touched_all) ** 2,
                               "pairs_to_recompute_per_batch": 1 - (1 - touched_one) ** 2},
    }


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n, child_argv, port=None, timeout=None):
    """One process per GPU when bench.py is started without a launcher:
    children get RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT
    exactly as torch.distributed.run sets them (127.0.0.1 rendezvous).  No
    GPU is touched here.  Returns non-zero if any rank fails."""
    import subprocess
    port = port or _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(child_argv, env=env))
    rcs = [None] * n
    try:
        for r, p in enumerate(procs):
            rcs[r] = p.wait(timeout=timeout)
            if rcs[r] != 0:  # a failed rank would leave the others waiting in a collective
                for q in procs:
                    if q.poll() is None:
                        q.kill()
    finally:
        for r, p in enumerate(procs):
            if p.poll() is None:
                p.kill()
            rcs[r] = p.wait()
    bad = [r for r, c in enumerate(rcs) if c != 0]
    if bad:
        print(f"bench: ranks {bad} failed (exit codes {[rcs[r] for r in bad]})", file=sys.stderr)
        return 1
    return 0


def config2_line(args, rank, world, local, device):
    """Config 2 (BASELINE configs[1]): Zipf 1M users x 100K items, 50M pairs
    per rank (weak scaling), d=5, w=4096 -- the round-1/2 headline, kept as a
    secondary ingest line with its own roofline; single-GPU extras (CSR and
    host-buffer ingest, query latency, all-pairs top-100 on this table)."""
    from mahout_amd import SketchTable, comm_unique_id
    c2 = argparse.Namespace(n_users=1_000_000, n_items=100_000, pairs=50_000_000)
    n, d, w = c2.n_items, 5, 4096
    table = SketchTable(n, depth=d, width=w, seed=42, device=local)
    if world > 1:
        uid = [comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        table.comm_init(uid[0], rank, world)
    items, users = rank_stream(c2, rank, world, device)
    npairs = int(items.numel())
    torch.cuda.synchronize()
    steps = max(args.steps, 10)
    m = ingest_steps(table, items, users, npairs, steps, max(args.warmup, 2), world, BREAKDOWN)
    value = npairs * world * steps / m["elapsed_s"]
    roof = build_roofline(table, npairs, m["build_ms"], m["build_n"], BUILD_KERNELS,
                          "pmc_summary_config2.json")
    table_bytes_u32 = n * d * w * 4
    out = {
        "workload": f"config 2: Zipf {c2.n_users} users x {n} items, {npairs} pairs per rank, d={d} w={w}; unordered "
                    "COO (item, user) stream -> finished sketch table + norms (+ packed all-reduce with N ranks)",
        "scaling": "weak", "steps": steps, "updates_per_s": value, "ms_per_step": m["ms_per_step"],
        "roofline": roof,
        "step_roofline": {"algorithmic_bytes": npairs * 16 + table.stats()["stored_bytes"],
                          "basis": "stream read once (16 B/pair) + counters written once at stored width",
                          "achieved_GBps": (npairs * 16 + table.stats()["stored_bytes"]) / (m["ms_per_step"] * 1e-3) / 1e9,
                          "frac": (npairs * 16 + table.stats()["stored_bytes"]) / (m["ms_per_step"] * 1e-3) / 1e9
                          / HBM_PEAK_GBPS,
                          "u32_priced_frac": (npairs * 16 + table_bytes_u32) / (m["ms_per_step"] * 1e-3) / 1e9
                          / HBM_PEAK_GBPS},
        "breakdown_ms_per_step": m["breakdown_ms_per_step"],
        "allreduce_ms_per_step": m["allreduce_ms_per_step"],
    }
    if world > 1:
        mw = table.stats()["merge_words"]
        out["merge"] = {"allreduce_bytes_per_step": mw * 8, "u32_table_bytes": table_bytes_u32,
                        "payload_ratio": mw * 8 / table_bytes_u32}
    if rank == 0 and world == 1 and not args.no_extras:
        extras = {}
        off, ckeys = csr_on_device(items, users, n)
        # CSR (DataModel layout) ingest of the same stream: no partition pass
        table.reset()
        table.ingest_csr_device(off, ckeys)
        table.finalize()
        table.synchronize()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            table.reset()
            table.ingest_csr_device(off, ckeys)
            table.finalize()
        table.synchronize()
        dt = time.perf_counter() - t0
        extras["csr_updates_per_s"] = npairs * steps / dt
        extras["csr_ms_per_step"] = dt * 1e3 / steps
        del off, ckeys
        # the same stream handed over in HOST memory (cms_ingest: PCIe copy +
        # validation + the device path), i.e. the JNI boundary's rate
        h_items = items.cpu().numpy()
        h_users = users.cpu().numpy()
        table.reset()
        table.ingest(h_items, h_users)
        table.finalize()
        t0 = time.perf_counter()
        for _ in range(3):
            table.reset()
            table.ingest(h_items, h_users)
            table.finalize()
        dt = time.perf_counter() - t0
        extras["host_buffers_updates_per_s"] = npairs * 3 / dt
        del h_items, h_users
        extras["query_latency"] = query_latency(table, n)
        # all-pairs top-100 over the config-2 table: per-row slab path, then
        # the symmetric streaming pass (each unordered pair once)
        extras["allpairs_top100_cfg2"] = allpairs_measure(table, 0, n, 100, n, d, w)
        t0 = time.perf_counter()
        _, _, cnt_all = table.top_k_all_device(100)
        dt = time.perf_counter() - t0
        extras["allpairs_top100_cfg2_streaming"] = {
            "wall_s": dt, "unique_item_pair_cosines_per_s": n * (n - 1) / 2 / dt,
            "full_lists": int((cnt_all == 100).sum().item())}
        out["extras"] = extras
    table.close()
    torch.cuda.empty_cache()
    if "extras" in out:
        # the reference's per-owner-shape mode at this scale (SURVEY 8(f) rank
        # 2), on the same stream, with the fixed-shape table released first
        progress("config 2: per-owner shapes")
        out["extras"]["per_owner_shapes_cfg2"] = per_owner_scale(items, users, n, c2.n_users)
    del items, users
    torch.cuda.empty_cache()
    return out


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # self-launch: one rank per GPU; this parent never initialises HIP
        have = visible_gpu_count()
        if have < args.gpus:
            print(f"bench: --gpus {args.gpus} but only {have} GPU(s) visible", file=sys.stderr)
            sys.exit(2)
        sys.exit(spawn_ranks(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    torch.cuda.set_device(local)
    device = f"cuda:{local}"
    if world > 1:
        dist.init_process_group("gloo", init_method="env://")  # control plane only; data path is RCCL in the lib

    from mahout_amd import SketchTable, comm_unique_id

    def bar():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    def max_over_ranks(x):
        if world == 1:
            return x
        v = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
        return float(v.item())

    # secondary lines first (their tables are freed before the 82 GB headline table)
    progress("config 2 line")
    config2 = None if args.no_config2 else config2_line(args, rank, world, local, device)
    cfg1 = None
    progress("config 1")
    if rank == 0 and world == 1 and not args.no_config1 and not args.no_extras:
        cfg1 = config1()

    if args.no_headline:
        if rank == 0:
            print(json.dumps({"metric": METRIC, "value": None, "note": "--no-headline (profiling aid)",
                              "config2": config2, "config1": cfg1}))
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    # ---- headline: config 3's shape ----
    progress("headline ingest")
    n, d, w = args.n_items, args.depth, args.width
    table = SketchTable(n, depth=d, width=w, seed=42, device=local)
    if world > 1:
        uid = [comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        table.comm_init(uid[0], rank, world)
    items, users = config3_shard(n, args.n_users, args.pairs, rank, world, device)
    npairs = int(items.numel())
    torch.cuda.synchronize()
    m = ingest_steps(table, items, users, npairs, args.steps, args.warmup, world, BREAKDOWN)
    value = args.pairs * args.steps / m["elapsed_s"]  # the whole stream per step, over all ranks
    roof = build_roofline(table, npairs, m["build_ms"], m["build_n"], BUILD_KERNELS, "pmc_summary.json")
    st = table.stats()
    stored = int(st["stored_bytes"])
    step_bytes = npairs * 16 + stored  # per GPU: its shard read once + its full table written once
    u32_step_bytes = npairs * 16 + n * d * w * 4  # SURVEY 8(d)'s B_g (4 B per counter)
    result = {
        "metric": METRIC,
        "value": value,
        "unit": "updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": m["ms_per_step"],
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,  # no published number for this path
        "dtype": "u32",
        "data": "synthetic Zipf stream (items ~ rank^-1.1, users ~ rank^-0.9), generated on the GPU, resident in HBM",
        "config": {
            "workload": f"config 3 shape (@1M items): Zipf {args.n_users} users x {n} items, {args.pairs}-pair stream "
                        f"user-hash sharded over {world} GPU(s) ({npairs} pairs on rank {rank}), d={d} w={w}; one "
                        "step = reset + unordered COO shard -> finished sketch table + norms"
                        + (" + packed RCCL all-reduce of the counters" if world > 1 else ""),
            "n_items": n, "n_users": args.n_users, "pairs": args.pairs, "pairs_per_rank": npairs, "depth": d,
            "width": w,
            "sharding": "user-hash (splitmix64) across ranks; RCCL all-reduce of the counters, counter-width-adaptive "
                        "packed (bit-identical to a u32 sum)",
        },
        "roofline": roof,
        "step_roofline": {"algorithmic_bytes_per_gpu": step_bytes,
                          "basis": "shard read once (16 B/pair) + every counter written once at stored width",
                          "achieved_GBps": step_bytes / (m["ms_per_step"] * 1e-3) / 1e9,
                          "frac": step_bytes / (m["ms_per_step"] * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                          "u32_priced_bytes_per_gpu": u32_step_bytes,
                          "u32_priced_GBps": u32_step_bytes / (m["ms_per_step"] * 1e-3) / 1e9},
        "breakdown_ms_per_step": m["breakdown_ms_per_step"],
        "breakdown_source": m["breakdown_source"],
        "allreduce_ms_per_step": m["allreduce_ms_per_step"],
        "table": {"stored_bytes": stored, "hot_rows": int(st["hot_rows"]), "u32_bytes": n * d * w * 4},
    }
    if world > 1:
        mw = st["merge_words"]
        result["merge"] = {"allreduce_bytes_per_step": mw * 8, "u32_table_bytes": n * d * w * 4,
                           "payload_ratio": mw * 8 / (n * d * w * 4)}
    progress("headline done; CPU baseline")
    if rank == 0 and not args.no_cpu_baseline:
        # bounded sample of the same workload: the owners [0, 65536) of rank 0's
        # shard (IDs are a seeded permutation of popularity ranks, so an ID
        # prefix is a popularity-unbiased sample)
        off, ckeys = csr_prefix_on_device(items, users, 65536)
        result["cpu_baseline"] = cpu_baseline(off, ckeys, args)
        result["cpu_baseline"]["sample"] = ("owners [0, 65536) of the config-3-shape stream (rank 0's shard), in ID "
                                            "order, blocks of 512 / 4096 owners, ~3 s per leg; value = faithful mode "
                                            "(fp64 sketch per owner, 128-bit BigInteger-equivalent hash) on "
                                            f"{result['cpu_baseline']['cores']} threads")
        result["vs_cpu_baseline"] = value / result["cpu_baseline"]["value"]
        del off, ckeys
    # device memory in use on the busiest rank (hipMemGetInfo: the library's
    # allocations and torch's), with this rank's input stream still resident
    result["memory"] = {"total_gb": torch.cuda.mem_get_info(device)[1] / 1e9,
                        "used_after_ingest_gb": max_over_ranks(hbm_used_gb(device)),
                        "basis": "max over ranks of (total - free) from hipMemGetInfo"}
    cos_cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.no_cosine_1m:
        cos_cpu = cosine_cpu_baseline(items, users, n, d, w)
    del items, users
    torch.cuda.empty_cache()
    progress("config 4 / 5")
    if not args.no_cosine_1m:
        try:
            table.release_scratch()
            cos = cosine_1m(args, table, local, device, rank, world, bar, max_over_ranks)
            cos["cpu_baseline"] = cos_cpu
            if rank == 0:
                result["cosine"] = cos
                result["memory"]["used_during_cosine_gb"] = cos.get("hbm_used_gb")
        except Exception as e:  # the headline line must still be printed
            if rank == 0:
                result["cosine"] = {"error": f"{type(e).__name__}: {e}"}
    table.close()
    if config2 is not None:
        result["config2"] = config2
    if cfg1 is not None:
        result["config1"] = cfg1
    if rank == 0:
        cos = result.get("cosine") or {}
        if "unique_item_pair_cosines_per_s" in cos:  # the metric's cosine half as top-level keys
            result["cosines_per_s"] = cos["unique_item_pair_cosines_per_s"]
            result["cosine_wall_s"] = cos["wall_s"]
            result["cosine_first_job_s"] = cos["first_job_s"]
            result["cosine_roofline"] = {k: cos["roofline"].get(k) for k in
                                         ("bound", "achieved", "peak", "unit", "frac", "avg_launch_ms",
                                          "pmc_mfma_busy_frac", "pmc_l2_hit")}
            result["cosine_roofline"]["kernel"] = "k_cosine_sym fp4"
        result["summary"] = summary(result)
        # the whole record (config 1/2 extras, the cosine and config-5 objects)
        # goes to stderr and, with --detail-out, to a file; stdout ends with
        # ONE compact line (<= COMPACT_LIMIT chars) that the driver parses
        full = json.dumps(result)
        print("bench-detail: " + full, file=sys.stderr, flush=True)
        if args.detail_out:
            with open(args.detail_out, "w") as f:
                f.write(full + "\n")
        print(json.dumps(compact_line(result)), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _r(x, nd=4):
    return None if x is None else float(f"{x:.{nd}g}")


COMPACT_LIMIT = 7000  # the driver's stdout tail window is ~8 KB; the line must fit it whole

# keys of the full record carried verbatim by the compact line
_COMPACT_TOP = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                "vs_baseline", "dtype", "data", "config", "roofline", "step_roofline", "breakdown_ms_per_step",
                "allreduce_ms_per_step", "table", "vs_cpu_baseline", "memory", "merge", "cosines_per_s",
                "cosine_wall_s", "cosine_first_job_s", "cosine_roofline")


def compact_line(res):
    """The one JSON line the driver parses: the contract's keys, the build
    and step rooflines, the CPU baseline with its modes, the cosine keys and
    the summary of every other line. Long prose fields are shortened and the
    full record is printed separately (stderr / --detail-out)."""
    out = {k: res[k] for k in _COMPACT_TOP if k in res}
    if "config" in out:
        cfg = dict(out["config"])
        cfg.pop("sharding", None)
        out["config"] = cfg
    if "roofline" in out:
        out["roofline"] = {k: v for k, v in out["roofline"].items() if k != "algorithmic_bytes_basis"}
    cb = res.get("cpu_baseline")
    if cb:
        out["cpu_baseline"] = {k: cb.get(k) for k in ("value", "unit", "cores", "kind", "sample", "best_updates_per_s")}
        out["cpu_baseline"]["modes"] = {m: {k: _r(v) if isinstance(v, float) else v for k, v in mv.items()}
                                        for m, mv in (cb.get("modes") or {}).items()}
        out["cpu_baseline"]["host"] = cb.get("host")
    out["summary"] = res.get("summary") or summary(res)
    out["detail"] = "full record on stderr ('bench-detail: ' line) and in --detail-out"
    s = json.dumps(out)
    # shed optional keys (never the contract's) until the line fits
    for k in ("memory", "table", "breakdown_ms_per_step", "step_roofline"):
        if len(s) <= COMPACT_LIMIT:
            break
        if k == "step_roofline" and "step_roofline" in out:
            out[k] = {kk: out[k].get(kk) for kk in ("achieved_GBps", "frac")}
        else:
            out.pop(k, None)
        s = json.dumps(out)
    if len(s) > COMPACT_LIMIT and "cpu_baseline" in out:
        out["cpu_baseline"].pop("modes", None)
        out["cpu_baseline"]["sample"] = str(out["cpu_baseline"].get("sample"))[:120]
    return out


def summary(res):
    """Compact figures of the whole line (configs 3, 4, 5, 2, 1, CPU
    baselines), printed last so a truncated stdout tail still holds them."""
    out = {"cfg3_updates_per_s": _r(res.get("value")), "cfg3_ms_per_step": _r(res.get("ms_per_step")),
           "cfg3_build_frac": _r((res.get("roofline") or {}).get("frac"), 3),
           "cfg3_step_frac": _r((res.get("step_roofline") or {}).get("frac"), 3),
           "cfg3_breakdown_ms": {k: _r(v, 3) for k, v in (res.get("breakdown_ms_per_step") or {}).items()}}
    cos = res.get("cosine") or {}
    if "wall_s" in cos:
        rf = cos.get("roofline") or {}
        out.update({"cfg4_cosines_per_s": _r(cos.get("unique_item_pair_cosines_per_s")),
                    "cfg4_wall_s": _r(cos.get("wall_s")), "cfg4_first_job_s": _r(cos.get("first_job_s")),
                    "cfg4_fp4_frac": _r(rf.get("frac"), 3), "cfg4_fp4_avg_launch_ms": _r(rf.get("avg_launch_ms")),
                    "cfg4_int8_frac": _r((cos.get("roofline_int8_waves") or {}).get("frac"), 3),
                    "cfg4_mixed_peak_frac": _r(cos.get("frac_mixed_peak_per_gpu"), 3),
                    "cfg4_full_lists": cos.get("full_lists")})
        st = cos.get("config5_streaming") or {}
        if st:
            out.update({"cfg5_sustained_updates_per_s": _r(st.get("sustained_updates_per_s")),
                        "cfg5_steady_updates_per_s": _r(st.get("steady_updates_per_s")),
                        "cfg5_refresh_latency_s": _r(st.get("refresh_latency_s")),
                        "cfg5_refresh_pair_rate_vs_whole_job": _r(st.get("refresh_pair_rate_vs_whole_job"), 3),
                        "cfg5_refresh_class_weighted_rate": _r(st.get("refresh_class_weighted_rate_vs_whole_job"), 3),
                        "cfg5_whole_job_s": _r(st.get("keep_lists_whole_job_s"))})
        if cos.get("cpu_baseline"):
            out["cfg4_cpu_pairs_per_s"] = _r(cos["cpu_baseline"].get("value"))
    elif cos:
        out["cfg4_error"] = str(cos.get("error"))[:200]
    c2 = res.get("config2") or {}
    if c2:
        out["cfg2_updates_per_s"] = _r(c2.get("updates_per_s"))
        po = ((c2.get("extras") or {}).get("per_owner_shapes_cfg2") or {})
        if po.get("all_pairs"):
            out["cfg2_per_owner_all_pairs_s"] = _r(po["all_pairs"].get("s"))
            out["cfg2_per_owner_ordered_pairs_per_s"] = _r(po["all_pairs"].get("ordered_pairs_per_s"))
    rc1 = ((res.get("config1") or {}).get("recommender") or {})
    if rc1.get("gpu"):
        out["cfg1_recommend_all_users_s"] = _r(rc1["gpu"].get("all_users_s"))
    if res.get("cpu_baseline"):
        out["cfg3_cpu_updates_per_s"] = _r(res["cpu_baseline"].get("value"))
    if res.get("merge"):
        out["merge_payload_ratio"] = _r(res["merge"].get("payload_ratio"), 3)
        out["allreduce_ms_per_step"] = _r(res.get("allreduce_ms_per_step"))
    return out


if __name__ == "__main__":
    main()
