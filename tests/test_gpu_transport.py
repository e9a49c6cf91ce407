"""GPU, 2-3 processes on one device: the whole multi-rank life cycle through a
caller-supplied communicator (cms_comm_init_transport, torch.distributed gloo
as the transport).

This is the rank logic cms_finalize / cms_top_k_all run over RCCL on an 8-GPU
node -- the packed counter merge, the delta-log exchange of a merged table
(config 5's streaming batches) and the collective all-pairs top-k (partial
lists all-gathered and merged, in rounds when world * k exceeds one merge
workgroup) -- driven with several ranks sharing the one GPU of a test box.
Every rank must end with the unsharded result bit for bit:
  counters   == oracle DoubleCountMinSketch.update over the whole stream
               (`T/impl/common/DoubleCountMinSketch.java:72-80`)
  top-k      == a single-rank handle's cms_top_k_all, and the oracle's
               TopItems.getTopUsers on sampled rows (`TopItems.java:91-136`);
  refresh    == cms_top_k_all on the same table (cms_top_k_refresh after the
               delta exchange: kept lists + the touched owners' pairs).
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _same(a, b):
    return bool(np.all((a == b) | (np.isnan(a) & np.isnan(b))))


def _worker(rank, world, port, q, case):
    import torch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from mahout_amd import SketchTable
        from mahout_amd.sketch import shard_of_keys
        from mahout_amd.synth import zipf_stream
        from mahout_amd.transport import TorchDistTransport
        n, d, w, npairs, vmax, k = case
        items, users = zipf_stream(20000, n, npairs, seed=n + k)
        vals = np.random.Generator(np.random.PCG64(5)).integers(1, vmax + 1, size=items.size).astype(np.float32)
        mine = shard_of_keys(users, world) == rank
        torch.cuda.init()
        bulk = npairs * 6 // 10
        # streaming batches after the merge: one through the owner-grouped
        # path (>= 32768 pairs), the rest through plain atomics
        cuts = [bulk, bulk + 60_000, bulk + 70_000, bulk + 75_000, npairs]
        tr = TorchDistTransport()
        res = {}
        with SketchTable(n, depth=d, width=w, seed=42, device=0) as t:
            tr.attach(t)
            sel = mine.copy()
            sel[bulk:] = False
            t.ingest(items[sel], users[sel], vals[sel])
            t.finalize()  # packed all-reduce through the transport
            res["merge_bytes"] = tr.bytes_moved
            t.top_k_refresh(k)  # collective whole job; every rank keeps the 2k-deep lists
            for lo, hi in zip(cuts[:-1], cuts[1:]):
                m = np.zeros(npairs, bool)
                m[lo:hi] = mine[lo:hi]
                t.ingest(items[m], users[m], vals[m])
            before = tr.bytes_moved
            t.finalize()  # delta-log exchange through the transport
            res["delta_bytes"] = tr.bytes_moved - before
            got = t.read_counters()
            ids, sc, cnt = t.top_k_all(k)  # collective: partial lists gathered and merged
            # collective incremental refresh: only pairs with an owner any rank's batches touched
            fids, fsc, fcnt = t.top_k_refresh(k)
            res["refresh_stats"] = t.refresh_stats()
        res["refresh_vs_all"] = bool(np.array_equal(fcnt, cnt)) and all(
            fids[r, :cnt[r]].tolist() == ids[r, :cnt[r]].tolist() and _same(fsc[r, :cnt[r]], sc[r, :cnt[r]])
            for r in range(n))
        a, b = O.hash_params(42, d)
        full = O.build_table(n, d, w, a, b, items, users, vals)
        res["counters"] = bool(np.array_equal(got, full))
        with SketchTable(n, depth=d, width=w, seed=42, device=0) as ref:
            ref.ingest(items, users, vals)
            ref.finalize()
            rids, rsc, rcnt = ref.top_k_all(k)
        res["topk_vs_single_rank"] = bool(np.array_equal(cnt, rcnt)) and all(
            ids[r, :cnt[r]].tolist() == rids[r, :rcnt[r]].tolist() and _same(sc[r, :cnt[r]], rsc[r, :rcnt[r]])
            for r in range(n))
        ok = True
        for r in list(range(0, n, max(1, n // 11))) + [n - 1]:
            sims = O.similarities_row(full, r)
            eids, esc = O.top_users(np.arange(n), sims, k)
            ok &= ids[r, :cnt[r]].tolist() == eids.tolist() and _same(sc[r, :cnt[r]], esc)
        res["topk_vs_oracle"] = bool(ok)
        q.put((rank, res))
    except Exception as e:  # noqa: BLE001
        import traceback
        traceback.print_exc()
        q.put((rank, {"error": repr(e)}))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,case", [
    (2, (1500, 4, 256, 300_000, 3, 40)),    # multi-limb owners, lists from every shard kind
    (3, (900, 3, 512, 250_000, 2, 400)),    # world * k = 1200 > 1024: the merge runs in rounds
])
def test_transport_merge_delta_exchange_collective_top_k(world, case):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, case)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=500) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, r in res:
        assert "error" not in r, (rank, r)
        assert r["counters"], (rank, r)
        assert r["topk_vs_single_rank"], (rank, r)
        assert r["topk_vs_oracle"], (rank, r)
        assert r["refresh_vs_all"], (rank, r)
        assert r["refresh_stats"][2] == 1, (rank, r)  # one whole job, then an incremental refresh
        n, d, w = case[:3]
        assert 0 < r["merge_bytes"] < n * d * w * 4  # the packed merge moved less than the u32 table
        assert 0 < r["delta_bytes"] < n * d * w * 4  # the exchange moved the logs (20 B/pair), not a table


def _po_worker(rank, world, port, q):
    import torch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from mahout_amd import SketchTable
        from mahout_amd.synth import movielens_like, to_csr
        from mahout_amd.transport import TorchDistTransport
        torch.cuda.init()
        users, items, ratings = movielens_like(700, 900, 30_000, seed=11, min_per_user=5)
        uid = np.unique(users)
        rows = np.searchsorted(uid, users)
        order = np.lexsort((items, rows))
        off, keys, vals = to_csr(rows[order], items[order], uid.size, ratings[order])
        k, n = 20, uid.size
        res = {}
        tr = TorchDistTransport()

        def job(collective):
            with SketchTable.per_owner_shapes(n, seed=42, owner_ids=uid, device=0) as t:
                t.ingest_csr(off, keys, vals)  # every rank holds the whole DataModel
                t.configure_owner_shapes(1.0, 900)
                if collective:
                    tr.attach(t)
                t.finalize()
                shapes = t.owner_shapes()[2:]
                return t.top_k_all(k), shapes
        (ids, sc, cnt), shapes = job(True)
        (rids, rsc, rcnt), _ = job(False)
        res["vs_single_rank"] = bool(np.array_equal(cnt, rcnt) and np.array_equal(ids, rids) and _same(sc, rsc))
        a, b = O.hash_params(42, 32)
        ok = True
        for r in [0, 1, 255, 256, 257, 511, 512, n // 2, n - 1]:
            sims = np.array([O.per_owner_similarity(off, keys, vals, shapes, a, b, r, c) for c in range(n)])
            sims[r] = np.nan  # TopItems skips the query owner itself
            eids, esc = O.top_users(uid, sims, k)
            ok &= ids[r, :cnt[r]].tolist() == eids.tolist() and _same(sc[r, :cnt[r]], esc)
        res["vs_oracle"] = bool(ok)
        q.put((rank, res))
    except Exception as e:  # noqa: BLE001
        import traceback
        traceback.print_exc()
        q.put((rank, {"error": repr(e)}))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_transport_per_owner_shapes_collective_top_k():
    """Per-owner shapes (CosineCM with CountMinSketchConfig, asymmetric
    userSimilarity(u1, u2), `T/impl/similarity/CosineCM.java:83-96`) on 2
    ranks: the all-pairs top-k sharded by query rows and gathered equals the
    single-rank job and the oracle's TopItems loop on rows of both shards."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_po_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=500) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, r in res:
        assert "error" not in r, (rank, r)
        assert r["vs_single_rank"], (rank, r)
        assert r["vs_oracle"], (rank, r)
