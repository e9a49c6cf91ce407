"""GPU: the RCCL data path itself, on a real one-rank communicator.

RCCL refuses two ranks on one device, so the multi-process tests
(test_gpu_transport.py, test_gpu_merge.py) drive the rank logic through a
caller transport.  Here the handle asks for the collective path at world 1
(CMS_FLAG_COLLECTIVE_SINGLE_RANK) and cms_comm_init builds a real RCCL
communicator, so every collective call site of the library runs through RCCL:

  cms_finalize (first)  -> merge_packed: ncclAllReduce of the per-owner bounds
                           and of the packed counter words (the linearity of
                           DoubleCountMinSketch.update, `T/impl/common/DoubleCountMinSketch.java:72-80`)
  cms_finalize (later)  -> dlog_exchange: ncclAllGather of the delta-log
                           counts and of the logged (row, key, value) batches
  cms_top_k_all / refresh -> top_k_all_job: ncclAllGather of the partial
                           lists, then the exact merge (`TopItems.java:91-136`)
  cms_destroy           -> ncclCommDestroy

With one participant every collective is an identity, so each result must
equal the plain single-GPU path and the oracle bit for bit;
cms_stats.collective_calls counts the calls that went through the
communicator and comm_kind names RCCL.
"""
import os

import numpy as np
import pytest

from mahout_amd import SketchTable, comm_unique_id
from mahout_amd.synth import zipf_stream

pytestmark = pytest.mark.gpu

# a box without a routed interface still bootstraps over loopback
os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")


def _same(a, b):
    return bool(np.all((a == b) | (np.isnan(a) & np.isnan(b))))


def _lists_equal(x, y):
    return all(np.array_equal(p, q, equal_nan=True) for p, q in zip(x, y))


@pytest.mark.parametrize("n,d,w,vmax,k", [(1500, 4, 256, 3, 30), (700, 5, 1024, 1, 100)])
def test_rccl_one_rank_merge_delta_log_collective_top_k(oracle, n, d, w, vmax, k):
    items, users = zipf_stream(20000, n, 400_000, seed=n + 7)
    items = items.astype(np.int64)
    users = users.astype(np.int64)
    vals = np.random.Generator(np.random.PCG64(n)).integers(1, vmax + 1, items.size).astype(np.float32)
    bulk = 300_000  # >= 262144 pairs: the partition + row build, then the packed merge
    cuts = [bulk, bulk + 50_000, bulk + 60_000, items.size]  # grouped (>= 32768) and atomic batches
    a, b = oracle.hash_params(42, d)
    with SketchTable(n, depth=d, width=w, seed=42, collective_single_rank=True) as t, \
            SketchTable(n, depth=d, width=w, seed=42) as plain:
        t.comm_init(comm_unique_id(), 0, 1)
        st = t.stats()
        assert st["comm_kind"] == 1 and st["world"] == 1 and st["collective_calls"] == 0, st
        t.ingest(items[:bulk], users[:bulk], vals[:bulk])
        t.finalize()  # packed merge over ncclAllReduce
        st = t.stats()
        merge_calls = st["collective_calls"]
        assert merge_calls >= 2 and st["merge_words"] > 0, st
        full = oracle.build_table(n, d, w, a, b, items[:bulk], users[:bulk], vals[:bulk])
        assert np.array_equal(t.read_counters(), full)
        first = t.top_k_refresh(k)  # whole job through the collective merge; 2k-deep lists kept
        assert t.stats()["collective_calls"] > merge_calls
        # streaming batches into the merged table: applied locally and logged
        for lo, hi in zip(cuts[:-1], cuts[1:]):
            t.ingest(items[lo:hi], users[lo:hi], vals[lo:hi])
        before = t.stats()["collective_calls"]
        t.finalize()  # delta-log exchange over ncclAllGather (no other rank's batches to apply)
        assert t.stats()["collective_calls"] >= before + 4  # counts + rows + keys + values
        full = oracle.build_table(n, d, w, a, b, items, users, vals)
        assert np.array_equal(t.read_counters(), full)
        plain.ingest(items, users, vals)
        plain.finalize()
        assert np.array_equal(plain.read_counters(), full)
        got = t.top_k_all(k)  # collective: partial list all-gathered, merged
        want = plain.top_k_all(k)
        assert _lists_equal(got, want)
        ids, sc, cnt = got
        for r in (0, 1, n // 3, n - 1):
            sims = oracle.similarities_row(full, r)
            eids, esc = oracle.top_users(np.arange(n), sims, k)
            assert ids[r, :cnt[r]].tolist() == eids.tolist() and _same(sc[r, :cnt[r]], esc), r
        refreshed = t.top_k_refresh(k)  # kept lists + the touched owners' pairs, collectively
        assert _lists_equal(refreshed, got)
        touched, _, whole_jobs = t.refresh_stats()
        assert whole_jobs == 1 and 0 < touched <= n  # a 100K-pair Zipf stream touches (nearly) every owner
        assert not _lists_equal(first, got)  # the batches did change the lists
        s = t.similarities(1, np.arange(n))
        e = oracle.similarities_row(full, 1)
        e[1] = oracle.cosine_cm(full[1], full[1])
        assert _same(s, e)


def test_rccl_one_rank_per_owner_shapes(oracle):
    """Per-owner shapes (CosineCM with CountMinSketchConfig) with an RCCL
    communicator: the all-pairs top-k splits query rows over the ranks and
    all-gathers the lists through RCCL -- at one rank, the plain job's lists."""
    from mahout_amd.synth import movielens_like, to_csr
    users, items, ratings = movielens_like(500, 700, 20_000, seed=4, min_per_user=5)
    uid = np.unique(users)
    rows = np.searchsorted(uid, users)
    order = np.lexsort((items, rows))
    off, keys, vals = to_csr(rows[order], items[order], uid.size, ratings[order])
    n, k = uid.size, 20

    def job(collective):
        with SketchTable(n, seed=42, owner_ids=uid, per_owner=True, collective_single_rank=collective) as t:
            if collective:
                t.comm_init(comm_unique_id(), 0, 1)
            t.ingest_csr(off, keys, vals)
            t.configure_owner_shapes(1.0, 700)
            t.finalize()
            out = t.top_k_all(k)
            return out, t.stats()["collective_calls"]
    got, calls = job(True)
    want, calls0 = job(False)
    assert calls > 0 and calls0 == 0
    assert _lists_equal(got, want)


def test_rccl_flag_rules():
    """The flag is refused with fp64 counters; without it a world of 1
    detaches (no communicator, the single-GPU path)."""
    from mahout_amd._lib import CmsError
    with pytest.raises(CmsError):
        SketchTable(100, depth=4, width=256, counters="f64", collective_single_rank=True)
    with SketchTable(100, depth=4, width=256) as t:
        t.comm_init(comm_unique_id(), 0, 1)
        assert t.stats()["comm_kind"] == 0
