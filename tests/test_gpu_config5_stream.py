"""Config 5 at its stated volume on one GPU (BASELINE.json configs[4]): the
config-3/4 table (500M-pair Zipf bulk build, 10M users x 1M items, d=5,
w=8192), then the whole 1B-pair incremental stream in 10M-pair batches --
exactly the batches bench.py's streaming_refresh pushes through the live
table (seeds 555_000 + b; grouped by owner, k_ingest_sorted) -- and a
periodic refresh.

The streamed table is what the bench's refreshes read, so it is checked the
way the domain allows at a size the oracle cannot hold:
  * checksum of checksums: every update adds its increment once to each of
    the d rows (`T/impl/common/DoubleCountMinSketch.java:72-80`), so each row
    of all 1M sketches sums to the owner's pair count over bulk + stream;
  * storage capacity: no owner's largest counter exceeds what its stored
    form holds (list rows the stream touched were widened, 1/2/4-bit and u8
    rows promoted before they could overflow);
  * the 16 hottest owners, 32 random owners and 16 owners that were list rows
    after the bulk build and were then touched by the stream, bit for bit
    against oracle.build_table over every (owner, key) pair of bulk + stream
    (regenerated from the seeds and filtered on the device; the oracle adds
    each distinct key's multiplicity once -- the same integer counters, as
    integer addition commutes);
  * cms_top_k_refresh after one further 1.25M-pair batch equals
    cms_top_k_all on the streamed table, every list.
"""
import numpy as np
import pytest

from mahout_amd import SketchTable
from mahout_amd.synth import zipf_stream_torch

pytestmark = pytest.mark.gpu

N_USERS, N_ITEMS, N_PAIRS, D, W, SEED, K = 10_000_000, 1_000_000, 500_000_000, 5, 8192, 42, 100
STREAM, BATCH = 1_000_000_000, 10_000_000
CHUNK = 16384
CAP = {"u32": 2 ** 32 - 1, "u16": 65535, "u8": 255, "u4": 15, "u2": 3, "u1": 1}


def _same(a, b):
    return bool(np.all((a == b) | (np.isnan(a) & np.isnan(b))))


def _batches():
    """bench.py streaming_refresh's sustained stream (world 1)."""
    nb = (STREAM + BATCH - 1) // BATCH
    for b in range(nb):
        yield zipf_stream_torch(N_USERS, N_ITEMS, min(BATCH, STREAM - b * BATCH), seed=555_000 + b, device="cuda")


@pytest.mark.timeout(1200)
def test_config5_full_stream_table(oracle):
    import torch

    items, users = zipf_stream_torch(N_USERS, N_ITEMS, N_PAIRS, seed=20261015, device="cuda")  # bench's headline
    counts_d = torch.bincount(items, minlength=N_ITEMS)
    t = SketchTable(N_ITEMS, depth=D, width=W, seed=SEED)
    try:
        t.ingest_device_rows(items, users, None, N_PAIRS)
        t.finalize()
        forms0, _ = t.owner_forms()
        assert (forms0 == SketchTable.FORMS.index("list")).sum() > N_ITEMS // 2
        bulk_counts = counts_d.cpu().numpy()

        # the whole 1B-pair stream, 10M pairs per batch, into the live table
        streamed = 0
        for bi, bu in _batches():
            t.ingest_device_rows(bi.contiguous(), bu.contiguous(), None, int(bi.numel()))
            counts_d += torch.bincount(bi, minlength=N_ITEMS)
            streamed += int(bi.numel())
            del bi, bu
        t.finalize()
        t.synchronize()
        assert streamed == STREAM
        counts = counts_d.cpu().numpy()
        assert int(counts.sum()) == N_PAIRS + STREAM
        assert t.stats()["pairs_ingested"] == N_PAIRS + STREAM

        # 1. every row of every owner sums to its pair count; largest counters
        rowmax = torch.empty(N_ITEMS, dtype=torch.int64, device="cuda")
        buf = torch.empty((CHUNK, D, W), dtype=torch.int32, device="cuda")
        for o in range(0, N_ITEMS, CHUNK):
            c = min(CHUNK, N_ITEMS - o)
            v = t.read_counters_device(o, c, buf[:c])
            sums = (v.to(torch.int64) & 0xFFFFFFFF).sum(dim=2)
            assert torch.equal(sums, counts_d[o:o + c, None].expand(c, D)), o
            rowmax[o:o + c] = (v.view(c, -1).to(torch.int64) & 0xFFFFFFFF).amax(dim=1)
        del buf, v, sums
        rowmax = rowmax.cpu().numpy()

        # 2. no stored form past its capacity, and each narrow form's bound holds
        forms, bound = t.owner_forms()
        for code, name in enumerate(SketchTable.FORMS):
            sel = forms == code
            if name == "list" or not sel.any():
                continue
            assert rowmax[sel].max() <= CAP[name], name
            if name not in ("u32", "u16"):  # u16 rows are kept below 2^16 by their mass bound, not cbound
                assert (rowmax[sel] <= bound[sel]).all(), name
        touched = counts > bulk_counts
        assert (forms[touched] != SketchTable.FORMS.index("list")).any()  # the stream widened list rows

        # 3. sampled owners bit for bit: keys of bulk + stream regenerated and
        # counted per (sampled owner, user) on the device
        rng = np.random.default_rng(2028)
        hot = np.argsort(counts)[-16:]
        rand = rng.choice(np.flatnonzero(counts), 32, replace=False)
        was_list = np.flatnonzero((forms0 == SketchTable.FORMS.index("list")) & touched)
        lst = rng.choice(was_list, 16, replace=False)
        sample = np.unique(np.concatenate([hot, rand, lst]))
        pos = torch.full((N_ITEMS,), -1, dtype=torch.int64, device="cuda")
        pos[torch.from_numpy(sample).cuda()] = torch.arange(sample.size, device="cuda")
        hist = torch.zeros(sample.size * N_USERS, dtype=torch.int64, device="cuda")

        def collect(it_, us):
            p = pos[it_]
            sel = p >= 0
            idx = p[sel] * N_USERS + us[sel]
            hist.index_add_(0, idx, torch.ones_like(idx))

        collect(items, users)
        del items, users
        for bi, bu in _batches():
            collect(bi, bu)
            del bi, bu
        a, b = oracle.hash_params(SEED, D)
        for j, owner in enumerate(sample.tolist()):
            h = hist[j * N_USERS:(j + 1) * N_USERS]
            keys = torch.nonzero(h).flatten()
            mult = h[keys].cpu().numpy()
            keys = keys.cpu().numpy().astype(np.int64)
            assert int(mult.sum()) == int(counts[owner]), owner
            # float32 multiplicities stay exact below 2^24: split larger ones
            reps = (mult + (1 << 23) - 1) >> 23
            k2 = np.repeat(keys, reps)
            v2 = np.full(k2.size, 1 << 23, np.int64)
            v2[np.cumsum(reps) - 1] = mult - (reps - 1) * (1 << 23)
            want = oracle.build_table(1, D, W, a, b, np.zeros(k2.size, np.int64), k2, v2.astype(np.float32))
            np.testing.assert_array_equal(t.read_counters(owner, 1), want, err_msg=str(owner))
        del hist, pos
        torch.cuda.empty_cache()
        t.release_scratch()

        # 4. the periodic refresh on the streamed table: one further batch, then
        # the incremental lists equal the whole job's, every one of the 1M
        t.top_k_refresh(K)  # whole job: keeps the 2k-deep lists
        bi, bu = zipf_stream_torch(N_USERS, N_ITEMS, 1_250_000, seed=777_000, device="cuda")
        t.ingest_device_rows(bi.contiguous(), bu.contiguous(), None, int(bi.numel()))
        t.finalize()
        got = t.top_k_refresh(K)
        touched_n, redone, full = t.refresh_stats()
        assert full == 1 and 0 < touched_n < N_ITEMS // 2 and redone == 0
        ids, sc, cnt = got
        rids, rsc, rcnt = t.top_k_all(K)
        assert np.array_equal(cnt, rcnt)
        assert np.array_equal(ids, rids)
        assert _same(sc, rsc)
        assert t.stats()["topk_redo"] == 0
    finally:
        t.close()
        torch.cuda.empty_cache()
