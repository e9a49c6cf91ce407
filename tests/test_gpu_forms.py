"""GPU: narrow storage forms of the sketch table (u8, 4-bit, 2-bit and 1-bit
rows, and sparse list rows, inside their u16 slots; cms_internal.h TableView,
cms_build.hip byte-form path, cms_table.hip widen_rows).

The form a row is stored in is an implementation detail: every counter must
read back as DoubleCountMinSketch's value (`T/impl/common/DoubleCountMinSketch.java:72-80`)
whatever path wrote it, and every similarity / top-k must be bit-identical to
the oracle and to a handle that never uses forms (CMS_NO_FORMS=1).  The cases:
a fresh build with owners in every class (2-bit, 4-bit, u8, u16, u32 hot),
then incremental batches that push 2-bit rows past 3, 4-bit rows past 15 and
u8 rows past 255
(widening in place), and a large batch into the live table (the accumulate
build, which widens every touched form row first).
"""
import os

import numpy as np
import pytest

from mahout_amd import SketchTable
from mahout_amd.synth import zipf_stream

pytestmark = pytest.mark.gpu


def _same(a, b):
    return bool(np.all((a == b) | (np.isnan(a) & np.isnan(b))))


def _stream(n, n_keys, pairs, seed):
    items, users = zipf_stream(n_keys, n, pairs, seed=seed)
    return items.astype(np.int64), users.astype(np.int64)


def _handle(n, d, w, forms, lists=True):
    """forms=False: CMS_NO_FORMS=1 (every narrow row u16); lists=False:
    CMS_LIST_KEYS=0 (the byte-class owners take the dense 1/2/4-bit rows)."""
    saved = {k: os.environ.pop(k, None) for k in ("CMS_NO_FORMS", "CMS_LIST_KEYS")}
    if not forms:
        os.environ["CMS_NO_FORMS"] = "1"
    if not lists:
        os.environ["CMS_LIST_KEYS"] = "0"
    try:
        return SketchTable(n, depth=d, width=w, seed=42)
    finally:
        for k, v in saved.items():
            os.environ.pop(k, None)
            if v is not None:
                os.environ[k] = v


@pytest.mark.parametrize("lists", [True, False])
@pytest.mark.parametrize("n,d,w", [(3000, 5, 1024), (1500, 4, 256)])
def test_forms_build_incremental_accumulate_bit_exact(oracle, n, d, w, lists):
    rng = np.random.Generator(np.random.PCG64(n))
    # Zipf: a few hot owners (u32), a band of u16 owners, many u8 / nibble owners
    items, users = _stream(n, 20000, 600_000, seed=n)
    a, b = oracle.hash_params(42, d)
    stream = [(items, users, np.ones(items.size, np.float32))]
    with _handle(n, d, w, True, lists) as t, _handle(n, d, w, False) as plain:
        for x in (t, plain):
            x.ingest(items, users)
            x.finalize()
        st = t.stats()
        # lists are stored where no larger than the owner's dense 1-/2-bit row:
        # owners of <= 127 keys at d=5, w=1024, none at d=4, w=256 (>= 33 keys)
        small_form = "list_rows" if lists and w >= 1024 else "crumb_rows"
        assert st[small_form] > 0 and st["nibble_rows"] > 0 and st["u8_rows"] > 0 and st["hot_rows"] > 0, st
        assert lists or st["list_rows"] == 0, st
        assert st["bit_rows"] + st["crumb_rows"] + st["list_rows"] + st["nibble_rows"] + st["u8_rows"] + \
            st["hot_rows"] < n  # and u16 rows
        ps = plain.stats()
        assert ps["bit_rows"] == 0 and ps["crumb_rows"] == 0 and ps["nibble_rows"] == 0 and ps["u8_rows"] == 0
        assert ps["list_rows"] == 0
        assert st["stored_bytes"] < plain.stats()["stored_bytes"]
        exp = oracle.build_table(n, d, w, a, b, *[np.concatenate(c) for c in zip(*stream)])
        assert np.array_equal(t.read_counters(), exp)
        # batches: (1) small values onto nibble rows (some stay nibble, some pass 15),
        # (2) weights pushing u8 rows past 255, (3) the owner-grouped atomic path,
        # (4) a large batch -> accumulate build
        nib_rows = np.flatnonzero(np.abs(exp).max(axis=(1, 2)) < 16)
        u8_rows = np.flatnonzero((exp.max(axis=(1, 2)) >= 16) & (exp.max(axis=(1, 2)) < 256))
        batches = [
            (rng.choice(nib_rows, 3000), rng.integers(0, 20000, 3000), rng.integers(1, 3, 3000)),
            # half of the u8 rows get weights that push them past 255 (the other half stays u8)
            (rng.choice(u8_rows[: max(1, u8_rows.size // 2)], 2000), rng.integers(0, 50, 2000),
             rng.integers(1, 200, 2000)),
            # >= 32768 pairs into the live table: grouped by owner, k_ingest_sorted
            (rng.choice(nib_rows, 40000), rng.integers(0, 20000, 40000), np.ones(40000, np.int64)),
        ]
        bi, bu = _stream(n, 20000, 300_000, seed=n + 1)
        batches.append((bi, bu, np.ones(bi.size, np.int64)))
        seen = []
        for step, (r, k, v) in enumerate(batches):
            r = r.astype(np.int64)
            k = k.astype(np.int64)
            v = v.astype(np.float32)
            for x in (t, plain):
                x.ingest(r, k, v)
                x.finalize()
            stream.append((r, k, v))
            exp = oracle.build_table(n, d, w, a, b, *[np.concatenate(c) for c in zip(*stream)])
            got = t.read_counters()
            assert np.array_equal(got, exp), step
            assert np.array_equal(plain.read_counters(), exp), step
            for q in (0, int(r[0]), n - 1):
                s1 = t.similarities(q, np.arange(n))
                assert _same(s1, plain.similarities(q, np.arange(n))), (step, q)
                ref = oracle.similarities_row(exp, q)
                ref[q] = oracle.cosine_cm(exp[q], exp[q])
                assert _same(s1, ref), (step, q)
            seen.append(t.stats())
        # the atomic batches widen only the rows they could push past their form,
        # into the narrowest form that holds the new bound (a 2-bit row lifted to
        # 4..15 becomes 4-bit); a list row takes no in-place add (any add widens it)
        small = [x["nibble_rows"] + x["crumb_rows"] + x["bit_rows"] + x["list_rows"] for x in seen]
        assert 0 < small[0] <= st["nibble_rows"] + st["crumb_rows"] + st["bit_rows"] + st["list_rows"]
        assert seen[0][small_form] < st[small_form]
        assert u8_rows.size < 2 or 0 < seen[1]["u8_rows"] < seen[0]["u8_rows"]
        assert seen[1]["hot_rows"] >= st["hot_rows"]
        assert small[2] <= small[1]
        # the accumulate build widens every touched form row (u16 or hot)
        assert small[3] <= small[2]
        # the all-pairs job over form rows equals the form-free handle's
        k = 20
        got = t.top_k_all(k)
        want = plain.top_k_all(k)
        assert all(np.array_equal(x, y, equal_nan=True) for x, y in zip(got, want))


@pytest.mark.parametrize("mode", ["bits", "nobits", "lists"])
def test_forms_point_queries_and_device_read(oracle, monkeypatch, mode):
    """Point queries (DoubleCountMinSketch.get, :94-103) and the device
    counter read on 2-bit, 4-bit and u8 rows, with and without 1-bit rows
    (owners of <= 64 keys try them first unless CMS_BIT_KEYS=0), or with the
    byte-class owners as list rows, then a batch that widens some of every form."""
    import torch
    if mode == "nobits":
        monkeypatch.setenv("CMS_BIT_KEYS", "0")
    n, d, w = 2000, 4, 512
    items, users = _stream(n, 5000, 300_000, seed=3)  # > 262143 pairs: the row build (smaller batches: atomics)
    a, b = oracle.hash_params(42, d)
    exp = oracle.build_table(n, d, w, a, b, items, users)
    with _handle(n, d, w, True, mode == "lists") as t:
        t.ingest(items, users)
        t.finalize()
        st = t.stats()
        if mode == "lists":  # owners of <= 31 keys (2 + 8 m bytes <= their 256-B 1-bit row), then 1-/2-bit rows
            assert st["list_rows"] > 0 and st["crumb_rows"] > 0, st
        else:
            assert st["nibble_rows"] > 0 and st["crumb_rows"] > 0 and (st["bit_rows"] > 0) == (mode == "bits"), st
            assert st["list_rows"] == 0, st
        dev = t.read_counters_device(0, n).cpu().numpy()
        assert np.array_equal(dev.astype(np.float64), exp)
        for r in (0, 5, 400, n - 1):
            for key in (0, 1, 17, 4999, -3):
                assert t.point_query(r, key) == oracle.sketch_get(exp[r], a, b, key)
        t.ingest_csr(np.zeros(n + 1, np.int64), np.zeros(0, np.int64))  # an empty CSR batch changes nothing
        t.finalize()
        assert np.array_equal(t.read_counters(), exp)
        # a small batch (atomics) onto every row: rows it could push past their
        # form are widened in place, the others keep it; all stay exact
        rng = np.random.Generator(np.random.PCG64(9))
        br = rng.integers(0, n, 3000).astype(np.int64)
        bk = rng.integers(0, 5000, 3000).astype(np.int64)
        t.ingest(br, bk)
        t.finalize()
        exp2 = oracle.build_table(n, d, w, a, b, np.concatenate([items, br]), np.concatenate([users, bk]))
        assert np.array_equal(t.read_counters(), exp2)
        for r in (0, 5, 400, n - 1):
            s1 = t.similarities(r, np.arange(n))
            ref = oracle.similarities_row(exp2, r)
            ref[r] = oracle.cosine_cm(exp2[r], exp2[r])
            assert _same(s1, ref), r
        torch.cuda.synchronize()


@pytest.mark.parametrize("lists,w", [(False, 256), (True, 1024)])
def test_accumulate_build_zero_valued_form_rows(oracle, lists, w):
    """A CSR batch into a live table with forms (the accumulate build) where
    narrow owners' keys all carry 0.0: the build rewrites every owner that has
    keys through its u16 image, so those rows must be widened first even though
    the batch adds no mass to them (update(key, 0.0) leaves the counters as
    they were, DoubleCountMinSketch.java:72-80)."""
    n, d = 1500, 4
    items, users = _stream(n, 5000, 300_000, seed=11)
    a, b = oracle.hash_params(42, d)
    exp = oracle.build_table(n, d, w, a, b, items, users)
    with _handle(n, d, w, True, lists) as t:
        t.ingest(items, users)
        t.finalize()
        st = t.stats()
        if lists:
            assert st["list_rows"] > 0 and st["nibble_rows"] > 0, st
        else:
            assert st["bit_rows"] > 0 and st["crumb_rows"] > 0 and st["nibble_rows"] > 0, st
        mx = exp.max(axis=(1, 2))
        # owners in the 1-/2-bit, 4-bit and u8 forms
        picks = [np.flatnonzero(mx == 1)[:2], np.flatnonzero((mx >= 2) & (mx <= 3))[:2],
                 np.flatnonzero((mx >= 4) & (mx <= 15))[:2], np.flatnonzero((mx >= 16) & (mx <= 255))[:2]]
        zero_rows = np.concatenate(picks).astype(np.int64)
        assert zero_rows.size >= 6
        rng = np.random.Generator(np.random.PCG64(5))
        rows, keys, vals = [], [], []
        for r in range(n):
            if r in set(zero_rows.tolist()):
                k = rng.integers(0, 5000, 7)
                rows.append(np.full(k.size, r)), keys.append(k), vals.append(np.zeros(k.size))
            elif r % 5 == 0:
                k = rng.integers(0, 5000, 3)
                rows.append(np.full(k.size, r)), keys.append(k), vals.append(np.ones(k.size))
        br = np.concatenate(rows).astype(np.int64)
        bk = np.concatenate(keys).astype(np.int64)
        bv = np.concatenate(vals).astype(np.float32)
        off = np.zeros(n + 1, np.int64)
        np.add.at(off, br + 1, 1)
        off = np.cumsum(off)
        t.ingest_csr(off, bk, bv)  # rows ascending already: the CSR order
        t.finalize()
        exp2 = oracle.build_table(n, d, w, a, b, np.concatenate([items, br]), np.concatenate([users, bk]),
                                  np.concatenate([np.ones(items.size, np.float32), bv]))
        got = t.read_counters()
        assert np.array_equal(got[zero_rows], exp2[zero_rows])
        assert np.array_equal(got, exp2)
        for r in zero_rows[::2]:
            s1 = t.similarities(int(r), np.arange(n))
            ref = oracle.similarities_row(exp2, int(r))
            ref[r] = oracle.cosine_cm(exp2[r], exp2[r])
            assert _same(s1, ref), r


def test_mid_class_list_rows(oracle):
    """Mid-class owners (257..1024 keys, unit increments) whose key-bucket
    list is smaller than their 4-bit row are stored as list rows by
    k_build_mid (cms_build.hip): counters, point queries, similarities
    (list x list included) and the all-pairs top-k equal the oracle and a
    form-free handle; a batch then widens the touched list rows in place and
    an accumulating CSR batch widens every touched one to u16."""
    n, d, w = 2000, 4, 4096
    items, users = _stream(n, 20000, 1_200_000, seed=21)
    a, b = oracle.hash_params(42, d)
    exp = oracle.build_table(n, d, w, a, b, items, users)
    counts = np.bincount(items, minlength=n)
    with _handle(n, d, w, True) as t, _handle(n, d, w, False) as plain:
        for x in (t, plain):
            x.ingest(items, users)
            x.finalize()
        st = t.stats()
        mid = np.flatnonzero((counts > 256) & (counts <= 1024))
        assert mid.size > 100 and st["list_rows"] > mid.size // 2, (mid.size, st)
        assert st["stored_bytes"] < plain.stats()["stored_bytes"]
        assert np.array_equal(t.read_counters(), exp)
        for r in (int(mid[0]), int(mid[-1]), n - 1):
            for key in (0, 1, 17, 19999, -3):
                assert t.point_query(r, key) == oracle.sketch_get(exp[r], a, b, key)
            s1 = t.similarities(r, np.arange(n))
            ref = oracle.similarities_row(exp, r)
            ref[r] = oracle.cosine_cm(exp[r], exp[r])
            assert _same(s1, ref), r
            assert _same(s1, plain.similarities(r, np.arange(n))), r
        got = t.top_k_all(20)
        want = plain.top_k_all(20)
        assert all(np.array_equal(x, y, equal_nan=True) for x, y in zip(got, want))
        # a small batch onto mid list rows: widened to the narrowest dense form
        rng = np.random.Generator(np.random.PCG64(4))
        br = rng.choice(mid, 5000).astype(np.int64)
        bk = rng.integers(0, 20000, 5000).astype(np.int64)
        for x in (t, plain):
            x.ingest(br, bk)
            x.finalize()
        exp2 = oracle.build_table(n, d, w, a, b, np.concatenate([items, br]), np.concatenate([users, bk]))
        assert t.stats()["list_rows"] < st["list_rows"]
        assert np.array_equal(t.read_counters(), exp2)
        r = int(br[0])
        s1 = t.similarities(r, np.arange(n))
        ref = oracle.similarities_row(exp2, r)
        ref[r] = oracle.cosine_cm(exp2[r], exp2[r])
        assert _same(s1, ref)
