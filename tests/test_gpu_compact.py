"""GPU: the compact row layout (cms_internal.h TableView: each narrow row at
an arena offset of its own, sized by what its form can need) holds the same
table as whole u16 slots per row (CMS_NO_COMPACT=1), through every writer of
the table:

  * the fresh build (list, 1/2/4-bit and u8 rows packed end to end, the mid
    class in whole slots, hot rows in u32 slots);
  * the small-batch atomics and the owner-grouped incremental batch
    (k_ingest_sorted): a touched row without a slot of its own first moves to
    one at the arena's end (widen_rows), whatever its form;
  * the accumulate build (every touched row moves to a u16 slot);
  * the packed merge (cms_finalize_with, one rank): the rows are laid out
    anew by their merged field widths and stored as u8 / 4-bit rows;
  * a byte-class list row whose 4-bit count overflows (k_build_bytes keeps
    it a list: its capacity is the list's).

After each stage the two layouts' tables, forms, norms (through the
similarities) and top-k lists are equal bit for bit, sampled rows equal the
oracle's rebuild, and the compact table's allocation stays a fraction of the
slot layout's.
"""
import numpy as np
import pytest

from mahout_amd.synth import zipf_stream

pytestmark = pytest.mark.gpu


def same(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return a.shape == b.shape and bool(np.all((a == b) | (np.isnan(a) & np.isnan(b))))


def _state(t, n):
    import torch
    q = np.array([0, 1, 2, 7, 100, n // 2, n - 1])
    tab = t.read_counters_device()  # (stays on the device)
    sims = np.stack([t.similarities(int(x), np.arange(n)) for x in q])
    ids, sc, cnt = t.top_k_all(20)
    st = t.stats()
    torch.cuda.synchronize()
    return tab, sims, (ids, sc, cnt), st, t.owner_forms()


def _equal(a, b, forms=True):
    import torch
    assert torch.equal(a[0], b[0])
    assert same(a[1], b[1])
    assert np.array_equal(a[2][2], b[2][2]) and np.array_equal(a[2][0], b[2][0]) and same(a[2][1], b[2][1])
    if forms:
        assert np.array_equal(a[4][0], b[4][0])  # the same form per row


def test_compact_layout_equals_slots_through_every_writer(oracle, monkeypatch):
    from mahout_amd import SketchTable
    n, d, w = 20000, 5, 4096
    items, users = zipf_stream(2_000_000, n, 2_000_000, seed=17)
    rng = np.random.Generator(np.random.PCG64(4))
    # the incremental batches: owners of every class, rows new to the table
    # among them (the zero row), one owner past 2^16 (promoted to a u32 slot)
    small_i = rng.integers(0, n, 20_000).astype(np.int64)
    small_u = rng.integers(0, 2_000_000, small_i.size).astype(np.int64)
    mid_i = np.concatenate([rng.integers(0, n, 200_000), np.full(70_000, 5)]).astype(np.int64)
    mid_u = rng.integers(0, 2_000_000, mid_i.size).astype(np.int64)
    acc_i, acc_u = zipf_stream(2_000_000, n, 2_000_000, seed=18)
    stages = {}
    for compact in (True, False):
        monkeypatch.setenv("CMS_NO_COMPACT", "0" if compact else "1")
        got = []
        with SketchTable(n, depth=d, width=w, seed=42) as t:
            t.ingest(items, users)  # fresh build
            t.finalize()
            got.append(_state(t, n))
            t.ingest(small_i, small_u)  # small batch: global atomics
            t.finalize()
            got.append(_state(t, n))
            t.ingest(mid_i, mid_u)  # owner-grouped incremental batch (k_ingest_sorted)
            t.finalize()
            got.append(_state(t, n))
            t.ingest(acc_i, acc_u)  # accumulate build into the live table
            t.finalize()
            got.append(_state(t, n))
        with SketchTable(n, depth=d, width=w, seed=42) as t:  # merge through a one-rank caller collective
            t.ingest(items, users)
            t.finalize_with(lambda ptr, count: None)
            got.append(_state(t, n))
        stages[compact] = got
    for i, (a, b) in enumerate(zip(stages[True], stages[False])):
        _equal(a, b, forms=i < 4)  # (the merge stores u8 / 4-bit rows only in the compact layout)
    # the compact fresh table is a fraction of the slot layout's allocation
    fresh_c, fresh_s = stages[True][0][3], stages[False][0][3]
    assert fresh_c["table_bytes"] * 4 < fresh_s["table_bytes"], (fresh_c["table_bytes"], fresh_s["table_bytes"])
    assert fresh_c["stored_bytes"] == fresh_s["stored_bytes"]
    # the merged compact table stores u8 / 4-bit rows (the slot layout keeps u16)
    merged_c = stages[True][4][3]
    assert merged_c["u8_rows"] + merged_c["nibble_rows"] > 0
    # sampled rows against the oracle after every incremental stage
    a, b = oracle.hash_params(42, d)
    sel = np.array([0, 1, 5, 100, n - 1])
    all_i = np.concatenate([items, small_i, mid_i, acc_i])
    all_u = np.concatenate([users, small_u, mid_u, acc_u])
    m = np.isin(all_i, sel)
    exp = oracle.build_table(sel.size, d, w, a, b, np.searchsorted(sel, all_i[m]), all_u[m], None)
    assert same(stages[True][3][0][sel].cpu().numpy().astype(np.float64), exp)


def test_compact_merge_forms_equal_oracle(oracle, monkeypatch):
    """The one-rank packed merge of a compact table: rows re-laid out by their
    merged widths (u8 and 4-bit forms, the zero row for owners without keys)
    read back as the oracle's table, with the oracle's similarities."""
    from mahout_amd import SketchTable
    monkeypatch.setenv("CMS_NO_COMPACT", "0")
    n, d, w = 3000, 4, 1024
    items, users = zipf_stream(500_000, n - 200, 600_000, seed=23)  # the last 200 owners stay empty
    a, b = oracle.hash_params(7, d)
    exp = oracle.build_table(n, d, w, a, b, items, users, None)
    with SketchTable(n, depth=d, width=w, seed=7) as t:
        t.ingest(items, users)
        t.finalize_with(lambda ptr, count: None)
        got = t.read_counters()
        st = t.stats()
        assert st["u8_rows"] + st["nibble_rows"] > 0, st
        assert same(got, exp)
        for q in (0, 5, n - 300, n - 1):
            ref = oracle.similarities_row(exp, q)
            ref[q] = oracle.cosine_cm(exp[q], exp[q])
            assert same(t.similarities(q, np.arange(n)), ref), q


@pytest.mark.parametrize("vmm", [True, False])
def test_compact_arena_regrows_and_shrinks(oracle, monkeypatch, vmm):
    """One handle through a large fresh build, resets and small ones (after
    three small layouts in a row the arena gives back what it no longer
    needs: unmapped chunks, or a smaller hipMalloc with CMS_NO_VMM=1),
    incremental batches that move rows to slots
    of their own (the arena grows), and a large build again -- each stage
    bit-exact against the oracle's rebuild."""
    from mahout_amd import SketchTable
    monkeypatch.setenv("CMS_NO_VMM", "0" if vmm else "1")
    monkeypatch.setenv("CMS_NO_COMPACT", "0")
    n, d, w = 30000, 5, 4096
    a, b = oracle.hash_params(11, d)
    big_i, big_u = zipf_stream(1_000_000, n, 3_000_000, seed=31)
    small_i, small_u = zipf_stream(1_000_000, 300, 400_000, seed=32)  # owners 0..299 only
    rng = np.random.Generator(np.random.PCG64(33))
    more_i = rng.integers(0, n, 100_000).astype(np.int64)
    more_u = rng.integers(0, 1_000_000, more_i.size).astype(np.int64)
    sel = np.array([0, 1, 2, 150, 299, 5000, n - 1])

    def check(t, items, users):
        m = np.isin(items, sel)
        exp = oracle.build_table(sel.size, d, w, a, b, np.searchsorted(sel, items[m]), users[m], None)
        got = t.read_counters_device()[sel].cpu().numpy().astype(np.float64)
        assert same(got, exp)
        return t.stats()["table_bytes"]

    with SketchTable(n, depth=d, width=w, seed=11) as t:
        t.ingest(big_i, big_u)
        t.finalize()
        tb_big = check(t, big_i, big_u)
        for _ in range(3):  # the third small layout in a row gives the big one's memory back
            t.reset()
            t.ingest(small_i, small_u)
            t.finalize()
            tb_small = check(t, small_i, small_u)
        assert tb_small < tb_big, (tb_small, tb_big)
        t.ingest(more_i, more_u)  # touched rows without a slot of their own move to one
        t.finalize()
        tb_more = check(t, np.concatenate([small_i, more_i]), np.concatenate([small_u, more_u]))
        assert tb_more > tb_small
        t.reset()
        t.ingest(big_i, big_u)
        t.finalize()
        check(t, big_i, big_u)
