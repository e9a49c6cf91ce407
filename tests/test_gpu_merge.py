"""GPU, 2 processes on one device: the counter-width-adaptive merge.

cms_finalize's multi-rank merge packs each owner's counters into bit fields
of the width its global bound needs and sums the packed u64 words.  Here the
same code (cms_merge.hip) runs through cms_finalize_with, with gloo over
127.0.0.1 as the transport, so two ranks can share the one GPU of a test box
(RCCL refuses two ranks on one device).  Each rank builds the partial table
of its user-hash shard; after the merge every rank must hold the unsharded
table bit for bit, and its norms must give the unsharded similarities.
"""
import ctypes
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


def _hip_runtime():
    """The HIP runtime already mapped into this process (the one torch and
    libmahout_cms.so share), for the test transport's device<->host copies."""
    with open("/proc/self/maps") as f:
        for line in f:
            path = line.split()[-1]
            if "libamdhip64.so" in path:
                lib = ctypes.CDLL(path)
                lib.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
                lib.hipMemcpy.restype = ctypes.c_int
                return lib
    raise RuntimeError("libamdhip64 not mapped")


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
        n, d, w, npairs, vmax = case[:5]
        refresh_k = case[5] if len(case) > 5 else 0
        items, users = zipf_stream(30000, n, npairs, seed=n)
        vals = None
        if vmax > 1:
            vals = np.random.Generator(np.random.PCG64(3)).integers(1, vmax + 1, size=items.size).astype(np.float32)
        mine = shard_of_keys(users, world) == rank
        torch.cuda.init()
        hip = _hip_runtime()
        moved = []

        def allreduce(ptr, count):
            host = np.empty(count, np.int64)
            assert hip.hipMemcpy(host.ctypes.data, ptr, count * 8, 2) == 0  # device -> host
            t = torch.from_numpy(host)
            dist.all_reduce(t)  # u64 sums (two's complement: same bits)
            assert hip.hipMemcpy(ptr, host.ctypes.data, count * 8, 1) == 0  # host -> device
            moved.append(count)

        with SketchTable(n, depth=d, width=w, seed=42, device=0) as t:
            t.ingest(items[mine], users[mine], None if vals is None else vals[mine])
            pre = t.stats()  # the local table's narrow forms (w % 32 == 0: 1-/2-/4-bit and u8 rows)
            if refresh_k:
                # kept refresh lists of the LOCAL (shard) table; the merge below
                # replaces the table, so the next refresh must be a whole job
                t.finalize()
                t.top_k_refresh(refresh_k)
            t.finalize_with(allreduce)
            post = t.stats()
            got = t.read_counters()
            sims = t.similarities(1, np.arange(n))
            if refresh_k:
                lists = t.top_k_refresh(refresh_k)
                full_jobs = t.refresh_stats()[2]
                whole = t.top_k_all(refresh_k)
        a, b = O.hash_params(42, d)
        full = O.build_table(n, d, w, a, b, items, users, vals)
        exp = O.similarities_row(full, 1)
        exp[1] = O.cosine_cm(full[1], full[1])
        ok_t = bool(np.array_equal(got, full))
        # k_merge_unpack writes every narrow row back as u16 (hidx kFormU16) or a
        # hot slot -- or, with compact rows (w % 32 == 0), as u8 / 4-bit rows
        # where the merged field width allows (never 1-/2-bit or list rows)
        forms = ("bit_rows", "crumb_rows", "nibble_rows", "u8_rows")
        if w % 32 == 0 and npairs // world >= 262144:  # a bulk build per rank: narrow forms exist before the merge
            ok_t = ok_t and sum(pre[f] for f in forms) > 0
        after = ("bit_rows", "crumb_rows", "list_rows") if w % 32 == 0 else forms
        ok_t = ok_t and all(post[f] == 0 for f in after)
        ok_s = bool(np.all((sims == exp) | (np.isnan(sims) & np.isnan(exp))))
        if refresh_k:
            ids, sc, cnt = lists
            ok_s = ok_s and full_jobs == 2
            ok_s = ok_s and all(np.array_equal(x, y, equal_nan=True) for x, y in zip(lists, whole))
            for row in (0, 1, n // 2, n - 1):  # TopItems.getTopUsers over the merged table
                er = O.similarities_row(full, row)
                eids, esc = O.top_users(np.arange(n, dtype=np.int64), er, refresh_k)
                ok_s = ok_s and ids[row, :cnt[row]].tolist() == eids.tolist()
                ok_s = ok_s and np.array_equal(sc[row, :cnt[row]], esc, equal_nan=True)
        q.put((rank, ok_t, ok_s, moved))
    except Exception as e:  # noqa: BLE001
        import traceback
        traceback.print_exc()
        q.put((rank, False, False, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", [(800, 4, 512, 200_000, 1), (300, 5, 1000, 150_000, 5), (64, 3, 128, 400_000, 1),
                                  (800, 4, 512, 200_000, 2, 20),  # + refresh lists across the merge
                                  (1500, 4, 512, 700_000, 1)])   # bulk builds: 1-/2-/4-bit and u8 rows merged
def test_packed_merge_two_ranks_bit_exact(case):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, case)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, ok_t, ok_s, moved in res:
        assert ok_t and ok_s, (rank, moved)
    n, d, w = case[:3]
    words = res[0][3][1]
    assert words < n * d * w / 2  # the packed payload is well under the u32 table's n*d*w/2 u64 words
