"""CPU, world_size 2 over gloo: the multi-GPU data path's semantics.

Each rank keeps the pairs whose key (user) hashes to it (cms_shard_of_key,
the function libmahout_cms.so shards with), builds a full-shape partial
table, and the tables are summed with one all-reduce -- the RCCL step of
cms_finalize.  Counters are integers, so the merged table must equal the
unsharded one bit for bit, for every rank count."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from mahout_amd import shard_of_key
        from mahout_amd.synth import zipf_stream
        items, users = zipf_stream(2000, 300, 40000, seed=11)
        a, b = O.hash_params(42, 4)
        mine = np.array([shard_of_key(int(u), world) == rank for u in users])
        part = O.build_table(300, 4, 256, a, b, items[mine], users[mine])
        t = torch.from_numpy(part.astype(np.int64))
        dist.all_reduce(t)  # integer sum, as ncclAllReduce(ncclUint32, ncclSum)
        full = O.build_table(300, 4, 256, a, b, items, users)
        q.put((rank, bool(np.array_equal(t.numpy(), full.astype(np.int64))), int(mine.sum())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_user_hash_sharding_allreduce_is_exact(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res)
    assert sum(n for _, _, n in res) == 40000


def test_bench_config3_shards_partition_the_global_stream():
    """bench.config3_shard: for any world size the ranks' shards partition the
    same global stream, each pair on the rank its user hashes to."""
    import sys as _sys
    import os as _os
    _sys.path.insert(0, _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
    import bench
    from mahout_amd.sketch import shard_of_keys
    n_items, n_users, total = 1000, 5000, 200_000
    gi, gu = bench.config3_shard(n_items, n_users, total, 0, 1, "cpu", seed=5)
    glob = np.sort(gi.numpy() * n_users + gu.numpy())
    for world in (2, 3):
        parts = []
        for r in range(world):
            i, u = bench.config3_shard(n_items, n_users, total, r, world, "cpu", seed=5)
            assert np.all(shard_of_keys(u.numpy(), world) == r)
            parts.append(i.numpy() * n_users + u.numpy())
        assert np.array_equal(np.sort(np.concatenate(parts)), glob)


def _transport_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from mahout_amd import shard_of_key
        from mahout_amd.synth import zipf_stream
        from mahout_amd.transport import TorchDistTransport
        tr = TorchDistTransport(host=True)  # the product's transport, host buffers
        n, d, w = 300, 4, 256
        items, users = zipf_stream(2000, n, 40000, seed=13)
        a, b = O.hash_params(42, d)
        mine = np.array([shard_of_key(int(u), world) == rank for u in users])
        part = O.build_table(n, d, w, a, b, items[mine], users[mine]).astype(np.uint64).reshape(n, d * w)
        # 1. the bounds all-reduce (cms_merge.hip): local mass and local max per owner
        bnd = np.concatenate([part.sum(axis=1), part.max(axis=1)]).astype(np.uint64)
        tr.allreduce(bnd.ctypes.data, bnd.size)
        bound = np.minimum(bnd[:n], bnd[n:])
        # 2. the packed all-reduce: b(o) = bit_length(bound(o))-bit fields,
        # floor(64/b) per u64 word, field f of word i = counter f*NW + i
        words, layout = [], []
        for o in range(n):
            bits = int(bound[o]).bit_length()
            if bits == 0:
                layout.append((0, 0, 0))
                continue
            per = 64 // bits
            nw = -(-(d * w) // per)
            c = np.zeros(nw * per, np.uint64)
            c[:d * w] = part[o]
            f = c.reshape(per, nw)  # f[k][i] = counter k*nw + i
            wv = np.zeros(nw, np.uint64)
            for k in range(per):
                wv |= f[k] << np.uint64(k * bits)
            layout.append((len(words), nw, bits))
            words.extend(wv.tolist())
        packed = np.array(words, np.uint64)
        tr.allreduce(packed.ctypes.data, packed.size)
        merged = np.zeros((n, d * w), np.uint64)
        for o, (w0, nw, bits) in enumerate(layout):
            if bits == 0:
                continue
            per = 64 // bits
            wv = packed[w0:w0 + nw]
            mask = np.uint64((1 << bits) - 1)
            f = np.stack([(wv >> np.uint64(k * bits)) & mask for k in range(per)])
            merged[o] = f.reshape(-1)[:d * w]
        full = O.build_table(n, d, w, a, b, items, users).astype(np.uint64).reshape(n, d * w)
        # 3. the all-gather (collective top-k partial lists): rank order
        mine_b = np.full(16, rank + 1, np.uint8)
        got = np.zeros(16 * world, np.uint8)
        tr.allgather(mine_b.ctypes.data, got.ctypes.data, 16)
        q.put((rank, bool(np.array_equal(merged, full)), bool((got == np.repeat(np.arange(1, world + 1), 16)).all()),
               int(packed.size), n * d * w))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e), False, 0, 0))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_transport_packed_merge_on_host(world):
    """The product's caller transport (mahout_amd.transport, host buffers)
    carrying the packed merge's two all-reduces and the top-k all-gather over
    gloo: u64 sums of counter-width-packed words are the packed merged table
    (no carry crosses a field, cms_merge.hip), so the unpacked result equals
    the unsharded oracle table (DoubleCountMinSketch.update,
    `T/impl/common/DoubleCountMinSketch.java:72-80`), and the all-gather
    stacks the ranks' buffers in rank order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_transport_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, merged_ok, gather_ok, words, counters in res:
        assert merged_ok is True, (rank, merged_ok)
        assert gather_ok, rank
        assert 0 < words < counters / 2  # the packed payload is a fraction of the u32 table's
