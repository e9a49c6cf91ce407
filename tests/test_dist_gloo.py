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
