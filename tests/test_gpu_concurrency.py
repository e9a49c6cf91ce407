"""Drop-in concurrency (SURVEY §8(b) "Threading"): Taste calls a similarity
from many threads at once (MultithreadedBatchItemSimilarities.java:78, the
evaluator's pool, AbstractDifferenceRecommenderEvaluator.java:192-193).  After
cms_finalize the point queries take the handle's lock shared and run on
leased per-call streams and scratch, so 8 Python threads (ctypes drops the
GIL around every call) must get exactly the serial answers."""
import threading

import numpy as np
import pytest

from mahout_amd import SketchTable
from mahout_amd.synth import zipf_stream

pytestmark = pytest.mark.gpu


def same(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return a.shape == b.shape and bool(np.all((a == b) | (np.isnan(a) & np.isnan(b))))


@pytest.mark.parametrize("counters", ["u32", "f64"])
def test_eight_threads_equal_serial(counters):
    n, d, w = 1500, 5, 1024
    items, users = zipf_stream(5000, n, 200_000, seed=21)
    vals = np.random.Generator(np.random.PCG64(21)).integers(1, 6, size=items.size).astype(np.float32)
    rng = np.random.Generator(np.random.PCG64(22))
    with SketchTable(n, depth=d, width=w, seed=42, counters=counters) as t:
        t.ingest(items, users, vals)
        t.finalize()
        queries = []
        for i in range(240):
            kind = i % 3
            q = int(rng.integers(0, n))
            if kind == 0:
                queries.append(("sims", q, rng.integers(0, n, 300)))
            elif kind == 1:
                queries.append(("point", q, int(users[rng.integers(0, users.size)])))
            else:
                queries.append(("est", q, rng.integers(0, n, 12), np.unique(users[rng.integers(0, users.size, 50)])))

        def run(qr):
            if qr[0] == "sims":
                return t.similarities(qr[1], qr[2])
            if qr[0] == "point":
                return np.array([t.point_query(qr[1], qr[2])])
            return t.estimate_preferences(qr[1], qr[2], qr[3], (1.0, 5.0))

        serial = [run(qr) for qr in queries]
        results = [None] * len(queries)
        errors = []

        def worker(tid):
            try:
                for i in range(tid, len(queries), 8):
                    results[i] = run(queries[i])
            except Exception as e:  # noqa: BLE001
                errors.append(repr(e))

        ths = [threading.Thread(target=worker, args=(i,)) for i in range(8)]
        for th in ths:
            th.start()
        for th in ths:
            th.join(timeout=120)
        assert not errors, errors
        for i, (a, b) in enumerate(zip(results, serial)):
            assert a is not None and same(a, b), (i, queries[i][0])
        # a writer between the readers: the table changes, the next reads see it
        t.ingest(items[:1000], users[:1000], vals[:1000])
        t.finalize()
        assert t.similarities(0, np.arange(5)).shape == (5,)
