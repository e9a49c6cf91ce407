"""Diagnose an all-pairs mismatch: slab values vs oracle for the returned ids."""
import sys
import numpy as np
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import torch  # noqa
from mahout_amd import SketchTable
from mahout_amd.synth import zipf_stream
from oracle import oracle as O

n, d, w, vmax, seed = [int(x) for x in sys.argv[1:6]]
q0 = int(sys.argv[6]) if len(sys.argv) > 6 else 5
O.build()
items, users = zipf_stream(3000, n, 300_000, seed=seed)
vals = np.random.Generator(np.random.PCG64(seed)).integers(1, vmax + 1, size=items.size).astype(np.float32)
a, b = O.hash_params(42, d)
ot = O.build_table(n, d, w, a, b, items, users, vals)
with SketchTable(n, depth=d, width=w, seed=42) as t:
    t.ingest(items, users, vals)
    t.finalize()
    k = min(n - 1, 1024)
    ids, sc, cnt = t.top_k_rows(q0, n - q0, k)
    print("stats", t.stats())
    bad = 0
    for q in range(q0, n):
        sims = O.similarities_row(ot, q, False)
        got = ids[q - q0, :cnt[q - q0]]
        gs = sc[q - q0, :cnt[q - q0]]
        exp_at_got = sims[got]
        wrong = ~((exp_at_got == gs) | (np.isnan(exp_at_got) & np.isnan(gs)))
        eids, esc = O.top_users(np.arange(n), sims, k)
        if wrong.any() or got.tolist() != eids.tolist():
            bad += 1
            if bad <= 8:
                wi = np.nonzero(wrong)[0]
                print("row", q, "value-mismatches", wi.size, "first cols", got[wi[:6]].tolist(),
                      "got", gs[wi[:3]].tolist(), "exp", exp_at_got[wi[:3]].tolist(),
                      "order-ok", got.tolist() == eids.tolist())
    print("bad rows", bad, "of", n - q0)
