"""Generates tests/golden/golden_cms.json -- the committed parity fixtures.

Provenance of every value (the reference is Java; no JDK exists in this
image and no reference test exercises the sketch path):

  jdk_random      published java.util.Random known answers (JDK behaviour the
                  reference relies on at HashFunctionBuilder.java:27,46-47);
                  NOT derived from the oracle -- they pin it.
  reference_kats  known answers held by the reference's own tests for the
                  exact cosine the sketch reproduces when it is collision
                  free: VectorSimilarityMeasuresTest.java:108-114 and
                  ItemSimilarityJobTest.java:103-165 (input lines included).
  hash_*, sketch_*, cosine_*, top_users_*
                  outputs of the CPU restatement oracle/cms_oracle.c
                  (regression vectors; cross-checked against the pure-Python
                  big-integer restatement oracle/java_ref.py when generated).

Run:  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import java_ref as J  # noqa: E402
from oracle import oracle as O  # noqa: E402

EDGE_KEYS = [0, 1, -1, 2, 1000, -1000, 943, 1682, 2 ** 31 - 1, -(2 ** 31), 2 ** 62, -(2 ** 62),
             9223372036854775783, 9223372036854775782, 9223372036854775807, -9223372036854775808,
             -9223372036854775783, -9223372036854775784, 123456789012345678, -987654321098765432]


def main():
    out = {}
    out["jdk_random"] = {
        "new Random(0).nextLong()": -4962768465676381896,
        "new Random(42).nextLong()": -5025562857975149833,
        "new Random(42).nextInt()": -1170105035,
    }
    out["reference_kats"] = {
        "VectorSimilarityMeasuresTest.testCosineSimilarity": {
            "source": "mr/src/test/java/org/apache/mahout/math/hadoop/similarity/cooccurrence/measures/"
                      "VectorSimilarityMeasuresTest.java:108-114",
            "a": [0, 2, 0, 0, 8, 3, 0, 6, 0, 1, 2, 2, 0],
            "b": [3, 0, 0, 0, 7, 0, 2, 2, 1, 3, 2, 1, 1],
            "cosine": 0.769846046,
            "epsilon": 1e-6,
        },
        "ItemSimilarityJobTest.testCompleteJob": {
            "source": "mr/src/test/java/org/apache/mahout/cf/taste/hadoop/similarity/item/ItemSimilarityJobTest.java:"
                      "103-165",
            "lines": ["2,1,1", "1,2,1", "3,4,1", "1,3,2", "2,3,1"],
            "pairs": [[1, 3, 0.45], [2, 3, 0.89]],
            "epsilon": 0.01,
        },
    }
    seeds = [0, 1, 42, -7, 2 ** 40 + 3, 20261015]
    hp = {}
    for s in seeds:
        a, b = O.hash_params(s, 8)
        pa, pb = J.hash_params(s, 8)
        assert list(a) == pa and list(b) == pb, s
        hp[str(s)] = {"a": [int(x) for x in a], "b": [int(x) for x in b]}
    out["hash_params_depth8"] = hp
    rng = np.random.Generator(np.random.PCG64(7))
    keys = EDGE_KEYS + [int(x) for x in rng.integers(-2 ** 63, 2 ** 63 - 1, size=44, dtype=np.int64)]
    hidx = {}
    a, b = O.hash_params(42, 5)
    for w in [1, 40, 1000, 1024, 4096, 8192, 39, 32768]:
        got = O.hash_keys(a, b, w, np.array(keys, np.int64))
        for i, k in enumerate(keys):
            assert [J.hash_(int(a[r]), int(b[r]), w, k) for r in range(5)] == list(got[i]), (w, k)
        hidx[str(w)] = got.tolist()
    out["hash_indices_seed42_depth5"] = {"keys": keys, "by_width": hidx}

    # small integer-valued model (owners x keys), d=4, w=64 so collisions happen
    owners = np.array([0, 0, 0, 1, 1, 2, 2, 2, 2, 3, 3, 1, 0], np.int64)
    okeys = np.array([5, 17, 99, 5, 23, 17, 99, 5, 64, 1, 2, 99, 5], np.int64)
    vals = np.array([1, 3, 2, 5, 4, 1, 1, 2, 5, 3, 3, 1, 4], np.float32)
    ha, hb = O.hash_params(42, 4)
    table = O.build_table(4, 4, 64, ha, hb, owners, okeys, vals)
    cos = [[O.cosine_cm(table[i], table[j]) for j in range(4)] for i in range(4)]
    out["sketch_small"] = {
        "seed": 42, "depth": 4, "width": 64, "owners": owners.tolist(), "keys": okeys.tolist(),
        "vals": vals.tolist(), "counters": table.astype(np.int64).tolist(),
        "cosine_cm": [[None if np.isnan(x) else float(x) for x in row] for row in cos],
        "point_query": {str(k): [O.sketch_get(table[i], ha, hb, k) for i in range(4)] for k in [5, 17, 99, 7]},
    }
    ids = np.arange(10, dtype=np.int64)
    scores = np.array([0.5, np.nan, 0.9, 0.5, 0.9, 0.1, 0.5, -0.2, 0.9, 0.5])
    ti, ts = O.top_users(ids, scores, 4)
    out["top_users_ties"] = {"ids": ids.tolist(), "scores": [None if np.isnan(x) else x for x in scores], "k": 4,
                             "expect_ids": ti.tolist(), "expect_scores": ts.tolist()}
    out["shape_from_delta_epsilon"] = {
        str(w): O.shape_from_delta_epsilon(np.exp(-5.0), np.e / w) for w in [39, 40, 43, 78, 1024, 4096, 8192]}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden_cms.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", path)


if __name__ == "__main__":
    main()
