"""CPU: the precomputed-similarity consumer -- GenericItemSimilarity over
ItemItemSimilarity records (T/impl/similarity/GenericItemSimilarity.java:71-95,
172-256) and TopItems.getTopItemItemSimilarities (TopItems.java:145-174) --
restated in mahout_amd.taste, checked here against direct statements of their
rules.  (The GPU lists feeding it are checked in tests/test_gpu_refresh.py.)"""
import math

import numpy as np
import pytest

from mahout_amd.taste import (GenericItemSimilarity, ItemItemSimilarity, get_top_item_item_similarities,
                              similarities_from_top_k)


def test_item_item_similarity_range_check():
    ItemItemSimilarity(1, 2, -1.0)
    ItemItemSimilarity(1, 2, 1.0)
    for bad in (1.0000001, -1.5, math.nan):
        with pytest.raises(ValueError):
            ItemItemSimilarity(1, 2, bad)


def test_generic_item_similarity_map_rules():
    sims = [ItemItemSimilarity(5, 3, 0.5), ItemItemSimilarity(3, 5, 0.25),  # later value wins, either order
            ItemItemSimilarity(7, 7, 0.1),                                  # self: skipped (assumed 1.0)
            ItemItemSimilarity(3, 9, -0.75)]
    g = GenericItemSimilarity(sims)
    assert g.itemSimilarity(3, 5) == 0.25 and g.itemSimilarity(5, 3) == 0.25
    assert g.itemSimilarity(9, 3) == -0.75
    assert g.itemSimilarity(7, 7) == 1.0 and g.itemSimilarity(4, 4) == 1.0
    assert math.isnan(g.itemSimilarity(5, 9))
    assert g.allSimilarItemIDs(3).tolist() == [5, 9]
    assert g.allSimilarItemIDs(7).tolist() == []
    np.testing.assert_array_equal(g.itemSimilarities(3, [5, 9, 4]), [0.25, -0.75, math.nan])


def test_top_item_item_similarities_distinct_values():
    rng = np.random.default_rng(4)
    vals = rng.permutation(np.linspace(-1, 1, 500))
    sims = [ItemItemSimilarity(i, i + 1000, v) for i, v in enumerate(vals)]
    for how_many in (1, 7, 100, 499, 500, 800):
        got = get_top_item_item_similarities(how_many, iter(sims))
        want = sorted(vals, reverse=True)[:how_many]
        assert [s.value for s in got] == want


def test_top_item_item_similarities_ties_follow_the_jdk_heap():
    # Traced by hand through java.util.PriorityQueue (reverseOrder comparator):
    # (2,.5) then (3,.9) then (4,.5) are admitted while not full; the third add
    # overflows and poll() removes the heap head, (2,.5) -- the array is then
    # [(4,.5), (3,.9)]; (5,.5) is refused once full ('>' in TopItems.java:155).
    sims = [ItemItemSimilarity(1, 2, 0.5), ItemItemSimilarity(1, 3, 0.9), ItemItemSimilarity(1, 4, 0.5),
            ItemItemSimilarity(1, 5, 0.5)]
    got = get_top_item_item_similarities(2, iter(sims))
    assert [(s.itemID2, s.value) for s in got] == [(3, 0.9), (4, 0.5)]
    g = GenericItemSimilarity(iter(sims), maxToKeep=2)
    assert g.itemSimilarity(1, 3) == 0.9 and g.itemSimilarity(1, 4) == 0.5 and math.isnan(g.itemSimilarity(1, 2))


def test_similarities_from_top_k_lists():
    ids = np.array([[2, 1], [0, 2], [0, 0]], np.int64)
    sc = np.array([[0.5, 0.25], [0.25, 0.125], [0.5, 0.0]])
    cnt = np.array([2, 2, 1], np.int32)
    owner_ids = np.array([10, 20, 30])
    recs = list(similarities_from_top_k(ids, sc, cnt, owner_ids))
    assert [(r.itemID1, r.itemID2, r.value) for r in recs] == [(10, 2, 0.5), (10, 1, 0.25), (20, 0, 0.25),
                                                               (20, 2, 0.125), (30, 0, 0.5)]
