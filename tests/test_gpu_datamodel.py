"""SURVEY section 8 row A10 end to end on the GPU: a MovieLens-shaped text
file through FileDataModel(transpose=True) -- delimiter from the first line,
Long.parseLong / Float.parseFloat, last value wins, `user,item,` removals,
comments and blank lines (T/impl/model/file/FileDataModel.java:175-221,
394-535) -- into the sketch-cosine ItemSimilarity (taste.CosineCM over the
transposed model), checked against the oracle built from the file's
ground truth (known by construction, not by parsing the file again)."""
import numpy as np
import pytest

from mahout_amd.datamodel import FileDataModel
from mahout_amd.synth import movielens_like
from mahout_amd.taste import CosineCM, FixedShapeConfig, HashFunctionBuilder

pytestmark = pytest.mark.gpu


def write_movielens_file(path, delim=","):
    """Returns {(user, item): value} of the preferences the file leaves."""
    users, items, ratings = movielens_like()
    rng = np.random.Generator(np.random.PCG64(77))
    half = rng.random(users.size) < 0.2  # some half-star ratings (value - 0.5)
    vals = np.where(half, ratings - 0.5, ratings).astype(np.float32)
    truth = {(int(u), int(i)): float(v) for u, i, v in zip(users, items, vals)}
    ops = []  # (order key, line)
    for (u, i), v in truth.items():
        t = rng.random()
        if rng.random() < 0.05:  # an earlier, overridden value
            ops.append((t * 0.5, f"{u}{delim}{i}{delim}{rng.integers(1, 6)}"))
            t = 0.5 + t * 0.5
        s = f"{v:.1f}" if v != int(v) or rng.random() < 0.5 else f"{int(v)}"
        ops.append((t, f"{u}{delim}{i}{delim}{s}"))
    # removed preferences: written, then removed later
    gone = []
    for k in range(3000):
        u, i = int(rng.integers(1, 944)), int(rng.integers(20000, 20100))
        if (u, i) in truth:
            continue
        ops.append((rng.random() * 0.5, f"{u}{delim}{i}{delim}3"))
        ops.append((0.5 + rng.random() * 0.5, f"{u}{delim}{i}{delim}"))
        gone.append((u, i))
    ops.sort(key=lambda x: x[0])
    lines = ["# MovieLens-shaped stand-in (u.data is not available offline)", ""]
    for n, (_, ln) in enumerate(ops):
        lines.append(ln)
        if n % 997 == 0:
            lines.append("# comment")
        if n % 1499 == 0:
            lines.append("")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    return truth, gone


@pytest.mark.parametrize("delim", [",", "\t"])
def test_file_data_model_transposed_item_similarity_end_to_end(oracle, tmp_path, delim):
    path = str(tmp_path / "ratings.csv")
    truth, gone = write_movielens_file(path, delim)
    model = FileDataModel(path, transpose=True)  # owners = items, keys = users
    # ground truth in the transposed orientation
    item_ids = np.array(sorted({i for _, i in truth} | {i for _, i in gone}), np.int64)
    assert np.array_equal(model.getUserIDs(), item_ids)  # emptied items stay in the model
    row_of = {int(x): r for r, x in enumerate(item_ids)}
    rows = np.array([row_of[i] for (_, i) in truth], np.int64)
    keys = np.array([u for (u, _) in truth], np.int64)
    vals = np.array(list(truth.values()), np.float32)
    d, w = 4, 1024
    a, b = oracle.hash_params(42, d)
    exp = oracle.build_table(item_ids.size, d, w, a, b, rows, keys, vals)
    sim = CosineCM(model, FixedShapeConfig(d, w), HashFunctionBuilder(42))
    try:
        assert np.array_equal(sim.table.read_counters(), exp)  # half stars: counters in units of 1/2
        rng = np.random.Generator(np.random.PCG64(5))
        for q in rng.integers(0, item_ids.size, 12).tolist() + [row_of[gone[0][1]]]:
            got = sim.itemSimilarities(int(item_ids[q]), item_ids)
            ref = oracle.similarities_row(exp, q)
            ref[q] = oracle.cosine_cm(exp[q], exp[q])
            assert np.all((got == ref) | (np.isnan(got) & np.isnan(ref))), f"item row {q}"
            ids = sim.mostSimilarUserIDs(int(item_ids[q]), 10)
            eids, _ = oracle.top_users(item_ids, oracle.similarities_row(exp, q), 10)
            assert ids.tolist() == eids.tolist()
        # an item whose every preference was removed: all-zero sketch, NaN similarities
        assert np.isnan(sim.itemSimilarity(int(gone[0][1]), int(item_ids[0])))
    finally:
        sim.close()
