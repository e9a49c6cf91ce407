"""CPU: input handling and options of the job drivers (mahout_amd/jobs.py),
following ToEntityPrefsMapper (T/hadoop/ToEntityPrefsMapper.java:58-80),
ToUserVectorsReducer (T/hadoop/item/ToUserVectorsReducer.java:66-80) and
ItemSimilarityJob's options (T/hadoop/similarity/item/ItemSimilarityJob.java:97-130)."""
import numpy as np
import pytest

from mahout_amd.jobs import SKETCH_COSINE, ItemSimilarityJob, read_item_prefs


def test_read_item_prefs_mapper_semantics(tmp_path):
    d = tmp_path / "in"
    d.mkdir()
    # tab or comma delimits; a missing preference is 1.0; a trailing empty field is dropped
    (d / "a").write_text("1,10,3\n1\t11\t2.5\n2,10\n3,12,4,\n3,10,1\n")
    (d / "_SUCCESS").write_text("")
    (d / ".crc").write_text("x")
    items, off, keys, vals = read_item_prefs(str(d))
    assert items.tolist() == [10, 11, 12]
    assert off.tolist() == [0, 3, 4, 5]
    assert keys.tolist() == [1, 2, 3, 1, 3]
    assert vals.tolist() == [3.0, 1.0, 1.0, 2.5, 4.0]
    # booleanData: every value 1; minPrefsPerUser drops users 2 (1 item)
    items, off, keys, vals = read_item_prefs(str(d), boolean_data=True, min_prefs_per_user=2)
    assert items.tolist() == [10, 11, 12] and keys.tolist() == [1, 3, 1, 3]
    assert set(vals.tolist()) == {1.0}


def test_read_item_prefs_last_line_wins_and_errors(tmp_path):
    p = tmp_path / "p.txt"
    p.write_text("1,10,3\n1,10,5\n")
    _, _, _, vals = read_item_prefs(str(p))
    assert vals.tolist() == [5.0]
    p.write_text("1,10,3\n\n")
    with pytest.raises(ValueError):  # Long.parseLong("") in the mapper
        read_item_prefs(str(p))


def test_item_similarity_job_options(tmp_path):
    job = ItemSimilarityJob()
    with pytest.raises(ValueError):
        job.run(["--input", "x", "--output", "y", "--similarityClassname", "SIMILARITY_COOCCURRENCE"])
    with pytest.raises(ValueError):
        job.run(["--input", "x", "--output", "y", "-s", SKETCH_COSINE, "-m", "0"])
    with pytest.raises(ValueError):
        job.run(["--input", "x", "--bogus", "1"])
    with pytest.raises(ValueError):
        job.run(["--output", "y", "-s", SKETCH_COSINE])
    assert np.array_equal(read_item_prefs(str(_write(tmp_path)))[0], [5])


def _write(tmp_path):
    p = tmp_path / "one.txt"
    p.write_text("1,5,1\n")
    return p
