"""CPU: FileDataModel / GenericDataModel semantics the sketch path reads
(T/impl/model/file/FileDataModel.java:394-535, GenericDataModel.java:80-137)."""
import numpy as np

from mahout_amd.datamodel import FileDataModel, GenericDataModel


def write(tmp_path, lines):
    p = tmp_path / "prefs.csv"
    p.write_text("\n".join(lines) + "\n")
    return str(p)


def test_sorted_owners_and_keys(tmp_path):
    m = FileDataModel(write(tmp_path, ["3,9,1", "1,5,2", "1,2,3", "2,7,4"]))
    assert m.getUserIDs().tolist() == [1, 2, 3]
    ids, vals = m.getPreferencesFromUser(1)
    assert ids.tolist() == [2, 5] and vals.tolist() == [3.0, 2.0]


def test_last_value_wins_and_removal(tmp_path):
    m = FileDataModel(write(tmp_path, ["1,5,2", "1,5,4", "1,6,1", "1,6,", "# comment", "", "2\t5\t1"]))
    ids, vals = m.getPreferencesFromUser(1)
    assert ids.tolist() == [5] and vals.tolist() == [4.0]
    assert m.getUserIDs().tolist() == [1, 2]


def test_transpose(tmp_path):
    m = FileDataModel(write(tmp_path, ["2,1,1", "1,2,1", "3,4,1", "1,3,2", "2,3,1"]), transpose=True)
    assert m.getUserIDs().tolist() == [1, 2, 3, 4]  # items became owners
    ids, vals = m.getPreferencesFromUser(3)
    assert ids.tolist() == [1, 2] and vals.tolist() == [2.0, 1.0]


def test_generic_csr_layout():
    m = GenericDataModel({10: {3: 1.0, 1: 2.0}, 4: {1: 5.0}})
    assert m.getUserIDs().tolist() == [4, 10]
    assert m.offsets.tolist() == [0, 1, 3]
    assert m.keys.tolist() == [1, 1, 3]
    assert m.values.dtype == np.float32
