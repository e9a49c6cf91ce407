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
    m = FileDataModel(write(tmp_path, ["1,5,2", "1,5,4", "1,6,1", "1,6,", "# comment", "", "2,5,1", "3,7,2", "3,7,"]))
    ids, vals = m.getPreferencesFromUser(1)
    assert ids.tolist() == [5] and vals.tolist() == [4.0]
    # user 3 lost its only preference but stays (GenericDataModel.toDataMap keeps the emptied collection)
    assert m.getUserIDs().tolist() == [1, 2, 3]
    assert m.getPreferencesFromUser(3)[0].size == 0


def test_delimiter_from_first_line_and_boolean_files(tmp_path):
    """FileDataModel.determineDelimiter (:344-352): ',' if the first data
    line holds one, else tab -- and only that character splits every line;
    a first line without a third token makes a boolean model (:210-214)."""
    import pytest
    m = FileDataModel(write(tmp_path, ["# c", "", "1\t5\t2.5", "2\t5\t1"]))
    assert m.getPreferencesFromUser(1)[1].tolist() == [2.5]
    with pytest.raises(ValueError):  # '1,2' is not a long once tab is the delimiter
        FileDataModel(write(tmp_path, ["1\t5\t2", "1,2\t7\t1"]))
    b = FileDataModel(write(tmp_path, ["1,5", "1,6", "2,5", "1,6,"]))
    assert not b.hasPreferenceValues()
    assert b.getPreferencesFromUser(1)[0].tolist() == [5]
    from mahout_amd.taste import CosineCM, FixedShapeConfig, HashFunctionBuilder
    with pytest.raises(ValueError):  # CosineCM.java:38 checkArgument(hasPreferenceValues)
        CosineCM(b, FixedShapeConfig(2, 64), HashFunctionBuilder(1))


def test_java_parse_float_and_long():
    """Float.parseFloat: trimmed, sign, NaN/Infinity, hex significands,
    f/F/d/D suffixes, one rounding of the exact decimal to float32 (no
    decimal -> double -> float double rounding); Long.parseLong: digits and
    an optional sign only, within range."""
    import pytest
    from fractions import Fraction
    from mahout_amd.datamodel import java_parse_float as pf, java_parse_long as pl
    assert pf(" 3.5 ") == np.float32(3.5) and pf("2.5f") == np.float32(2.5) and pf("4D") == np.float32(4.0)
    assert pf("0x1p-2") == np.float32(0.25) and pf("-0x1.8p1") == np.float32(-3.0)
    assert np.isnan(pf("NaN")) and pf("-Infinity") == -np.inf and pf("1e39") == np.inf
    assert pf("1.4e-45") == np.float32(1e-45) and pf("7e-46") == 0.0
    assert str(pf("-0")) == "-0.0"
    # a decimal just above a float32 midpoint whose nearest double IS the midpoint:
    # Java rounds the exact value up; decimal -> double -> float would round to even (down)
    lo = np.float32(1.0)
    hi = np.nextafter(lo, np.float32(2.0))
    mid = (Fraction(1) + Fraction(float(hi))) / 2
    s = "1.000000059604644775390625000000000001"  # mid + 1e-36
    assert Fraction(s) > mid and float(Fraction(s)) == float(mid)
    assert pf(s) == hi and np.float32(float(s)) == lo
    for bad in ["", "3.5.1", "1e", "0x", "abc", "4,5"]:
        with pytest.raises(ValueError):
            pf(bad)
    assert pl("+5") == 5 and pl("-9223372036854775808") == -2 ** 63
    for bad in [" 5", "5 ", "9223372036854775808", "1.0", "0x10", ""]:
        with pytest.raises(ValueError):
            pl(bad)


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


def test_min_max_and_preference_value():
    from mahout_amd.datamodel import GenericDataModel
    m = GenericDataModel({1: {10: 2.5, 11: 0.5}, 2: {10: 4.0}})
    assert m.getMinPreference() == 0.5 and m.getMaxPreference() == 4.0
    assert m.getPreferenceValue(1, 11) == 0.5
    assert m.getPreferenceValue(2, 11) is None


def test_estimate_preference_oracle_hand_kat(oracle):
    """doEstimatePreference on a collision-free sketch by hand: the point
    query returns the exact rating, the sketch cosine the exact cosine."""
    import math
    import numpy as np
    keys = [101, 202, 303]
    d, w = 3, 4096
    seed = None
    for s in range(1, 5000):
        a, b = oracle.hash_params(s, d)
        h = oracle.hash_keys(a, b, w, np.array(keys, np.int64))
        if all(len(set(h[:, r].tolist())) == len(keys) for r in range(d)):
            seed = s
            break
    a, b = oracle.hash_params(seed, d)
    # user 0 rated 101 -> 3; user 1 rated 101 -> 4, 202 -> 2; user 2 rated 101 -> 1, 202 -> 5, 303 -> 2
    rows = np.array([0, 1, 1, 2, 2, 2], np.int64)
    ks = np.array([101, 101, 202, 101, 202, 303], np.int64)
    vals = np.array([3, 4, 2, 1, 5, 2], np.float32)
    t = oracle.build_table(3, d, w, a, b, rows, ks, vals)
    s1 = 12.0 / (3.0 * math.sqrt(20.0))         # cosine(u0, u1): every row equal
    s2 = 3.0 / (3.0 * math.sqrt(30.0))          # cosine(u0, u2)
    exp = np.float32((s1 * 2.0 + s2 * 5.0) / (s1 + s2))
    got = oracle.estimate_preference(t, a, b, 0, [1, 2, 0], 202)
    assert got == exp
    assert math.isnan(oracle.estimate_preference(t, a, b, 0, [1, 2], 303))  # one data point only
    assert oracle.estimate_preference(t, a, b, 0, [1, 2], 202, capper=(1.0, 2.5)) == np.float32(2.5)


def test_counter_units_picks_exact_u32_or_fp64():
    """taste.counter_units: exact u32 counters in units of 2^-s while every
    preference is a non-negative multiple of 2^-s and every owner's total
    stays below 2^32 units; DoubleCountMinSketch's fp64 counters otherwise."""
    import numpy as np
    from mahout_amd.taste import counter_units
    off = np.array([0, 2, 4], np.int64)
    assert counter_units(off, None) == (0, "u32")
    assert counter_units(off, np.array([1, 2, 3, 4], np.float32)) == (0, "u32")
    assert counter_units(off, np.array([0.5, 2, 3, 4.5], np.float32)) == (1, "u32")
    assert counter_units(off, np.array([0.1, 2, 3, 4], np.float32)) == (27, "u32")  # small masses still fit
    assert counter_units(np.array([0, 400], np.int64), np.full(400, 0.1, np.float32)) == (0, "f64")  # 2^32 units
    assert counter_units(off, np.array([-1, 2, 3, 4], np.float32)) == (0, "f64")
    assert counter_units(off, np.array([np.nan, 2, 3, 4], np.float32)) == (0, "f64")
    assert counter_units(np.array([0, 0, 4], np.int64), np.array([1e9, 2e9, 3e9, 4], np.float32)) == (0, "f64")
