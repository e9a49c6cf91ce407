"""The bench's final stdout line stays small enough for the driver to parse
(r05's 20.4 KB line left BENCH_r05.parsed null) and carries the contract's
keys. Built here from a committed full record of a real GPU run."""
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "roofline", "step_roofline", "cpu_baseline", "cosines_per_s",
            "cosine_wall_s", "cosine_first_job_s", "cosine_roofline", "summary")


def _full_record():
    with open(os.path.join(ROOT, "profiles", "r05", "bench_s6.json")) as f:
        return json.load(f)


def test_compact_line_size_and_keys():
    import bench
    full = _full_record()
    assert len(json.dumps(full)) > 15000  # the record that did not parse
    line = bench.compact_line(full)
    s = json.dumps(line)
    assert len(s) <= bench.COMPACT_LIMIT < 8081
    for k in REQUIRED:
        assert k in line, k
    assert json.loads(s) == line
    rf = line["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in rf, k
    cb = line["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample", "modes"):
        assert k in cb, k
    assert line["value"] == full["value"] and line["ms_per_step"] == full["ms_per_step"]
    assert "workload" in line["config"]
    assert "cfg4_wall_s" in line["summary"] and "cfg2_per_owner_all_pairs_s" in line["summary"]


def test_compact_line_sheds_optional_keys():
    import bench
    full = _full_record()
    full["table"] = {"pad": "x" * 9000}  # an oversized optional field is dropped, not the contract's keys
    line = bench.compact_line(full)
    assert len(json.dumps(line)) <= bench.COMPACT_LIMIT
    assert "table" not in line and "roofline" in line and "cpu_baseline" in line
