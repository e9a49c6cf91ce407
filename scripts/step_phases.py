"""Per-step phase durations of the headline ingest from a rocprofv3 kernel
trace (scripts/profile_r03.sh ingest): for every step, the build scope
(first build-kernel start -> last build-kernel end: k_build_rows on the
handle's stream, k_build_nibbles / k_build_mid / k_build_bytes on the side
stream, which overlap) and the partition (k_hot_sample start -> k_p2_scatter
end), so the bench's build roofline (algorithmic bytes / scope time) can be
recomputed from the committed trace.

usage: python scripts/step_phases.py gpurun_out/prof_ingest/trace/run_kernel_trace.csv"""
import csv
import statistics
import sys

BUILD = ("k_build_rows", "k_build_nibbles", "k_build_mid", "k_build_bytes")
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
steps, part = [], []
cur_b, cur_p = None, None
for r in rows:
    name, t0, t1 = r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if "k_hot_sample" in name:
        cur_p = [t0, t0]
        if cur_b:
            steps.append(cur_b)
            cur_b = None
    if "k_p2_scatter" in name and cur_p:
        cur_p[1] = t1
        part.append(cur_p[1] - cur_p[0])
        cur_p = None
    if any(b in name for b in BUILD):
        cur_b = [t0, t1] if cur_b is None else [min(cur_b[0], t0), max(cur_b[1], t1)]
if cur_b:
    steps.append(cur_b)
build = [(b - a) / 1e6 for a, b in steps]
print(f"steps {len(build)}; build scope ms: median {statistics.median(build):.3f}, all {[round(x, 3) for x in build]}")
print(f"partition ms: median {statistics.median(part) / 1e6:.3f}")
