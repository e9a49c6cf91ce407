"""Per-kernel average duration (us) of each rocprofv3 run under gpurun_out/kt/
(scripts/ktrace_variant.sh), cms kernels only."""
import csv
import glob
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/kt"
runs = {}
for f in sorted(glob.glob(os.path.join(root, "*", "**", "run_kernel_stats.csv"), recursive=True)):
    name = os.path.relpath(f, root).split(os.sep)[0]
    runs[name] = {r["Name"].split("(")[0]: float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(f))}
kernels = sorted({k for r in runs.values() for k in r if "cms::" in k}, key=lambda k: -max(r.get(k, 0) for r in runs.values()))
print("| kernel | " + " | ".join(runs) + " |")
for k in kernels[:14]:
    print(f"| {k} | " + " | ".join(f"{runs[r].get(k, 0):.1f}" for r in runs) + " |")
