"""Top kernels (average us, calls) of the rocprofv3 kernel_stats.csv files
under a directory."""
import csv
import glob
import os
import sys

root = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
for f in sorted(glob.glob(os.path.join(root, "**", "*kernel_stats.csv"), recursive=True)):
    rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
    print(f)
    for r in rows[:n]:
        print(f"  {float(r['AverageNs']) / 1e3:10.1f} us x{int(r['Calls']):4d}  {r['Name'].split('(')[0][:90]}")
