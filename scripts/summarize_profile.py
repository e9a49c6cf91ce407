"""Summarise a scripts/profile.sh run (gpurun_out/prof) into profiles/<tag>/.

Writes kernel_stats.csv (rocprofv3 --stats), pmc_summary.json (per-kernel
average FETCH_SIZE / WRITE_SIZE per dispatch) and a short summary.md.
HBM bytes per launch = 2 * FETCH_SIZE + WRITE_SIZE (KiB): on gfx950
FETCH_SIZE reports half the bytes of wide coalesced streaming reads and
WRITE_SIZE is exact for 16-B stores (MI355X_MICROARCH.md, HBM section).
"""
import collections
import csv
import json
import os
import shutil
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
tag = sys.argv[2] if len(sys.argv) > 2 else "r01"
suffix = sys.argv[3] if len(sys.argv) > 3 else ""  # e.g. "_config2": kernel_stats_config2.csv, pmc_summary_config2.json
dst = os.path.join("profiles", tag)
os.makedirs(dst, exist_ok=True)


def _find(sub, name):
    """rocprofv3 writes <dir>/<host>/<pid>/run_*.csv or <dir>/run_*.csv by version."""
    import glob
    hits = sorted(glob.glob(os.path.join(src, sub, "**", name), recursive=True))
    if not hits:
        raise SystemExit(f"no {name} under {os.path.join(src, sub)}")
    return hits[-1]


shutil.copy(_find("trace", "run_kernel_stats.csv"), os.path.join(dst, f"kernel_stats{suffix}.csv"))
pmc = collections.defaultdict(dict)
for sub, ctr in [("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")]:
    acc = collections.defaultdict(list)
    for row in csv.DictReader(open(_find(sub, "run_counter_collection.csv"))):
        if row["Counter_Name"] == ctr:
            acc[row["Kernel_Name"].split("(")[0]].append(float(row["Counter_Value"]))
    for k, v in acc.items():
        pmc[k][ctr + "_KiB_avg"] = sum(v) / len(v)
        pmc[k]["dispatches"] = len(v)
stats = {r["Name"].split("(")[0]: r for r in csv.DictReader(open(_find("trace", "run_kernel_stats.csv")))}
out = {}
for k, v in pmc.items():
    f, w = v.get("FETCH_SIZE_KiB_avg", 0.0), v.get("WRITE_SIZE_KiB_avg", 0.0)
    out[k] = dict(v, hbm_bytes_per_launch=(2 * f + w) * 1024,
                  avg_ns=float(stats[k]["AverageNs"]) if k in stats else None)
json.dump(out, open(os.path.join(dst, f"pmc_summary{suffix}.json"), "w"), indent=1, sort_keys=True)
with open(os.path.join(dst, f"summary{suffix}.md"), "w") as fh:
    fh.write("| kernel | calls | avg us | FETCH KiB | WRITE KiB | HBM bytes/launch (2F+W) |\n|---|---|---|---|---|---|\n")
    for k, r in sorted(stats.items(), key=lambda kv: -float(kv[1]["TotalDurationNs"])):
        p = out.get(k, {})
        fh.write(f"| {k} | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | {p.get('FETCH_SIZE_KiB_avg', 0):.0f} | "
                 f"{p.get('WRITE_SIZE_KiB_avg', 0):.0f} | {p.get('hbm_bytes_per_launch', 0):.3e} |\n")
print(open(os.path.join(dst, f"summary{suffix}.md")).read())
