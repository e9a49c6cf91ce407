"""Summarise a profile_r05.sh ingest_sq pass (one rocprofv3 --pmc run of SQ
counters) into a JSON of per-kernel averages per dispatch plus the ratios the
design notes quote: lds_bank_conflict_frac = SQ_LDS_BANK_CONFLICT /
SQ_LDS_IDX_ACTIVE, wait_any_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES,
active_inst_frac = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES.
usage: summarize_sq.py <pass dir> <out.json>"""
import collections
import csv
import glob
import json
import os
import sys

src, out = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(lambda: collections.defaultdict(set))
for f in sorted(glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k][r["Counter_Name"]].add((f, r["Dispatch_Id"]))
res = {}
for k, c in acc.items():
    avg = {n: v / max(1, len(disp[k][n])) for n, v in c.items()}
    rec = dict(avg)
    if avg.get("SQ_LDS_IDX_ACTIVE"):
        rec["lds_bank_conflict_frac"] = avg.get("SQ_LDS_BANK_CONFLICT", 0.0) / avg["SQ_LDS_IDX_ACTIVE"]
    if avg.get("SQ_WAVE_CYCLES"):
        rec["wait_any_frac"] = avg.get("SQ_WAIT_ANY", 0.0) / avg["SQ_WAVE_CYCLES"]
        rec["active_inst_frac"] = avg.get("SQ_ACTIVE_INST_ANY", 0.0) / avg["SQ_WAVE_CYCLES"]
    res[k] = rec
json.dump(res, open(out, "w"), indent=1, sort_keys=True)
for k in sorted(res, key=lambda k: -res[k].get("SQ_BUSY_CYCLES", 0))[:8]:
    r = res[k]
    print(k[:48], {x: round(r[x], 3) for x in ("lds_bank_conflict_frac", "wait_any_frac", "active_inst_frac") if x in r})
