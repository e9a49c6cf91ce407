"""Summarise scripts/cos_pmc_r02.sh passes into profiles/<tag>/cosine_pmc_summary.json:
per kernel (averaged over dispatches) the raw counters plus
  mfma_busy_frac  = SQ_VALU_MFMA_BUSY_CYCLES / (kernel cycles x 1024 SIMDs),
                    kernel cycles = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs)
  clock_ghz       = GRBM_GUI_ACTIVE / 8 / dispatch duration
  wait_any_frac, wait_inst_any_frac, active_inst_frac (of SQ_WAVE_CYCLES)
  lds_bank_conflict_frac = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  l2_hit = TCC_HIT / (TCC_HIT + TCC_MISS)
  fetch_bytes = 2 x FETCH_SIZE (gfx950 correction, MI355X_MICROARCH.md HBM)."""
import collections
import csv
import glob
import json
import os
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/cos_pmc"
tag = sys.argv[2] if len(sys.argv) > 2 else "r02"
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(lambda: collections.defaultdict(set))
dur = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(src, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0]
        if "k_cosine" not in n:
            continue
        acc[n][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[n][r["Counter_Name"]].add((f, r["Dispatch_Id"]))
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            dur[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) if "End_Timestamp" in r else None)
out = {}
for n, c in acc.items():
    avg = {k: v / max(1, len(disp[n][k])) for k, v in c.items()}
    rec = {"counters_avg_per_dispatch": avg, "dispatches": max(len(s) for s in disp[n].values())}
    g = avg.get("GRBM_GUI_ACTIVE")
    if g and avg.get("SQ_VALU_MFMA_BUSY_CYCLES") is not None:
        rec["mfma_busy_frac"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / 8 * 1024)
    ds = [x for x in dur[n] if x]
    if g and ds:
        rec["clock_ghz"] = g / 8 / (sum(ds) / len(ds))
    wc = avg.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if k in avg:
                rec[k.lower().replace("sq_", "") + "_frac"] = avg[k] / wc
    if avg.get("SQ_LDS_IDX_ACTIVE"):
        rec["lds_bank_conflict_frac"] = avg.get("SQ_LDS_BANK_CONFLICT", 0) / avg["SQ_LDS_IDX_ACTIVE"]
    if "TCC_HIT_sum" in avg:
        rec["l2_hit"] = avg["TCC_HIT_sum"] / max(1.0, avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
    if "FETCH_SIZE" in avg:
        rec["fetch_bytes_per_dispatch"] = 2 * avg["FETCH_SIZE"] * 1024
    out[n] = rec
os.makedirs(os.path.join("profiles", tag), exist_ok=True)
json.dump(out, open(os.path.join("profiles", tag, "cosine_pmc_summary.json"), "w"), indent=1, sort_keys=True)
for n, r in out.items():
    print(n, {k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items() if k != "counters_avg_per_dispatch"})
