#!/bin/bash
# Kernel-trace stats of the packed-merge kernels (scripts/merge_payload.py, G ranks on one GPU).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/mp
rm -rf $OUT && mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- \
    python3 scripts/merge_payload.py ${G:-2} > $OUT/run.log 2>&1 \
  && python3 - <<'P'
import csv, glob
f = glob.glob("gpurun_out/mp/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if "merge" in n or "promote" in n:
        print(f'{float(r["AverageNs"])/1e3:9.1f} us  x{r["Calls"]:>3}  {n.split("(")[0]}')
P
