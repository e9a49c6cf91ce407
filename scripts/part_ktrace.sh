#!/bin/bash
# EXPERIMENT: kernel-trace averages of the ingest step with and without the
# hot-owner routing of the partition (CMS_NO_HOT_ROUTING=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/pkt*
for mode in hot twopass; do
OUT=gpurun_out/pkt_$mode
mkdir -p $OUT
echo "== $mode"
if [ $mode = twopass ]; then export CMS_NO_HOT_ROUTING=1; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras --no-cosine-1m ${BENCH_ARGS} \
    > $OUT/bench.json 2> $OUT/trace.log \
  && OUT=$OUT python3 - <<'P' || exit 1
import csv, glob
f = glob.glob(""+__import__("os").environ["OUT"]+"/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if n.startswith("cms::"):
        print(f'{float(r["AverageNs"])/1e3:9.1f} us  x{r["Calls"]:>3}  {n.split("(")[0]}')
P
done
