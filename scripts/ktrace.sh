#!/bin/bash
# Kernel-trace pass only (no counters) over a short ingest bench, then the
# per-kernel averages of the cms:: kernels.  For quick A/B of ingest kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/kt*
for lib in "" ${LIBS}; do
OUT=gpurun_out/kt${lib:+_$(basename $lib .so)}
mkdir -p $OUT
echo "== lib ${lib:-default}"
MAHOUT_CMS_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- \
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
