#!/bin/bash
# rocprofv3 passes over a short bench run: (1) kernel-trace + stats,
# (2) FETCH_SIZE, (3) WRITE_SIZE (separate PMC passes; no sys/runtime trace).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
BENCH="bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras --no-cosine-1m ${BENCH_ARGS}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $BENCH \
    > $OUT/trace.log 2>&1 && echo "trace ok" \
  && timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $BENCH \
    > $OUT/fetch.log 2>&1 && echo "fetch ok" \
  && timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $BENCH \
    > $OUT/write.log 2>&1 && echo "write ok"
