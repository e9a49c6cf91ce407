#!/bin/bash
# HIP API + kernel trace of a short config-2 ingest bench (no counters), for
# finding host-side waits between the step's launches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/ht
rm -rf $OUT && mkdir -p $OUT
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace -d $OUT -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras --no-cosine-1m > $OUT/bench.json 2> $OUT/trace.log
