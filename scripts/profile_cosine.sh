#!/bin/bash
# rocprofv3 kernel trace of the config-4 all-pairs top-k (1M items) and its
# HBM counters (separate PMC passes), for profiles/<round>/cosine_*.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_cos
mkdir -p $OUT
ARGS="${COS_ARGS:-1000000 500000000 8192 100}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 scripts/topk_all_probe.py $ARGS \
    > $OUT/trace.log 2>&1 && echo "trace ok"
