#!/bin/bash
# Wave-state counters of the config-2 ingest kernels (one PMC pass, kernel trace only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/build_pmc
mkdir -p $OUT
BENCH="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --no-cosine-1m"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS -d $OUT/p1 -o run --output-format csv -- python3 $BENCH > $OUT/p1.log 2>&1 && echo "pass 1 ok"
