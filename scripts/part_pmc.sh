#!/bin/bash
# Wave-state and LDS counters of the config-2 ingest kernels: two PMC passes
# (kernel trace only), summarized per kernel by scripts/pmc_brief.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/part_pmc
rm -rf $OUT; mkdir -p $OUT
BENCH="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --no-cosine-1m"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS -d $OUT/p1 -o run --output-format csv -- python3 $BENCH > $OUT/p1.out 2>&1 \
  && timeout -k 10 300 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_MISC -d $OUT/p2 -o run --output-format csv -- python3 $BENCH > $OUT/p2.out 2>&1 \
  && python3 scripts/pmc_brief.py $OUT/p1 $OUT/p2
