#!/bin/bash
# PMC passes over the config-4 job (scripts/cos_job_probe.py): MFMA busy,
# LDS activity / conflicts / issue stalls, wait breakdown, L2 hit rate,
# memory-side fetch.  One counter group per pass, kernel trace only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/cos_pmc
mkdir -p $OUT
ARGS="${COS_ARGS:-1000000 500000000 8192 100}"
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 scripts/cos_job_probe.py $ARGS \
      > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  echo "pass $i ok"
done
