#!/bin/bash
# PMC counters for the all-pairs kernels (one counter group per pass; kernel
# trace only, no runtime/sys trace).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/cos_pmc
mkdir -p $OUT
i=0
for grp in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_INST_LDS SQ_WAVE_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 scripts/cosine_probe.py 1000000 500000000 8192 1024 500000 > $OUT/p$i.log 2>&1 || exit 1
  echo "pass $i ok"
done
