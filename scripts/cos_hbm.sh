#!/bin/bash
# HBM traffic and L2 hit rate of the config-4 all-pairs kernels (separate PMC
# passes, kernel trace only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/cos_hbm
mkdir -p $OUT
ARGS="${COS_ARGS:-1000000 500000000 8192 100}"
i=0
for grp in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 scripts/topk_all_probe.py $ARGS > $OUT/p$i.log 2>&1 || exit 1
  echo "pass $i ok"
done
