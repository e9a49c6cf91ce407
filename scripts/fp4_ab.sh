#!/bin/bash
# EXPERIMENT: cms_top_k_all at 1M, fp4 waves on vs off, and fp4 kernel parts toggled
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/topk_all_probe.py > gpurun_out/fp4_on.json 2>&1 || exit 1
CMS_BOUND_ANALYSIS=1 python -m mahout_amd.build_lib > gpurun_out/analysis_build.log 2>&1 || exit 1
CMS_NO_FP4=1 timeout -k 10 300 python scripts/topk_all_probe.py > gpurun_out/fp4_off.json 2>&1 || exit 1
for m in ${MODES:-1 2}; do
  CMS_COS_MODE=$m timeout -k 10 300 python scripts/topk_all_probe.py > gpurun_out/fp4_mode_$m.json 2>&1 || exit 1
done
