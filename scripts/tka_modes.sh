#!/bin/bash
# EXPERIMENT: cms_top_k_all at 1M with kernel parts toggled (CMS_COS_MODE)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
# the knobs exist only in the bound-analysis build of the library
CMS_BOUND_ANALYSIS=1 python -m mahout_amd.build_lib > gpurun_out/analysis_build.log 2>&1 || exit 1
for m in ${MODES:-0 4}; do
  CMS_COS_MODE=$m timeout -k 10 300 python scripts/topk_all_probe.py 1000000 500000000 8192 100 > gpurun_out/tka_mode_$m.json 2>&1 || exit 1
  echo "mode $m: $(tail -1 gpurun_out/tka_mode_$m.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["wall_s"],2), round(d["timing_ms"]["topk_all_waves"]))')"
done
