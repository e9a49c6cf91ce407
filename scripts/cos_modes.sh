#!/bin/bash
# EXPERIMENT: bound analysis of k_cosine_big (loads / MFMA / epilogue toggled off)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for m in 0 1 2 4 6 3; do
  CMS_COS_MODE=$m timeout -k 10 300 python scripts/cosine_probe.py ${N:-1000000} ${P:-500000000} ${W:-8192} ${Q:-2048} ${Q0:-500000} > gpurun_out/mode_$m.json 2>&1 || exit 1
  echo "mode $m: $(tail -1 gpurun_out/mode_$m.json)"
done
