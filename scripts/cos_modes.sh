#!/bin/bash
# EXPERIMENT: bound analysis of k_cosine_big (loads / MFMA / epilogue toggled off)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
# the knobs exist only in the bound-analysis build of the library
CMS_BOUND_ANALYSIS=1 python -m mahout_amd.build_lib > gpurun_out/analysis_build.log 2>&1 || exit 1
for bk in ${BKS:-64 128}; do
for m in ${MODES:-0 1 6}; do
  CMS_COS_BK=$bk CMS_COS_MODE=$m timeout -k 10 300 python scripts/cosine_probe.py ${N:-1000000} ${P:-500000000} ${W:-8192} ${Q:-2048} ${Q0:-500000} > gpurun_out/mode_${bk}_$m.json 2>&1 || exit 1
  echo "bk $bk mode $m: $(tail -1 gpurun_out/mode_${bk}_$m.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["mfma_ms"],1), round(d["limbs_ms"],1))')"
done
done
