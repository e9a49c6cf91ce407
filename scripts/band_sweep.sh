#!/bin/bash
# EXPERIMENT: wave-band schedule sweep for cms_top_k_all at 1M items
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
# the knobs exist only in the bound-analysis build of the library
CMS_BOUND_ANALYSIS=1 python -m mahout_amd.build_lib > gpurun_out/analysis_build.log 2>&1 || exit 1
for b in ${BANDS:-25,32 50,64 100,128}; do
  CMS_BAND=$b timeout -k 10 300 python scripts/topk_all_probe.py 1000000 500000000 8192 100 > gpurun_out/band_$b.json 2>&1 || exit 1
  echo "band $b: $(tail -1 gpurun_out/band_$b.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["wall_s"],2), round(d["waves_TOPS"]), d["stats"]["topk_redo"], d["spot_check_rows_equal"])')"
done
