#!/bin/bash
# EXPERIMENT: bound analysis of the config-4 job's symmetric waves: the
# bound-analysis build (CMS_BOUND_ANALYSIS) with parts of k_cosine_big
# switched off by CMS_COS_MODE (bit0 loads, bit1 MFMA, bit2 epilogue).
# Results are wrong by design in modes != 0; only the wave timings matter.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CMS_BOUND_ANALYSIS=1 python -m mahout_amd.build_lib > gpurun_out/analysis_build.log 2>&1 || exit 1
for m in ${MODES:-0 4 2 1}; do
  CMS_COS_MODE=$m timeout -k 10 300 python -u scripts/cos_job_probe.py 1000000 500000000 8192 100 0 > gpurun_out/jmode_$m.json 2> gpurun_out/jmode_$m.err || exit 1
  echo "mode $m: $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); t=d["timing_ms"]; print({k: round(v[0]) for k,v in t.items()})' gpurun_out/jmode_$m.json)"
done
