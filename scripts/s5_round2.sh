#!/bin/bash
# Session-5 GPU batch: transport + per-owner tests, the no-write build bound,
# the per-owner mode at config-2 scale.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_transport.py tests/test_gpu_per_owner.py -x -v -p no:cacheprovider \
  --timeout 600 --timeout-method thread > gpurun_out/po.log 2>&1 || { tail -40 gpurun_out/po.log; exit 1; }
tail -3 gpurun_out/po.log
bash scripts/ab_env.sh base:X=1 nowrite:@CMS_BUILD_NOWRITE || exit 1
timeout -k 10 300 python -u scripts/po_scale_probe.py 64 > gpurun_out/po_scale.json 2> gpurun_out/po_scale.err || { tail -20 gpurun_out/po_scale.err; exit 1; }
cat gpurun_out/po_scale.json; tail -2 gpurun_out/po_scale.err
