#!/bin/bash
# Session-5 GPU batch: the whole GPU suite, then the headline ingest twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/pytest_gpu.log | head -30; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
bash scripts/ab_env.sh base:X=1 base2:X=2 ${ARMS}
