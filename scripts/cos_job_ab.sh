#!/bin/bash
# EXPERIMENT: top-k tests, then the config-4 job (scripts/cos_job_probe.py)
# with and without an env knob (AB_ENV, e.g. CMS_NO_I8BLK=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize_1m.py -m gpu -x -v -p no:cacheprovider \
    --timeout 400 --timeout-method thread -k "${TESTS:-top_k_all or all_pairs or fullsize}" > gpurun_out/pytest_cos.log 2>&1 \
  && echo "tests ok" \
  && timeout -k 10 400 python -u scripts/cos_job_probe.py 1000000 500000000 8192 100 1 > gpurun_out/cos_a.json 2> gpurun_out/cos_a.err \
  && echo "A: $(tail -c 600 gpurun_out/cos_a.json)" \
  && env ${AB_ENV:-CMS_NOTHING=1} timeout -k 10 400 python -u scripts/cos_job_probe.py 1000000 500000000 8192 100 1 > gpurun_out/cos_b.json 2> gpurun_out/cos_b.err \
  && echo "B (${AB_ENV}): $(tail -c 600 gpurun_out/cos_b.json)"
