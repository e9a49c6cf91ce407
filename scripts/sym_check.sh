#!/bin/bash
# EXPERIMENT: k_cosine_sym correctness (top-k tests, default and with the old
# waves) and the config-4 job A/B (CMS_OLD_SYM=1 = k_cosine_big waves).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider \
    --timeout 300 --timeout-method thread -k "top_k_all or all_pairs" > gpurun_out/pytest_sym.log 2>&1 \
  && echo "sym tests ok" \
  && CMS_OLD_SYM=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread -k "top_k_all" > gpurun_out/pytest_oldsym.log 2>&1 \
  && echo "old-sym tests ok" \
  && timeout -k 10 400 python -u scripts/cos_job_probe.py 1000000 500000000 8192 100 1 > gpurun_out/cos_a.json 2> gpurun_out/cos_a.err \
  && echo "A: $(tail -c 700 gpurun_out/cos_a.json)" \
  && timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize_1m.py -m gpu -x -q -p no:cacheprovider --timeout 500 --timeout-method thread > gpurun_out/pytest_sym1m.log 2>&1 \
  && echo "1M test ok"
