#!/bin/bash
# EXPERIMENT: partition tests + config-2 bench A/B of the hot-owner routing
# (CMS_NO_HOT_ROUTING=1 is the plain two-pass partition).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v -p no:cacheprovider \
    --timeout 300 --timeout-method thread -k "${TESTS:-partition or ingest or fullsize}" > gpurun_out/pytest_part.log 2>&1 \
  && echo "tests ok" \
  && timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --no-cosine-1m > gpurun_out/bench_hot.json 2> gpurun_out/bench_hot.err \
  && CMS_NO_HOT_ROUTING=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --no-cosine-1m > gpurun_out/bench_twopass.json 2> gpurun_out/bench_twopass.err \
  && python3 scripts/bench_brief.py gpurun_out/bench_hot.json gpurun_out/bench_twopass.json
