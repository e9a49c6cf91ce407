#!/bin/bash
# One GPU-box session: parity tests, smoke, a short bench, a rocprofv3 summary.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
  && echo "pytest gpu ok" \
  && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
  && echo "smoke ok" \
  && timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err \
  && echo "bench ok" && cat gpurun_out/bench.json
