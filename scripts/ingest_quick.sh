#!/bin/bash
# Ingest parity tests + the config-2 bench line alone (no extras / cosine).
# BENCH_ENV (optional) is prepended to a second bench run for A/B experiments.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --no-cosine-1m"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "ingest or csr or values or accumulate or movielens" --timeout 120 --timeout-method thread > gpurun_out/iq_tests.log 2>&1 \
  && tail -1 gpurun_out/iq_tests.log \
  && timeout -k 10 300 $B > gpurun_out/iq_bench.json 2> gpurun_out/iq_bench.err \
  && { [ -z "$BENCH_ENV" ] || timeout -k 10 300 env $BENCH_ENV $B > gpurun_out/iq_bench_b.json 2>> gpurun_out/iq_bench.err; } \
  && python scripts/bench_brief.py gpurun_out/iq_bench.json gpurun_out/iq_bench_b.json
