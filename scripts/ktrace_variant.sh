#!/bin/bash
# EXPERIMENT: rocprofv3 kernel trace of the headline ingest with the product
# library and with each bound-analysis variant in _variants/ (MAHOUT_CMS_LIB);
# per-kernel average durations side by side (scripts/ktrace_table.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --no-config1 --no-config2 --no-cosine-1m"
rm -rf gpurun_out/kt && mkdir -p gpurun_out/kt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt/base -o run --output-format csv -- $B > gpurun_out/kt/base.log 2>&1 || exit 1
for v in "$@"; do
  MAHOUT_CMS_LIB=_variants/lib_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt/$v -o run --output-format csv -- $B > gpurun_out/kt/$v.log 2>&1 || exit 1
done
