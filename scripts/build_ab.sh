#!/bin/bash
# EXPERIMENT: the headline ingest (config-3 shape) with bound-analysis library
# variants built by scripts/build_variants.sh into _variants/ (MAHOUT_CMS_LIB):
# the k_build_rows time of each, beside the product library's.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
B="python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras --no-config1 --no-config2 --no-cosine-1m"
timeout -k 10 200 $B > gpurun_out/ab/base.json 2> gpurun_out/ab/base.err || exit 1
for v in "$@"; do
  MAHOUT_CMS_LIB=_variants/lib_$v.so timeout -k 10 200 $B > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err || exit 1
done
python scripts/bench_brief.py gpurun_out/ab/*.json
