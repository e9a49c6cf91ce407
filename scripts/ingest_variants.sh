#!/bin/bash
# EXPERIMENT: config-2 ingest step with library variants (MAHOUT_CMS_LIB)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in "" ${LIBS}; do
  MAHOUT_CMS_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --no-cosine-1m > gpurun_out/iv.json 2>&1 || exit 1
  echo "lib '${lib:-default}': $(tail -1 gpurun_out/iv.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e9,2), d["breakdown_ms_per_step"])')"
done
