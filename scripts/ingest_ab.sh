#!/bin/bash
# EXPERIMENT: config-2 and config-3-shaped ingest steps, default library vs ${LIBS} (MAHOUT_CMS_LIB)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
C3="--n-items 1000000 --n-users 10000000 --pairs 500000000 --width 8192"
for shape in "" "$C3"; do
  for lib in "" ${LIBS}; do
    MAHOUT_CMS_LIB=$lib timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras --no-cosine-1m $shape > gpurun_out/iab.json 2>&1 || exit 1
    echo "shape '${shape:-config2}' lib '${lib:-default}': $(tail -1 gpurun_out/iab.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e9,2), round(d["ms_per_step"],3), d["breakdown_ms_per_step"])')"
  done
done
