#!/bin/bash
# EXPERIMENT: the headline ingest line under environment settings, one run per
# argument ("NAME=VALUE ..." or "base"), e.g. CMS_SLICE_KEYS=32768.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/envab
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras --no-config1 --no-cosine-1m"
i=0
for e in "$@"; do
  i=$((i+1))
  if [ "$e" = base ]; then timeout -k 10 200 $B > gpurun_out/envab/$i.json 2>/dev/null || exit 1
  else env $e timeout -k 10 200 $B > gpurun_out/envab/$i.json 2>/dev/null || exit 1; fi
  echo "$e: $(python scripts/bench_brief.py gpurun_out/envab/$i.json)"
  python -c "import json; d=json.load(open('gpurun_out/envab/$i.json')); c=d['config2']; print('   config2', round(c['updates_per_s']/1e9,2), c['breakdown_ms_per_step'])"
done
