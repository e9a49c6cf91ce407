#!/bin/bash
# EXPERIMENT: the config-4 job (scripts/cos_job_probe.py, one table build,
# first + timed job) under environment settings, one run per argument
# ("NAME=VALUE ..." or "base"); prints wall and per-phase ms of each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cenv
i=0
for e in "$@"; do
  i=$((i+1))
  if [ "$e" = base ]; then timeout -k 10 300 python -u scripts/cos_job_probe.py 1000000 500000000 8192 100 0 > gpurun_out/cenv/$i.json 2> gpurun_out/cenv/$i.err || exit 1
  else env $e timeout -k 10 300 python -u scripts/cos_job_probe.py 1000000 500000000 8192 100 0 > gpurun_out/cenv/$i.json 2> gpurun_out/cenv/$i.err || exit 1; fi
  python - "$e" gpurun_out/cenv/$i.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2])); t = d["timing_ms"]
print(sys.argv[1], "wall", round(d["wall_timed_s"], 3), "first", round(d["wall_first_s"], 3), "f4", round(t["topk_all_waves_f4"][0]),
      "i8", round(t["topk_all_waves_i8"][0]), "multi", round(t["topk_all_multi_rows"][0]), "full", d["full_lists"], flush=True)
PY
done
