#!/bin/bash
# EXPERIMENT: the config-4 job (scripts/cos_job_probe.py, one untimed warm
# call) under several library builds / env settings.  VARIANTS is a
# ';'-separated list of "label|lib path or -|ENV=VAL ..." entries.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
IFS=';' read -ra VS <<< "$VARIANTS"
for v in "${VS[@]}"; do
  IFS='|' read -r label lib envs <<< "$v"
  [ "$lib" = "-" ] && lib=""
  env MAHOUT_CMS_LIB=$lib $envs timeout -k 10 ${VTIMEOUT:-150} python -u scripts/cos_job_probe.py 1000000 500000000 8192 100 0 \
      > gpurun_out/var_$label.json 2> gpurun_out/var_$label.err || { echo "$label failed"; exit 1; }
  echo "$label: $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); t=d["timing_ms"]; print(round(d["wall_timed_s"],3), {k: round(v[0]) for k,v in t.items() if v[0]}, d["stats"]["topk_redo"])' gpurun_out/var_$label.json)"
done
