#!/bin/bash
# Bound analysis of the symmetric waves: the config-4 job (cos_job_probe.py)
# on the main library and on k_cosine_sym probe builds (CMS_SYM_PROBE bit
# flags, cms_cosine_sym.hip), each arm under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ARMS=${ARMS:-"main $(ls ab/*.so 2>/dev/null | tr '\n' ' ')"}
for arm in $ARMS; do
  envs=()
  case "$arm" in
    main) tag=main ;;
    *) envs=(MAHOUT_CMS_LIB="$PWD/$arm"); tag=$(basename "$arm" .so) ;;
  esac
  env "${envs[@]}" timeout -k 10 240 python -u scripts/cos_job_probe.py 1000000 500000000 8192 100 0 \
      > gpurun_out/sym_${tag}.json 2> gpurun_out/sym_${tag}.err || { echo "arm $tag failed"; tail -5 gpurun_out/sym_${tag}.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'first', round(d['wall_first_s'],3), 'steady', round(d['wall_timed_s'],3), {k: round(v[0],1) for k, v in d['timing_ms'].items()})" gpurun_out/sym_${tag}.json $tag
done
