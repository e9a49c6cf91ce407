#!/bin/bash
# EXPERIMENT: k_build_rows store forms (CMS_BUILD_SV 0: 8-B stores, 1: 16-B, 2: 16-B non-temporal)
# on the config-2 and config-3 ingest steps, after the ingest parity tests under each form.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
C3="--n-items 1000000 --n-users 10000000 --pairs 500000000 --width 8192"
for sv in 1 2; do
  CMS_BUILD_SV=$sv timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider \
    -k "ingest or csr or values or accumulate or movielens or full" --timeout 200 --timeout-method thread > gpurun_out/sab_tests_$sv.log 2>&1 || { tail -20 gpurun_out/sab_tests_$sv.log; exit 1; }
  echo "tests sv=$sv: $(tail -1 gpurun_out/sab_tests_$sv.log)"
done
for shape in "" "$C3"; do
  for sv in 0 1 2 0; do
    CMS_BUILD_SV=$sv timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --no-cosine-1m $shape > gpurun_out/sab.json 2>/dev/null || exit 1
    echo "shape '${shape:-config2}' sv $sv: $(tail -1 gpurun_out/sab.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e9,2), round(d["ms_per_step"],3), d["breakdown_ms_per_step"])')"
  done
done
