#!/bin/bash
# top-k parity tests, then the config-4 probe twice: default and with AB_ENV
# (e.g. AB_ENV=CMS_NO_RECT=1) for an A/B of the all-pairs kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "top_k or all_pairs" --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 \
  && tail -1 gpurun_out/ab_tests.log \
  && timeout -k 10 300 python scripts/topk_all_probe.py > gpurun_out/ab_a.json 2> gpurun_out/ab.err \
  && { [ -z "$AB_ENV" ] || timeout -k 10 300 env $AB_ENV python scripts/topk_all_probe.py > gpurun_out/ab_b.json 2>> gpurun_out/ab.err; } \
  && python - <<'PY'
import json, os
for f in ["gpurun_out/ab_a.json", "gpurun_out/ab_b.json"]:
    if os.path.exists(f):
        d = json.load(open(f)); t = d["timing_ms"]
        print(f, "wall", round(d["wall_s"], 3), "f4", round(t["topk_all_waves_f4"]), "i8", round(t["topk_all_waves_i8"]),
              "multi", round(t["topk_all_multi_rows"]), "spot", d["spot_check_rows_equal"], "full", d["full_lists"])
PY
