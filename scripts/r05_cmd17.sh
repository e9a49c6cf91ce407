set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 - > gpurun_out/rec.json 2> gpurun_out/rec.err <<'PY'
import json, sys
sys.path.insert(0, ".")
import bench
print(json.dumps(bench.config1_recommender()))
PY
rc=$?; tail -c 1500 gpurun_out/rec.json; tail -5 gpurun_out/rec.err; [ $rc -eq 0 ] || exit $rc
STEPS="ab" ARMS="main env:CMS_MID_U8_IMAGE=1 main env:CMS_MID_U8_IMAGE=1" bash scripts/r05_iter.sh
