#!/bin/bash
# Session-5 probes: config-3 ingest at several hot-slice sizes, the owners'
# largest-counter histogram (operand classes), a config-5 refresh breakdown.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s5
export TMPDIR=/tmp
B="python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras --no-config1 --no-config2 --no-cosine-1m"
for sk in ${SLICES:-16384 32768 65536}; do
  CMS_SLICE_KEYS=$sk timeout -k 10 200 $B > gpurun_out/s5/slice_$sk.json 2> gpurun_out/s5/slice_$sk.err || exit 1
  echo "slice $sk ok"
done
for v in $VARIANTS; do
  MAHOUT_CMS_LIB=_variants/lib_$v.so timeout -k 10 200 $B > gpurun_out/s5/var_$v.json 2> gpurun_out/s5/var_$v.err || exit 1
  echo "variant $v ok"
done
python scripts/bench_brief.py gpurun_out/s5/slice_*.json gpurun_out/s5/var_*.json
if [ -n "$HIST" ]; then
  timeout -k 10 300 python scripts/rowmax_hist.py > gpurun_out/s5/rowmax.json 2> gpurun_out/s5/rowmax.err || exit 1
  cat gpurun_out/s5/rowmax.json
fi
if [ -n "$REFRESH" ]; then
  timeout -k 10 400 python scripts/refresh_probe.py 1 > gpurun_out/s5/refresh.log 2>&1 || exit 1
  tail -40 gpurun_out/s5/refresh.log
fi
