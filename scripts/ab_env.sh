#!/bin/bash
# EXPERIMENT: the headline ingest (config-3 shape) under several settings.
# Each argument is one arm: "name:VAR=val,VAR2=val" (environment) or
# "name:@lib" (library _variants/lib_<lib>.so).  Optional TESTS="<pytest -k expr>"
# runs those GPU tests first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "$TESTS" > gpurun_out/ab/pytest.log 2>&1 || { tail -30 gpurun_out/ab/pytest.log; exit 1; }
  tail -2 gpurun_out/ab/pytest.log
fi
B="python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-extras --no-config1 --no-config2 --no-cosine-1m"
for arm in "$@"; do
  name=${arm%%:*}
  spec=${arm#*:}
  if [ "${spec:0:1}" = "@" ]; then
    MAHOUT_CMS_LIB=_variants/lib_${spec:1}.so timeout -k 10 200 $B > gpurun_out/ab/$name.json 2> gpurun_out/ab/$name.err || exit 1
  else
    env $(echo "$spec" | tr ',' ' ') timeout -k 10 200 $B > gpurun_out/ab/$name.json 2> gpurun_out/ab/$name.err || exit 1
  fi
  echo "$name ok"
done
for arm in "$@"; do python scripts/bench_brief.py gpurun_out/ab/${arm%%:*}.json; done
