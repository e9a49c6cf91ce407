#!/bin/bash
# Round-4 iteration on a GPU box: parity tests, smoke, a kernel trace of the
# headline ingest, then the full bench.  Each GPU step has its own time limit.
# A test FAILURE (pytest exit 1) still lets the measurements run; a crash,
# abort, fault or time limit (any other non-zero status) ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-tests}
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended with status $rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/smoke.log; exit 1; }
echo "smoke ok"
rm -rf gpurun_out/prof_ingest
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ingest -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras --no-config1 --no-config2 --no-cosine-1m \
    > gpurun_out/prof_ingest.log 2>&1 || { echo "ingest trace failed"; exit 1; }
echo "ingest trace ok"
timeout -k 10 700 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err \
  || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
echo "bench ok"
python -c "import json; print(json.dumps(json.load(open('gpurun_out/bench.json'))['summary']))"
# A/B arms of the ingest step: ARMS (default: the main library, every variant
# library under ab/, then env:NAME=VALUE arms on the main library); variant
# libraries are built on the CPU side with build_lib.py --define ... --out ab/<name>.so
ARMS=${ARMS:-"main $(ls ab/*.so 2>/dev/null | tr '\n' ' ')"}
for arm in $ARMS; do
  envs=()
  case "$arm" in
    main) tag=main ;;
    env:*) envs=("${arm#env:}"); tag=$(echo "${arm#env:}" | tr '=' '_') ;;
    *) envs=(MAHOUT_CMS_LIB="$PWD/$arm"); tag=$(basename "$arm" .so) ;;
  esac
  env "${envs[@]}" timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras \
      --no-config1 --no-config2 --no-cosine-1m > gpurun_out/ab_${tag}.json 2> gpurun_out/ab_${tag}.err \
    || { echo "A/B arm $tag failed"; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], d.get('breakdown_ms_per_step'))" gpurun_out/ab_${tag}.json
done
exit $rc
