#!/bin/bash
# Round-6 iteration on a GPU box.  Steps (STEPS, space-separated, in order):
#   tests   -- pytest -m gpu ($TESTS, default tests/)
#   smoke   -- __graft_entry__.smoke()
#   trace   -- rocprofv3 kernel trace + stats of the headline ingest
#   prof_ingest / prof_cosine -- scripts/profile_r06.sh passes, summarized
#              into profiles/r06 (the bench step after them reads those)
#   ab      -- headline ingest bench per arm (ARMS: main, ab/*.so variant
#              libraries, env:NAME=VALUE arms)
#   bench   -- the full bench
# Each GPU step has its own time limit; a test FAILURE (pytest exit 1) lets
# the later steps run, any other non-zero status ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-"tests smoke ab"}
TESTS=${TESTS:-tests}
rc=0
for step in $STEPS; do
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest $TESTS -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread \
          > gpurun_out/pytest_gpu.log 2>&1
      rc=$?
      tail -3 gpurun_out/pytest_gpu.log
      grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu.log | head -20
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended with status $rc: stopping"; exit $rc; fi ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
        || { echo "smoke failed"; tail -5 gpurun_out/smoke.log; exit 1; }
      echo "smoke ok" ;;
    trace)
      rm -rf gpurun_out/prof_ingest
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ingest -o run --output-format csv -- \
          python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras --no-config1 --no-config2 --no-cosine-1m \
          > gpurun_out/prof_ingest.log 2>&1 || { echo "ingest trace failed"; exit 1; }
      python3 scripts/kstats.py gpurun_out/prof_ingest 30
      echo "ingest trace ok" ;;
    ab)
      ARMS=${ARMS:-"main $(ls ab/*.so 2>/dev/null | tr '\n' ' ')"}
      for arm in $ARMS; do
        envs=()
        case "$arm" in
          main) tag=main ;;
          env:*) IFS='+' read -r -a envs <<< "${arm#env:}"; tag=$(echo "${arm#env:}" | tr '=+/.' '____') ;;
          *) envs=(MAHOUT_CMS_LIB="$PWD/$arm"); tag=$(basename "$arm" .so) ;;
        esac
        env "${envs[@]}" timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras \
            --no-config1 --no-config2 --no-cosine-1m > gpurun_out/ab_${tag}.json 2> gpurun_out/ab_${tag}.err \
          || { echo "A/B arm $tag failed"; tail -5 gpurun_out/ab_${tag}.err; exit 1; }
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['ms_per_step'],3), d.get('breakdown_ms_per_step'))" gpurun_out/ab_${tag}.json
      done ;;
    ktrace)
      # per-arm kernel traces of the headline ingest (isolated kernel times
      # with a CMS_BUILD_SERIAL variant); table: scripts/ktrace_table.py
      KT_ARMS=${KT_ARMS:-${ARMS:-"main $(ls ab/*.so 2>/dev/null | tr '\n' ' ')"}}
      rm -rf gpurun_out/kt
      for arm in $KT_ARMS; do
        envs=()
        case "$arm" in
          main) tag=main ;;
          env:*) IFS='+' read -r -a envs <<< "${arm#env:}"; tag=$(echo "${arm#env:}" | tr '=+/.' '____') ;;
          *) envs=(MAHOUT_CMS_LIB="$PWD/$arm"); tag=$(basename "$arm" .so) ;;
        esac
        env "${envs[@]}" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt/$tag -o run --output-format csv -- \
            python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --no-config1 --no-config2 --no-cosine-1m \
            > gpurun_out/kt_$tag.log 2>&1 || { echo "ktrace arm $tag failed"; tail -5 gpurun_out/kt_$tag.log; exit 1; }
      done
      python3 scripts/ktrace_table.py gpurun_out/kt ;;
    prof_ingest)
      bash scripts/profile_r06.sh ingest || exit 1
      python3 scripts/summarize_profile.py gpurun_out/prof_ingest r06 || exit 1 ;;
    prof_cosine)
      bash scripts/profile_r06.sh cosine || exit 1
      python3 scripts/summarize_cos_pmc.py gpurun_out/prof_cosine r06 || exit 1 ;;
    bench)
      timeout -k 10 700 python bench.py --steps 10 --warmup 3 --detail-out gpurun_out/bench_detail.json > gpurun_out/bench.json 2> gpurun_out/bench.err \
        || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
      echo "bench ok"
      python3 -c "import json; print(json.dumps(json.load(open('gpurun_out/bench.json'))['summary']))" ;;
  esac
done
exit $rc
