#!/bin/bash
# Round-5 closing run on a GPU box: the whole -m gpu suite, smoke, the full
# bench line, then the config-4 job's rocprofv3 passes (kernel stats, MFMA /
# wait, LDS, L2, FETCH).  Each GPU step has its own time limit; a crash, fault
# or time limit ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended with status $rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 700 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err \
  || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
echo "bench ok"
python -c "import json; print(json.dumps(json.load(open('gpurun_out/bench.json'))['summary']))"
[ "${SKIP_COS_PROF:-0}" = 1 ] || bash scripts/profile_r05.sh cosine || exit 1
exit $rc
