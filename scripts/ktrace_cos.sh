#!/bin/bash
# EXPERIMENT: kernel trace of the config-4 job (scripts/cos_job_probe.py, first
# + timed job) with the environment given as arguments; top kernels by time.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/ktc && mkdir -p gpurun_out/ktc
env "${@:-CMS_NOTHING=1}" timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/ktc -o run --output-format csv -- \
    python3 scripts/cos_job_probe.py 1000000 500000000 8192 100 0 > gpurun_out/ktc/log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/ktc/**/run_kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in rows[:14]:
    print(f'{float(r["TotalDurationNs"])/1e6:10.1f} ms {int(r["Calls"]):5d} calls {float(r["AverageNs"])/1e6:9.2f} ms avg  {r["Name"][:90]}')
PY
