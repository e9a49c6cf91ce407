set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_per_owner.py > gpurun_out/pytest_po.log 2>&1 && tail -3 gpurun_out/pytest_po.log && \
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/po -o run --output-format csv -- python3 scripts/po_scale_probe.py 1024 120 20261015 > gpurun_out/po_probe.log 2>&1; rc=$?; tail -3 gpurun_out/po_probe.log; python3 scripts/kstats.py gpurun_out/po 10; exit $rc
