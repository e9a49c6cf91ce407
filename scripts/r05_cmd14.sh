set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_per_owner.py > gpurun_out/pytest_po.log 2>&1 && tail -2 gpurun_out/pytest_po.log && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/po -o run --output-format csv -- python3 scripts/po_scale_probe.py 1024 150 20261015 > gpurun_out/po_probe.log 2>&1; rc=$?; grep -v "^[WEI]2026" gpurun_out/po_probe.log | tail -3; python3 scripts/kstats.py gpurun_out/po 8; exit $rc
