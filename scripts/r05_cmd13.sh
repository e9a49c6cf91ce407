set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_per_owner.py > gpurun_out/pytest_po.log 2>&1 && tail -2 gpurun_out/pytest_po.log && \
CMS_PO_BOUND_ROWS=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_per_owner.py -k "big_queries or grouped or wide" > gpurun_out/pytest_po2.log 2>&1 && tail -2 gpurun_out/pytest_po2.log && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/po -o run --output-format csv -- python3 scripts/po_scale_probe.py 1024 120 20261015 > gpurun_out/po_probe.log 2>&1 && grep -v "^[WEI]2026" gpurun_out/po_probe.log | tail -3 && python3 scripts/kstats.py gpurun_out/po 8 && \
CMS_PO_BOUND_ROWS=2 timeout -k 10 600 python3 scripts/po_scale_probe.py 1024 120 20261015 > gpurun_out/po_probe2.log 2>&1 && tail -2 gpurun_out/po_probe2.log && \
CMS_PO_DENSE_X4=1 timeout -k 10 600 python3 scripts/po_scale_probe.py 1024 120 20261015 > gpurun_out/po_probe3.log 2>&1; rc=$?; tail -2 gpurun_out/po_probe3.log; exit $rc
