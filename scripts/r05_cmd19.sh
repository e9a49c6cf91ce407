set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 scripts/po_scale_probe.py 1024 150 20261015 > gpurun_out/po_main.log 2>&1 && grep -o '"all_pairs": {"s": [0-9.]*' gpurun_out/po_main.log && \
MAHOUT_CMS_LIB=$PWD/ab/po32k.so timeout -k 10 300 python3 scripts/po_scale_probe.py 1024 150 20261015 > gpurun_out/po_32k.log 2>&1 && grep -o '"all_pairs": {"s": [0-9.]*' gpurun_out/po_32k.log
