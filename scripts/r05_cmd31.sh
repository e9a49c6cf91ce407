set -o pipefail
STEPS="tests ab" TESTS="tests/test_gpu_parity.py tests/test_gpu_forms.py tests/test_gpu_edges.py tests/test_gpu_fullsize.py tests/test_gpu_fullsize_1m.py tests/test_gpu_config5_stream.py tests/test_gpu_transport.py" ARMS="main ab/base.so env:CMS_EARLY_SLICES=0 main ab/base.so env:CMS_EARLY_SLICES=0" bash scripts/r05_iter.sh
