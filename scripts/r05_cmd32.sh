set -o pipefail
STEPS="tests ab" TESTS="tests/test_gpu_parity.py tests/test_gpu_forms.py tests/test_gpu_edges.py tests/test_gpu_fullsize.py tests/test_gpu_fullsize_1m.py tests/test_gpu_config5_stream.py" ARMS="main ab/base.so main ab/base.so main ab/base.so" bash scripts/r05_iter.sh
