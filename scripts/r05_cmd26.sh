set -o pipefail
CMS_BUILD_STREAMS=3 STEPS="tests ab" TESTS="tests/test_gpu_parity.py tests/test_gpu_forms.py tests/test_gpu_fullsize.py" ARMS="main env:CMS_BUILD_STREAMS=2 ab/base.so main env:CMS_BUILD_STREAMS=2 ab/base.so" bash scripts/r05_iter.sh
