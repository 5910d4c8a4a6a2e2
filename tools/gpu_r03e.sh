set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_binary.py tests/test_gpu_binary_errors.py tests/test_gpu_big_pages.py tests/test_gpu_nested.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03e_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r03e_tests.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="old new" bash tools/ab_bin.sh
