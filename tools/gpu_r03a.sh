# round-3 check: the spill / big-page tests, the whole -m gpu suite, C3 timing.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_spill.py tests/test_gpu_binary.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03a_spill.log 2>&1
rc=$?; echo "spill rc=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/r03a_spill.log | tail -25; tail -5 gpurun_out/r03a_spill.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03a_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r03a_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/wlbench.py c3 10 3 > gpurun_out/r03a_c3.log 2>&1
rc=$?; echo "c3 rc=$rc"; tail -3 gpurun_out/r03a_c3.log
timeout -k 10 300 python tools/wlbench.py c5 10 3 > gpurun_out/r03a_c5.log 2>&1
rc=$?; echo "c5 rc=$rc"; tail -3 gpurun_out/r03a_c5.log; exit $rc
