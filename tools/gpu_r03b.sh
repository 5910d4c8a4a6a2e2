# binary / spill parity, Utf8 kind timings, C2 headline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_spill.py tests/test_gpu_binary.py tests/test_gpu_bool.py tests/test_gpu_decode.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03b_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r03b_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/binbench.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --no-cpu --no-b12 --no-hard --no-c3 --no-c4 --no-c5 --no-encode --no-file > gpurun_out/r03b_c2.json 2> gpurun_out/r03b_c2.err
rc=$?; echo "c2 rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/r03b_c2.json'));print(d['value'],d['roofline']['frac'],d['roofline']['kernel_ms'])"
timeout -k 10 300 python tools/wlbench.py c5 10 3 2>&1 | grep -v amdgpu.ids
