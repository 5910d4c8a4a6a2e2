# full -m gpu suite, C2 headline, Utf8 kinds, C5
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03c_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r03c_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu --no-b12 --no-hard --no-c3 --no-c4 --no-c5 --no-encode --no-file > gpurun_out/r03c_c2.json 2> gpurun_out/r03c_c2.err
rc=$?; echo "c2 rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/r03c_c2.json'));print(d['value'],d['roofline']['frac'],d['roofline']['kernel_ms'])"
timeout -k 10 200 python tools/binbench.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python tools/wlbench.py c5 10 3 2>&1 | grep -v amdgpu.ids
