set -o pipefail
SB_DEBUG_VNONE=1 timeout -k 10 120 python -u tools/vn_debug.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_encode_adaptive.py tests/test_gpu_encode.py tests/test_lz4c.py > gpurun_out/enc_tests.log 2>&1; tail -2 gpurun_out/enc_tests.log
A="--no-cpu --no-b12 --no-hard --no-c3 --no-c4 --no-file --no-encode --steps 5"
for v in "X=1" "SB_LZ4E_NO_STAGE=1"; do env $v timeout -k 10 200 python -u bench.py $A > gpurun_out/c5e.json 2>/dev/null || exit 1; python -c "import json,sys; d=json.load(open(\"gpurun_out/c5e.json\"))[\"c5_mixed_64col\"]; print(\"$v\", d[\"ms_per_step\"], d[\"encode_gpu_GBps\"], d[\"encode_gpu_ms\"], d[\"encode_byte_identical\"])"; done
