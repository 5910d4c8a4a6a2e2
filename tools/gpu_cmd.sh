bash tools/gpu_tests.sh h1 -m gpu tests/test_gpu_decode.py tests/test_gpu_lz4_long.py tests/test_gpu_binary.py tests/test_gpu_configs.py tests/test_gpu_spill.py > /dev/null; rc=$?; tail -2 gpurun_out/h1.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python tools/c3bench.py 100000000 2>&1 | grep -v amdgpu.ids
for m in own torch; do
SB_BENCH_STREAMS=$m timeout -k 10 300 python bench.py --no-cpu --no-b12 --no-hard --no-c4 --no-encode --no-file --steps 10 > gpurun_out/ab_$m.json 2>/dev/null || exit 1
python -c "
import json; d=json.loads(open('gpurun_out/ab_$m.json').read().strip().splitlines()[-1])
print('$m', 'c3', d['c3_f64_utf8_lz4_nullable']['ms_per_step'], 'c5', d['c5_mixed_64col']['ms_per_step'], 'enc', d['c5_mixed_64col']['encode_gpu_GBps'])"
done
