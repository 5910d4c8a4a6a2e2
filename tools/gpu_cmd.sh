bash tools/gpu_tests.sh pt1 -m gpu tests/test_gpu_decode.py tests/test_gpu_spill.py tests/test_gpu_configs.py tests/test_gpu_table.py tests/test_oracle_kat.py -k "atas or f64 or float or double or c5 or table" > /dev/null; rc=$?; tail -2 gpurun_out/pt1.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python tools/kindbench.py 8388608 float64:patas,float64:lz4 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --no-cpu --no-b12 --no-hard --no-c3 --no-c4 --no-encode --no-file --steps 10 > gpurun_out/pt1.json 2>/dev/null || exit 1
python -c "
import json; d=json.loads(open('gpurun_out/pt1.json').read().strip().splitlines()[-1]); x=d['c5_mixed_64col']; print('c5', x['ms_per_step'], x['roofline_frac'], x['bit_exact'])"
