bash tools/gpu_tests.sh bl1 -m gpu tests/test_gpu_binary.py tests/test_gpu_binary_errors.py tests/test_gpu_utf8.py tests/test_gpu_big_pages.py tests/test_gpu_table.py > /dev/null; rc=$?; tail -2 gpurun_out/bl1.log; [ $rc = 0 ] || exit $rc
PA_AMD_LIB=pa_amd/variants/libsb_phases.so timeout -k 10 200 python tools/binphases.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --no-cpu --no-b12 --no-hard --no-c3 --no-c4 --no-encode --no-file --steps 10 > gpurun_out/bl1.json 2>/dev/null || exit 1
python -c "
import json; d=json.loads(open('gpurun_out/bl1.json').read().strip().splitlines()[-1]); x=d['c5_mixed_64col']; print('c5', x['ms_per_step'], x['roofline_frac'], x['bit_exact'])"
