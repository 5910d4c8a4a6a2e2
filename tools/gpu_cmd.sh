bash tools/gpu_tests.sh w1 -m gpu tests/test_gpu_encode.py tests/test_gpu_encode_adaptive.py tests/test_gpu_encode_binary_bool.py tests/test_lz4c.py > /dev/null; rc=$?; tail -2 gpurun_out/w1.log; [ $rc = 0 ] || exit $rc
bash tools/gpu_r04.sh prof c5e3 tools/c5enc.py > /dev/null; grep "c5 encode" gpurun_out/c5e3_kt.log
timeout -k 10 300 python bench.py --no-cpu --no-b12 --no-hard --no-c3 --no-c4 --no-file --no-c5 --steps 5 > gpurun_out/w1_bench.json 2>&1; python -c "
import json; d=json.loads(open('gpurun_out/w1_bench.json').read().strip().splitlines()[-1]); print(json.dumps(d.get('encode_gpu')))"
