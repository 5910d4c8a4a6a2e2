# Device-encode check: the encode parity tests, then the bench's encode and C5
# legs (no CPU legs), then the C5 decode units timed alone.
set -o pipefail
mkdir -p gpurun_out
tag=${1:-enc}
timeout -k 10 500 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_encode.py tests/test_gpu_encode_adaptive.py tests/test_gpu_encode_binary_bool.py > gpurun_out/${tag}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu --no-b12 --no-hard --no-c3 --no-c4 --no-file --steps 10 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -5 gpurun_out/${tag}_bench.err; exit 1; }
python -c "
import json
d=json.loads(open('gpurun_out/${tag}_bench.json').read().strip().splitlines()[-1])
c5=d.get('c5_mixed_64col',{}); print('C5 ms', c5.get('ms_per_step'), 'enc GB/s', c5.get('encode_gpu_GBps'), 'ident', c5.get('encode_byte_identical'))
print(json.dumps(d.get('encode_gpu')))"
timeout -k 10 200 python tools/c5units.py > gpurun_out/${tag}_c5units.log 2>&1; rc=$?; cat gpurun_out/${tag}_c5units.log | grep -v amdgpu.ids; exit $rc
