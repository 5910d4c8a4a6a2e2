# Encode parity tests, then C2 / C5 device encode timings against variant
# libraries (pa_amd/variants/libsb_<name>.so): bash tools/gpu_enc_ab.sh name ...
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_gpu_encode.py tests/test_gpu_encode_adaptive.py tests/test_gpu_encode_binary_bool.py tests/test_gpu_encode_list.py > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc = 0 ] || exit $rc
for v in "$@" cur; do
  if [ "$v" = cur ]; then lib=""; else lib=pa_amd/variants/libsb_$v.so; fi
  PA_AMD_LIB=$lib timeout -k 10 150 python tools/enc_c2.py > gpurun_out/ab_c2_$v.log 2>&1 || { tail -5 gpurun_out/ab_c2_$v.log; exit 1; }
  echo "$v C2: $(python -c "import json,sys; d=json.loads(open('gpurun_out/ab_c2_$v.log').read().strip().splitlines()[-1]); print({k: (v['ms_per_call'], v['byte_identical_to_host']) for k, v in d.items() if 'ms_per_call' in v})")"
done
bash tools/gpu_c5enc_ab.sh "$@" cur
