#!/bin/bash
# A/B of decode-kernel variant libraries (pa_amd/variants/libsb_<name>.so;
# "cur" = the in-tree library): per variant, the TESTS pytest selection
# (bit-exactness first, when set), then SCRIPT (a timing script and its
# args).  bash tools/gpu_ab.sh name ...   e.g.
#   TESTS="tests/test_gpu_configs.py -k c4" SCRIPT="tools/c4bench.py" bash tools/gpu_ab.sh cur vecdw
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = cur ]; then lib=""; else lib=pa_amd/variants/libsb_$v.so; fi
  echo "== $v"
  if [ -n "$TESTS" ]; then
    PA_AMD_LIB=$lib timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
      $TESTS > gpurun_out/ab_check_$v.log 2>&1 || { tail -15 gpurun_out/ab_check_$v.log; exit 1; }
    tail -1 gpurun_out/ab_check_$v.log
  fi
  PA_AMD_LIB=$lib timeout -k 10 200 python -u $SCRIPT > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/ab_$v.log
done
