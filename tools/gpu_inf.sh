#!/bin/bash
# k_inflate evidence for C3 (LZ4 Float64 + Utf8): the columns timed alone per
# library (args: variant names under pa_amd/variants, "cur" = in-tree), the
# per-phase cycle split (libsb_phases.so, SB_INF_PHASES) and two passes of SQ
# counters (tools/pmc_sq.sh).  ROWS (default 20M) sizes the columns.
set -o pipefail
mkdir -p gpurun_out
rows=${ROWS:-20000000}
for v in "$@"; do
  if [ "$v" = cur ]; then lib=""; else lib=pa_amd/variants/libsb_$v.so; fi
  echo "== $v"
  if [ -n "$CHECK" ]; then  # bit-exact first: the C3 config tests and the long-literal LZ4 tests
    PA_AMD_LIB=$lib timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
      tests/test_gpu_configs.py -k c3 tests/test_gpu_lz4_long.py > gpurun_out/inf_check_$v.log 2>&1 || { tail -15 gpurun_out/inf_check_$v.log; exit 1; }
    tail -1 gpurun_out/inf_check_$v.log
  fi
  PA_AMD_LIB=$lib timeout -k 10 200 python -u tools/c3bench.py $rows > gpurun_out/inf_$v.log 2>&1 || { tail -5 gpurun_out/inf_$v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/inf_$v.log
done
if [ -f pa_amd/variants/libsb_phases.so ] && [ -z "$NO_PHASES" ]; then
  PA_AMD_LIB=pa_amd/variants/libsb_phases.so timeout -k 10 200 python -u tools/infphases.py $rows > gpurun_out/inf_phases.log 2>&1 || { tail -5 gpurun_out/inf_phases.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/inf_phases.log
fi
if [ -z "$NO_PMC" ]; then
  bash tools/pmc_sq.sh k_inflate tools/c3bench.py $rows || exit 1
fi
