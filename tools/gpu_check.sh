#!/bin/bash
# One GPU round trip: the -m gpu suite, then the Patas column bench (and its
# phase variant when built), then a C5-only bench line.  Each step under its
# own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 60 python -u tools/patasbench.py > gpurun_out/pb.log 2>&1 || { cat gpurun_out/pb.log; exit 1; }
if [ -f pa_amd/variants/libsb_patph.so ]; then
  PA_AMD_LIB=pa_amd/variants/libsb_patph.so timeout -k 10 60 python -u tools/patasbench.py >> gpurun_out/pb.log 2>&1 || { cat gpurun_out/pb.log; exit 1; }
fi
grep -v amdgpu.ids gpurun_out/pb.log
if [ -n "$BENCH_ARGS" ]; then
  timeout -k 10 300 python -u bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
