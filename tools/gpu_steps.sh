# GPU session steps: bash tools/gpu_steps.sh <step> ...
#   tests "<pytest -k expr>" <files...>  : pytest subset (-m gpu), log under gpurun_out/
#   c3ab "<lib ...>" [rows]              : tools/c3bench.py per library (PA_AMD_LIB)
#   phases [rows]                        : tools/infphases.py on pa_amd/variants/libsb_phases.so
#   prof <tag> <script args...>          : rocprofv3 --kernel-trace --stats of a python script
set -o pipefail
mkdir -p gpurun_out
step=$1; shift
case $step in
  tests)
    k=$1; shift
    timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -k "$k" "$@" > gpurun_out/steps_tests.log 2>&1
    rc=$?; tail -4 gpurun_out/steps_tests.log; exit $rc ;;
  c3ab)
    for L in $1; do
      echo "== $L"
      PA_AMD_LIB=$L timeout -k 10 200 python tools/c3bench.py ${2:-100000000} 2>&1 | grep -v amdgpu.ids || exit 1
    done ;;
  prof)  # prof <tag> <python args...>: rocprofv3 kernel trace + stats of a python command, per-kernel summary
    tag=$1; script=$2; shift 2
    R=$GRAFT_REPO_ROOT
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${tag}_kt -o k -- python3 $R/$script "$@" > $R/gpurun_out/${tag}_kt.log 2>&1 || { echo "prof failed"; tail -5 $R/gpurun_out/${tag}_kt.log; exit 1; }
    cd $R && python3 tools/prof_summary.py trace gpurun_out/${tag}_kt/k_kernel_trace.csv 1 gpurun_out/${tag}_kernels.json | head -60 ;;
  phases)
    PA_AMD_LIB=pa_amd/variants/libsb_phases.so timeout -k 10 200 python tools/infphases.py ${1:-10000000} 2>&1 | grep -v amdgpu.ids ;;
esac
