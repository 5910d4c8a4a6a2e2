# Utf8 C5-kind decode timings and their kernel split (rocprofv3 kernel trace).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/binbench.py > gpurun_out/binbench.log 2>&1 || { tail -5 gpurun_out/binbench.log; exit 1; }
cat gpurun_out/binbench.log | grep -v amdgpu.ids
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/binprof -o k -- python3 tools/binbench.py > gpurun_out/binprof.log 2>&1 || { tail -5 gpurun_out/binprof.log; exit 1; }
python3 tools/prof_summary.py trace $(ls gpurun_out/binprof/*kernel_trace.csv) 4 gpurun_out/binprof.json | head -60
