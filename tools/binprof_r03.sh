# rocprofv3 kernel stats of the Utf8 C5-kind decodes, one kind per run
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for k in ${KINDS:-dict freq one}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/binprof_$k -o k -- python3 tools/binbench.py 8388608 $k > gpurun_out/binprof_$k.log 2>&1 || { echo "prof $k failed"; tail -3 gpurun_out/binprof_$k.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/binprof_$k.log | tail -1
  grep -h "k_bin\|k_utf8\|k_inflate" gpurun_out/binprof_$k/k_kernel_stats.csv | cut -d, -f1-4
done
