# usage: bash tools/stab.sh "variant ..." [kernel]: kernel time per decode-kernel variant on C4 (20M rows)
set -o pipefail
mkdir -p gpurun_out
k=${2:-k_list_levels}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in $1; do
  SB_NOCHECK=1 PA_AMD_LIB=pa_amd/variants/libsb_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stab_$v -o x -- python3 tools/c4bench.py 50000000 > gpurun_out/stab_$v.log 2>&1 || echo "($v: python failed; kernels still traced)"
  echo "== $v $(grep ms/step gpurun_out/stab_$v.log)"; grep $k gpurun_out/stab_$v/x_kernel_stats.csv | cut -d, -f1-4
done
