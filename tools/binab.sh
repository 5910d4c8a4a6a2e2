# usage: bash tools/binab.sh "variant ...": C5 Utf8 kinds per binary-kernel variant (kernel trace)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in $1; do
  PA_AMD_LIB=pa_amd/variants/libsb_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/binab_$v -o x -- python3 tools/binbench.py > gpurun_out/binab_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/binab_$v.log; exit 1; }
  echo "== $v"; grep -E "^(dict|freq|one|lz4):" gpurun_out/binab_$v.log
  grep -E "k_bin" gpurun_out/binab_$v/x_kernel_stats.csv | cut -d, -f1-4
done
