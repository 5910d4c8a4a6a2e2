set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in $1; do
  PA_AMD_LIB=pa_amd/variants/libsb_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lvab_$v -o x -- python3 tools/c4bench.py 20000000 > gpurun_out/lvab_$v.log 2>&1 || exit 1
  echo "== $v $(grep ms/step gpurun_out/lvab_$v.log)"; grep k_list_levels gpurun_out/lvab_$v/x_kernel_stats.csv | cut -d, -f1-4
done
