# usage: bash tools/abrun.sh "variant ..." "workload ..."
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_$(date +%H%M%S).txt
for v in $1; do
  echo "== $v" >> $out
  PA_AMD_LIB=pa_amd/variants/libsb_$v.so timeout -k 10 200 python tools/kbench.py 100000000 $2 >> $out 2>&1 || { echo "variant $v failed"; tail -5 $out; exit 1; }
done
grep -v amdgpu.ids $out
