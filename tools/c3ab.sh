# usage: bash tools/c3ab.sh "variant ..." [rows]: c3bench per decode-kernel variant
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/c3ab_$(date +%H%M%S).txt
for v in $1; do
  echo "== $v" >> $out
  PA_AMD_LIB=pa_amd/variants/libsb_$v.so timeout -k 10 200 python tools/c3bench.py ${2:-100000000} >> $out 2>&1 || { echo "variant $v failed"; tail -5 $out; exit 1; }
done
grep -v amdgpu.ids $out
