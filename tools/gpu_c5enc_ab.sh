# C5 table encode A/B over encoder variant libraries (pa_amd/variants/libsb_<name>.so;
# "cur" = the in-tree library): bash tools/gpu_c5enc_ab.sh name ...
set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do
  for v in "$@"; do
    if [ "$v" = cur ]; then lib=""; else lib=pa_amd/variants/libsb_$v.so; fi
    PA_AMD_LIB=$lib timeout -k 10 150 python tools/c5enc.py > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
    echo "$v: $(grep 'c5 encode' gpurun_out/ab_$v.log)"
  done
done
