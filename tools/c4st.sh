set -o pipefail
for v in base plain; do
  lib=pa_amd/libstrawboat_gpu.so; [ $v = plain ] && lib=pa_amd/variants/libsb_plain.so
  PA_AMD_LIB=$lib bash tools/kprof.sh c4s_$v python3 tools/c4bench.py | grep -E "list_(steps|levels)" | tail -1
  SB_LIST_OLD=1 PA_AMD_LIB=$lib bash tools/kprof.sh c4o_$v python3 tools/c4bench.py | grep -E "list_(steps|levels)" | tail -1
  grep -h ok= gpurun_out/kp_c4s_$v.log gpurun_out/kp_c4o_$v.log
done
