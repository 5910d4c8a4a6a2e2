bash tools/gpu_tests.sh z2 -m gpu tests/test_gpu_binary.py tests/test_gpu_binary_errors.py tests/test_gpu_configs.py tests/test_gpu_table.py tests/test_gpu_utf8.py tests/test_gpu_shard.py > /dev/null; rc=$?; tail -3 gpurun_out/z2.log; [ $rc = 0 ] || exit $rc
PA_AMD_LIB=pa_amd/variants/libsb_phases.so timeout -k 10 200 python tools/binphases.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python tools/c5units.py > gpurun_out/z2_c5units.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/z2_c5units.log; exit $rc
