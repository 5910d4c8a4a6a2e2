set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_encode_adaptive.py tests/test_gpu_encode.py tests/test_gpu_encode_list.py > gpurun_out/ed_tests.log 2>&1; rc=$?; tail -3 gpurun_out/ed_tests.log; [ $rc = 0 ] || exit $rc
for v in old newph oldph; do echo "== $v"; done
PA_AMD_LIB=pa_amd/variants/libsb_oldph.so timeout -k 10 120 python tools/encphases.py > gpurun_out/ed_oldph.log 2>&1 || exit 1
PA_AMD_LIB=pa_amd/variants/libsb_newph.so timeout -k 10 120 python tools/encphases.py > gpurun_out/ed_newph.log 2>&1 || exit 1
PA_AMD_LIB=pa_amd/variants/libsb_old.so timeout -k 10 120 python tools/enc_c2.py > gpurun_out/ed_old.log 2>&1 || exit 1
timeout -k 10 120 python tools/enc_c2.py > gpurun_out/ed_new.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ed_oldph.log gpurun_out/ed_newph.log gpurun_out/ed_old.log gpurun_out/ed_new.log
