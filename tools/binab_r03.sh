# A/B of the Utf8 C5-kind decodes: fused / two-pass x wave / block emission
set -o pipefail
run() { echo "== $1"; timeout -k 10 200 python tools/binbench.py 2>&1 | grep -v amdgpu.ids || exit 1; }
run fused_wave
SB_NO_BIN_FUSED=1 run twopass_wave
PA_AMD_LIB=pa_amd/variants/libsb_blockemit.so run fused_block
SB_NO_BIN_FUSED=1 PA_AMD_LIB=pa_amd/variants/libsb_blockemit.so run twopass_block
