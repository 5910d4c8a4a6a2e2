# A/B of the Utf8 C5-kind decodes between library variants
set -o pipefail
for v in $VARIANTS; do echo "== $v"; PA_AMD_LIB=pa_amd/variants/libsb_$v.so timeout -k 10 200 python tools/binbench.py 2>&1 | grep -v amdgpu.ids || exit 1; done
