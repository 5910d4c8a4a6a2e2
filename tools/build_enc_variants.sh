#!/bin/bash
# Builds encoder variants (sb_encode_adapt.hip with extra flags) as separate
# libraries: bash tools/build_enc_variants.sh name:-DFLAG ...
set -e
cd "$(dirname "$0")/../pa_amd"
make -s
mkdir -p variants _build/variants
build() {
  name=$1; shift
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function "$@" -x hip -c csrc/sb_encode_adapt.hip -o _build/variants/enc_$name.o
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o variants/libsb_$name.so _build/variants/enc_$name.o $(ls _build/*.o | grep -v sb_encode_adapt) -l:liblz4.so.1 -l:libzstd.so.1 -lpthread
}
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  build $name $flags &
done
wait
ls variants
