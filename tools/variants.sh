#!/bin/bash
# Build kernel variants of libplakar_cdc.so: tools/variants.sh NAME "-DFLAG=V ..." [NAME "FLAGS"]...
# Output: plakar_amd/_lib/variants/NAME.so (select with PLAKAR_CDC_LIB=...).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/plakar_amd/_lib/variants"
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I "$ROOT/include" $flags \
    -o "$ROOT/plakar_amd/_lib/variants/$name.so" \
    "$ROOT/plakar_amd/csrc/cdc_kernels.hip" "$ROOT/plakar_amd/csrc/cdc_digest.hip" "$ROOT/plakar_amd/csrc/cdc_api.cpp" &
done
wait
ls -la "$ROOT/plakar_amd/_lib/variants"
