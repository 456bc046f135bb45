#!/bin/bash
# Build libsbft_gpuverify variants of the verify kernel (occupancy etc.) into tools/variants/.
# Usage: tools/build_variants.sh "w2:-DSBFT_VERIFY_WAVES=2" "w3:-DSBFT_VERIFY_WAVES=3" ...
set -e
cd "$(dirname "$0")/../smartbft_amd/csrc"
make -s
mkdir -p ../../tools/variants
rm -f ../../tools/variants/*.so
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  (d=/tmp/sbft_var_$name; mkdir -p $d
   hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -I../../include -mllvm -pragma-unroll-threshold=1000000 $flags -c -o $d/pv.o p256_verify.hip
   hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/variants/lib_$name.so $d/pv.o build/p256_keyed.o build/p256_sign.o build/p256_selftest.o build/sha256.o build/gpuverify.o build/verifier.o) &
done
wait
ls ../../tools/variants
