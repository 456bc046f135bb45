#!/bin/bash
# Build libsbft_gpuverify variants of the verify and keyed kernels (occupancy etc.) into tools/variants/.
# Usage: tools/build_variants.sh "w2:-DSBFT_VERIFY_WAVES=2" "w3:-DSBFT_VERIFY_WAVES=3" ...
set -e
cd "$(dirname "$0")/../smartbft_amd/csrc"
make -s
mkdir -p ../../tools/variants
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  rm -f ../../tools/variants/lib_$name.so
  (d=/tmp/sbft_var_$name; mkdir -p $d
   F="-O3 -fPIC -std=c++17 --offload-arch=gfx950 -I../../include -mllvm -pragma-unroll-threshold=1000000 $flags"
   hipcc $F -c -o $d/pv.o p256_verify.hip &
   hipcc $F -c -o $d/pk.o p256_keyed.hip &
   wait
   hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/variants/lib_$name.so $d/pv.o $d/pk.o build/p256_sign.o build/p256_selftest.o build/sha256.o build/gpuverify.o build/verifier.o) &
done
wait
ls ../../tools/variants
