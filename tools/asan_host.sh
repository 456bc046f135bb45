#!/bin/bash
# Host code under AddressSanitizer (CPU only; GPU sanitizers are not available on the pool):
# gpuverify.cpp and verifier.cpp rebuilt with -Xarch_host -fsanitize=address and linked with the
# regular device objects into a scratch library, then the CPU test suite runs against it with
# the ASan runtime preloaded into the interpreter (SBFT_GV_LIB selects the library).
set -e
cd "$(dirname "$0")/.."
make -s -C smartbft_amd/csrc
out=${ASAN_DIR:-/tmp/sbft_asan}
mkdir -p "$out"
for f in gpuverify verifier; do
  /opt/rocm/bin/hipcc -O1 -g -fPIC -std=c++17 --offload-arch=gfx950 -Iinclude -Xarch_host -fsanitize=address \
    -Xarch_host -fno-omit-frame-pointer -c -o "$out/$f.o" smartbft_amd/csrc/$f.cpp
done
b=smartbft_amd/csrc/build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -shared-libasan -fsanitize=address -fno-gpu-sanitize \
  -o "$out/libsbft_asan.so" $b/p256_keyed.o $b/p256_verify.o $b/p256_sign.o $b/p256_selftest.o $b/sha256.o \
  "$out/gpuverify.o" "$out/verifier.o"
rt=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
SBFT_GV_LIB="$out/libsbft_asan.so" LD_PRELOAD="$rt" ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 \
  python -m pytest tests -q -m "not gpu" -p no:cacheprovider "$@"
