// Issue rates of the 32-bit VALU instructions SHA-256 is made of, on gfx950: 8 independent
// chains per lane, 8 waves per SIMD (256 CUs x 8 workgroups of 256 threads), inline asm so
// the instruction is exactly the one named. Reports T lane-ops/s and cycles per wave64
// instruction per SIMD at the 2.4 GHz peak clock. (Diagnostics for the SHA-256 roofline.)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s\n", hipGetErrorString(e_)); return 1; } } while (0)
constexpr int ITERS = 2048;

#define KERNEL3(NAME, ASM)                                                                    \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t seed) {                \
        uint32_t x[8];                                                                         \
        _Pragma("unroll") for (int j = 0; j < 8; ++j) x[j] = seed + threadIdx.x * (j + 3);     \
        const uint32_t y = seed ^ blockIdx.x, z = seed * 5u + 1u;                              \
        for (int i = 0; i < ITERS; ++i) {                                                      \
            _Pragma("unroll") for (int j = 0; j < 8; ++j) asm volatile(ASM : "+v"(x[j]) : "v"(y), "v"(z)); \
        }                                                                                      \
        uint32_t s = 0;                                                                        \
        _Pragma("unroll") for (int j = 0; j < 8; ++j) s ^= x[j];                               \
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                        \
    }

KERNEL3(k_alignbit, "v_alignbit_b32 %0, %0, %0, 7")
KERNEL3(k_bitop3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")
KERNEL3(k_add3, "v_add3_u32 %0, %0, %1, %2")
KERNEL3(k_perm, "v_perm_b32 %0, %0, %1, %2")
KERNEL3(k_bfi, "v_bfi_b32 %0, %0, %1, %2")
KERNEL3(k_xad, "v_xad_u32 %0, %0, %1, %2")
KERNEL3(k_lshl_or, "v_lshl_or_b32 %0, %0, 3, %1")
KERNEL3(k_xor, "v_xor_b32 %0, %0, %1")
KERNEL3(k_add, "v_add_u32 %0, %0, %1")
KERNEL3(k_lshr, "v_lshrrev_b32 %0, 3, %0")
KERNEL3(k_xor_e64, "v_xor_b32_e64 %0, %0, %1")

template <class K>
static int run(const char* name, K kern, uint32_t* d, int cus) {
    const int blocks = cus * 8;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, 1u);
    CHK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CHK(hipEventRecord(a));
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, 2u + r);
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms;
        CHK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    const double ops = (double)blocks * 256 * ITERS * 8;
    const double tops = ops / (best * 1e-3) / 1e12;
    const double cyc = (double)cus * 4 * 2.4e9 * (best * 1e-3) / (ops / 64);
    printf("%-16s %8.3f ms %7.2f T lane-ops/s  %.2f cycles/wave-instr/SIMD @2.4GHz\n", name, best, tops, cyc);
    return 0;
}

int main() {
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t* d;
    CHK(hipMalloc(&d, (size_t)cus * 8 * 256 * 4));
    run("v_xor_b32", k_xor, d, cus);
    run("v_xor_b32_e64", k_xor_e64, d, cus);
    run("v_add_u32", k_add, d, cus);
    run("v_lshrrev_b32", k_lshr, d, cus);
    run("v_alignbit_b32", k_alignbit, d, cus);
    run("v_bitop3_b32", k_bitop3, d, cus);
    run("v_add3_u32", k_add3, d, cus);
    run("v_perm_b32", k_perm, d, cus);
    run("v_bfi_b32", k_bfi, d, cus);
    run("v_xad_u32", k_xad, d, cus);
    run("v_lshl_or_b32", k_lshl_or, d, cus);
    return 0;
}
