// Issue rates of the instructions a radix-2^29 field product is made of, on gfx950: the 64-bit
// mads, 64-bit shifts, shift-adds and the 32-bit logic around them, plus candidate
// replacements (24-bit mads, f64 FMA, dot products). 8 independent chains per lane (or 1 for
// the "dep" rows: a dependent chain, i.e. the latency-bound case), 8 waves per SIMD unless the
// row says otherwise. Inline asm so the instruction is exactly the one named. Reports cycles per
// wave64 instruction per SIMD at the 2.4 GHz peak clock. (Diagnostics for the verify roofline.)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s\n", hipGetErrorString(e_)); return 1; } } while (0)

// 64-bit accumulator chains: x[j] (u64) updated by ASM with 32-bit operands y, z
#define K64(NAME, CH, ASM)                                                                     \
    __global__ __launch_bounds__(256) void NAME(uint64_t* out, uint32_t seed, int iters) {                \
        uint64_t x[CH];                                                                        \
        _Pragma("unroll") for (int j = 0; j < CH; ++j) x[j] = seed + threadIdx.x * (j + 3);    \
        uint32_t y = seed ^ blockIdx.x, z = seed * 5u + 1u;                                    \
        asm volatile("" : "+v"(y), "+v"(z));                                                   \
        for (int i = 0; i < iters; i += 16) _Pragma("unroll") for (int r = 0; r < 16; ++r) {       \
            _Pragma("unroll") for (int j = 0; j < CH; ++j) asm volatile(ASM : "+v"(x[j]) : "v"(y), "v"(z) : "vcc"); \
        }                                                                                      \
        uint64_t s = 0;                                                                        \
        _Pragma("unroll") for (int j = 0; j < CH; ++j) s ^= x[j];                              \
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                        \
    }
// same with an SGPR operand
#define K64S(NAME, CH, ASM)                                                                    \
    __global__ __launch_bounds__(256) void NAME(uint64_t* out, uint32_t seed, int iters) {                \
        uint64_t x[CH];                                                                        \
        _Pragma("unroll") for (int j = 0; j < CH; ++j) x[j] = seed + threadIdx.x * (j + 3);    \
        uint32_t y = seed ^ threadIdx.x, z = seed * 5u + 1u;                                   \
        asm volatile("" : "+v"(y), "+s"(z));                                                   \
        for (int i = 0; i < iters; i += 16) _Pragma("unroll") for (int r = 0; r < 16; ++r) {       \
            _Pragma("unroll") for (int j = 0; j < CH; ++j) asm volatile(ASM : "+v"(x[j]) : "v"(y), "s"(z) : "vcc"); \
        }                                                                                      \
        uint64_t s = 0;                                                                        \
        _Pragma("unroll") for (int j = 0; j < CH; ++j) s ^= x[j];                              \
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                        \
    }
// 32-bit chains
#define K32(NAME, CH, ASM)                                                                     \
    __global__ __launch_bounds__(256) void NAME(uint64_t* out, uint32_t seed, int iters) {                \
        uint32_t x[CH];                                                                        \
        _Pragma("unroll") for (int j = 0; j < CH; ++j) x[j] = seed + threadIdx.x * (j + 3);    \
        uint32_t y = seed ^ blockIdx.x, z = seed * 5u + 1u;                                    \
        asm volatile("" : "+v"(y), "+v"(z));                                                   \
        for (int i = 0; i < iters; i += 16) _Pragma("unroll") for (int r = 0; r < 16; ++r) {       \
            _Pragma("unroll") for (int j = 0; j < CH; ++j) asm volatile(ASM : "+v"(x[j]) : "v"(y), "v"(z) : "vcc"); \
        }                                                                                      \
        uint32_t s = 0;                                                                        \
        _Pragma("unroll") for (int j = 0; j < CH; ++j) s ^= x[j];                              \
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                        \
    }

K64(k_mad_i64, 8, "v_mad_i64_i32 %0, vcc, %1, %2, %0")
K64S(k_mad_i64_s, 8, "v_mad_i64_i32 %0, vcc, %1, %2, %0")
K64(k_mad_u64, 8, "v_mad_u64_u32 %0, vcc, %1, %2, %0")
K64(k_mad_i64_dep, 1, "v_mad_i64_i32 %0, vcc, %1, %2, %0")
K64(k_mad_i64_dep2, 2, "v_mad_i64_i32 %0, vcc, %1, %2, %0")
K64(k_mad_i64_dep4, 4, "v_mad_i64_i32 %0, vcc, %1, %2, %0")
K64(k_ashr64, 8, "v_ashrrev_i64 %0, 29, %0")
K64(k_lshr64, 8, "v_lshrrev_b64 %0, 29, %0")
K64(k_lshl_add64, 8, "v_lshl_add_u64 %0, %0, 2, %0")
K64(k_mov64, 8, "v_mov_b64 %0, %0")
K64(k_fma64, 8, "v_fma_f64 %0, %0, %0, %0")
K64(k_mul_f64, 8, "v_mul_f64 %0, %0, %0")
K32(k_add_co, 8, "v_add_co_u32 %0, vcc, %0, %1")
K32(k_addc, 8, "v_addc_co_u32 %0, vcc, %0, %1, vcc")
K32(k_and, 8, "v_and_b32 %0, %0, %1")
K32(k_and_k, 8, "v_and_b32 %0, 0x1fffffff, %0")
K32(k_ashr32, 8, "v_ashrrev_i32 %0, 29, %0")
K32(k_mul_lo, 8, "v_mul_lo_u32 %0, %0, %1")
K32(k_mul_hi, 8, "v_mul_hi_u32 %0, %0, %1")
K32(k_mad_u24, 8, "v_mad_u32_u24 %0, %0, %1, %2")
K32(k_mul_u24, 8, "v_mul_u32_u24 %0, %0, %1")
K32(k_mul_hi_u24, 8, "v_mul_hi_u32_u24 %0, %0, %1")
K32(k_dot2_u16, 8, "v_dot2_u32_u16 %0, %1, %2, %0")
K32(k_dot4_u8, 8, "v_dot4_u32_u8 %0, %1, %2, %0")
K32(k_lshl_add32, 8, "v_lshl_add_u32 %0, %1, 3, %0")
K32(k_alignbit, 8, "v_alignbit_b32 %0, %1, %0, 29")
K32(k_bfe, 8, "v_bfe_u32 %0, %0, 3, 29")
K32(k_sub, 8, "v_sub_u32 %0, %1, %0")

// actual shader clock: s_memtime (core clocks) against s_memrealtime (100 MHz) around a long
// mad loop on every wave; reported per wave as MHz.
__global__ __launch_bounds__(256) void k_clock(uint64_t* out, uint32_t seed, int iters) {
    uint64_t x[8];
    _Pragma("unroll") for (int j = 0; j < 8; ++j) x[j] = seed + threadIdx.x * (j + 3);
    uint32_t y = seed ^ blockIdx.x, z = seed * 5u + 1u;
    asm volatile("" : "+v"(y), "+v"(z));
    const uint64_t c0 = clock64(), w0 = wall_clock64();
    for (int i = 0; i < iters; ++i) {
        _Pragma("unroll") for (int j = 0; j < 8; ++j) asm volatile("v_mad_i64_i32 %0, vcc, %1, %2, %0" : "+v"(x[j]) : "v"(y), "v"(z) : "vcc");
    }
    const uint64_t c1 = clock64(), w1 = wall_clock64();
    uint64_t s = 0;
    _Pragma("unroll") for (int j = 0; j < 8; ++j) s ^= x[j];
    if (threadIdx.x == 0) out[blockIdx.x] = ((c1 - c0) * 100ull) / (w1 - w0 ? w1 - w0 : 1);  // MHz
    else if (s == 0x12345) out[blockIdx.x] = s;
}

static double g_mhz = 2400.0;

template <class K>
static int run(const char* name, K kern, uint64_t* d, int cus, int ch, int wg_per_cu = 8) {
    const int blocks = cus * wg_per_cu;
    // ~2-4 ms per launch: 8 waves/SIMD x 8 chains x 16k iterations at ~5 cycles
    const int iters = (16384 * 8 / ch) * 8 / wg_per_cu;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, 1u, 64);
    CHK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
        CHK(hipEventRecord(a));
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, 2u + r, iters);
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms;
        CHK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    const double ops = (double)blocks * 256 * iters * ch;
    const double cyc = (double)cus * 4 * 2.4e9 * (best * 1e-3) / (ops / 64);
    printf("%-20s ch=%d waves/SIMD=%d %8.3f ms  %6.2f cyc/wave-instr @2.4GHz  %6.2f @%.0fMHz\n", name, ch,
           wg_per_cu, best, cyc, cyc * g_mhz / 2400.0, g_mhz);
    return 0;
}

int main() {
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint64_t* d;
    CHK(hipMalloc(&d, (size_t)cus * 8 * 256 * 8));
    {
        const int blocks = cus * 8;
        hipLaunchKernelGGL(k_clock, dim3(blocks), dim3(256), 0, 0, d, 1u, 64);
        hipLaunchKernelGGL(k_clock, dim3(blocks), dim3(256), 0, 0, d, 1u, 32768);
        CHK(hipDeviceSynchronize());
        uint64_t* h = new uint64_t[blocks];
        CHK(hipMemcpy(h, d, blocks * 8, hipMemcpyDeviceToHost));
        double sum = 0;
        uint64_t mn = ~0ull, mx = 0;
        for (int i = 0; i < blocks; ++i) { sum += h[i]; mn = h[i] < mn ? h[i] : mn; mx = h[i] > mx ? h[i] : mx; }
        g_mhz = sum / blocks;
        printf("shader clock under a mad loop: mean %.0f MHz (min %llu, max %llu)\n", g_mhz,
               (unsigned long long)mn, (unsigned long long)mx);
        delete[] h;
    }
    run("v_mad_i64_i32", k_mad_i64, d, cus, 8);
    run("v_mad_i64_i32", k_mad_i64, d, cus, 8, 2);
    run("v_mad_i64_i32 sgpr", k_mad_i64_s, d, cus, 8);
    run("v_mad_u64_u32", k_mad_u64, d, cus, 8);
    run("v_mad_i64 dep1", k_mad_i64_dep, d, cus, 1);
    run("v_mad_i64 dep1", k_mad_i64_dep, d, cus, 1, 2);
    run("v_mad_i64 dep2", k_mad_i64_dep2, d, cus, 2, 2);
    run("v_mad_i64 dep4", k_mad_i64_dep4, d, cus, 4, 2);
    run("v_mad_i64 dep1", k_mad_i64_dep, d, cus, 1, 4);
    run("v_mad_i64 dep2", k_mad_i64_dep2, d, cus, 2, 4);
    run("v_mad_i64 dep4", k_mad_i64_dep4, d, cus, 4, 4);
    run("v_mad_i64_i32", k_mad_i64, d, cus, 8, 4);
    run("v_ashrrev_i64", k_ashr64, d, cus, 8);
    run("v_lshrrev_b64", k_lshr64, d, cus, 8);
    run("v_lshl_add_u64", k_lshl_add64, d, cus, 8);
    run("v_mov_b64", k_mov64, d, cus, 8);
    run("v_fma_f64", k_fma64, d, cus, 8);
    run("v_mul_f64", k_mul_f64, d, cus, 8);
    run("v_add_co_u32", k_add_co, d, cus, 8);
    run("v_addc_co_u32", k_addc, d, cus, 8);
    run("v_and_b32", k_and, d, cus, 8);
    run("v_and_b32 lit", k_and_k, d, cus, 8);
    run("v_ashrrev_i32", k_ashr32, d, cus, 8);
    run("v_sub_u32", k_sub, d, cus, 8);
    run("v_mul_lo_u32", k_mul_lo, d, cus, 8);
    run("v_mul_hi_u32", k_mul_hi, d, cus, 8);
    run("v_mad_u32_u24", k_mad_u24, d, cus, 8);
    run("v_mul_u32_u24", k_mul_u24, d, cus, 8);
    run("v_mul_hi_u32_u24", k_mul_hi_u24, d, cus, 8);
    run("v_dot2_u32_u16", k_dot2_u16, d, cus, 8);
    run("v_dot4_u32_u8", k_dot4_u8, d, cus, 8);
    run("v_lshl_add_u32", k_lshl_add32, d, cus, 8);
    run("v_alignbit_b32", k_alignbit, d, cus, 8);
    run("v_bfe_u32", k_bfe, d, cus, 8);
    return 0;
}
