// Microbenchmark: peak v_mad_u64_u32 (32x32->64 + 64 accumulate) rate on gfx950,
// plus v_add_co/v_addc carry-chain rate. Used as the roofline "peak" for the
// P-256 verify kernel: the guides quote no integer-multiply rate.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

template <int ITERS>
__global__ __launch_bounds__(256) void k_mad(uint64_t* out, uint32_t seed) {
    uint32_t a = seed ^ threadIdx.x, b = seed * 7u + blockIdx.x;
    uint64_t acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = (uint64_t)(a + j) << 3;
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            // 8 independent chains; each step is one v_mad_u64_u32
            { uint64_t sc; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[j]), "=s"(sc) : "v"(a), "v"(b + j)); }
        }
    }
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s ^= acc[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int ITERS>
__global__ __launch_bounds__(256) void k_addc(uint32_t* out, uint32_t seed) {
    uint32_t x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = seed + threadIdx.x * (j + 1);
    uint32_t y = seed ^ blockIdx.x;
    for (int i = 0; i < ITERS; ++i) {
        // 8-limb carry chain: 1 v_add_co + 7 v_addc_co
        asm volatile(
            "v_add_co_u32 %0, vcc, %0, %8\n\t"
            "v_addc_co_u32 %1, vcc, %1, %8, vcc\n\t"
            "v_addc_co_u32 %2, vcc, %2, %8, vcc\n\t"
            "v_addc_co_u32 %3, vcc, %3, %8, vcc\n\t"
            "v_addc_co_u32 %4, vcc, %4, %8, vcc\n\t"
            "v_addc_co_u32 %5, vcc, %5, %8, vcc\n\t"
            "v_addc_co_u32 %6, vcc, %6, %8, vcc\n\t"
            "v_addc_co_u32 %7, vcc, %7, %8, vcc\n\t"
            : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7])
            : "v"(y) : "vcc");
    }
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s ^= x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int ITERS>
__global__ __launch_bounds__(256) void k_add3(uint32_t* out, uint32_t seed) {
    uint32_t x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = seed + threadIdx.x * (j + 1);
    uint32_t y = seed ^ blockIdx.x;
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
            asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x[j]) : "v"(y), "v"(x[(j + 1) & 7]));
    }
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s ^= x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// 64-bit arithmetic shift (the radix-2^29 carry step): 8 independent chains
template <int ITERS>
__global__ __launch_bounds__(256) void k_ashr64(uint64_t* out, uint32_t seed) {
    int64_t x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = ((int64_t)(seed ^ threadIdx.x) << 40) * (j + 1);
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) asm volatile("v_ashrrev_i64 %0, 1, %0" : "+v"(x[j]));
    }
    int64_t s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s ^= x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// signed 32x32+64 mad (the radix-2^29 product), compiler-scheduled: 8 independent chains
template <int ITERS>
__global__ __launch_bounds__(256) void k_madi(uint64_t* out, uint32_t seed) {
    int32_t a = (int32_t)(seed ^ threadIdx.x), b = (int32_t)(seed * 7u + blockIdx.x);
    int64_t acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = (int64_t)(a + j) << 3;
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            acc[j] = (int64_t)a * (int64_t)(b + j) + acc[j];
            asm("" : "+v"(acc[j]));
        }
    }
    int64_t s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s ^= acc[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

// 32-bit and (the radix-2^29 mask)
template <int ITERS>
__global__ __launch_bounds__(256) void k_and(uint32_t* out, uint32_t seed) {
    uint32_t x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = seed + threadIdx.x * (j + 1);
    uint32_t y = seed ^ blockIdx.x;
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x[j]) : "v"(y));
    }
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s ^= x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    const int ITERS = 4096;
    const int blocks = 256 * 8 * 4;  // plenty of waves per SIMD
    const int threads = 256;
    void* d;
    CHK(hipMalloc(&d, (size_t)blocks * threads * 8));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    printf("device %s CUs %d clock %d kHz\n", prop.gcnArchName, prop.multiProcessorCount, prop.clockRate);
    auto timeit = [&](auto launch, double ops_per_thread_iter, const char* name) -> int {
        for (int w = 0; w < 2; ++w) launch();
        CHK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            CHK(hipEventRecord(e0));
            launch();
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        double ops = (double)blocks * threads * ITERS * ops_per_thread_iter;
        printf("%-16s %.3f ms  %.3f T lane-ops/s\n", name, best, ops / (best * 1e-3) / 1e12);
        return 0;
    };
    timeit([&] { k_mad<ITERS><<<blocks, threads>>>((uint64_t*)d, 1234u); }, 8, "v_mad_u64_u32");
    timeit([&] { k_addc<ITERS><<<blocks, threads>>>((uint32_t*)d, 1234u); }, 8, "v_add(c)_co_u32");
    timeit([&] { k_add3<ITERS><<<blocks, threads>>>((uint32_t*)d, 1234u); }, 8, "v_add3_u32");
    timeit([&] { k_ashr64<ITERS><<<blocks, threads>>>((uint64_t*)d, 1234u); }, 8, "v_ashrrev_i64");
    timeit([&] { k_madi<ITERS><<<blocks, threads>>>((uint64_t*)d, 1234u); }, 8, "v_mad_i64_i32");
    timeit([&] { k_and<ITERS><<<blocks, threads>>>((uint32_t*)d, 1234u); }, 8, "v_and_b32");
    CHK(hipFree(d));
    return 0;
}
