// valu_peak.hip -- measures the sustained int32 VALU issue rate of gfx950 with the
// scan kernel's instruction mix (v_xor_b32 + v_min3_u32 on wave-uniform operands), and
// the chip clock it runs at.  Prints lane-ops/s.  Diagnostic tool, not part of libdhtgpu.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int ILP>
__global__ __launch_bounds__(256) void k_valu(uint32_t* out, uint32_t seed, int iters, uint32_t s0, uint32_t s1) {
    uint32_t x[ILP], a[ILP];
#pragma unroll
    for (int i = 0; i < ILP; ++i) { x[i] = seed * (threadIdx.x + 1) + i; a[i] = ~0u; }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < ILP; ++i) {
            uint32_t p, q2;
            asm volatile("v_xor_b32 %0, %1, %2" : "=v"(p) : "s"(s0), "v"(x[i]));
            asm volatile("v_xor_b32 %0, %1, %2" : "=v"(q2) : "s"(s1), "v"(x[i]));
            asm volatile("v_min3_u32 %0, %1, %2, %3" : "=v"(a[i]) : "v"(a[i]), "v"(p), "v"(q2));
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < ILP; ++i) r ^= a[i];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int ILP>
__global__ __launch_bounds__(256) void k_valu_pk(uint32_t* out, uint32_t seed, int iters, uint32_t s0, uint32_t s1) {
    uint32_t x[ILP], a[ILP];
#pragma unroll
    for (int i = 0; i < ILP; ++i) { x[i] = seed * (threadIdx.x + 1) + i; a[i] = ~0u; }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < ILP; ++i) {
            uint32_t p;
            asm volatile("v_xor_b32 %0, %1, %2" : "=v"(p) : "s"(s0 + it), "v"(x[i]));
            asm volatile("v_pk_min_u16 %0, %1, %2" : "=v"(a[i]) : "v"(a[i]), "v"(p));
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < ILP; ++i) r ^= a[i];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

int main() {
    const int blocks = 256 * 8, iters = 4096;
    uint32_t* d;
    CHK(hipMalloc(&d, blocks * 256 * 4));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    for (int rep = 0; rep < 3; ++rep) {
        k_valu<8><<<blocks, 256>>>(d, 7, iters, 0x1234, 0x5678);
        CHK(hipEventRecord(e0));
        k_valu<8><<<blocks, 256>>>(d, 7, iters, 0x1234, 0x5678);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
        const double ops = (double)blocks * 256 * iters * 8 * 3;   // lane-ops
        printf("{\"valu_lane_ops_per_s\": %.4e, \"ms\": %.3f, \"implied_ghz_at_32_lanes_per_simd\": %.3f}\n",
               ops / (ms * 1e-3), ms, ops / (ms * 1e-3) / (256.0 * 4 * 32) / 1e9);
    }
    for (int rep = 0; rep < 3; ++rep) {
        k_valu_pk<8><<<blocks, 256>>>(d, 7, iters, 0x1234, 0x5678);
        CHK(hipEventRecord(e0));
        k_valu_pk<8><<<blocks, 256>>>(d, 7, iters, 0x1234, 0x5678);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
        const double ops = (double)blocks * 256 * iters * 8 * 2;   // lane-ops (xor + pk_min)
        printf("{\"mix\": \"xor+pk_min_u16\", \"valu_lane_ops_per_s\": %.4e, \"ms\": %.3f}\n", ops / (ms * 1e-3), ms);
    }
    return 0;
}
