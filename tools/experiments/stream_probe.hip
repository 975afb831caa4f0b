// stream_probe.hip -- how fast can one kernel read a word plane on this MI355X?  The floor under
// F2's and S1's streams: a 64 MB plane (the cfg-2 w0 plane, Infinity-Cache resident
// when read back to back) and a 1 GB plane (HBM), read once per launch by
//   * persistent blocks over contiguous ranges with a ring of RING 16-B loads per lane in flight
//     (F2 / S1's shape), at several blocks per CU, threads per block and ring depths;
//   * a classic grid of short-lived blocks, one 16-B load per lane per iteration, 4 in flight.
// Each configuration: 5 warm launches, then the mean of 20 by HIP events.  Prints GB/s.
// build: hipcc -O3 --offload-arch=gfx950 -o tools/experiments/stream_probe tools/experiments/stream_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int NT, int RING>
__global__ __launch_bounds__(NT) void k_ring(const uint4* __restrict__ p, uint64_t n16, uint64_t per_blk, uint32_t* out) {
    const uint64_t lo = (uint64_t)blockIdx.x * per_blk;
    const uint64_t hi = lo + per_blk < n16 ? lo + per_blk : n16;
    uint4 ring[RING];
    uint32_t acc = 0;
#pragma unroll
    for (int r = 0; r < RING; ++r) {
        uint64_t j = lo + (uint64_t)r * NT + threadIdx.x;
        ring[r] = p[j < hi ? j : hi - 1];
    }
    for (uint64_t c0 = lo; c0 < hi; c0 += (uint64_t)RING * NT) {
#pragma unroll
        for (int r = 0; r < RING; ++r) {
            acc ^= ring[r].x ^ ring[r].y ^ ring[r].z ^ ring[r].w;
            uint64_t j = c0 + (uint64_t)(r + RING) * NT + threadIdx.x;
            ring[r] = p[j < hi ? j : hi - 1];
        }
    }
    if (acc == 0x9E3779B9u) out[blockIdx.x] = acc;
}

template <int NT, int U>
__global__ __launch_bounds__(NT) void k_grid(const uint4* __restrict__ p, uint64_t n16, uint32_t* out) {
    const uint64_t base = (uint64_t)blockIdx.x * NT * U + threadIdx.x;
    uint32_t acc = 0;
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t j = base + (uint64_t)u * NT;
        v[u] = p[j < n16 ? j : n16 - 1];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    if (acc == 0x9E3779B9u) out[blockIdx.x] = acc;
}

template <typename F>
static double time_ms(F launch, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 5; ++i) launch();
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < reps; ++i) launch();
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return ms / reps;
}

template <int NT, int RING>
static void ring_case(const uint4* p, uint64_t n16, uint32_t* out, int cus, int bpc) {
    const uint64_t g = (uint64_t)cus * bpc;
    const uint64_t per = ((n16 + g - 1) / g + NT - 1) / NT * NT;
    const uint32_t nb = (uint32_t)((n16 + per - 1) / per);
    const double ms = time_ms([&] { k_ring<NT, RING><<<nb, NT>>>(p, n16, per, out); }, 20);
    printf("  ring  NT %4d RING %2d blocks/CU %d (%5u blocks, %6.1f KB/block in flight): %7.2f us  %6.0f GB/s\n", NT, RING, bpc,
           nb, NT * RING * 16 / 1024.0, ms * 1e3, n16 * 16 / (ms * 1e-3) / 1e9);
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t* out;
    CK(hipMalloc(&out, 1 << 20));
    for (uint64_t bytes : {64ull << 20, 1ull << 30}) {
        uint4* p;
        CK(hipMalloc(&p, bytes));
        CK(hipMemset(p, 1, bytes));
        const uint64_t n16 = bytes / 16;
        printf("plane %llu MB, %d CUs\n", (unsigned long long)(bytes >> 20), cus);
        ring_case<1024, 8>(p, n16, out, cus, 1);
        ring_case<1024, 4>(p, n16, out, cus, 1);
        ring_case<1024, 3>(p, n16, out, cus, 1);
        ring_case<1024, 2>(p, n16, out, cus, 1);
        ring_case<512, 4>(p, n16, out, cus, 1);
        ring_case<512, 8>(p, n16, out, cus, 1);
        ring_case<768, 4>(p, n16, out, cus, 1);
        ring_case<1024, 16>(p, n16, out, cus, 1);
        ring_case<512, 8>(p, n16, out, cus, 2);
        ring_case<512, 4>(p, n16, out, cus, 2);
        ring_case<512, 16>(p, n16, out, cus, 2);
        ring_case<256, 8>(p, n16, out, cus, 4);
        ring_case<256, 16>(p, n16, out, cus, 4);
        ring_case<512, 8>(p, n16, out, cus, 4);
        ring_case<1024, 8>(p, n16, out, cus, 2);
        for (int u : {1, 4}) {
            const uint32_t nb = (uint32_t)((n16 + 256 * u - 1) / (256 * u));
            const double ms = u == 1 ? time_ms([&] { k_grid<256, 1><<<nb, 256>>>(p, n16, out); }, 20)
                                     : time_ms([&] { k_grid<256, 4><<<nb, 256>>>(p, n16, out); }, 20);
            printf("  grid  NT  256 U %d (%u blocks): %7.2f us  %6.0f GB/s\n", u, nb, ms * 1e3, n16 * 16 / (ms * 1e-3) / 1e9);
        }
        const double e = time_ms([&] { hipLaunchKernelGGL((k_grid<256, 1>), dim3(1), dim3(256), 0, 0, p, (uint64_t)256, out); }, 50);
        printf("  empty-ish launch (1 block): %.2f us\n", e * 1e3);
        CK(hipFree(p));
    }
    return 0;
}
