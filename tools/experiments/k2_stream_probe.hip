// k2_stream_probe.hip -- the floor under K2: read a 4-B word-0 plane of 10^8 ids
// (400 MB) and write one byte per id (100 MB), with K2's access shape (a wave owns chunks of
// 64 x U uint4, grid-strided, the next chunk's loads issued before this chunk's stores) and no
// classification.  Variants: loads cached / non-temporal, stores cached / non-temporal / none,
// U, workgroups per CU, and a read-only pass of the same plane.  Each: 5 warm launches, then the
// mean of 20 by HIP events, reported as (read + written bytes) / time.
// build: hipcc -O3 --offload-arch=gfx950 -o tools/experiments/k2_stream_probe tools/experiments/k2_stream_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef unsigned int u4v __attribute__((ext_vector_type(4)));

template <uint32_t U, bool NTL, int ST>   // ST: 0 no store, 1 cached store, 2 non-temporal store
__global__ __launch_bounds__(256) void k_rw(const uint4* __restrict__ w04, uint64_t n4, uint32_t* __restrict__ out,
                                            uint32_t* sink) {
    constexpr uint64_t CH = 64 * U;
    const uint64_t nch = (n4 + CH - 1) / CH;
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t W = (uint64_t)gridDim.x * 4;
    uint64_t c = (uint64_t)blockIdx.x * 4 + wv;
    auto load = [&](uint64_t ch, uint4* v) {
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            uint64_t i4 = ch * CH + u * 64 + lane;
            i4 = i4 < n4 ? i4 : n4 - 1;
            if (NTL) {
                const u4v t = __builtin_nontemporal_load(reinterpret_cast<const u4v*>(w04 + i4));
                v[u] = make_uint4(t[0], t[1], t[2], t[3]);
            } else {
                v[u] = w04[i4];
            }
        }
    };
    uint4 v[U];
    load(c, v);
    uint32_t acc = 0;
    for (; c < nch; c += W) {
        uint4 nx[U];
        load(c + W, nx);
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const uint32_t p = (v[u].x >> 24) | ((v[u].y >> 24) << 8) | ((v[u].z >> 24) << 16) | ((v[u].w >> 24) << 24);
            const uint64_t i4 = c * CH + u * 64 + lane;
            if (ST == 0) acc ^= p;
            else if (i4 < n4) {
                if (ST == 2) __builtin_nontemporal_store(p, out + i4);
                else out[i4] = p;
            }
            v[u] = nx[u];
        }
    }
    if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc;
}

template <uint32_t U, bool NTL, int ST>
static int run(const uint4* p, uint64_t n4, uint32_t* out, uint32_t* sink, int cus, int per_cu, const char* name) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int grid = cus * per_cu;
    for (int i = 0; i < 5; ++i) k_rw<U, NTL, ST><<<grid, 256>>>(p, n4, out, sink);
    CK(hipEventRecord(a));
    for (int i = 0; i < 20; ++i) k_rw<U, NTL, ST><<<grid, 256>>>(p, n4, out, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= 20;
    const double bytes = 16.0 * n4 + (ST ? 4.0 * n4 : 0.0);
    printf("%-28s U=%u percu=%2d: %.4f ms  %7.0f GB/s  frac %.3f\n", name, U, per_cu, ms, bytes / ms / 1e6,
           bytes / ms / 1e6 / 8000.0);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return 0;
}

int main() {
    const uint64_t n = 100000000ull, n4 = n / 4;
    uint4* p;
    uint32_t *out, *sink;
    CK(hipMalloc(&p, 16 * n4));
    CK(hipMalloc(&out, 4 * n4));
    CK(hipMalloc(&sink, 1 << 20));
    CK(hipMemset(p, 0x5A, 16 * n4));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    for (int rep = 0; rep < 2; ++rep) {
        run<3, true, 0>(p, n4, out, sink, cus, 8, "read-only nt");
        run<3, false, 0>(p, n4, out, sink, cus, 8, "read-only");
        run<3, true, 1>(p, n4, out, sink, cus, 8, "nt load + store");
        run<3, true, 2>(p, n4, out, sink, cus, 8, "nt load + nt store");
        run<3, false, 2>(p, n4, out, sink, cus, 8, "load + nt store");
        run<3, true, 2>(p, n4, out, sink, cus, 4, "nt load + nt store");
        run<3, true, 2>(p, n4, out, sink, cus, 2, "nt load + nt store");
        run<2, true, 2>(p, n4, out, sink, cus, 8, "nt load + nt store");
        run<4, true, 2>(p, n4, out, sink, cus, 8, "nt load + nt store");
        run<4, true, 2>(p, n4, out, sink, cus, 4, "nt load + nt store");
        run<8, true, 2>(p, n4, out, sink, cus, 4, "nt load + nt store");
        run<8, true, 2>(p, n4, out, sink, cus, 2, "nt load + nt store");
        run<4, true, 1>(p, n4, out, sink, cus, 4, "nt load + store");
    }
    return 0;
}
