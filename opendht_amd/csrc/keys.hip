// keys.hip -- id-set layout kernels: synthetic generation, AoS(20 B big-endian) <->
// word-plane conversion, sortedness check.  All are HBM-streaming kernels: one id
// per thread, every plane access coalesced (lane i -> word i of a plane).
#include "dhtgpu_dev.h"
#include "dhtgpu_internal.h"

namespace dhtgpu {
namespace {

constexpr int kBlock = 256;

inline uint32_t grid_for(uint64_t n, uint64_t per_block) {
    uint64_t g = (n + per_block - 1) / per_block;
    if (g > 65535ull * 32) g = 65535ull * 32;
    return (uint32_t)(g ? g : 1);
}

__global__ __launch_bounds__(kBlock) void k_gen(uint64_t seed, uint64_t start, uint64_t n,
                                                uint32_t* __restrict__ planes, uint64_t stride) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * kBlock) {
        const uint64_t g = start + i;
        const uint64_t a = splitmix(seed, 3 * g), b = splitmix(seed, 3 * g + 1),
                       c = splitmix(seed, 3 * g + 2);
        planes[i] = (uint32_t)(a >> 32);
        planes[stride + i] = (uint32_t)a;
        planes[2 * stride + i] = (uint32_t)(b >> 32);
        planes[3 * stride + i] = (uint32_t)b;
        planes[4 * stride + i] = (uint32_t)(c >> 32);
    }
}

__global__ __launch_bounds__(kBlock) void k_pack(const uint32_t* __restrict__ aos, uint64_t n,
                                                 uint32_t* __restrict__ planes, uint64_t stride) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * kBlock) {
#pragma unroll
        for (int j = 0; j < DHT_W; ++j) planes[(uint64_t)j * stride + i] = __builtin_bswap32(aos[5 * i + j]);
    }
}

__global__ __launch_bounds__(kBlock) void k_unpack(const uint32_t* __restrict__ planes,
                                                   uint64_t stride, uint64_t first, uint64_t n,
                                                   uint32_t* __restrict__ aos) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * kBlock) {
#pragma unroll
        for (int j = 0; j < DHT_W; ++j)
            aos[5 * i + j] = __builtin_bswap32(planes[(uint64_t)j * stride + first + i]);
    }
}

__global__ __launch_bounds__(kBlock) void k_fill(uint32_t* __restrict__ p, uint64_t n, uint32_t v) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * kBlock)
        p[i] = v;
}

__global__ __launch_bounds__(kBlock) void k_check_sorted(const uint32_t* __restrict__ planes,
                                                         uint64_t stride, uint64_t n,
                                                         uint32_t* __restrict__ flag) {
    bool bad = false;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i + 1 < n;
         i += (uint64_t)gridDim.x * kBlock) {
        uint32_t a[DHT_W], b[DHT_W];
        load_id(planes, stride, i, a);
        load_id(planes, stride, i + 1, b);
        bad |= !lex_lt(a, b);
    }
    if (__ballot(bad) && lane_id() == 0) atomicOr(flag, 1u);
}

// ---- prefix selection (deterministic stream compaction, order preserving) -----------
constexpr uint32_t kSelPer = 4096;   // ids per block (256 threads x 16)

__device__ __forceinline__ bool sel_match(uint32_t w0, uint32_t pbits, uint32_t pval) {
    return pbits == 0 || (w0 >> (32 - pbits)) == pval;
}

__global__ __launch_bounds__(kBlock) void k_sel_count(const uint32_t* __restrict__ w0, uint64_t n, uint32_t pbits,
                                                      uint32_t pval, uint32_t* __restrict__ bcount) {
    __shared__ uint32_t c;
    if (threadIdx.x == 0) c = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kSelPer;
    uint32_t mine = 0;
    for (uint32_t e = threadIdx.x; e < kSelPer; e += kBlock)
        if (base + e < n && sel_match(w0[base + e], pbits, pval)) ++mine;
    atomicAdd(&c, mine);
    __syncthreads();
    if (threadIdx.x == 0) bcount[blockIdx.x] = c;
}

__global__ __launch_bounds__(1024) void k_sel_scan(uint32_t* __restrict__ a, uint32_t len,
                                                   unsigned long long* __restrict__ total) {
    __shared__ uint32_t scr[1024];
    uint32_t carry = 0;
    for (uint32_t b = 0; b < len; b += 1024) {
        const uint32_t i = b + threadIdx.x;
        const uint32_t v = i < len ? a[i] : 0;
        scr[threadIdx.x] = v;
        __syncthreads();
        for (uint32_t o = 1; o < 1024; o <<= 1) {
            const uint32_t x = threadIdx.x >= o ? scr[threadIdx.x - o] : 0;
            __syncthreads();
            scr[threadIdx.x] += x;
            __syncthreads();
        }
        if (i < len) a[i] = carry + scr[threadIdx.x] - v;
        carry += scr[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = carry;
}

// order-preserving compaction: within a block, chunks of 256 ids in index order; a
// chunk's matches are ranked by wave ballots + per-wave offsets in LDS
__global__ __launch_bounds__(kBlock) void k_sel_compact(const uint32_t* __restrict__ planes, uint64_t stride,
                                                        uint64_t n, uint32_t pbits, uint32_t pval,
                                                        const uint32_t* __restrict__ boff,
                                                        uint32_t* __restrict__ out, uint64_t out_stride,
                                                        uint32_t* __restrict__ gidx, uint64_t gbase) {
    __shared__ uint32_t wsum[kBlock / 64];
    __shared__ uint32_t run;
    if (threadIdx.x == 0) run = boff[blockIdx.x];
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kSelPer;
    const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
    for (uint32_t e0 = 0; e0 < kSelPer; e0 += kBlock) {
        const uint64_t i = base + e0 + threadIdx.x;
        const bool m = i < n && sel_match(planes[i], pbits, pval);
        const uint64_t bal = __ballot(m);
        const uint32_t before = (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[wave] = (uint32_t)__popcll(bal);
        __syncthreads();
        uint32_t woff = run;
        for (uint32_t w = 0; w < wave; ++w) woff += wsum[w];
        if (m) {
            const uint32_t pos = woff + before;
#pragma unroll
            for (int j = 0; j < DHT_W; ++j) out[(uint64_t)j * out_stride + pos] = planes[(uint64_t)j * stride + i];
            if (gidx) gidx[pos] = (uint32_t)(gbase + i);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t t = 0;
            for (uint32_t w = 0; w < kBlock / 64; ++w) t += wsum[w];
            run += t;
        }
        __syncthreads();
    }
}

}  // namespace

hipError_t launch_select_prefix(const uint32_t* planes, uint64_t stride, uint64_t n, uint32_t pbits,
                                uint32_t pval, uint32_t* scratch, unsigned long long* d_total,
                                uint32_t* out, uint64_t out_stride, uint32_t* gidx, uint64_t gbase,
                                hipStream_t s) {
    const uint32_t nblk = (uint32_t)((n + kSelPer - 1) / kSelPer);
    if (!nblk) return hipMemsetAsync(d_total, 0, 8, s);
    k_sel_count<<<nblk, kBlock, 0, s>>>(planes, n, pbits, pval, scratch);
    k_sel_scan<<<1, 1024, 0, s>>>(scratch, nblk, d_total);
    if (out) k_sel_compact<<<nblk, kBlock, 0, s>>>(planes, stride, n, pbits, pval, scratch, out, out_stride, gidx, gbase);
    return hipGetLastError();
}

uint64_t select_scratch_words(uint64_t n) { return (n + kSelPer - 1) / kSelPer + 1; }

hipError_t launch_gen(uint64_t seed, uint64_t start, uint64_t n, uint32_t* planes,
                      uint64_t stride, hipStream_t s) {
    if (!n) return hipSuccess;
    k_gen<<<grid_for(n, kBlock), kBlock, 0, s>>>(seed, start, n, planes, stride);
    return hipGetLastError();
}
hipError_t launch_pack(const uint8_t* ids20, uint64_t n, uint32_t* planes, uint64_t stride,
                       hipStream_t s) {
    if (!n) return hipSuccess;
    k_pack<<<grid_for(n, kBlock), kBlock, 0, s>>>((const uint32_t*)ids20, n, planes, stride);
    return hipGetLastError();
}
hipError_t launch_unpack(const uint32_t* planes, uint64_t stride, uint64_t first, uint64_t n,
                         uint8_t* out20, hipStream_t s) {
    if (!n) return hipSuccess;
    k_unpack<<<grid_for(n, kBlock), kBlock, 0, s>>>(planes, stride, first, n, (uint32_t*)out20);
    return hipGetLastError();
}
hipError_t launch_fill(uint32_t* p, uint64_t n, uint32_t v, hipStream_t s) {
    if (!n) return hipSuccess;
    k_fill<<<grid_for(n, kBlock), kBlock, 0, s>>>(p, n, v);
    return hipGetLastError();
}
hipError_t launch_check_sorted(const uint32_t* planes, uint64_t stride, uint64_t n,
                               uint32_t* d_flag, hipStream_t s) {
    if (n < 2) return hipSuccess;
    k_check_sorted<<<grid_for(n, kBlock), kBlock, 0, s>>>(planes, stride, n, d_flag);
    return hipGetLastError();
}

}  // namespace dhtgpu
