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

}  // namespace

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
