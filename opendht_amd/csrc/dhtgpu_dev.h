// dhtgpu_dev.h -- device-side helpers shared by the libdhtgpu kernels (gfx950).
//
// A 160-bit node id (dht::InfoHash, include/opendht/infohash.h:61-265) is held as
// five big-endian u32 words w0..w4 in word planes: word j of id i lives at
// planes[j*stride + i].  Lexicographic byte order (InfoHash::operator<, :107-113)
// is then lexicographic order over (w0..w4) as unsigned integers, and the XOR
// order of InfoHash::xorCmp (:179-194) is lexicographic order over (wj ^ tj).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DHT_W 5
#define DHT_NONE 0xFFFFFFFFu
#define DHTGPU_MAX_K_DEV 32u   // = DHTGPU_MAX_K of include/dhtgpu.h

namespace dhtgpu {

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// (a ^ t) < (b ^ t) over words [from, 5), then index; a/b/t are 5-word arrays.
__device__ __forceinline__ bool xor_less_from(const uint32_t* a, uint32_t ia, const uint32_t* b,
                                              uint32_t ib, const uint32_t* t, int from) {
#pragma unroll
    for (int j = 0; j < DHT_W; ++j) {
        if (j < from) continue;
        uint32_t da = a[j] ^ t[j], db = b[j] ^ t[j];
        if (da != db) return da < db;
    }
    return ia < ib;
}

// lexicographic a <= b (InfoHash::cmp(a, b) <= 0, infohash.h:149-151)
__device__ __forceinline__ bool lex_le(const uint32_t* a, const uint32_t* b) {
#pragma unroll
    for (int j = 0; j < DHT_W; ++j)
        if (a[j] != b[j]) return a[j] < b[j];
    return true;
}

// lexicographic a < b
__device__ __forceinline__ bool lex_lt(const uint32_t* a, const uint32_t* b) {
#pragma unroll
    for (int j = 0; j < DHT_W; ++j)
        if (a[j] != b[j]) return a[j] < b[j];
    return false;
}

// InfoHash::commonBits (infohash.h:154-176): leading zero bits of a ^ b, 160 if equal.
__device__ __forceinline__ uint32_t common_bits(const uint32_t* a, const uint32_t* b) {
    uint32_t r = 160;
    bool done = false;
#pragma unroll
    for (int j = 0; j < DHT_W; ++j) {
        uint32_t x = a[j] ^ b[j];
        if (!done && x) { r = 32u * j + __clz(x); done = true; }
    }
    return r;
}

__device__ __forceinline__ void load_id(const uint32_t* __restrict__ planes, uint64_t stride,
                                        uint64_t i, uint32_t* w) {
#pragma unroll
    for (int j = 0; j < DHT_W; ++j) w[j] = planes[(uint64_t)j * stride + i];
}

__device__ __forceinline__ uint64_t splitmix(uint64_t seed, uint64_t j) {
    uint64_t z = seed + (j + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

}  // namespace dhtgpu
