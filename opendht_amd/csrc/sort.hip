// sort.hip -- lexicographic sort of 160-bit node ids on gfx950.
//
// NodeCache keeps every known node in a std::map<InfoHash, weak_ptr<Node>> ordered by
// InfoHash::operator< (include/opendht/node_cache.h:43, include/opendht/infohash.h:107-113)
// and getCachedNodes walks it from lower_bound(target) (src/node_cache.cpp:42-74).  The device
// mirror of that map is the id set sorted lexicographically = by (w0, w1, w2, w3, w4) as
// unsigned words, plus the permutation back to the caller's order.
//
// Stable LSD radix sort over 8-bit digits, least significant first (byte 0 of w4 ... byte 3 of
// w0).  One pass = three kernels:
//   hist     per 4096-id tile, the digit histogram (LDS atomics) -> counts[digit][tile]
//   rowscan  one workgroup per digit: exclusive scan of its row over the tiles + row total
//   scatter  every tile re-reads its ids in index order, 256 at a time; a wave ranks equal
//            digits among its lanes with 8 ballots (bit-sliced match), the waves' per-digit
//            counts go through LDS in wave order, so the scatter is stable; the five key
//            words and the permutation word move to their slots.
// Passes over the two high words run first as a shortcut: when the 64-bit prefixes
// (w0, w1) of the sorted ids are all distinct (the case for random ids up to ~10^9) the
// order is already total; otherwise the full 20-pass sort runs from the original order.
// Every pass streams 24 B/id in and scatters 24 B/id out (HBM-bound; setup-time work).
#include "dhtgpu_dev.h"
#include "dhtgpu_internal.h"

namespace dhtgpu {
namespace {

constexpr uint32_t kSortThreads = 256;
constexpr uint32_t kSortItems = 16;
constexpr uint32_t kSortTile = kSortThreads * kSortItems;   // 4096 ids per tile
constexpr uint32_t kWaves = kSortThreads / 64;

__device__ __forceinline__ uint32_t digit_of(uint32_t w, uint32_t shift) { return (w >> shift) & 0xFFu; }

__global__ __launch_bounds__(kSortThreads) void k_sort_hist(const uint32_t* __restrict__ word, uint64_t n,
                                                            uint32_t shift, uint32_t ntiles,
                                                            uint32_t* __restrict__ counts) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kSortTile;
#pragma unroll
    for (uint32_t r = 0; r < kSortItems; ++r) {
        const uint64_t i = base + r * kSortThreads + threadIdx.x;
        if (i < n) atomicAdd(&h[digit_of(word[i], shift)], 1u);
    }
    __syncthreads();
    counts[(uint64_t)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}

// exclusive scan of counts[d][0 .. ntiles) in place; tot[d] = the row's sum
__global__ __launch_bounds__(1024) void k_sort_rowscan(uint32_t* __restrict__ counts, uint32_t ntiles,
                                                       uint32_t* __restrict__ tot) {
    __shared__ uint32_t wsum[16];
    uint32_t* row = counts + (uint64_t)blockIdx.x * ntiles;
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    uint32_t carry = 0;
    for (uint32_t c0 = 0; c0 < ntiles; c0 += 1024) {
        const uint32_t i = c0 + threadIdx.x;
        const uint32_t v = i < ntiles ? row[i] : 0u;
        uint32_t x = v;   // inclusive wave scan
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, o);
            if (lane >= (uint32_t)o) x += y;
        }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        uint32_t before = carry;
        for (uint32_t j = 0; j < w; ++j) before += wsum[j];
        uint32_t all = 0;
        for (uint32_t j = 0; j < 16; ++j) all += wsum[j];
        if (i < ntiles) row[i] = before + x - v;
        carry += all;
        __syncthreads();
    }
    if (threadIdx.x == 0) tot[blockIdx.x] = carry;
}

struct SortBufs {
    const uint32_t* in[6];   // five key planes + permutation
    uint32_t* out[6];
    uint64_t in_stride, out_stride;   // key planes: word j of id i at in[j][i] (planes are separate pointers)
};

__global__ __launch_bounds__(kSortThreads) void k_sort_scatter(SortBufs b, uint64_t n, uint32_t wsel, uint32_t shift,
                                                               uint32_t ntiles, const uint32_t* __restrict__ counts,
                                                               const uint32_t* __restrict__ tot) {
    __shared__ uint32_t base[256];
    __shared__ uint32_t wcnt[kWaves][256];
    __shared__ uint32_t scan_tmp[256];
    const uint32_t tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
    // digit bases: exclusive scan of the 256 row totals (every tile does it; 1 KB) + this tile's row prefix
    scan_tmp[tid] = tot[tid];
#pragma unroll
    for (uint32_t w = 0; w < kWaves; ++w) wcnt[w][tid] = 0;
    __syncthreads();
    uint32_t acc = 0;
    for (uint32_t j = 0; j < tid; ++j) acc += scan_tmp[j];
    base[tid] = acc + counts[(uint64_t)tid * ntiles + blockIdx.x];
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * kSortTile;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (uint32_t r = 0; r < kSortItems; ++r) {
        const uint64_t i = t0 + r * kSortThreads + tid;
        const bool valid = i < n;
        uint32_t v[6];
#pragma unroll
        for (int j = 0; j < 6; ++j) v[j] = valid ? b.in[j][i] : 0u;
        const uint32_t d = digit_of(v[wsel], shift);
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (uint32_t bit = 0; bit < 8; ++bit) {
            const uint64_t bb = __ballot((d >> bit) & 1u);
            peers &= ((d >> bit) & 1u) ? bb : ~bb;
        }
        const uint32_t rank = (uint32_t)__popcll(peers & lt);
        if (valid && rank == 0) wcnt[wv][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        if (valid) {
            uint32_t off = base[d] + rank;
            for (uint32_t w = 0; w < wv; ++w) off += wcnt[w][d];
#pragma unroll
            for (int j = 0; j < 6; ++j) b.out[j][off] = v[j];
        }
        __syncthreads();
        uint32_t add = 0;
#pragma unroll
        for (uint32_t w = 0; w < kWaves; ++w) {
            add += wcnt[w][tid];
            wcnt[w][tid] = 0;
        }
        base[tid] += add;
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_iota(uint32_t* __restrict__ p, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        p[i] = (uint32_t)i;
}

// flag |= 1 if two adjacent sorted ids share their first `words` words (2: the (w0, w1)
// shortcut is not total; 5: duplicated ids)
__global__ __launch_bounds__(256) void k_adjacent_equal(const uint32_t* __restrict__ planes, uint64_t stride, uint64_t n,
                                                        uint32_t words, uint32_t* __restrict__ flag) {
    bool eq = false;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i + 1 < n; i += (uint64_t)gridDim.x * 256) {
        bool e = true;
        for (uint32_t j = 0; j < words; ++j) e = e && planes[(uint64_t)j * stride + i] == planes[(uint64_t)j * stride + i + 1];
        eq |= e;
    }
    if (__ballot(eq) && lane_id() == 0) atomicOr(flag, 1u);
}

inline uint32_t grid256(uint64_t n) {
    uint64_t g = (n + 255) / 256;
    if (g > 8192) g = 8192;
    return (uint32_t)(g ? g : 1);
}

}  // namespace

size_t sort_scratch_bytes(uint64_t n) {
    const uint64_t ntiles = (n + kSortTile - 1) / kSortTile;
    // ping-pong key planes + permutation (6 words per id), counts[256][ntiles], totals, flag
    return (size_t)6 * 4 * (n ? n : 1) + (size_t)256 * 4 * (ntiles ? ntiles : 1) + 256 * 4 + 256;
}

hipError_t launch_sort_ids(const uint32_t* planes, uint64_t stride, uint64_t n, uint32_t* out_planes, uint64_t out_stride,
                           uint32_t* perm, void* scratch, int* unique, hipStream_t s) {
    *unique = 1;
    if (n == 0) return hipSuccess;
    if (n >= 0xFFFFFFFFull) return hipErrorInvalidValue;
    const uint32_t ntiles = (uint32_t)((n + kSortTile - 1) / kSortTile);
    uint8_t* w = static_cast<uint8_t*>(scratch);
    uint32_t* tmp = reinterpret_cast<uint32_t*>(w);                       // 6 arrays of n words
    uint32_t* counts = tmp + (size_t)6 * n;
    uint32_t* tot = counts + (size_t)256 * ntiles;
    uint32_t* flag = tot + 256;
    uint32_t* A[6];   // the output buffers (also the input copy)
    uint32_t* B[6];   // the scratch ping-pong buffers
    for (int j = 0; j < 5; ++j) A[j] = out_planes + (uint64_t)j * out_stride;
    A[5] = perm;
    for (int j = 0; j < 6; ++j) B[j] = tmp + (size_t)j * n;
    // sort by words [0, top]: LSD passes from byte 0 of word `top` to byte 3 of word 0; the input
    // is copied into A first, pass p reads A and writes B when p is even (B -> A when odd), so
    // the last pass of an even count (p odd) writes A
    auto run = [&](int top) -> hipError_t {
        for (int j = 0; j < 5; ++j) {
            hipError_t x = hipMemcpyAsync(A[j], planes + (uint64_t)j * stride, (size_t)n * 4, hipMemcpyDeviceToDevice, s);
            if (x != hipSuccess) return x;
        }
        k_iota<<<grid256(n), 256, 0, s>>>(A[5], n);
        int pass = 0;
        for (int word = top; word >= 0; --word) {
            for (uint32_t byte = 0; byte < 4; ++byte, ++pass) {
                SortBufs sb;
                for (int j = 0; j < 6; ++j) {
                    sb.in[j] = (pass & 1) ? B[j] : A[j];
                    sb.out[j] = (pass & 1) ? A[j] : B[j];
                }
                sb.in_stride = sb.out_stride = 0;
                k_sort_hist<<<ntiles, kSortThreads, 0, s>>>(sb.in[word], n, 8 * byte, ntiles, counts);
                k_sort_rowscan<<<256, 1024, 0, s>>>(counts, ntiles, tot);
                k_sort_scatter<<<ntiles, kSortThreads, 0, s>>>(sb, n, (uint32_t)word, 8 * byte, ntiles, counts, tot);
            }
        }
        return hipGetLastError();
    };
    auto adjacent_equal = [&](uint32_t words, uint32_t* out) -> hipError_t {
        hipError_t x = hipMemsetAsync(flag, 0, 4, s);
        if (x != hipSuccess) return x;
        k_adjacent_equal<<<grid256(n), 256, 0, s>>>(out_planes, out_stride, n, words, flag);
        if ((x = hipMemcpyAsync(out, flag, 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return x;
        return hipStreamSynchronize(s);
    };
    hipError_t e = run(1);   // the (w0, w1) shortcut
    uint32_t tie = 0;
    if (e == hipSuccess) e = adjacent_equal(2, &tie);
    if (e == hipSuccess && tie) {
        e = run(4);           // some 64-bit prefixes repeat: the full 160-bit sort
        uint32_t dup = 0;
        if (e == hipSuccess) e = adjacent_equal(5, &dup);
        *unique = dup ? 0 : 1;
    }
    return e;
}

}  // namespace dhtgpu
