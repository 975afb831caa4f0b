// table.hip -- routing-table kernels for gfx950.
//   K1r k_find_closest : RoutingTable::findClosestNodes (src/routing_table.cpp:110-150)
//   K2  k_classify     : RoutingTable::findBucket (:153-166) + InfoHash::commonBits
//                        (include/opendht/infohash.h:154-176) histogram
//   a8  k_cached       : NodeCache::getCachedNodes (src/node_cache.cpp:42-74)
#include "dhtgpu_dev.h"
#include "dhtgpu_internal.h"

namespace dhtgpu {
namespace {

// ---------------------------------------------------------------------------------
// K1r.  Semantics: j = findBucket(t); visit buckets in rounds
// r = 0,1,..: b_{j+r} then b_{j-1-r}, stopping after the first round in which the
// number of good nodes seen reaches `count` (or both sides run out); the answer is
// the min(count, C) XOR-closest good nodes of the visited contiguous bucket range,
// ascending -- exactly what the reference's insertion sort (find_if on xorCmp) yields.
// Buckets own contiguous node ranges [off[b], off[b+1]), so the visited range is one
// contiguous node slice.  One thread per target; the running top-K is a register
// list {d0, d1, idx} kept sorted by an unrolled compare-swap chain (static indices).
// ---------------------------------------------------------------------------------
struct Ent {
    uint32_t d0, d1, idx;
};

__device__ __forceinline__ bool ent_less(const Ent& a, const Ent& b,
                                         const uint32_t* __restrict__ np, uint64_t ns,
                                         const uint32_t* t) {
    if (b.idx == DHT_NONE) return a.idx != DHT_NONE;
    if (a.idx == DHT_NONE) return false;
    if (a.d0 != b.d0) return a.d0 < b.d0;
    if (a.d1 != b.d1) return a.d1 < b.d1;
    uint32_t wa[DHT_W], wb[DHT_W];
    load_id(np, ns, a.idx, wa);
    load_id(np, ns, b.idx, wb);
    return xor_less_from(wa, a.idx, wb, b.idx, t, 2);
}

template <uint32_t K>
__global__ __launch_bounds__(256) void k_find_closest(
    uint32_t nb, const uint32_t* __restrict__ fp, const uint32_t* __restrict__ off,
    const uint32_t* __restrict__ gcnt, const uint32_t* __restrict__ np, uint64_t ns,
    const uint8_t* __restrict__ good, const uint32_t* __restrict__ tp, uint64_t ts, uint32_t q,
    uint32_t count, uint32_t* __restrict__ out_idx, uint32_t* __restrict__ out_cnt) {
    const uint32_t qi = blockIdx.x * blockDim.x + threadIdx.x;
    if (qi >= q) return;
    uint32_t t[DHT_W];
    load_id(tp, ts, qi, t);

    // findBucket: the last bucket b >= 1 with first_b <= t, else bucket 0
    uint32_t j = 0;
    for (uint32_t step = 1u << 8; step; step >>= 1) {
        const uint32_t c = j + step;
        if (c < nb) {
            uint32_t f[DHT_W];
#pragma unroll
            for (int w = 0; w < DHT_W; ++w) f[w] = fp[(uint64_t)w * nb + c];
            if (lex_le(f, t)) j = c;
        }
    }
    // outward walk over per-bucket good counts
    uint32_t seen = 0;
    int itn = (int)j, itp = (int)j - 1;
    while (seen < count && (itn < (int)nb || itp >= 0)) {
        if (itn < (int)nb) seen += gcnt[itn++];
        if (itp >= 0) seen += gcnt[itp--];
    }
    const uint32_t lo = off[itp + 1], hi = off[itn];

    Ent e[K];
#pragma unroll
    for (uint32_t r = 0; r < K; ++r) e[r] = Ent{DHT_NONE, DHT_NONE, DHT_NONE};
    for (uint32_t i = lo; i < hi; ++i) {
        if (!good[i]) continue;
        Ent c{np[i] ^ t[0], np[ns + i] ^ t[1], i};
#pragma unroll
        for (uint32_t r = 0; r < K; ++r) {
            if (ent_less(c, e[r], np, ns, t)) {
                const Ent tmp = e[r];
                e[r] = c;
                c = tmp;
            }
        }
    }
    uint32_t n_out = 0;
#pragma unroll
    for (uint32_t r = 0; r < K; ++r) {
        if (r < count) {
            out_idx[(uint64_t)qi * count + r] = e[r].idx;
            n_out += e[r].idx != DHT_NONE;
        }
    }
    out_cnt[qi] = n_out;
}

// ---------------------------------------------------------------------------------
// K2.  HBM-streaming: each thread classifies 4 consecutive ids per step (5 x 16-B plane
// loads, one 4-B bucket store), with the next step's 5 loads issued before this step's
// work (two steps in flight per lane).  The grid is kClsPerCu = 32 workgroups per CU (four
// rounds of the eight that are resident at once): shorter grid-stride ranges per workgroup
// end together (measured, profiles/r03/experiments/k2_shapes.txt: 4 per CU 0.468 ms, 8 0.48,
// 16 0.44, 32 0.42-0.43, 64 without the look-ahead 0.43 ms).  Bucket
// firsts live in LDS; findBucket is a branch-light binary search.  commonBits is a clz
// over the first nonzero xor word; the heavy low bins (cb < 8 hold 255/256 of uniform ids)
// are counted with wave ballots, the rest with LDS atomics, then one global atomic per bin
// per workgroup.
// ---------------------------------------------------------------------------------
constexpr int kClsBlock = 256;
#ifndef DHT_K2_PERCU
#define DHT_K2_PERCU 32
#endif
#ifndef DHT_K2_AHEAD
#define DHT_K2_AHEAD 1
#endif
constexpr int kClsPerCu = DHT_K2_PERCU;
constexpr bool kClsAhead = DHT_K2_AHEAD != 0;   // the next step's loads issued before this step's work

__global__ __launch_bounds__(kClsBlock) void k_classify(
    const uint32_t* __restrict__ planes, uint64_t stride, uint64_t n, uint32_t nb,
    const uint32_t* __restrict__ fp, uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3,
    uint32_t m4, uint8_t* __restrict__ out_bucket, unsigned long long* __restrict__ hist) {
    __shared__ uint32_t sf[DHT_W * 256];
    __shared__ uint32_t sh[161];
    const uint64_t n4 = (n + 3) / 4;
    const uint64_t G = (uint64_t)gridDim.x * kClsBlock;
    uint64_t g = (uint64_t)blockIdx.x * kClsBlock + threadIdx.x;
    // the first step's loads ahead of the setup
    uint4 v[DHT_W];
#pragma unroll
    for (int w = 0; w < DHT_W; ++w)
        v[w] = g < n4 ? reinterpret_cast<const uint4*>(planes + (uint64_t)w * stride)[g] : make_uint4(0u, 0u, 0u, 0u);
    for (uint32_t i = threadIdx.x; i < DHT_W * nb; i += kClsBlock) sf[i] = fp[i];
    for (uint32_t i = threadIdx.x; i < 161; i += kClsBlock) sh[i] = 0;
    __syncthreads();
    const uint32_t my[DHT_W] = {m0, m1, m2, m3, m4};
    const uint32_t lane = lane_id();
    uint32_t low[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (; g - threadIdx.x < n4; g += G) {   // block-uniform: whole waves stay in the loop for the ballots
        const bool active = g < n4;
        const uint64_t gn = g + G;
        uint4 nx[DHT_W];
        if (kClsAhead) {
#pragma unroll
            for (int w = 0; w < DHT_W; ++w)
                nx[w] = gn < n4 ? reinterpret_cast<const uint4*>(planes + (uint64_t)w * stride)[gn] : make_uint4(0u, 0u, 0u, 0u);
        }
        uint32_t packed = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const uint64_t i = 4 * g + e;
            const bool valid = active && i < n;
            uint32_t id[DHT_W];
#pragma unroll
            for (int w = 0; w < DHT_W; ++w) id[w] = e == 0 ? v[w].x : e == 1 ? v[w].y : e == 2 ? v[w].z : v[w].w;
            // findBucket by binary search on word 0 of the firsts; words 1..4 only when word 0
            // ties (a first shares the id's top 32 bits: rare)
            uint32_t j = 0;
            for (uint32_t step = 128; step; step >>= 1) {
                const uint32_t c = j + step;
                if (c < nb) {
                    const uint32_t f0 = sf[c];
                    bool le = f0 < id[0];
                    if (f0 == id[0]) {
                        uint32_t f[DHT_W];
#pragma unroll
                        for (int w = 0; w < DHT_W; ++w) f[w] = sf[w * nb + c];
                        le = lex_le(f, id);
                    }
                    if (le) j = c;
                }
            }
            packed |= j << (8 * e);
            const uint32_t cb = common_bits(id, my);
#pragma unroll
            for (uint32_t b = 0; b < 8; ++b) low[b] += (uint32_t)__popcll(__ballot(valid && cb == b));
            if (valid && cb >= 8) atomicAdd(&sh[cb], 1u);
        }
        if (active && out_bucket) {
            if (4 * g + 3 < n) {
                *reinterpret_cast<uint32_t*>(out_bucket + 4 * g) = packed;
            } else {
                for (int e = 0; e < 4; ++e)
                    if (4 * g + e < n) out_bucket[4 * g + e] = (uint8_t)(packed >> (8 * e));
            }
        }
        if (kClsAhead) {
#pragma unroll
            for (int w = 0; w < DHT_W; ++w) v[w] = nx[w];
        } else {
#pragma unroll
            for (int w = 0; w < DHT_W; ++w)
                v[w] = gn < n4 ? reinterpret_cast<const uint4*>(planes + (uint64_t)w * stride)[gn] : make_uint4(0u, 0u, 0u, 0u);
        }
    }
    if (lane == 0) {
#pragma unroll
        for (uint32_t b = 0; b < 8; ++b)
            if (low[b]) atomicAdd(&sh[b], low[b]);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < 161; i += kClsBlock)
        if (sh[i]) atomicAdd(hist + i, (unsigned long long)sh[i]);
}

// ---------------------------------------------------------------------------------
// a8.  One thread per target: lower_bound over the lexicographically sorted planes,
// then the reference's two-pointer walk (take the XOR-closer of prev/next; accept
// iff the accept bit is set), emitting accepted nodes in walk order.  perm (nullable)
// maps a sorted position to the caller's index (an unsorted upload sorted on the
// device, sort.hip); accept and the output are in the caller's index space.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_cached(const uint32_t* __restrict__ planes,
                                                uint64_t stride, uint64_t n,
                                                const uint32_t* __restrict__ perm,
                                                const uint8_t* __restrict__ accept,
                                                const uint32_t* __restrict__ tp, uint64_t ts,
                                                uint32_t q, uint32_t count,
                                                uint32_t* __restrict__ out_idx,
                                                uint32_t* __restrict__ out_cnt) {
    const uint32_t qi = blockIdx.x * blockDim.x + threadIdx.x;
    if (qi >= q) return;
    uint32_t t[DHT_W];
    load_id(tp, ts, qi, t);
    uint64_t lo = 0, hi = n;   // first id >= t
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        uint32_t m[DHT_W];
        load_id(planes, stride, mid, m);
        if (lex_lt(m, t)) lo = mid + 1;
        else hi = mid;
    }
    const uint64_t END = n;
    uint64_t it_n = lo, it_p = lo;
    if (n != 0) it_p = it_p == 0 ? END : it_p - 1;
    uint32_t c = 0;
    while (c < count && (it_n != END || it_p != END)) {
        uint64_t it;
        if (it_p == END) {
            it = it_n++;
        } else if (it_n == END) {
            it = it_p;
            it_p = it_p == 0 ? END : it_p - 1;
        } else {
            uint32_t a[DHT_W], b[DHT_W];
            load_id(planes, stride, it_p, a);
            load_id(planes, stride, it_n, b);
            // InfoHash::xorCmp(it_p, it_n) < 0  (ids are unique, so no index tie)
            if (xor_less_from(a, 0, b, 1, t, 0)) {
                it = it_p;
                it_p = it_p == 0 ? END : it_p - 1;
            } else {
                it = it_n++;
            }
        }
        const uint32_t id = perm ? perm[it] : (uint32_t)it;
        if (!accept || accept[id]) out_idx[(uint64_t)qi * count + c++] = id;
    }
    out_cnt[qi] = c;
    for (uint32_t r = c; r < count; ++r) out_idx[(uint64_t)qi * count + r] = DHT_NONE;
}

}  // namespace

hipError_t launch_find_closest(uint32_t nb, const uint32_t* fp, const uint32_t* off,
                               const uint32_t* gcnt, const uint32_t* np, uint64_t ns,
                               const uint8_t* good, const uint32_t* tp, uint64_t ts, uint32_t q,
                               uint32_t count, uint32_t* out_idx, uint32_t* out_cnt,
                               hipStream_t s) {
    if (!q) return hipSuccess;
    const uint32_t grid = (q + 255) / 256;
    if (count <= 8)
        k_find_closest<8><<<grid, 256, 0, s>>>(nb, fp, off, gcnt, np, ns, good, tp, ts, q, count, out_idx, out_cnt);
    else if (count <= 16)
        k_find_closest<16><<<grid, 256, 0, s>>>(nb, fp, off, gcnt, np, ns, good, tp, ts, q, count, out_idx, out_cnt);
    else
        k_find_closest<32><<<grid, 256, 0, s>>>(nb, fp, off, gcnt, np, ns, good, tp, ts, q, count, out_idx, out_cnt);
    return hipGetLastError();
}

hipError_t launch_classify(const uint32_t* planes, uint64_t stride, uint64_t n, uint32_t nb,
                           const uint32_t* fp, const uint32_t* myid, uint8_t* out_bucket,
                           unsigned long long* hist, hipStream_t s) {
    if (!n) return hipSuccess;
    const uint64_t n4 = (n + 3) / 4;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    uint64_t grid = (n4 + kClsBlock - 1) / kClsBlock;
    const uint64_t full = (uint64_t)(cus > 0 ? cus : 256) * kClsPerCu;
    if (grid > full) grid = full;
    k_classify<<<(uint32_t)grid, kClsBlock, 0, s>>>(planes, stride, n, nb, fp, myid[0], myid[1],
                                                    myid[2], myid[3], myid[4], out_bucket, hist);
    return hipGetLastError();
}

hipError_t launch_cached(const uint32_t* planes, uint64_t stride, uint64_t n, const uint32_t* perm,
                         const uint8_t* accept, const uint32_t* tp, uint64_t ts, uint32_t q,
                         uint32_t count, uint32_t* out_idx, uint32_t* out_cnt, hipStream_t s) {
    if (!q) return hipSuccess;
    k_cached<<<(q + 255) / 256, 256, 0, s>>>(planes, stride, n, perm, accept, tp, ts, q, count, out_idx, out_cnt);
    return hipGetLastError();
}

}  // namespace dhtgpu
