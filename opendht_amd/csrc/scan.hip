// scan.hip -- K1 xor_topk_scan and K3 topk_merge for gfx950.
//
// K1 restates std::partial_sort(ids, ids+k, ids+n, [t](a,b){ return t.xorCmp(a,b) < 0; })
// (InfoHash::xorCmp, include/opendht/infohash.h:179-194) for a batch of
// targets; its body (scan_dev.h) streams the w0 plane through LDS and keeps every target's
// exact top-k in registers.  When the batch has too few targets to fill the chip the id
// range is split across workgroups and the per-split lists are merged by K3.
#include "scan_dev.h"

namespace dhtgpu {
namespace {

using scan::WAVES;
using scan::TILE;

template <uint32_t K, uint32_t T>
__global__ __launch_bounds__(WAVES * 64, 4) void k_scan(
    const uint32_t* __restrict__ ids, uint64_t is, uint64_t n, uint64_t split_len,
    const uint32_t* __restrict__ tp, uint64_t ts, uint32_t q, uint32_t k,
    uint32_t* __restrict__ out_idx, uint32_t* __restrict__ out_cnt, uint32_t* __restrict__ out_rec,
    const uint32_t* __restrict__ gidx, uint32_t idx_base) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[scan::lds_words<T>()];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t id_begin = (uint64_t)blockIdx.y * split_len;
    const uint64_t id_end = n < id_begin + split_len ? n : id_begin + split_len;
    scan::ScanOut o{out_idx, out_cnt, gidx, idx_base, out_rec, (uint64_t)blockIdx.y * q, idx_base};
    scan::scan_run<K, T>(lds, ids, is, id_begin, id_end, tp, ts, nullptr, (blockIdx.x * WAVES + wave) * T, q, k, o);
}

// K3: one wave per target; candidates staged in LDS as {w0^t .. w4^t, idx}; the rank
// of each valid candidate (number of strictly closer candidates) is its output slot.
__global__ __launch_bounds__(64) void k_merge(const uint32_t* __restrict__ rec, uint32_t lists,
                                              uint32_t q, uint32_t kin,
                                              const uint32_t* __restrict__ tp, uint64_t ts,
                                              uint32_t k, uint32_t* __restrict__ out_idx,
                                              uint32_t* __restrict__ out_cnt) {
    extern __shared__ uint32_t sm[];
    const uint32_t qi = blockIdx.x, lane = lane_id();
    const uint32_t C = lists * kin;
    uint32_t t[DHT_W];
    load_id(tp, ts, qi, t);
    uint32_t nvalid = 0;
    for (uint32_t c0 = 0; c0 < C; c0 += 64) {
        const uint32_t c = c0 + lane;
        bool v = false;
        if (c < C) {
            const uint32_t l = c / kin, r = c % kin;
            const uint32_t* src = rec + (((uint64_t)l * q + qi) * kin + r) * 6;
            const uint32_t idx = src[5];
            v = idx != DHT_NONE;
#pragma unroll
            for (int w = 0; w < DHT_W; ++w) sm[c * 6 + w] = src[w] ^ t[w];
            sm[c * 6 + 5] = idx;
        }
        nvalid += (uint32_t)__popcll(__ballot(v));
    }
    __syncthreads();
    for (uint32_t c0 = 0; c0 < C; c0 += 64) {
        const uint32_t c = c0 + lane;
        if (c >= C) continue;
        uint32_t key[6];
#pragma unroll
        for (int w = 0; w < 6; ++w) key[w] = sm[c * 6 + w];
        if (key[5] == DHT_NONE) continue;
        uint32_t rank = 0;
        for (uint32_t o = 0; o < C; ++o) {
            const uint32_t* kk = sm + o * 6;
            if (kk[5] == DHT_NONE) continue;
            bool less = false, decided = false;
#pragma unroll
            for (int w = 0; w < 6; ++w) {
                if (!decided && kk[w] != key[w]) {
                    less = kk[w] < key[w];
                    decided = true;
                }
            }
            rank += less;
        }
        if (rank < k) out_idx[(uint64_t)qi * k + rank] = key[5];
    }
    const uint32_t nout = nvalid < k ? nvalid : k;
    if (lane >= nout && lane < k) out_idx[(uint64_t)qi * k + lane] = DHT_NONE;
    for (uint32_t r = 64 + lane; r < k; r += 64)
        if (r >= nout) out_idx[(uint64_t)qi * k + r] = DHT_NONE;
    if (lane == 0) out_cnt[qi] = nout;
}

// K3 over sorted lists (every producer in this library writes its lists ascending in XOR
// order, DHT_NONE after the valid entries): the exact top-k is the first k picks of a k-way
// merge of the lists' heads.  G lanes per target (G = the power of two >= lists), lane j walking
// list j: its list {w0 ^ t0, w1 ^ t1, idx} is staged in LDS, and each of the k rounds takes the
// group minimum of the heads by an xor butterfly over (word-0 distance, word-1 distance, idx).
// Two heads of different ids that tie on both distances (never on hash-distributed ids) send
// the round to the full five-word compare (words 2..4 from the records).  64 / G targets per
// wave, four waves per block; against the pairwise rank (k_merge, one 64-thread block per
// target, C^2 LDS compares) this is k rounds of log2(G) shuffles.
constexpr int kMergeThreads = 256;

template <uint32_t G>
__global__ __launch_bounds__(kMergeThreads) void k_merge_heads(const uint32_t* __restrict__ rec, uint32_t lists,
                                                                uint32_t q, uint32_t kin, const uint32_t* __restrict__ tp,
                                                                uint64_t ts, uint32_t k, uint32_t* __restrict__ out_idx,
                                                                uint32_t* __restrict__ out_cnt) {
    extern __shared__ uint32_t sm[];   // [thread][kin][3]
    constexpr uint32_t TPW = 64 / G;
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    const uint32_t g = lane / G, j = lane % G;
    const uint32_t qi = (blockIdx.x * (kMergeThreads / 64) + wv) * TPW + g;
    const bool tv = qi < q, lv = tv && j < lists;
    const uint32_t qc = tv ? qi : 0u;
    const uint32_t t0 = tp[qc], t1 = tp[ts + qc];
    uint32_t* my = sm + threadIdx.x * kin * 3;
    const uint32_t* src = rec + ((uint64_t)(lv ? j : 0u) * q + qc) * kin * 6;
    for (uint32_t r = 0; r < kin; ++r) {
        const uint2 w01 = *reinterpret_cast<const uint2*>(src + r * 6);
        const uint32_t ix = lv ? src[r * 6 + 5] : DHT_NONE;
        const bool none = ix == DHT_NONE;
        my[3 * r] = none ? DHT_NONE : w01.x ^ t0;
        my[3 * r + 1] = none ? DHT_NONE : w01.y ^ t1;
        my[3 * r + 2] = ix;
    }
    uint32_t p = 0;
    uint32_t h0 = my[0], h1 = my[1], hi = my[2];
    uint32_t cnt = 0;
    for (uint32_t r = 0; r < k; ++r) {   // wave-uniform
        uint32_t m0 = h0, m1 = h1, mi = hi;
        bool tie = false;
#pragma unroll
        for (uint32_t o = 1; o < G; o <<= 1) {
            const uint32_t p0 = (uint32_t)__shfl_xor((int)m0, (int)o), p1 = (uint32_t)__shfl_xor((int)m1, (int)o);
            const uint32_t pi = (uint32_t)__shfl_xor((int)mi, (int)o);
            tie = tie || (p0 == m0 && p1 == m1 && pi != mi && pi != DHT_NONE && mi != DHT_NONE);
            const bool less = p0 < m0 || (p0 == m0 && (p1 < m1 || (p1 == m1 && pi < mi)));
            if (less) { m0 = p0; m1 = p1; mi = pi; }
        }
        const uint64_t gmask = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << (g * G);
        if (__ballot(tie) & gmask) {
            // both distances tie between different ids: the group minimum by the full key
            uint32_t f[DHT_W + 1];
            f[0] = h0; f[1] = h1; f[DHT_W] = hi;
            for (int w = 2; w < DHT_W; ++w)
                f[w] = hi == DHT_NONE ? DHT_NONE : src[p * 6 + w] ^ tp[(uint64_t)w * ts + qc];
#pragma unroll
            for (uint32_t o = 1; o < G; o <<= 1) {
                uint32_t pf[DHT_W + 1];
                for (int w = 0; w <= DHT_W; ++w) pf[w] = (uint32_t)__shfl_xor((int)f[w], (int)o);
                bool less = false, decided = false;
                for (int w = 0; w <= DHT_W; ++w) {
                    if (!decided && pf[w] != f[w]) { less = pf[w] < f[w]; decided = true; }
                }
                if (less)
                    for (int w = 0; w <= DHT_W; ++w) f[w] = pf[w];
            }
            m0 = f[0]; m1 = f[1]; mi = f[DHT_W];
        }
        if (mi == DHT_NONE) continue;   // this target's lists are exhausted (group-uniform)
        if (tv && j == 0) out_idx[(uint64_t)qi * k + r] = mi;
        ++cnt;
        if (hi == mi && lv) {   // the winning list advances (global indices are distinct across lists)
            ++p;
            if (p < kin) { h0 = my[3 * p]; h1 = my[3 * p + 1]; hi = my[3 * p + 2]; }
            else { h0 = DHT_NONE; h1 = DHT_NONE; hi = DHT_NONE; }
        }
    }
    if (tv && j == 0) {
        for (uint32_t r = cnt; r < k; ++r) out_idx[(uint64_t)qi * k + r] = DHT_NONE;
        out_cnt[qi] = cnt;
    }
}

__global__ __launch_bounds__(256) void k_map_idx(uint32_t* __restrict__ idx, uint64_t m,
                                                 const uint32_t* __restrict__ gidx, uint32_t base) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < m && idx[i] != DHT_NONE) idx[i] = gidx ? gidx[idx[i]] : idx[i] + base;
}

// candidate records {w0..w4, global idx} of local indices.  aos (nullable): the set's ids as 24-B
// records (k_pack_aos), one 24-B read per candidate instead of five 4-B reads from the planes
// (each its own 64-B sector: the planes gather of 65,536 x 8 records took 62 us on a 2^24 set)
__global__ __launch_bounds__(256) void k_rec_from_idx(const uint32_t* __restrict__ idx, uint64_t m,
                                                      const uint32_t* __restrict__ planes,
                                                      uint64_t stride, uint32_t base,
                                                      const uint32_t* __restrict__ gidx,
                                                      const uint2* __restrict__ aos,
                                                      uint32_t* __restrict__ rec) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    const uint32_t x = idx[i];
    const bool none = x == DHT_NONE;
    uint2* out = reinterpret_cast<uint2*>(rec + i * 6);
    if (aos) {
        const uint2* a = aos + (uint64_t)(none ? 0u : x) * 3;
        const uint2 r0 = a[0], r1 = a[1], r2 = a[2];
        out[0] = none ? make_uint2(DHT_NONE, DHT_NONE) : r0;
        out[1] = none ? make_uint2(DHT_NONE, DHT_NONE) : r1;
        out[2] = make_uint2(none ? DHT_NONE : r2.x, none ? DHT_NONE : (gidx ? gidx[x] : x + base));
        return;
    }
#pragma unroll
    for (int w = 0; w < DHT_W; ++w) rec[i * 6 + w] = none ? DHT_NONE : planes[(uint64_t)w * stride + x];
    rec[i * 6 + 5] = none ? DHT_NONE : (gidx ? gidx[x] : x + base);
}

// the id set as 24-B records {w0..w4, 0} (built once per set for record-mode calls)
__global__ __launch_bounds__(256) void k_pack_aos(const uint32_t* __restrict__ planes, uint64_t stride, uint64_t n,
                                                  uint2* __restrict__ aos) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint2* o = aos + i * 3;
    o[0] = make_uint2(planes[i], planes[stride + i]);
    o[1] = make_uint2(planes[2 * stride + i], planes[3 * stride + i]);
    o[2] = make_uint2(planes[4 * stride + i], 0u);
}

template <uint32_t K>
hipError_t launch_scan_k(const uint32_t* ids, uint64_t is, uint64_t n, const ScanPlan& p,
                         const uint32_t* tp, uint64_t ts, uint32_t q, uint32_t k,
                         uint32_t* out_idx, uint32_t* out_cnt, uint32_t* out_rec,
                         const uint32_t* gidx, uint32_t idx_base, hipStream_t s) {
    dim3 grid(p.blocks_x, p.splits);
    k_scan<K, kScanTargets><<<grid, WAVES * 64, 0, s>>>(ids, is, n, p.split_len, tp, ts, q, k,
                                                        out_idx, out_cnt, out_rec, gidx, idx_base);
    return hipGetLastError();
}

}  // namespace

ScanPlan plan_scan(uint64_t n, uint32_t q, uint32_t k, int num_cus) {
    ScanPlan p;
    const uint32_t per_block = WAVES * kScanTargets;
    p.blocks_x = (q + per_block - 1) / per_block;
    const uint64_t ntiles = (n + TILE - 1) / TILE;
    // aim for >= 2 workgroups per CU; never split below one tile per workgroup
    const uint64_t want = (uint64_t)(num_cus > 0 ? num_cus : 256) * 2;
    uint64_t splits = (want + p.blocks_x - 1) / p.blocks_x;
    if (splits > ntiles) splits = ntiles ? ntiles : 1;
    // K3 stages every split's k records of a target in LDS (24 B each)
    const uint64_t kk = k ? k : 1, cap = kLdsBytes / (kk * 24);
    if (splits > cap) splits = cap;
    if (splits < 1) splits = 1;
    const uint64_t tiles_per = (ntiles + splits - 1) / splits;
    p.split_len = (tiles_per ? tiles_per : 1) * TILE;
    p.splits = (uint32_t)((n + p.split_len - 1) / p.split_len);
    if (p.splits == 0) p.splits = 1;
    return p;
}

hipError_t launch_scan(const uint32_t* ids, uint64_t is, uint64_t n, const ScanPlan& p,
                       const uint32_t* tp, uint64_t ts, uint32_t q, uint32_t k,
                       uint32_t* out_idx, uint32_t* out_cnt, uint32_t* out_rec,
                       const uint32_t* gidx, uint32_t idx_base, hipStream_t s) {
    if (k <= 8) return launch_scan_k<8>(ids, is, n, p, tp, ts, q, k, out_idx, out_cnt, out_rec, gidx, idx_base, s);
    if (k <= 16) return launch_scan_k<16>(ids, is, n, p, tp, ts, q, k, out_idx, out_cnt, out_rec, gidx, idx_base, s);
    return launch_scan_k<32>(ids, is, n, p, tp, ts, q, k, out_idx, out_cnt, out_rec, gidx, idx_base, s);
}

hipError_t launch_map_idx(uint32_t* idx, uint64_t m, const uint32_t* gidx, uint32_t base, hipStream_t s) {
    if (!m || (!gidx && !base)) return hipSuccess;
    k_map_idx<<<(uint32_t)((m + 255) / 256), 256, 0, s>>>(idx, m, gidx, base);
    return hipGetLastError();
}

hipError_t launch_rec_from_idx(const uint32_t* idx, uint64_t m, const uint32_t* planes,
                               uint64_t stride, uint32_t base, const uint32_t* gidx, uint32_t* rec,
                               hipStream_t s, const uint32_t* aos) {
    if (!m) return hipSuccess;
    k_rec_from_idx<<<(uint32_t)((m + 255) / 256), 256, 0, s>>>(idx, m, planes, stride, base, gidx,
                                                               reinterpret_cast<const uint2*>(aos), rec);
    return hipGetLastError();
}

hipError_t launch_pack_aos(const uint32_t* planes, uint64_t stride, uint64_t n, uint32_t* aos, hipStream_t s) {
    if (!n) return hipSuccess;
    k_pack_aos<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(planes, stride, n, reinterpret_cast<uint2*>(aos));
    return hipGetLastError();
}

hipError_t launch_merge(const uint32_t* rec, uint32_t lists, uint32_t q, uint32_t kin,
                        const uint32_t* tp, uint64_t ts, uint32_t k, uint32_t* out_idx,
                        uint32_t* out_cnt, hipStream_t s) {
    if (lists <= 64 && kin <= 32) {   // the heads merge (sorted lists)
        uint32_t G = 1;
        while (G < lists) G <<= 1;
        const uint32_t tpb = (kMergeThreads / 64) * (64 / G);
        const dim3 grid((q + tpb - 1) / tpb), blk(kMergeThreads);
        const size_t lds = (size_t)kMergeThreads * kin * 3 * sizeof(uint32_t);
        static std::once_flag once[kMaxDevices];
        const hipError_t e = per_device_once(once, [] {
            const void* fs[] = {(const void*)k_merge_heads<1>, (const void*)k_merge_heads<2>, (const void*)k_merge_heads<4>,
                                (const void*)k_merge_heads<8>, (const void*)k_merge_heads<16>, (const void*)k_merge_heads<32>,
                                (const void*)k_merge_heads<64>};
            for (const void* f : fs) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
        });
        if (e != hipSuccess) return e;
        switch (G) {
            case 1: k_merge_heads<1><<<grid, blk, lds, s>>>(rec, lists, q, kin, tp, ts, k, out_idx, out_cnt); break;
            case 2: k_merge_heads<2><<<grid, blk, lds, s>>>(rec, lists, q, kin, tp, ts, k, out_idx, out_cnt); break;
            case 4: k_merge_heads<4><<<grid, blk, lds, s>>>(rec, lists, q, kin, tp, ts, k, out_idx, out_cnt); break;
            case 8: k_merge_heads<8><<<grid, blk, lds, s>>>(rec, lists, q, kin, tp, ts, k, out_idx, out_cnt); break;
            case 16: k_merge_heads<16><<<grid, blk, lds, s>>>(rec, lists, q, kin, tp, ts, k, out_idx, out_cnt); break;
            case 32: k_merge_heads<32><<<grid, blk, lds, s>>>(rec, lists, q, kin, tp, ts, k, out_idx, out_cnt); break;
            default: k_merge_heads<64><<<grid, blk, lds, s>>>(rec, lists, q, kin, tp, ts, k, out_idx, out_cnt); break;
        }
        return hipGetLastError();
    }
    // many lists (the K1 scan's id-range splits at tiny k): the pairwise rank
    const size_t lds = (size_t)lists * kin * 6 * sizeof(uint32_t);
    if (lds > kLdsBytes) return hipErrorInvalidValue;
    k_merge<<<q, 64, lds, s>>>(rec, lists, q, kin, tp, ts, k, out_idx, out_cnt);
    return hipGetLastError();
}

}  // namespace dhtgpu
