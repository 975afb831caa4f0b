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

__global__ __launch_bounds__(256) void k_map_idx(uint32_t* __restrict__ idx, uint64_t m,
                                                 const uint32_t* __restrict__ gidx, uint32_t base) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < m && idx[i] != DHT_NONE) idx[i] = gidx ? gidx[idx[i]] : idx[i] + base;
}

__global__ __launch_bounds__(256) void k_rec_from_idx(const uint32_t* __restrict__ idx, uint64_t m,
                                                      const uint32_t* __restrict__ planes,
                                                      uint64_t stride, uint32_t base,
                                                      const uint32_t* __restrict__ gidx,
                                                      uint32_t* __restrict__ rec) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    const uint32_t x = idx[i];
#pragma unroll
    for (int w = 0; w < DHT_W; ++w) rec[i * 6 + w] = x == DHT_NONE ? DHT_NONE : planes[(uint64_t)w * stride + x];
    rec[i * 6 + 5] = x == DHT_NONE ? DHT_NONE : (gidx ? gidx[x] : x + base);
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
                               hipStream_t s) {
    if (!m) return hipSuccess;
    k_rec_from_idx<<<(uint32_t)((m + 255) / 256), 256, 0, s>>>(idx, m, planes, stride, base, gidx, rec);
    return hipGetLastError();
}

hipError_t launch_merge(const uint32_t* rec, uint32_t lists, uint32_t q, uint32_t kin,
                        const uint32_t* tp, uint64_t ts, uint32_t k, uint32_t* out_idx,
                        uint32_t* out_cnt, hipStream_t s) {
    const size_t lds = (size_t)lists * kin * 6 * sizeof(uint32_t);
    if (lds > kLdsBytes) return hipErrorInvalidValue;
    k_merge<<<q, 64, lds, s>>>(rec, lists, q, kin, tp, ts, k, out_idx, out_cnt);
    return hipGetLastError();
}

}  // namespace dhtgpu
