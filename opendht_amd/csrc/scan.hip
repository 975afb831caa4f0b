// scan.hip -- K1 xor_topk_scan and K3 topk_merge for gfx950.
//
// K1 restates std::partial_sort(ids, ids+k, ids+n, [t](a,b){ return t.xorCmp(a,b) < 0; })
// (InfoHash::xorCmp, include/opendht/infohash.h:179-194) for a batch of
// targets.  Design (integer compare-select; MFMA deliberately unused):
//   * ids are streamed as the w0 word plane (4 B/id) through a double-buffered LDS
//     tile shared by the 8 waves of a workgroup; each lane reads 16 ids per chunk with
//     4 conflict-free ds_read_b128;
//   * each wave owns kScanTargets targets whose w0 word and current k-th distance
//     (threshold) are wave-uniform (SGPRs); per (id, target) pair the hot loop costs a
//     v_xor_b32 plus half a v_min3_u32 (1.5 VALU ops), and one compare per target per
//     16-id chunk decides whether any lane holds a candidate;
//   * the exact top-k of each target is register-resident and lane-distributed (lane r
//     holds rank r as {w0 distance, id index}) and is updated by ballot + shuffle
//     insertion; ties on the w0 distance are resolved by a full 160-bit compare that
//     reads the remaining planes (rare: < 1 in 10^3 insertions at N = 2^24);
//   * when the batch has too few targets to fill the chip the id range is split across
//     workgroups and the per-split lists are merged by K3.
#include "dhtgpu_dev.h"
#include "dhtgpu_internal.h"

namespace dhtgpu {
namespace {

constexpr uint32_t WAVES = kScanWaves;
constexpr uint32_t TILE = kTile;
constexpr uint32_t CHUNK = 2048;       // ids per chunk per wave (32 per lane, 16 packed words)

// Is the (w0-distance-equal) entry `ei` closer to the target than candidate `ci`?
// Full compare on words 1..4, then index (ties only for duplicated ids).
__device__ __forceinline__ bool entry_closer_full(const uint32_t* __restrict__ ids, uint64_t is,
                                               uint32_t ei, uint32_t ci,
                                               const uint32_t* __restrict__ tp, uint64_t ts,
                                               uint32_t qi) {
    uint32_t a[DHT_W], b[DHT_W], t[DHT_W];
    load_id(ids, is, ei, a);
    load_id(ids, is, ci, b);
    load_id(tp, ts, qi, t);
    return xor_less_from(a, ei, b, ci, t, 1);
}

// Number of filled slots of a lane-distributed list (entries are filled front to back).
template <uint32_t K>
__device__ __forceinline__ uint32_t list_count(uint32_t ei, uint32_t lane) {
    return (uint32_t)__popcll(__ballot(lane < K && ei != DHT_NONE));
}

// Insert candidate (cd = w0 distance, ci = id index) into the lane-distributed sorted
// list {ed, ei} (lane r holds rank r).  thr (wave-uniform) becomes the K-th w0 distance
// once the list is full.  Returns the new list length.
template <uint32_t K>
__device__ __forceinline__ uint32_t topk_insert(uint32_t& ed, uint32_t& ei, uint32_t& thr,
                                                uint32_t cd, uint32_t ci, uint32_t lane,
                                                const uint32_t* __restrict__ ids, uint64_t is,
                                                const uint32_t* __restrict__ tp, uint64_t ts,
                                                uint32_t qi) {
    const uint32_t cnt = list_count<K>(ei, lane);
    const bool valid = lane < cnt;
    bool closer = valid && ed < cd;
    if (valid && ed == cd) closer = entry_closer_full(ids, is, ei, ci, tp, ts, qi);
    const uint32_t pos = (uint32_t)__popcll(__ballot(closer));
    if (pos >= K) return cnt;
    const uint32_t ud = __shfl_up(ed, 1), ui = __shfl_up(ei, 1);
    if (lane == pos) {
        ed = cd;
        ei = ci;
    } else if (lane > pos) {
        ed = ud;
        ei = ui;
    }
    const uint32_t ncnt = cnt + 1 < K ? cnt + 1 : K;
    thr = ncnt == K ? (uint32_t)__builtin_amdgcn_readlane((int)ed, K - 1) : DHT_NONE;
    return ncnt;
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// Hide a wave-uniform value from loop-invariant code motion, so per-target slow-path
// addresses are formed where they are used instead of being hoisted into SGPRs.
__device__ __forceinline__ uint32_t opaque(uint32_t x) {
    asm volatile("" : "+s"(x));
    return x;
}

// two packed u16 lanes: elementwise min (v_pk_min_u16)
__device__ __forceinline__ uint32_t pk_min(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a),
                                                                  __builtin_bit_cast(u16x2, b)));
}
// both halves <- min(lo, hi) (v_pk_min_u16 with op_sel half swap)
__device__ __forceinline__ uint32_t pk_min_halves(uint32_t a) {
    const u16x2 x = __builtin_bit_cast(u16x2, a);
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(x, __builtin_shufflevector(x, x, 1, 0)));
}

// LDS tile image (per buffer): w0[TILE] u32 followed by p16[TILE/2] u32, where p16 word m
// packs the top 16 bits of ids 2m (low half) and 2m+1 (high half).
constexpr uint32_t TILE_WORDS = TILE + TILE / 2;

template <uint32_t K, uint32_t T>
__global__ __launch_bounds__(WAVES * 64, 4) void k_scan(
    const uint32_t* __restrict__ ids, uint64_t is, uint64_t n, uint64_t split_len,
    const uint32_t* __restrict__ tp, uint64_t ts, uint32_t q, uint32_t k,
    uint32_t* __restrict__ out_idx, uint32_t* __restrict__ out_cnt, uint32_t* __restrict__ out_rec,
    uint32_t idx_base) {
    // [tile buffer 0 | tile buffer 1 | per-wave target w0 words]
    __shared__ __attribute__((aligned(16))) uint32_t lds[2 * TILE_WORDS + WAVES * T];

    const uint32_t lane = lane_id();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t id_begin = (uint64_t)blockIdx.y * split_len;
    const uint64_t id_end = n < id_begin + split_len ? n : id_begin + split_len;
    const uint32_t qbase = (blockIdx.x * WAVES + wave) * T;

    // wave-uniform per-target state: packed top-16 target, exact w0 threshold, count
    // st[j] = (top 16 bits of target w0) << 16 | (top 16 bits of the K-th w0 distance);
    // one SGPR per target keeps the hot loop free of SGPR spills.  The exact 32-bit
    // threshold is rebuilt from the register list (lane K-1) in the slow path.
    uint32_t st[T], ed[T], ei[T];
    uint32_t full = 0;   // bit j: target j's list holds K entries
    uint32_t* const twords = lds + 2 * TILE_WORDS + wave * T;
    if (lane < T) twords[lane] = tp[qbase + lane < q ? qbase + lane : q - 1];
#pragma unroll
    for (uint32_t j = 0; j < T; ++j) {
        const uint32_t qi = qbase + j < q ? qbase + j : q - 1;
        const uint32_t tw = __builtin_amdgcn_readfirstlane(tp[qi]);
        st[j] = (tw & 0xFFFF0000u) | 0xFFFFu;
        ed[j] = DHT_NONE;
        ei[j] = DHT_NONE;
    }

    const uint64_t ntiles = id_end > id_begin ? (id_end - id_begin + TILE - 1) / TILE : 0;
    // staging: thread h loads ids [4h, 4h+4) and [4(h+512), ...) of the tile's w0 plane
    uint4 pf0 = make_uint4(0, 0, 0, 0), pf1 = pf0;
    auto stage = [&](uint32_t* buf) {
        reinterpret_cast<uint4*>(buf)[threadIdx.x] = pf0;
        reinterpret_cast<uint4*>(buf)[threadIdx.x + WAVES * 64] = pf1;
        uint2* p16 = reinterpret_cast<uint2*>(buf + TILE);
        p16[threadIdx.x] = make_uint2((pf0.y & 0xFFFF0000u) | (pf0.x >> 16), (pf0.w & 0xFFFF0000u) | (pf0.z >> 16));
        p16[threadIdx.x + WAVES * 64] =
            make_uint2((pf1.y & 0xFFFF0000u) | (pf1.x >> 16), (pf1.w & 0xFFFF0000u) | (pf1.z >> 16));
    };
    if (ntiles) {
        const uint4* src = reinterpret_cast<const uint4*>(ids + id_begin);
        pf0 = src[threadIdx.x];
        pf1 = src[threadIdx.x + WAVES * 64];
        stage(lds);
    }
    __syncthreads();

    for (uint64_t t = 0; t < ntiles; ++t) {
        const uint64_t tb = id_begin + t * TILE;
        if (t + 1 < ntiles) {
            const uint4* src = reinterpret_cast<const uint4*>(ids + tb + TILE);
            pf0 = src[threadIdx.x];
            pf1 = src[threadIdx.x + WAVES * 64];
        }
        const uint32_t* bufw = lds + (t & 1) * TILE_WORDS;          // w0 words
        const uint4* bufp = reinterpret_cast<const uint4*>(bufw + TILE);  // packed top-16 words

#pragma unroll 1
        for (uint32_t c = 0; c < TILE / CHUNK; ++c) {
            // lane l holds ids c*CHUNK + r*512 + 8l + {0..7}, r = 0..3, as 16 packed words
            uint32_t x[16];
#pragma unroll
            for (uint32_t r = 0; r < 4; ++r) {
                const uint4 v = bufp[c * (CHUNK / 8) + r * 64 + lane];
                x[4 * r + 0] = v.x;
                x[4 * r + 1] = v.y;
                x[4 * r + 2] = v.z;
                x[4 * r + 3] = v.w;
            }
            const uint64_t cbase = tb + c * CHUNK;
            const uint64_t left = id_end > cbase ? id_end - cbase : 0;
            const uint32_t rem = left < CHUNK ? (uint32_t)left : CHUNK;

#pragma unroll
            for (uint32_t j = 0; j < T; ++j) {
                // hot loop: 1 v_xor_b32 + 1 v_pk_min_u16 per two (id, target) pairs
                const uint32_t tj = opaque((st[j] & 0xFFFF0000u) | (st[j] >> 16));   // t16 in both halves (SGPR)
                uint32_t a = x[0] ^ tj;
#pragma unroll
                for (uint32_t s = 1; s < 16; ++s) a = pk_min(a, x[s] ^ tj);
                a = pk_min_halves(a);
                // a = (m << 16) | m with m the lane's min top-16 distance; pass iff m <= thr >> 16
                const uint64_t lm = __ballot(a <= ((st[j] << 16) | 0xFFFFu));
                if (lm && ((full >> j) & 1u)) {
                    uint32_t thr = (uint32_t)__builtin_amdgcn_readlane((int)ed[j], K - 1);
                    // steady state (rare; mostly 16-bit false positives): for each flagged
                    // lane L, lanes 0..31 check L's 32 ids with the exact w0 word from LDS
                    const uint32_t qj = opaque(qbase) + j;
                    const uint32_t qi = qj < q ? qj : q - 1;
                    const uint32_t t0 = __builtin_amdgcn_readfirstlane(twords[j]);
                    uint64_t fl = lm;
                    while (fl) {
                        const uint32_t L = (uint32_t)__ffsll((long long)fl) - 1;
                        fl &= fl - 1;
                        const uint32_t sl = lane & 31;
                        const uint32_t off = (sl >> 3) * 512 + 8 * L + (sl & 7);
                        const uint32_t d = bufw[c * CHUNK + off] ^ t0;
                        uint64_t cm = __ballot(lane < 32 && off < rem && d <= thr);
                        while (cm) {
                            const uint32_t i = (uint32_t)__ffsll((long long)cm) - 1;
                            cm &= cm - 1;
                            const uint32_t cd = (uint32_t)__builtin_amdgcn_readlane((int)d, i);
                            if (cd <= thr) {
                                const uint32_t coff = (i >> 3) * 512 + 8 * L + (i & 7);
                                topk_insert<K>(ed[j], ei[j], thr, cd, (uint32_t)(cbase + coff),
                                               lane, ids, is, tp, ts, qi);
                            }
                        }
                    }
                    st[j] = (st[j] & 0xFFFF0000u) | (thr >> 16);
                } else if (lm) {
                    // warm-up (list not yet full): exact w0 compare of every slot, then
                    // serial insertion bounded by a bisection threshold
                    const uint32_t qj = opaque(qbase) + j;
                    const uint32_t qi = qj < q ? qj : q - 1;
                    const uint32_t t0 = __builtin_amdgcn_readfirstlane(twords[j]);
                    // the lane's 8 w0 distances of row r (ids c*CHUNK + r*512 + 8*lane + e)
                    auto row = [&](uint32_t r, uint32_t* d) {
                        const uint4 u0 = *reinterpret_cast<const uint4*>(bufw + c * CHUNK + r * 512 + 8 * lane);
                        const uint4 u1 = *reinterpret_cast<const uint4*>(bufw + c * CHUNK + r * 512 + 8 * lane + 4);
                        d[0] = u0.x ^ t0; d[1] = u0.y ^ t0; d[2] = u0.z ^ t0; d[3] = u0.w ^ t0;
                        d[4] = u1.x ^ t0; d[5] = u1.y ^ t0; d[6] = u1.z ^ t0; d[7] = u1.w ^ t0;
                    };
                    uint32_t thr = DHT_NONE;
                    uint32_t lim = DHT_NONE;
                    {
                        // Warm-up: the K-th smallest per-lane minimum v* bounds the K-th
                        // smallest distance of the chunk (K ids lie at or below it), so
                        // ids above v* cannot enter the top-K; find v* by bisection.
                        uint32_t av = DHT_NONE;
#pragma unroll 1
                        for (uint32_t r = 0; r < 4; ++r) {
                            uint32_t d[8];
                            row(r, d);
#pragma unroll
                            for (uint32_t e = 0; e < 8; ++e)
                                if (r * 512 + 8 * lane + e < rem) av = min(av, d[e]);
                        }
                        const bool has = 8 * lane < rem;
                        if ((uint32_t)__popcll(__ballot(has)) >= K) {
                            uint32_t v = 0;
                            for (int bit = 31; bit >= 0; --bit) {
                                const uint32_t tryv = v | ((1u << bit) - 1u);
                                if ((uint32_t)__popcll(__ballot(has && av <= tryv)) < K) v |= 1u << bit;
                            }
                            lim = min(lim, v);
                        }
                    }
                    uint32_t bits = 0;
#pragma unroll 1
                    for (uint32_t r = 0; r < 4; ++r) {
                        uint32_t d[8];
                        row(r, d);
#pragma unroll
                        for (uint32_t e = 0; e < 8; ++e)
                            bits |= (uint32_t)((d[e] <= lim) && r * 512 + 8 * lane + e < rem) << (8 * r + e);
                    }
                    for (;;) {
                        const uint64_t m = __ballot(bits != 0);
                        if (!m) break;
                        const uint32_t L = (uint32_t)__ffsll((long long)m) - 1;
                        const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)bits, L);
                        const uint32_t s = (uint32_t)__ffs(b) - 1;
                        if (lane == L) bits &= bits - 1;
                        const uint32_t off = (s >> 3) * 512 + 8 * L + (s & 7);
                        const uint32_t cd = bufw[c * CHUNK + off] ^ t0;
                        if (cd <= thr &&
                            topk_insert<K>(ed[j], ei[j], thr, cd, (uint32_t)(cbase + off), lane, ids,
                                           is, tp, ts, qi) == K)
                            full |= 1u << j;
                    }
                    st[j] = (st[j] & 0xFFFF0000u) | (thr >> 16);
                }
            }
        }
        if (t + 1 < ntiles) stage(lds + ((t + 1) & 1) * TILE_WORDS);
        __syncthreads();
    }

    // write results
#pragma unroll
    for (uint32_t j = 0; j < T; ++j) {
        const uint32_t qi = qbase + j;
        if (qi >= q) continue;
        const uint32_t cntj = list_count<K>(ei[j], lane);
        if (out_rec) {
            if (lane < k) {
                uint32_t* r = out_rec + (((uint64_t)blockIdx.y * q + qi) * k + lane) * 6;
                if (lane < cntj) {
#pragma unroll
                    for (int w = 0; w < DHT_W; ++w) r[w] = ids[(uint64_t)w * is + ei[j]];
                    r[5] = ei[j] + idx_base;
                } else {
#pragma unroll
                    for (int w = 0; w < 6; ++w) r[w] = DHT_NONE;
                }
            }
        } else {
            if (lane < k) out_idx[(uint64_t)qi * k + lane] = lane < cntj ? ei[j] + idx_base : DHT_NONE;
            if (lane == 0) out_cnt[qi] = cntj < k ? cntj : k;
        }
    }
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
                         uint32_t idx_base, hipStream_t s) {
    dim3 grid(p.blocks_x, p.splits);
    k_scan<K, kScanTargets><<<grid, WAVES * 64, 0, s>>>(ids, is, n, p.split_len, tp, ts, q, k,
                                                        out_idx, out_cnt, out_rec, idx_base);
    return hipGetLastError();
}

}  // namespace

ScanPlan plan_scan(uint64_t n, uint32_t q, int num_cus) {
    ScanPlan p;
    const uint32_t per_block = WAVES * kScanTargets;
    p.blocks_x = (q + per_block - 1) / per_block;
    const uint64_t ntiles = (n + TILE - 1) / TILE;
    // aim for >= 2 workgroups per CU; never split below one tile per workgroup
    const uint64_t want = (uint64_t)(num_cus > 0 ? num_cus : 256) * 2;
    uint64_t splits = (want + p.blocks_x - 1) / p.blocks_x;
    if (splits > ntiles) splits = ntiles ? ntiles : 1;
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
                       uint32_t idx_base, hipStream_t s) {
    if (k <= 8) return launch_scan_k<8>(ids, is, n, p, tp, ts, q, k, out_idx, out_cnt, out_rec, idx_base, s);
    if (k <= 16) return launch_scan_k<16>(ids, is, n, p, tp, ts, q, k, out_idx, out_cnt, out_rec, idx_base, s);
    return launch_scan_k<32>(ids, is, n, p, tp, ts, q, k, out_idx, out_cnt, out_rec, idx_base, s);
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
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    k_merge<<<q, 64, lds, s>>>(rec, lists, q, kin, tp, ts, k, out_idx, out_cnt);
    return hipGetLastError();
}

}  // namespace dhtgpu
