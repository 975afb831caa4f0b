// scan_dev.h -- the K1 streaming-scan body (device code), shared by the plain K1 launch
// (scan.hip: one role per workgroup from blockIdx) and K6's fallback pass (batch.hip: roles
// sized at run time from a device-side target count).
//
// K1 restates std::partial_sort(ids, ids+k, ids+n, [t](a,b){ return t.xorCmp(a,b) < 0; })
// (InfoHash::xorCmp, include/opendht/infohash.h:179-194) for a batch of
// targets.  Design (integer compare-select; MFMA deliberately unused):
//   * ids are streamed as the w0 word plane (4 B/id) through a double-buffered LDS tile
//     shared by the 8 waves of a workgroup; each lane reads 16 packed words per chunk with
//     4 conflict-free ds_read_b128;
//   * each wave owns kScanTargets targets whose w0 word and current k-th distance
//     (threshold) are wave-uniform (SGPRs); per (id, target) pair the hot loop costs a
//     v_xor_b32 plus half a v_pk_min_u16, and one compare per target per 32-id lane chunk
//     decides whether any lane holds a candidate;
//   * the exact top-k of each target is register-resident and lane-distributed (lane r
//     holds rank r as {w0 distance, id index}) and is updated by ballot + shuffle
//     insertion; ties on the w0 distance are resolved by a full 160-bit compare that reads
//     the remaining planes (rare: < 1 in 10^3 insertions at N = 2^24).
#pragma once
#include "dhtgpu_dev.h"
#include "dhtgpu_internal.h"

namespace dhtgpu {
namespace scan {

constexpr uint32_t WAVES = kScanWaves;
constexpr uint32_t TILE = kTile;
constexpr uint32_t CHUNK = 2048;   // ids per chunk per wave (32 per lane, 16 packed words)
// LDS tile image (per buffer): w0[TILE] u32 followed by p16[TILE/2] u32, where p16 word m
// packs the top 16 bits of ids 2m (low half) and 2m+1 (high half).
constexpr uint32_t TILE_WORDS = TILE + TILE / 2;
// workgroup LDS: two tile buffers, then per wave T target w0 words and T target indices
template <uint32_t T>
constexpr uint32_t lds_words() { return 2 * TILE_WORDS + 2 * WAVES * T; }

// Is the (w0-distance-equal) entry `ei` closer to the target than candidate `ci`?
// Full compare on words 1..4, then index (ties only for duplicated ids).
__device__ __forceinline__ bool entry_closer_full(const uint32_t* __restrict__ ids, uint64_t is, uint32_t ei,
                                                  uint32_t ci, const uint32_t* __restrict__ tp, uint64_t ts,
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

// Insert candidate (cd = w0 distance, ci = id index) into the lane-distributed sorted list
// {ed, ei} (lane r holds rank r).  thr (wave-uniform) becomes the K-th w0 distance once the
// list is full.  Returns the new list length.
template <uint32_t K>
__device__ __forceinline__ uint32_t topk_insert(uint32_t& ed, uint32_t& ei, uint32_t& thr, uint32_t cd, uint32_t ci,
                                                uint32_t lane, const uint32_t* __restrict__ ids, uint64_t is,
                                                const uint32_t* __restrict__ tp, uint64_t ts, uint32_t qi) {
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

// record store that is visible to another workgroup of the same launch once the storing
// wave's vmcnt is drained (sc1: written through to the memory side, MI355X_MICROARCH
// "inter-workgroup visibility")
__device__ __forceinline__ void store_sc1(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Where one role of the scan writes its results.
struct ScanOut {
    uint32_t* out_idx;        // final form: out_idx[qr * k + r] (mapped), out_cnt[qr]
    uint32_t* out_cnt;
    const uint32_t* gidx;     // final form: index map (nullable) ...
    uint32_t base;            // ... or offset
    uint32_t* rec;            // record form (non-null): rec[((rec_base + qc) * k + r) * 6 + {w0..w4, idx + rec_idx_base}]
    uint64_t rec_base;
    uint32_t rec_idx_base;
};

// One role: the workgroup's WAVES x T targets (wave w owns compact targets qbase_w + j,
// j < T, of q; compact target qc is target tlist[qc] of the planes tp, or qc itself when
// tlist is null) against ids [id_begin, id_end).  Every thread of the workgroup calls it.
template <uint32_t K, uint32_t T>
__device__ void scan_run(uint32_t* lds, const uint32_t* __restrict__ ids, uint64_t is, uint64_t id_begin,
                         uint64_t id_end, const uint32_t* __restrict__ tp, uint64_t ts,
                         const uint32_t* __restrict__ tlist, uint32_t qbase, uint32_t q, uint32_t k,
                         const ScanOut& o) {
    const uint32_t lane = lane_id();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    qbase = __builtin_amdgcn_readfirstlane(qbase);   // wave-uniform by contract
    q = __builtin_amdgcn_readfirstlane(q);
    // targets of this wave actually present (wave-uniform; the others are skipped)
    const uint32_t nv = q > qbase ? (q - qbase < T ? q - qbase : T) : 0u;

    // wave-uniform per-target state: packed top-16 target, exact w0 threshold, count
    // st[j] = (top 16 bits of target w0) << 16 | (top 16 bits of the K-th w0 distance);
    // one SGPR per target keeps the hot loop free of SGPR spills.  The exact 32-bit
    // threshold is rebuilt from the register list (lane K-1) in the slow path.
    uint32_t st[T], ed[T], ei[T];
    uint32_t full = 0;   // bit j: target j's list holds K entries
    uint32_t* const twords = lds + 2 * TILE_WORDS + wave * T;
    uint32_t* const treal = lds + 2 * TILE_WORDS + WAVES * T + wave * T;
    if (lane < T && nv) {
        const uint32_t qc = qbase + (lane < nv ? lane : nv - 1);
        const uint32_t qr = tlist ? tlist[qc] : qc;
        treal[lane] = qr;
        twords[lane] = tp[qr];
    }
    // the wave's own LDS words: visible to its lanes after the workgroup barrier below
#pragma unroll
    for (uint32_t j = 0; j < T; ++j) {
        st[j] = 0xFFFFu;
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
#pragma unroll
    for (uint32_t j = 0; j < T; ++j) {
        const uint32_t tw = __builtin_amdgcn_readfirstlane(twords[j < nv ? j : 0]);
        st[j] = (tw & 0xFFFF0000u) | 0xFFFFu;
    }

    for (uint64_t t = 0; t < ntiles; ++t) {
        const uint64_t tb = id_begin + t * TILE;
        if (t + 1 < ntiles) {
            const uint4* src = reinterpret_cast<const uint4*>(ids + tb + TILE);
            pf0 = src[threadIdx.x];
            pf1 = src[threadIdx.x + WAVES * 64];
        }
        const uint32_t* bufw = lds + (t & 1) * TILE_WORDS;                 // w0 words
        const uint4* bufp = reinterpret_cast<const uint4*>(bufw + TILE);   // packed top-16 words

#pragma unroll 1
        for (uint32_t c = 0; c < TILE / CHUNK; ++c) {
            if (!nv) break;
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
                if (j >= nv) continue;   // wave-uniform
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
                    const uint32_t qi = __builtin_amdgcn_readfirstlane(treal[opaque(j)]);
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
                                topk_insert<K>(ed[j], ei[j], thr, cd, (uint32_t)(cbase + coff), lane, ids, is, tp,
                                               ts, qi);
                            }
                        }
                    }
                    st[j] = (st[j] & 0xFFFF0000u) | (thr >> 16);
                } else if (lm) {
                    // warm-up (list not yet full): exact w0 compare of every slot, then
                    // serial insertion bounded by a bisection threshold
                    const uint32_t qi = __builtin_amdgcn_readfirstlane(treal[opaque(j)]);
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
                            topk_insert<K>(ed[j], ei[j], thr, cd, (uint32_t)(cbase + off), lane, ids, is, tp, ts,
                                           qi) == K)
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
        if (j >= nv) continue;
        const uint32_t qc = qbase + j;
        const uint32_t cntj = list_count<K>(ei[j], lane);
        if (o.rec) {
            if (lane < k) {
                uint32_t* r = o.rec + ((o.rec_base + qc) * k + lane) * 6;
                if (lane < cntj) {
#pragma unroll
                    for (int w = 0; w < DHT_W; ++w) store_sc1(r + w, ids[(uint64_t)w * is + ei[j]]);
                    store_sc1(r + 5, ei[j] + o.rec_idx_base);
                } else {
#pragma unroll
                    for (int w = 0; w < 6; ++w) store_sc1(r + w, DHT_NONE);
                }
            }
        } else {
            const uint32_t qr = __builtin_amdgcn_readfirstlane(treal[j]);
            if (lane < k) {
                uint32_t v = DHT_NONE;
                if (lane < cntj) v = o.gidx ? o.gidx[ei[j]] : ei[j] + o.base;
                o.out_idx[(uint64_t)qr * k + lane] = v;
            }
            if (lane == 0) o.out_cnt[qr] = cntj < k ? cntj : k;
        }
    }
    __syncthreads();   // the tile buffers and target words are reused by the caller's next role
}

}  // namespace scan
}  // namespace dhtgpu
