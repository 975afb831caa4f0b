// batch.hip -- K6: per-batch target-prefix filter + exact XOR top-k (gfx950).
//
// Same results as K1 / K4+K5: for every target the k ids closest by XOR distance,
// ascending -- std::partial_sort over InfoHash::xorCmp (include/opendht/infohash.h:179-194,
// SURVEY §8 a12), equal ids tie-broken by lower index.  Nothing persists between calls:
// every call reads the raw id planes once and answers the batch.
//
// Why it is exact.  Let sub(t, l) be the ids whose first l bits equal the target's.
// Every id inside sub(t, l) agrees with t on bits [0, l) and every id outside differs at
// some bit < l, so every id inside is XOR-closer than every id outside; hence if
// |sub(t, l)| >= k, the top-k of t lies inside sub(t, l).  K6 fixes one mark level Lm for
// the batch (about 4k ids per level-Lm subtree on uniform ids), and
//   F1  marks the level-Lm prefix of every target in a 2^Lm-bit bitmap and partitions
//       the targets by their top b1 bits (b1 <= Lm);
//   F2  streams the id word plane w0 once (4 B/id); an id survives iff its level-Lm
//       prefix is marked -- i.e. it lies in sub(t, Lm) of some target.  Survivors are
//       partitioned by their top b1 bits into per-block runs (the block's ids stay in
//       registers between its histogram and its scatter);
//   F3  one workgroup per partition gathers the partition's survivor runs into LDS,
//       counting-sorts them by the remaining Lm - b1 prefix bits, and answers each of the
//       partition's targets from its subtree sub(t, Lm), which is complete in LDS: the
//       exact top-k of the subtree's candidates keyed by (w0 ^ t0, words 1..4 ^ t, idx);
//       words 1..4 are read from the planes only when two w0 distances tie.  A target
//       whose subtree holds fewer than min(k, n) ids (or whose partition overflows the
//       LDS stage -- strongly clustered ids) is appended to a fallback list;
//   F4  answers the fallback list by an exact brute-force pass over all ids (one
//       workgroup per target; on uniform ids the list is empty and F4 exits at once).
// F3 also clears the bitmap words it owns, so the bitmap is all-zero between calls.
//
// Algorithmic bytes per call: n * 4 (w0) + q * 4 (target w0) + survivors * 16 (written
// and re-read as {w0, idx}) + q * k * 4 (results).  On uniform ids the survivor fraction
// is 1 - exp(-q / 2^Lm) (12 % at the cfg-2 batch).
#include "dhtgpu_dev.h"
#include "dhtgpu_internal.h"

#include <cmath>

namespace dhtgpu {
namespace {

constexpr int kF1Threads = 256;
constexpr int kF1Per = 4;
constexpr uint32_t kF1Chunk = kF1Threads * kF1Per;   // targets per F1 block
constexpr int kF2Threads = 1024;
constexpr int kF2Per = 32;
constexpr uint32_t kF2Chunk = kF2Threads * kF2Per;   // ids per F2 block (kept in registers)
constexpr int kF3Threads = 1024;
constexpr uint32_t kF3Cap = 8192;                    // survivors per partition staged in LDS
constexpr int kF3Per = kF3Cap / kF3Threads;
constexpr int kF4Threads = 256;
constexpr uint32_t kMaxLm = 19;                      // 2^19-bit bitmap = 64 KB of LDS in F2
constexpr uint32_t kMaxSubBits = 11;                 // F3 sub-prefix histogram <= 2048 bins
constexpr uint32_t kMaxBlk2 = 8192;                  // F2 blocks (n <= 2^28)
constexpr uint32_t kMaxBlk1 = 4096;                  // F1 blocks (q <= 2^22)
constexpr uint32_t kLdsMax = 160 * 1024;

__device__ __forceinline__ uint32_t top_bits(uint32_t w, uint32_t b) { return b ? w >> (32 - b) : 0u; }

// Exclusive scan of a[0, len) in LDS by a block of NT threads; returns the total.  Every
// thread must call it.  wsum: NT / 64 + 1 words of LDS scratch.
template <int NT>
__device__ uint32_t scan_lds(uint32_t* a, uint32_t len, uint32_t* wsum) {
    constexpr int NW = NT / 64;
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    const uint32_t per = (len + NT - 1) / NT;
    const uint32_t b = threadIdx.x * per;
    const uint32_t e = b + per < len ? b + per : len;
    uint32_t s = 0;
    for (uint32_t i = b; i < e; ++i) s += a[i];
    uint32_t x = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    if (threadIdx.x < 64) {
        const uint32_t v = lane < (uint32_t)NW ? wsum[lane] : 0u;
        uint32_t xv = v;
#pragma unroll
        for (int o = 1; o < NW; o <<= 1) {
            const uint32_t y = __shfl_up(xv, o);
            if (lane >= (uint32_t)o) xv += y;
        }
        if (lane < (uint32_t)NW) wsum[lane] = xv - v;
        if (lane == (uint32_t)NW - 1) wsum[NW] = xv;
    }
    __syncthreads();
    uint32_t run = wsum[w] + x - s;
    for (uint32_t i = b; i < e; ++i) {
        const uint32_t v = a[i];
        a[i] = run;
        run += v;
    }
    const uint32_t total = wsum[NW];
    __syncthreads();
    return total;
}

// largest r in [0, len) with a[r] <= j (a ascending, a[0] = 0 <= j)
__device__ __forceinline__ uint32_t run_of(const uint32_t* a, uint32_t len, uint32_t j) {
    uint32_t lo = 0, hi = len;   // invariant a[lo] <= j, answer < hi
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] <= j) lo = mid;
        else hi = mid;
    }
    return lo;
}

// ---- F1: mark target prefixes, partition targets -----------------------------------
__global__ __launch_bounds__(kF1Threads) void k_f1_targets(const uint32_t* __restrict__ tw0, uint32_t q, uint32_t Lm,
                                                          uint32_t b1, uint32_t* __restrict__ bitmap,
                                                          uint32_t* __restrict__ tab1, uint32_t nblk1,
                                                          uint2* __restrict__ treg, uint32_t* __restrict__ fb_count) {
    extern __shared__ uint32_t sh[];   // hist[np + 1] | wsum
    const uint32_t np = 1u << b1;
    uint32_t* hist = sh;
    uint32_t* wsum = sh + np + 1;
    for (uint32_t i = threadIdx.x; i <= np; i += kF1Threads) hist[i] = 0;
    if (blockIdx.x == 0 && threadIdx.x < 2) fb_count[threadIdx.x] = 0;   // fallback count, survivor count
    __syncthreads();
    const uint32_t base = blockIdx.x * kF1Chunk;
    const uint32_t m = q - base < kF1Chunk ? q - base : kF1Chunk;
    uint32_t v[kF1Per], rk[kF1Per];
#pragma unroll
    for (int e = 0; e < kF1Per; ++e) {
        const uint32_t j = e * kF1Threads + threadIdx.x;
        if (j < m) {
            v[e] = tw0[base + j];
            const uint32_t pre = top_bits(v[e], Lm);
            atomicOr(bitmap + (pre >> 5), 1u << (pre & 31));
            rk[e] = atomicAdd(hist + top_bits(v[e], b1), 1u);
        }
    }
    __syncthreads();
    scan_lds<kF1Threads>(hist, np, wsum);
    hist[np] = m;   // written by every thread, same value
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < np; p += kF1Threads)
        tab1[(uint64_t)p * nblk1 + blockIdx.x] = (hist[p] << 16) | (hist[p + 1] - hist[p]);
#pragma unroll
    for (int e = 0; e < kF1Per; ++e) {
        const uint32_t j = e * kF1Threads + threadIdx.x;
        if (j < m) treg[base + hist[top_bits(v[e], b1)] + rk[e]] = make_uint2(v[e], base + j);
    }
}

// ---- F2: stream w0, keep ids in marked subtrees, partition them ----------------------
__global__ __launch_bounds__(kF2Threads) void k_f2_filter(const uint32_t* __restrict__ w0, uint64_t n, uint32_t Lm,
                                                         uint32_t b1, const uint32_t* __restrict__ bitmap,
                                                         uint32_t nwords, uint32_t* __restrict__ tab2,
                                                         uint32_t nblk2, uint2* __restrict__ ireg) {
    extern __shared__ uint32_t sh[];   // bm[nwords] | hist[np + 1] | wsum
    const uint32_t np = 1u << b1;
    uint32_t* bm = sh;
    uint32_t* hist = sh + nwords;
    uint32_t* wsum = hist + np + 1;
    const uint64_t base = (uint64_t)blockIdx.x * kF2Chunk;
    const uint32_t m = (uint32_t)(n - base < kF2Chunk ? n - base : kF2Chunk);
    // id loads first (16 B per lane, all in flight), then the bitmap copy
    uint32_t v[kF2Per];
#pragma unroll
    for (int e = 0; e < kF2Per / 4; ++e) {
        const uint32_t j = e * 4 * kF2Threads + 4 * threadIdx.x;
        if (j + 3 < m) {
            const uint4 x = *reinterpret_cast<const uint4*>(w0 + base + j);
            v[4 * e] = x.x; v[4 * e + 1] = x.y; v[4 * e + 2] = x.z; v[4 * e + 3] = x.w;
        } else {
#pragma unroll
            for (int f = 0; f < 4; ++f) v[4 * e + f] = j + f < m ? w0[base + j + f] : 0u;
        }
    }
    if ((nwords & 3) == 0) {
        for (uint32_t i = threadIdx.x * 4; i < nwords; i += kF2Threads * 4)
            *reinterpret_cast<uint4*>(bm + i) = *reinterpret_cast<const uint4*>(bitmap + i);
    } else {
        for (uint32_t i = threadIdx.x; i < nwords; i += kF2Threads) bm[i] = bitmap[i];
    }
    for (uint32_t i = threadIdx.x; i <= np; i += kF2Threads) hist[i] = 0;
    __syncthreads();
    uint32_t rk[kF2Per];
#pragma unroll
    for (int e = 0; e < kF2Per; ++e) {
        const uint32_t j = (e / 4) * 4 * kF2Threads + 4 * threadIdx.x + (e % 4);
        rk[e] = DHT_NONE;
        if (j < m) {
            const uint32_t pre = top_bits(v[e], Lm);
            if ((bm[pre >> 5] >> (pre & 31)) & 1u) rk[e] = atomicAdd(hist + top_bits(v[e], b1), 1u);
        }
    }
    __syncthreads();
    const uint32_t tot = scan_lds<kF2Threads>(hist, np, wsum);
    hist[np] = tot;
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < np; p += kF2Threads)
        tab2[(uint64_t)p * nblk2 + blockIdx.x] = (hist[p] << 16) | (hist[p + 1] - hist[p]);
#pragma unroll
    for (int e = 0; e < kF2Per; ++e) {
        if (rk[e] != DHT_NONE) {
            const uint32_t j = (e / 4) * 4 * kF2Threads + 4 * threadIdx.x + (e % 4);
            ireg[base + hist[top_bits(v[e], b1)] + rk[e]] = make_uint2(v[e], (uint32_t)(base + j));
        }
    }
}

// ---- candidate order ------------------------------------------------------------------
// full XOR order of ids ia, ib (local indices) whose w0 distances are da, db
__device__ __forceinline__ bool id_less(uint32_t da, uint32_t ia, uint32_t db, uint32_t ib,
                                        const uint32_t* __restrict__ planes, uint64_t stride, const uint32_t* t) {
    if (da != db) return da < db;
    if (ia == ib) return false;
    uint32_t wa[DHT_W], wb[DHT_W];
    load_id(planes, stride, ia, wa);
    load_id(planes, stride, ib, wb);
    return xor_less_from(wa, ia, wb, ib, t, 1);
}

__device__ __forceinline__ uint32_t map_out(uint32_t x, const uint32_t* __restrict__ gidx, uint32_t base) {
    return gidx ? gidx[x] : x + base;
}

__device__ __forceinline__ void load_target(const uint32_t* __restrict__ tp, uint64_t ts, uint32_t qi, uint32_t* t) {
#pragma unroll
    for (int j = 0; j < DHT_W; ++j) t[j] = __builtin_amdgcn_readfirstlane(tp[(uint64_t)j * ts + qi]);
}

// ---- F3: one workgroup per partition --------------------------------------------------
struct F3Args {
    const uint2* ireg; const uint32_t* tab2; uint32_t nblk2;
    const uint2* treg; const uint32_t* tab1; uint32_t nblk1;
    uint32_t Lm, b1;
    uint32_t* bitmap; uint32_t nwords;
    const uint32_t* planes; uint64_t stride; uint64_t n;
    const uint32_t* tp; uint64_t ts; uint32_t k;
    const uint32_t* gidx; uint32_t base;
    uint32_t* out_idx; uint32_t* out_cnt;
    uint32_t* fb_count; uint32_t* fb_list;   // fb_count[0] = fallback targets, fb_count[1] = survivors
};

__global__ __launch_bounds__(kF3Threads) void k_f3_answer(F3Args a) {
    extern __shared__ uint32_t sh[];
    const uint32_t p = blockIdx.x, np = gridDim.x;
    const uint32_t sb = a.Lm - a.b1, nsub = 1u << sb;
    uint32_t* tpk = sh;                       // [nblk1] packed target runs
    uint32_t* toff = tpk + a.nblk1;           // [nblk1 + 1]
    uint32_t* ipk = toff + a.nblk1 + 1;       // [nblk2] packed survivor runs
    uint32_t* ioff = ipk + a.nblk2;           // [nblk2 + 1]
    uint32_t* sofs = ioff + a.nblk2 + 1;      // [nsub + 1]
    uint32_t* wsum = sofs + nsub + 1;         // [17]
    uint2* S = reinterpret_cast<uint2*>(sh + ((a.nblk1 * 2 + a.nblk2 * 2 + nsub + 2 + 2 + 17 + 1) & ~1u));
    // the bitmap is no longer read in this call: clear this block's share of it
    for (uint32_t i = p + np * threadIdx.x; i < a.nwords; i += np * kF3Threads) a.bitmap[i] = 0;
    for (uint32_t b = threadIdx.x; b < a.nblk1; b += kF3Threads) {
        const uint32_t x = a.tab1[(uint64_t)p * a.nblk1 + b];
        tpk[b] = x;
        toff[b] = x & 0xFFFFu;
    }
    for (uint32_t b = threadIdx.x; b < a.nblk2; b += kF3Threads) {
        const uint32_t x = a.tab2[(uint64_t)p * a.nblk2 + b];
        ipk[b] = x;
        ioff[b] = x & 0xFFFFu;
    }
    for (uint32_t i = threadIdx.x; i <= nsub; i += kF3Threads) sofs[i] = 0;
    __syncthreads();
    const uint32_t mt = scan_lds<kF3Threads>(toff, a.nblk1, wsum);
    if (mt == 0) return;   // no targets in this partition (block-uniform)
    const uint32_t m = scan_lds<kF3Threads>(ioff, a.nblk2, wsum);
    if (threadIdx.x == 0) {
        toff[a.nblk1] = mt;
        ioff[a.nblk2] = m;
        atomicAdd(a.fb_count + 1, m);
    }
    __syncthreads();
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    constexpr uint32_t NWV = kF3Threads / 64;
    auto target_at = [&](uint32_t j) -> uint2 {
        const uint32_t b = run_of(toff, a.nblk1, j);
        return a.treg[(uint64_t)b * kF1Chunk + (tpk[b] >> 16) + (j - toff[b])];
    };
    if (m > kF3Cap) {
        // strongly clustered ids: this partition's targets take the exact brute-force path
        for (uint32_t j = threadIdx.x; j < mt; j += kF3Threads) {
            const uint2 te = target_at(j);
            a.fb_list[atomicAdd(a.fb_count, 1u)] = te.y;
        }
        return;
    }
    // gather the survivor runs (registers), histogram by sub-prefix, place sorted in LDS
    uint2 e[kF3Per];
    uint32_t rk[kF3Per];
#pragma unroll
    for (int r = 0; r < kF3Per; ++r) {
        const uint32_t j = r * kF3Threads + threadIdx.x;
        if (j < m) {
            const uint32_t b = run_of(ioff, a.nblk2, j);
            e[r] = a.ireg[(uint64_t)b * kF2Chunk + (ipk[b] >> 16) + (j - ioff[b])];
        }
    }
#pragma unroll
    for (int r = 0; r < kF3Per; ++r) {
        const uint32_t j = r * kF3Threads + threadIdx.x;
        if (j < m) rk[r] = atomicAdd(sofs + (top_bits(e[r].x, a.Lm) & (nsub - 1u)), 1u);
    }
    __syncthreads();
    scan_lds<kF3Threads>(sofs, nsub, wsum);
    if (threadIdx.x == 0) sofs[nsub] = m;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kF3Per; ++r) {
        const uint32_t j = r * kF3Threads + threadIdx.x;
        if (j < m) S[sofs[top_bits(e[r].x, a.Lm) & (nsub - 1u)] + rk[r]] = e[r];
    }
    __syncthreads();
    // answer: one wave per target
    const uint32_t want = a.n < a.k ? (uint32_t)a.n : a.k;
    for (uint32_t jt = wv; jt < mt; jt += NWV) {
        const uint2 te = target_at(jt);
        const uint32_t qi = __builtin_amdgcn_readfirstlane(te.y);
        const uint32_t t0 = __builtin_amdgcn_readfirstlane(te.x);
        const uint32_t s = top_bits(t0, a.Lm) & (nsub - 1u);
        const uint32_t lo = sofs[s], hi = sofs[s + 1], mm = hi - lo;
        if (mm < want) {
            if (lane == 0) a.fb_list[atomicAdd(a.fb_count, 1u)] = qi;
            continue;
        }
        uint32_t t[DHT_W];
        t[0] = t0;
#pragma unroll
        for (int w = 1; w < DHT_W; ++w) t[w] = __builtin_amdgcn_readfirstlane(a.tp[(uint64_t)w * a.ts + qi]);
        uint32_t* orow = a.out_idx + (uint64_t)qi * a.k;
        if (mm <= 64) {
            const bool act = lane < mm;
            const uint2 me = act ? S[lo + lane] : make_uint2(0u, 0u);
            const uint32_t md = me.x ^ t0;
            const unsigned long long key = ((unsigned long long)md << 32) | me.y;
            uint32_t rank = 0, eq = 0;
            for (uint32_t o = 0; o < mm; ++o) {
                const uint2 x = S[lo + o];
                const unsigned long long ko = ((unsigned long long)(x.x ^ t0) << 32) | x.y;
                rank += ko < key;
                eq += x.x == me.x;
            }
            if (__ballot(act && eq > 1)) {   // equal w0 words: rank by the full 160-bit key
                rank = 0;
                for (uint32_t o = 0; o < mm; ++o) {
                    const uint2 x = S[lo + o];
                    if (act && o != lane) rank += id_less(x.x ^ t0, x.y, md, me.y, a.planes, a.stride, t);
                }
            }
            if (act && rank < want) orow[rank] = map_out(me.y, a.gidx, a.base);
        } else {
            // large subtree (clustered ids): running lane-distributed top-`want` list
            uint32_t ed = DHT_NONE, ei = DHT_NONE, cnt = 0;
            for (uint32_t c = lo; c < hi; c += 64) {
                const bool v = c + lane < hi;
                const uint2 x = v ? S[c + lane] : make_uint2(0u, DHT_NONE);
                const uint32_t xd = x.x ^ t0, xi = x.y;
                uint32_t wd = cnt == want ? __builtin_amdgcn_readlane((int)ed, want - 1) : DHT_NONE;
                uint32_t wi = cnt == want ? __builtin_amdgcn_readlane((int)ei, want - 1) : DHT_NONE;
                uint64_t cm = __ballot(v && (cnt < want || id_less(xd, xi, wd, wi, a.planes, a.stride, t)));
                while (cm) {
                    const uint32_t l = (uint32_t)__ffsll((long long)cm) - 1;
                    cm &= cm - 1;
                    const uint32_t cd = __builtin_amdgcn_readlane((int)xd, l), ci = __builtin_amdgcn_readlane((int)xi, l);
                    if (cnt == want && !id_less(cd, ci, wd, wi, a.planes, a.stride, t)) continue;
                    const bool closer = lane < cnt && id_less(ed, ei, cd, ci, a.planes, a.stride, t);
                    const uint32_t pos = (uint32_t)__popcll(__ballot(closer));
                    const uint32_t ud = __shfl_up(ed, 1), ui = __shfl_up(ei, 1);
                    if (lane == pos) { ed = cd; ei = ci; }
                    else if (lane > pos) { ed = ud; ei = ui; }
                    cnt = cnt + 1 < want ? cnt + 1 : want;
                    wd = cnt == want ? __builtin_amdgcn_readlane((int)ed, want - 1) : DHT_NONE;
                    wi = cnt == want ? __builtin_amdgcn_readlane((int)ei, want - 1) : DHT_NONE;
                }
            }
            if (lane < want) orow[lane] = map_out(ei, a.gidx, a.base);
        }
        if (lane >= want && lane < a.k) orow[lane] = DHT_NONE;
        if (lane == 0) a.out_cnt[qi] = want;
    }
}

// ---- F4: exact brute force for the fallback targets -------------------------------------
// One workgroup per target: every thread keeps a sorted top-`want` list of its strided
// share of the ids in LDS (slot-major), then `want` rounds of a block arg-min merge.
__global__ __launch_bounds__(kF4Threads) void k_f4_fallback(const uint32_t* __restrict__ fb_count,
                                                           const uint32_t* __restrict__ fb_list,
                                                           const uint32_t* __restrict__ planes, uint64_t stride,
                                                           uint64_t n, const uint32_t* __restrict__ tp, uint64_t ts,
                                                           uint32_t k, const uint32_t* __restrict__ gidx,
                                                           uint32_t base, uint32_t* __restrict__ out_idx,
                                                           uint32_t* __restrict__ out_cnt) {
    extern __shared__ uint2 lst[];            // [want][kF4Threads], then red[kF4Threads / 64]
    const uint32_t cntq = *fb_count;
    const uint32_t want = n < k ? (uint32_t)n : k;
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    uint2* red = lst + (size_t)want * kF4Threads;
    for (uint32_t f = blockIdx.x; f < cntq; f += gridDim.x) {
        const uint32_t qi = fb_list[f];
        uint32_t t[DHT_W];
        load_target(tp, ts, qi, t);
        uint32_t c = 0, wd = DHT_NONE, wi = DHT_NONE;   // own list length and its worst entry
        for (uint64_t i = threadIdx.x; i < n; i += kF4Threads) {
            const uint32_t d = planes[i] ^ t[0];
            if (c == want && !id_less(d, (uint32_t)i, wd, wi, planes, stride, t)) continue;
            uint32_t pos = c < want ? c : want - 1;
            while (pos > 0) {
                const uint2 prev = lst[(pos - 1) * kF4Threads + threadIdx.x];
                if (!id_less(d, (uint32_t)i, prev.x, prev.y, planes, stride, t)) break;
                lst[pos * kF4Threads + threadIdx.x] = prev;
                --pos;
            }
            lst[pos * kF4Threads + threadIdx.x] = make_uint2(d, (uint32_t)i);
            if (c < want) ++c;
            if (c == want) {
                const uint2 w = lst[(want - 1) * kF4Threads + threadIdx.x];
                wd = w.x;
                wi = w.y;
            }
        }
        // merge: `want` rounds of block arg-min over the list heads
        uint32_t ptr = 0;
        for (uint32_t r = 0; r < want; ++r) {
            uint2 h = ptr < c ? lst[ptr * kF4Threads + threadIdx.x] : make_uint2(DHT_NONE, DHT_NONE);
            // wave arg-min (NONE idx = empty, farthest)
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) {
                const uint2 x = make_uint2(__shfl_xor(h.x, o), __shfl_xor(h.y, o));
                const bool take = x.y != DHT_NONE && (h.y == DHT_NONE || id_less(x.x, x.y, h.x, h.y, planes, stride, t));
                if (take) h = x;
            }
            if (lane == 0) red[wv] = h;
            __syncthreads();
            uint2 best = red[0];
            for (uint32_t w = 1; w < kF4Threads / 64; ++w) {
                const uint2 x = red[w];
                if (x.y != DHT_NONE && (best.y == DHT_NONE || id_less(x.x, x.y, best.x, best.y, planes, stride, t)))
                    best = x;
            }
            __syncthreads();
            if (ptr < c && lst[ptr * kF4Threads + threadIdx.x].y == best.y) ++ptr;   // indices are unique
            if (threadIdx.x == 0) out_idx[(uint64_t)qi * k + r] = map_out(best.y, gidx, base);
        }
        for (uint32_t r = want + threadIdx.x; r < k; r += kF4Threads) out_idx[(uint64_t)qi * k + r] = DHT_NONE;
        if (threadIdx.x == 0) out_cnt[qi] = want;
        __syncthreads();
    }
}

struct BatchPlan {
    uint32_t Lm, b1, nwords, nblk1, nblk2;
};

uint32_t floor_log2(uint64_t x) {
    uint32_t r = 0;
    while (x > 1) { x >>= 1; ++r; }
    return r;
}

BatchPlan plan_batch(uint64_t n, uint32_t q, uint32_t k) {
    BatchPlan P;
    // mark level: about 4k ids per level-Lm subtree
    const uint64_t per = 4ull * k;
    P.Lm = n >= per ? floor_log2(n / per) : 0;
    if (P.Lm > kMaxLm) P.Lm = kMaxLm;
    // survivors on uniform ids: n (1 - exp(-q / 2^Lm)); partitions of about kF3Cap / 2
    const double f = 1.0 - std::exp(-(double)q / (double)(1ull << P.Lm));
    const double surv = (double)n * f + 1.0;
    uint32_t b1 = 0;
    while (b1 < P.Lm && surv / (double)(1ull << b1) > kF3Cap / 2) ++b1;
    if (P.Lm > kMaxSubBits && b1 < P.Lm - kMaxSubBits) b1 = P.Lm - kMaxSubBits;
    if (b1 > 13) b1 = 13;
    P.b1 = b1;
    P.nwords = P.Lm >= 5 ? (1u << (P.Lm - 5)) : 1u;
    P.nblk1 = (q + kF1Chunk - 1) / kF1Chunk;
    P.nblk2 = (uint32_t)((n + kF2Chunk - 1) / kF2Chunk);
    return P;
}

size_t f3_lds(const BatchPlan& P) {
    const uint32_t nsub = 1u << (P.Lm - P.b1);
    const size_t words = ((size_t)(P.nblk1 * 2 + P.nblk2 * 2 + nsub + 2 + 2 + 17 + 1) & ~size_t(1));
    return words * 4 + (size_t)kF3Cap * 8;
}

}  // namespace

bool batch_supported(uint64_t n, uint32_t q, uint32_t k) {
    if (k == 0 || k > DHTGPU_MAX_K_DEV) return false;
    const BatchPlan P = plan_batch(n, q, k);
    if (P.nblk2 > kMaxBlk2 || P.nblk1 > kMaxBlk1) return false;
    if (P.Lm - P.b1 > 13) return false;
    return f3_lds(P) <= kLdsMax;
}

// workspace: bitmap (64 KB, all-zero between calls) | fb_count | fb_list[q] | treg[q] |
// tab1[np * nblk1] | tab2[np * nblk2] | ireg[nblk2 * kF2Chunk]
size_t batch_bytes(uint64_t n, uint32_t q, uint32_t k) {
    const BatchPlan P = plan_batch(n, q, k);
    const size_t np = 1ull << P.b1;
    return 65536 + 256 + (size_t)q * 4 + 16 + (size_t)q * 8 + 16 + np * P.nblk1 * 4 + 16 + np * P.nblk2 * 4 + 16 +
           (size_t)P.nblk2 * kF2Chunk * 8 + 256;
}

const uint32_t* batch_stats(const void* ws) {
    return reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(ws) + 65536);
}

hipError_t launch_batch_topk(void* ws, const uint32_t* planes, uint64_t stride, uint64_t n, const uint32_t* tp,
                             uint64_t ts, uint32_t q, uint32_t k, const uint32_t* gidx, uint32_t base,
                             uint32_t* out_idx, uint32_t* out_cnt, hipStream_t s, hipEvent_t* ev) {
    if (!q) return hipSuccess;
    const BatchPlan P = plan_batch(n, q, k);
    const uint32_t np = 1u << P.b1;
    uint8_t* w = static_cast<uint8_t*>(ws);
    auto take = [&](size_t bytes) {
        uint8_t* r = w;
        w += (bytes + 255) & ~size_t(255);
        return r;
    };
    uint32_t* bitmap = reinterpret_cast<uint32_t*>(take(65536));
    uint32_t* fb_count = reinterpret_cast<uint32_t*>(take(16));
    uint32_t* fb_list = reinterpret_cast<uint32_t*>(take((size_t)q * 4));
    uint2* treg = reinterpret_cast<uint2*>(take((size_t)q * 8));
    uint32_t* tab1 = reinterpret_cast<uint32_t*>(take((size_t)np * P.nblk1 * 4));
    uint32_t* tab2 = reinterpret_cast<uint32_t*>(take((size_t)np * (P.nblk2 ? P.nblk2 : 1) * 4));
    uint2* ireg = reinterpret_cast<uint2*>(take((size_t)(P.nblk2 ? P.nblk2 : 1) * kF2Chunk * 8));
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)k_f2_filter, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax);
        (void)hipFuncSetAttribute((const void*)k_f3_answer, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax);
        attr_set = true;
    }
    if (ev) (void)hipEventRecord(ev[0], s);
    k_f1_targets<<<P.nblk1, kF1Threads, (np + 1 + 17) * 4, s>>>(tp, q, P.Lm, P.b1, bitmap, tab1, P.nblk1, treg,
                                                                fb_count);
    if (ev) (void)hipEventRecord(ev[1], s);
    if (P.nblk2)
        k_f2_filter<<<P.nblk2, kF2Threads, (P.nwords + np + 1 + 17) * 4, s>>>(planes, n, P.Lm, P.b1, bitmap,
                                                                               P.nwords, tab2, P.nblk2, ireg);
    if (ev) (void)hipEventRecord(ev[2], s);
    F3Args a{ireg, tab2, P.nblk2, treg, tab1, P.nblk1, P.Lm, P.b1, bitmap, P.nwords, planes, stride, n,
             tp, ts, k, gidx, base, out_idx, out_cnt, fb_count, fb_list};
    k_f3_answer<<<np, kF3Threads, f3_lds(P), s>>>(a);
    if (ev) (void)hipEventRecord(ev[3], s);
    const uint32_t want = n < k ? (uint32_t)n : k;
    k_f4_fallback<<<64, kF4Threads, ((size_t)want * kF4Threads + kF4Threads / 64) * 8, s>>>(fb_count, fb_list, planes, stride, n, tp, ts, k, gidx, base, out_idx,
                                           out_cnt);
    if (ev) (void)hipEventRecord(ev[4], s);
    return hipGetLastError();
}

}  // namespace dhtgpu
