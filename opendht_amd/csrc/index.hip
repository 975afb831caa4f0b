// index.hip -- K4 bucket index + K5 trie-descent exact XOR k-NN (gfx950).
//
// Restates the same flat exact top-k as K1 (std::partial_sort over InfoHash::xorCmp,
// include/opendht/infohash.h:179-194) with O(k + B) work per target
// instead of O(N).
//
// Why it is exact.  For a target t and a set S of ids, let sub(P, l) be the ids whose
// first l bits equal those of P.  All ids of a subtree sub(t, l) agree with t on bits
// [0, l) while every id outside differs from t at some bit < l, so every id inside is
// XOR-closer than every id outside.  Hence if |sub(t, l)| >= k the top-k lies in
// sub(t, l).  K5 finds the deepest such l with a bucket directory (counts of every
// prefix of length <= B in O(1)), brute-forces the exact top-k inside that subtree, and
// when that subtree is large but its t-side child holds fewer than `need` ids, takes the
// child whole (all closer) and continues in the sibling subtree, following t's bits.
//
// K4 (index build) is a counting sort of the ids by their top B bits into 8-byte entries
// {w0, index} plus the 2^B + 1 entry prefix directory (two LDS-histogram passes, see
// below).  Order inside a bucket is irrelevant: candidates are ranked by (distance, index);
// the id words 1..4 are read from the resident planes only when two w0 distances tie.
#include "dhtgpu_dev.h"
#include "dhtgpu_internal.h"

#include <mutex>

namespace dhtgpu {
namespace {

constexpr int kBlk = 256;

// Two-pass partition by the top B = b1 + b2 bits (b1, b2 <= 12), all histograms in LDS and
// no global atomics:
//   P0  per block (8192 ids): LDS histogram of the top b1 bits -> column of H[bin][block]
//   P0r one block per bin: exclusive scan of H's row (offsets of each block inside the
//       bin) and the bin total
//   P0s one block: exclusive scan of the bin totals -> partition starts (pstart)
//   P1  per block: scatter every id to pstart[bin] + H[bin][block] + LDS rank as an
//       8-byte entry {w0, idx}
//   P2  one block per partition: LDS histogram of the next b2 bits -> directory entries
//       of the partition's 2^b2 buckets; the bucket permutation is built in LDS and the
//       entries are then GATHERED into bucket order, so every global write is coalesced.
//       (Partitions larger than the LDS permutation capacity -- clustered inputs -- take
//       a scatter path instead.)
// Ranks come from LDS atomics, so order inside a bucket is arbitrary; queries rank
// candidates by (distance, index), so results do not depend on it.
constexpr uint32_t kP1Tile = 8192;   // minimum ids per P0/P1 block (256 threads x 32); grown so nblk <= 2048
constexpr int kP2Blk = 1024;
constexpr int kP2Per = 16;          // entries per thread per batch: a ~16K partition is one batch
constexpr uint32_t kLdsMax = 160 * 1024;

__global__ __launch_bounds__(kBlk) void k_p0_hist(const uint32_t* __restrict__ w0, uint64_t n, uint32_t b1,
                                                 uint32_t nblk, uint32_t tile, uint32_t* __restrict__ H) {
    extern __shared__ uint32_t sh[];
    const uint32_t nbin = 1u << b1, shift = 32 - b1;
    for (uint32_t i = threadIdx.x; i < nbin; i += kBlk) sh[i] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * tile;
    const uint32_t cnt = (uint32_t)(n - base < tile ? n - base : tile);
    for (uint32_t e = threadIdx.x * 4; e < cnt; e += kBlk * 4) {
        if (e + 3 < cnt) {
            const uint4 v = *reinterpret_cast<const uint4*>(w0 + base + e);
            atomicAdd(sh + (v.x >> shift), 1u);
            atomicAdd(sh + (v.y >> shift), 1u);
            atomicAdd(sh + (v.z >> shift), 1u);
            atomicAdd(sh + (v.w >> shift), 1u);
        } else {
            for (uint32_t f = e; f < cnt; ++f) atomicAdd(sh + (w0[base + f] >> shift), 1u);
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nbin; i += kBlk) H[(uint64_t)i * nblk + blockIdx.x] = sh[i];
}

// exclusive scan of `len` values in place (single block of 1024 threads); returns total
__device__ uint32_t block_scan_inplace(uint32_t* __restrict__ a, uint32_t len, uint32_t* scr) {
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
    return carry;
}

// exclusive scan of `len` values in place by a block of NT threads; returns the total
template <int NT>
__device__ uint32_t block_scan_nt(uint32_t* __restrict__ a, uint32_t len, uint32_t* scr) {
    uint32_t carry = 0;
    for (uint32_t b = 0; b < len; b += NT) {
        const uint32_t i = b + threadIdx.x;
        const uint32_t v = i < len ? a[i] : 0;
        scr[threadIdx.x] = v;
        __syncthreads();
        for (uint32_t o = 1; o < (uint32_t)NT; o <<= 1) {
            const uint32_t x = threadIdx.x >= o ? scr[threadIdx.x - o] : 0;
            __syncthreads();
            scr[threadIdx.x] += x;
            __syncthreads();
        }
        if (i < len) a[i] = carry + scr[threadIdx.x] - v;
        carry += scr[NT - 1];
        __syncthreads();
    }
    return carry;
}

__global__ __launch_bounds__(1024) void k_p0_rowscan(uint32_t* __restrict__ H, uint32_t nblk,
                                                    uint32_t* __restrict__ pcount) {
    __shared__ uint32_t scr[1024];
    const uint32_t total = block_scan_inplace(H + (uint64_t)blockIdx.x * nblk, nblk, scr);
    if (threadIdx.x == 0) pcount[blockIdx.x] = total;
}

__global__ __launch_bounds__(1024) void k_p0_scan(uint32_t* __restrict__ pcount, uint32_t nbin,
                                                 uint32_t* __restrict__ pstart, uint64_t n) {
    __shared__ uint32_t scr[1024];
    for (uint32_t i = threadIdx.x; i < nbin; i += 1024) pstart[i] = pcount[i];
    __syncthreads();
    block_scan_inplace(pstart, nbin, scr);
    if (threadIdx.x == 0) pstart[nbin] = (uint32_t)n;
}

// P1: the block's tile is counting-sorted by partition in LDS first, so that every
// partition run is then written to HBM contiguously by consecutive lanes (runs are
// short -- tile / 2^b1 entries -- and scattered 8-byte stores would leave partial lines).
constexpr uint32_t kP1Stage = 8192;   // entries staged in LDS per round (64 KB)

__global__ __launch_bounds__(kBlk) void k_p1_scatter(const uint32_t* __restrict__ w0, uint64_t n, uint32_t b1,
                                                    uint32_t nblk, uint32_t tile, const uint32_t* __restrict__ H,
                                                    const uint32_t* __restrict__ pstart,
                                                    uint2* __restrict__ tmp) {
    extern __shared__ uint32_t sh[];   // [gbase 2^b1 | lcnt 2^b1 | loff 2^b1 | scan scratch kBlk | stage]
    const uint32_t nbin = 1u << b1, shift = 32 - b1;
    uint32_t* gbase = sh;
    uint32_t* lcnt = sh + nbin;
    uint32_t* loff = sh + 2 * nbin;
    uint32_t* scr = sh + 3 * nbin;
    uint2* stage = reinterpret_cast<uint2*>(scr + kBlk);
    for (uint32_t i = threadIdx.x; i < nbin; i += kBlk) gbase[i] = pstart[i] + H[(uint64_t)i * nblk + blockIdx.x];
    const uint64_t base0 = (uint64_t)blockIdx.x * tile;
    const uint32_t mt = (uint32_t)(n - base0 < tile ? n - base0 : tile);
    constexpr uint32_t PER = kP1Stage / kBlk;   // 32 ids per thread per round
    for (uint32_t r0 = 0; r0 < mt; r0 += kP1Stage) {
        const uint32_t m = mt - r0 < kP1Stage ? mt - r0 : kP1Stage;
        const uint64_t base = base0 + r0;
        for (uint32_t i = threadIdx.x; i < nbin; i += kBlk) lcnt[i] = 0;
        __syncthreads();
        // ids base + 4*threadIdx.x + 1024*e + f  (coalesced 16-B loads, all issued first)
        uint32_t v[PER];
#pragma unroll
        for (uint32_t e = 0; e < PER / 4; ++e) {
            const uint32_t j = e * 4 * kBlk + 4 * threadIdx.x;
            if (j + 3 < m) {
                const uint4 x = *reinterpret_cast<const uint4*>(w0 + base + j);
                v[4 * e] = x.x; v[4 * e + 1] = x.y; v[4 * e + 2] = x.z; v[4 * e + 3] = x.w;
            } else {
#pragma unroll
                for (uint32_t f = 0; f < 4; ++f) v[4 * e + f] = j + f < m ? w0[base + j + f] : 0;
            }
        }
#pragma unroll
        for (uint32_t e = 0; e < PER; ++e) {
            const uint32_t j = (e / 4) * 4 * kBlk + 4 * threadIdx.x + (e % 4);
            if (j < m) atomicAdd(lcnt + (v[e] >> shift), 1u);
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < nbin; i += kBlk) loff[i] = lcnt[i];
        __syncthreads();
        block_scan_nt<kBlk>(loff, nbin, scr);
        for (uint32_t i = threadIdx.x; i < nbin; i += kBlk) lcnt[i] = 0;
        __syncthreads();
#pragma unroll
        for (uint32_t e = 0; e < PER; ++e) {
            const uint32_t j = (e / 4) * 4 * kBlk + 4 * threadIdx.x + (e % 4);
            if (j < m) {
                const uint32_t d = v[e] >> shift;
                stage[loff[d] + atomicAdd(lcnt + d, 1u)] = make_uint2(v[e], (uint32_t)(base + j));
            }
        }
        __syncthreads();
        // write out in partition order: consecutive lanes -> consecutive addresses of a run
        for (uint32_t j = threadIdx.x; j < m; j += kBlk) {
            const uint2 e = stage[j];
            const uint32_t d = e.x >> shift;
            tmp[gbase[d] + (j - loff[d])] = e;
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < nbin; i += kBlk) gbase[i] += lcnt[i];
        __syncthreads();
    }
}

__global__ __launch_bounds__(kP2Blk) void k_p2_buckets(const uint2* __restrict__ tmp,
                                                      const uint32_t* __restrict__ pstart, uint32_t b1,
                                                      uint32_t b2, uint32_t perm_cap, uint32_t* __restrict__ dir,
                                                      uint2* __restrict__ pairs, uint64_t n) {
    extern __shared__ uint32_t sh[];   // [cnt 2^b2 | offsets 2^b2 | scan scratch kP2Blk | perm]
    const uint32_t p = blockIdx.x;
    const uint32_t nsub = 1u << b2, shift = 32 - b1 - b2, mask = nsub - 1u;
    uint32_t* cnt = sh;
    uint32_t* off = sh + nsub;
    uint32_t* scr = sh + 2 * nsub;
    uint32_t* perm = scr + kP2Blk;
    const uint32_t lo = pstart[p], hi = pstart[p + 1], m = hi - lo;
    constexpr uint32_t BATCH = kP2Blk * kP2Per;
    for (uint32_t i = threadIdx.x; i < nsub; i += kP2Blk) cnt[i] = 0;
    __syncthreads();
    // histogram: each thread keeps kP2Per loads in flight per batch
    for (uint32_t b = 0; b < m; b += BATCH) {
        uint32_t key[kP2Per];
#pragma unroll
        for (int e = 0; e < kP2Per; ++e) {
            const uint32_t j = b + e * kP2Blk + threadIdx.x;
            key[e] = j < m ? tmp[lo + j].x : 0;
        }
#pragma unroll
        for (int e = 0; e < kP2Per; ++e)
            if (b + e * kP2Blk + threadIdx.x < m) atomicAdd(cnt + ((key[e] >> shift) & mask), 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nsub; i += kP2Blk) off[i] = cnt[i];
    __syncthreads();
    block_scan_nt<kP2Blk>(off, nsub, scr);
    for (uint32_t i = threadIdx.x; i < nsub; i += kP2Blk) {
        dir[((uint64_t)p << b2) + i] = lo + off[i];
        cnt[i] = 0;
    }
    if (p == gridDim.x - 1 && threadIdx.x == 0) dir[(uint64_t)gridDim.x << b2] = (uint32_t)n;
    __syncthreads();
    if (m <= perm_cap) {
        // bucket permutation in LDS, then a gather (reads inside the partition's slice)
        // with coalesced writes
        for (uint32_t b = 0; b < m; b += BATCH) {
            uint32_t key[kP2Per];
#pragma unroll
            for (int e = 0; e < kP2Per; ++e) {
                const uint32_t j = b + e * kP2Blk + threadIdx.x;
                key[e] = j < m ? tmp[lo + j].x : 0;
            }
#pragma unroll
            for (int e = 0; e < kP2Per; ++e) {
                const uint32_t j = b + e * kP2Blk + threadIdx.x;
                if (j < m) {
                    const uint32_t sb = (key[e] >> shift) & mask;
                    perm[off[sb] + atomicAdd(cnt + sb, 1u)] = j;
                }
            }
        }
        __syncthreads();
        for (uint32_t b = 0; b < m; b += BATCH) {
            uint2 v[kP2Per];
#pragma unroll
            for (int e = 0; e < kP2Per; ++e) {
                const uint32_t j = b + e * kP2Blk + threadIdx.x;
                v[e] = j < m ? tmp[lo + perm[j]] : make_uint2(0, 0);
            }
#pragma unroll
            for (int e = 0; e < kP2Per; ++e) {
                const uint32_t j = b + e * kP2Blk + threadIdx.x;
                if (j < m) pairs[lo + j] = v[e];
            }
        }
    } else {
        for (uint32_t b = 0; b < m; b += BATCH) {
            uint2 v[kP2Per];
#pragma unroll
            for (int e = 0; e < kP2Per; ++e) {
                const uint32_t j = b + e * kP2Blk + threadIdx.x;
                v[e] = j < m ? tmp[lo + j] : make_uint2(0, 0);
            }
#pragma unroll
            for (int e = 0; e < kP2Per; ++e) {
                const uint32_t j = b + e * kP2Blk + threadIdx.x;
                if (j < m) {
                    const uint32_t sb = (v[e].x >> shift) & mask;
                    pairs[lo + off[sb] + atomicAdd(cnt + sb, 1u)] = v[e];
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------------
// K5: one wave per target.  Bucket entries are (w0, idx) pairs; a candidate's key is
// (w0 ^ t0, then the remaining words ^ t, then idx).  Only when two candidates' w0
// distances tie are their words 1..4 gathered from the resident id planes.
// ---------------------------------------------------------------------------------
struct Cand {
    uint32_t d0, idx;
};

__device__ __forceinline__ Cand cand_none() { return Cand{DHT_NONE, DHT_NONE}; }

// strict order: a closer than b.  NONE entries are farthest.
__device__ __forceinline__ bool cand_less(const Cand& a, const Cand& b, const uint32_t* __restrict__ planes,
                                          uint64_t stride, const uint32_t* t) {
    if (b.idx == DHT_NONE) return a.idx != DHT_NONE;
    if (a.idx == DHT_NONE) return false;
    if (a.d0 != b.d0) return a.d0 < b.d0;
    uint32_t wa[DHT_W], wb[DHT_W];
    load_id(planes, stride, a.idx, wa);
    load_id(planes, stride, b.idx, wb);
    return xor_less_from(wa, a.idx, wb, b.idx, t, 1);
}

__device__ __forceinline__ Cand cand_readlane(const Cand& a, uint32_t l) {
    return Cand{(uint32_t)__builtin_amdgcn_readlane((int)a.d0, l), (uint32_t)__builtin_amdgcn_readlane((int)a.idx, l)};
}

__device__ __forceinline__ Cand load_cand(const uint2* __restrict__ pairs, uint32_t pos, uint32_t t0) {
    const uint2 e = pairs[pos];
    return Cand{e.x ^ t0, e.y};
}

// Append the `take` closest ids of bucket entries [lo, hi) (ascending) to the
// lane-distributed result list at slots [base, base + take).  `wl` is this wave's
// 64-entry LDS scratch (u64).
__device__ void select_range(const uint2* __restrict__ pairs, uint32_t lo, uint32_t hi,
                             const uint32_t* __restrict__ planes, uint64_t stride, const uint32_t* t,
                             uint32_t take, uint32_t base, uint32_t lane, uint32_t& res,
                             unsigned long long* wl) {
    const uint32_t m = hi - lo;
    if (m <= 64) {
        // packed key (w0 distance << 32 | idx); rank = number of smaller keys, read from LDS
        const Cand mine = lane < m ? load_cand(pairs, lo + lane, t[0]) : cand_none();
        const unsigned long long key = ((unsigned long long)mine.d0 << 32) | mine.idx;
        wl[lane] = key;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        uint32_t rank = 0, eq = 0;
        uint32_t o = 0;
        for (; o + 4 <= m; o += 4) {
#pragma unroll
            for (uint32_t u = 0; u < 4; ++u) {
                const unsigned long long ko = wl[o + u];
                rank += ko < key;
                eq += (uint32_t)(ko >> 32) == mine.d0;
            }
        }
        for (; o < m; ++o) {
            const unsigned long long ko = wl[o];
            rank += ko < key;
            eq += (uint32_t)(ko >> 32) == mine.d0;
        }
        if (__ballot(lane < m && eq > 1)) {
            // equal w0 distances (rare): exact rank by the full 160-bit key
            rank = 0;
            for (uint32_t q2 = 0; q2 < m; ++q2) {
                const unsigned long long ko = wl[q2];
                const Cand other{(uint32_t)(ko >> 32), (uint32_t)ko};
                if (lane < m && q2 != lane) rank += cand_less(other, mine, planes, stride, t);
            }
        }
        __builtin_amdgcn_wave_barrier();
        // route: the candidate of rank r (< take) goes to result slot base + r
        uint32_t* slot = reinterpret_cast<uint32_t*>(wl);
        if (lane < m && rank < take) slot[base + rank] = mine.idx;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        if (lane >= base && lane < base + take) res = slot[lane];
        __builtin_amdgcn_wave_barrier();
        return;
    }
    // large range (clustered inputs): running lane-distributed top-`take` list
    Cand ent = cand_none();
    uint32_t cnt = 0;
    for (uint32_t c = lo; c < hi; c += 64) {
        const bool v = c + lane < hi;
        const Cand mine = v ? load_cand(pairs, c + lane, t[0]) : cand_none();
        Cand worst = cnt == take ? cand_readlane(ent, take - 1) : cand_none();
        uint64_t cm = __ballot(v && (cnt < take || cand_less(mine, worst, planes, stride, t)));
        while (cm) {
            const uint32_t l = (uint32_t)__ffsll((long long)cm) - 1;
            cm &= cm - 1;
            const Cand cand = cand_readlane(mine, l);
            if (cnt == take && !cand_less(cand, worst, planes, stride, t)) continue;
            const bool closer = lane < cnt && cand_less(ent, cand, planes, stride, t);
            const uint32_t pos = (uint32_t)__popcll(__ballot(closer));
            const uint32_t ud = __shfl_up(ent.d0, 1), ui = __shfl_up(ent.idx, 1);
            if (lane == pos) ent = cand;
            else if (lane > pos) ent = Cand{ud, ui};
            cnt = cnt + 1 < take ? cnt + 1 : take;
            worst = cnt == take ? cand_readlane(ent, take - 1) : cand_none();
        }
    }
    const uint32_t idx_src = __shfl(ent.idx, (int)(lane >= base ? lane - base : 0));
    if (lane >= base && lane < base + cnt) res = idx_src;
}

__global__ __launch_bounds__(256) void k_query(const uint2* __restrict__ pairs, const uint32_t* __restrict__ dir,
                                              uint32_t B, uint64_t n, const uint32_t* __restrict__ planes,
                                              uint64_t stride, const uint32_t* __restrict__ tp, uint64_t ts,
                                              uint32_t q, uint32_t k, uint32_t* __restrict__ out_idx,
                                              uint32_t* __restrict__ out_cnt) {
    __shared__ unsigned long long wls[4 * 64];
    const uint32_t lane = lane_id();
    const uint32_t wv = threadIdx.x >> 6;
    unsigned long long* wl = wls + 64 * wv;
    const uint32_t qi = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + wv);
    if (qi >= q) return;
    uint32_t t[DHT_W];
#pragma unroll
    for (int j = 0; j < DHT_W; ++j) t[j] = __builtin_amdgcn_readfirstlane(tp[(uint64_t)j * ts + qi]);
    const uint32_t want = n < k ? (uint32_t)n : k;
    uint32_t res = DHT_NONE;   // lane r < want holds result rank r
    uint32_t got = 0;
    uint32_t p0 = t[0];        // prefix P: t with the branch bits flipped (within w0: levels <= B <= 32)
    uint32_t L = 0;
    while (got < want) {
        const uint32_t need = want - got;
        // lane l examines level L + l (<= B): range of prefix(P, level) from the directory
        const uint32_t level = L + lane;
        uint32_t lo = 0, hi = 0;
        if (level <= B) {
            const uint32_t topb = B ? p0 >> (32 - B) : 0;
            const uint32_t span = 1u << (B - level);
            const uint32_t v = topb & ~(span - 1u);
            lo = dir[v];
            hi = dir[v + span];
        }
        const uint64_t ok = __ballot(level <= B && hi - lo >= need);
        // counts are non-increasing in the level, so ok = lanes [0, x); level L has >= need
        const uint32_t x = (uint32_t)__popcll(ok);
        const uint32_t lp = L + x - 1;              // deepest level with >= need ids
        const uint32_t tlo = (uint32_t)__builtin_amdgcn_readlane((int)lo, x - 1);
        const uint32_t thi = (uint32_t)__builtin_amdgcn_readlane((int)hi, x - 1);
        if (lp == B || thi - tlo <= 64) {
            select_range(pairs, tlo, thi, planes, stride, t, need, got, lane, res, wl);
            got += need;
            break;
        }
        // subtree big but its t-side child (level lp + 1) holds < need ids: take the child
        // whole (every id in it is closer than the rest), continue in the sibling subtree
        const uint32_t clo = (uint32_t)__builtin_amdgcn_readlane((int)lo, x);
        const uint32_t chi = (uint32_t)__builtin_amdgcn_readlane((int)hi, x);
        if (chi > clo) select_range(pairs, clo, chi, planes, stride, t, chi - clo, got, lane, res, wl);
        got += chi - clo;
        p0 ^= 0x80000000u >> lp;
        L = lp + 1;
    }
    if (lane < k) out_idx[(uint64_t)qi * k + lane] = lane < want ? res : DHT_NONE;
    if (lane == 0) out_cnt[qi] = want;
}

}  // namespace

uint32_t index_bits(uint64_t n) {
    uint32_t lg = 0;
    while (lg < 63 && (1ull << (lg + 1)) <= n) ++lg;
    int b = (int)lg - 4;
    if (b < 1) b = 1;
    if (b > 24) b = 24;
    return (uint32_t)b;
}

static void index_split(uint64_t n, uint32_t B, uint32_t& b1, uint32_t& b2) {
    // partitions of ~2^14 ids: one register batch of a 1024-thread pass-2 block, and an
    // LDS permutation of <= 84 KB; b1, b2 <= 12 keep every LDS histogram within 32 KB
    uint32_t lg = 0;
    while (lg < 63 && (1ull << lg) < n) ++lg;
    int x = (int)lg - 14;
    if (x < (int)B - 12) x = (int)B - 12;
    if (x > 12) x = 12;
    if (x > (int)B) x = (int)B;
    if (x < 1) x = 1;   // B >= 1 (index_bits)
    b1 = (uint32_t)x;
    b2 = B - b1;
}

static uint32_t p1_tile(uint64_t n) {
    uint64_t t = kP1Tile;
    while ((n + t - 1) / t > 2048) t += kP1Tile;
    return (uint32_t)t;
}
static uint32_t p1_blocks(uint64_t n) { return (uint32_t)((n + p1_tile(n) - 1) / p1_tile(n)); }

// workspace: pairs (n x 8 B) | dir (2^B + 1) | tmp (n x 8 B) | H | pcount | pstart
size_t index_bytes(uint64_t n, uint32_t B) {
    uint32_t b1, b2;
    index_split(n, B, b1, b2);
    const uint64_t nb = 1ull << B, np = 1ull << b1, nblk = p1_blocks(n) ? p1_blocks(n) : 1;
    return (size_t)n * 8 * 2 + (nb + 1) * 4 + (np * nblk + 2 * np + 1) * 4 + 1024;
}

static void index_layout(void* ws, uint64_t n, uint32_t B, uint2*& pairs, uint32_t*& dir) {
    uint8_t* base = static_cast<uint8_t*>(ws);
    pairs = reinterpret_cast<uint2*>(base);
    dir = reinterpret_cast<uint32_t*>(base + (size_t)n * 8);
    (void)B;
}

std::once_flag g_idx_attr_once[kMaxDevices];   // k_p1_scatter / k_p2_buckets LDS attributes (per_device_once)

hipError_t launch_index_build(const uint32_t* planes, uint64_t stride, uint64_t n, uint32_t B, void* ws,
                              hipStream_t s, hipEvent_t* ev) {
    (void)stride;
    uint32_t b1, b2;
    index_split(n, B, b1, b2);
    const uint64_t nb = 1ull << B, np = 1ull << b1;
    const uint32_t nblk = p1_blocks(n);
    uint2* pairs;
    uint32_t* dir;
    index_layout(ws, n, B, pairs, dir);
    uint2* tmp = reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(dir) + (((nb + 1) * 4 + 15) & ~size_t(15)));
    uint32_t* H = reinterpret_cast<uint32_t*>(tmp + n);
    uint32_t* pcount = H + np * (nblk ? nblk : 1);
    uint32_t* pstart = pcount + np;
    // hipFuncSetAttribute applies to the device current at the call: once per device, from
    // whichever thread gets there first (a plain static flag raced between threads and skipped
    // every device after the first)
    {
        const hipError_t e = per_device_once(g_idx_attr_once, [] {
            (void)hipFuncSetAttribute((const void*)k_p2_buckets, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax);
            (void)hipFuncSetAttribute((const void*)k_p1_scatter, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax);
        });
        if (e != hipSuccess) return e;
    }
    if (ev) (void)hipEventRecord(ev[0], s);
    if (n) {
        k_p0_hist<<<nblk, kBlk, np * 4, s>>>(planes, n, b1, nblk, p1_tile(n), H);
        if (ev) (void)hipEventRecord(ev[1], s);
        k_p0_rowscan<<<(uint32_t)np, 1024, 0, s>>>(H, nblk, pcount);
    } else {
        if (ev) (void)hipEventRecord(ev[1], s);
        hipError_t e = hipMemsetAsync(pcount, 0, np * 4, s);
        if (e != hipSuccess) return e;
    }
    k_p0_scan<<<1, 1024, 0, s>>>(pcount, (uint32_t)np, pstart, n);
    if (ev) (void)hipEventRecord(ev[2], s);
    if (n)
        k_p1_scatter<<<nblk, kBlk, (3 * np + kBlk) * 4 + kP1Stage * 8, s>>>(planes, n, b1, nblk, p1_tile(n), H,
                                                                          pstart, tmp);
    if (ev) (void)hipEventRecord(ev[3], s);
    // LDS: fixed part + a permutation sized 1.25x the average partition + 512 (several
    // blocks per CU); larger partitions (clustered inputs) take the scatter path
    const uint32_t fixed = ((2u << b2) + kP2Blk) * 4;
    uint64_t cap = (n >> b1) + (n >> b1) / 4 + 512;
    if (cap > (kLdsMax - fixed) / 4) cap = (kLdsMax - fixed) / 4;
    k_p2_buckets<<<(uint32_t)np, kP2Blk, fixed + (uint32_t)cap * 4, s>>>(tmp, pstart, b1, b2, (uint32_t)cap, dir,
                                                                        pairs, n);
    if (ev) (void)hipEventRecord(ev[4], s);
    return hipGetLastError();
}

hipError_t launch_index_query(const void* ws, uint64_t n, uint32_t B, const uint32_t* planes, uint64_t stride,
                              const uint32_t* tp, uint64_t ts, uint32_t q, uint32_t k, uint32_t* out_idx,
                              uint32_t* out_cnt, hipStream_t s) {
    if (!q) return hipSuccess;
    uint2* pairs;
    uint32_t* dir;
    index_layout(const_cast<void*>(ws), n, B, pairs, dir);
    k_query<<<(q + 3) / 4, 256, 0, s>>>(pairs, dir, B, n, planes, stride, tp, ts, q, k, out_idx, out_cnt);
    return hipGetLastError();
}

}  // namespace dhtgpu
