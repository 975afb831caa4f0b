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
constexpr uint32_t kP1Tile = 8192;   // ids per P0/P1 block (256 threads x 32)
constexpr int kP2Blk = 1024;
constexpr uint32_t kLdsMax = 160 * 1024;

__global__ __launch_bounds__(kBlk) void k_p0_hist(const uint32_t* __restrict__ w0, uint64_t n, uint32_t b1,
                                                 uint32_t nblk, uint32_t* __restrict__ H) {
    extern __shared__ uint32_t sh[];
    const uint32_t nbin = 1u << b1, shift = 32 - b1;
    for (uint32_t i = threadIdx.x; i < nbin; i += kBlk) sh[i] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kP1Tile;
    const uint32_t cnt = (uint32_t)(n - base < kP1Tile ? n - base : kP1Tile);
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

__global__ __launch_bounds__(kBlk) void k_p1_scatter(const uint32_t* __restrict__ w0, uint64_t n, uint32_t b1,
                                                    uint32_t nblk, const uint32_t* __restrict__ H,
                                                    const uint32_t* __restrict__ pstart,
                                                    uint2* __restrict__ tmp) {
    extern __shared__ uint32_t sh[];   // [rank counters 2^b1 | base 2^b1]
    const uint32_t nbin = 1u << b1, shift = 32 - b1;
    uint32_t* cnt = sh;
    uint32_t* bb = sh + nbin;
    for (uint32_t i = threadIdx.x; i < nbin; i += kBlk) {
        cnt[i] = 0;
        bb[i] = pstart[i] + H[(uint64_t)i * nblk + blockIdx.x];
    }
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kP1Tile;
    const uint32_t m = (uint32_t)(n - base < kP1Tile ? n - base : kP1Tile);
    for (uint32_t e = threadIdx.x * 4; e < m; e += kBlk * 4) {
        uint32_t v[4];
        if (e + 3 < m) {
            const uint4 x = *reinterpret_cast<const uint4*>(w0 + base + e);
            v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
        } else {
            for (uint32_t f = 0; f < 4; ++f) v[f] = e + f < m ? w0[base + e + f] : 0;
        }
#pragma unroll
        for (uint32_t f = 0; f < 4; ++f) {
            if (e + f >= m) break;
            const uint32_t d = v[f] >> shift;
            tmp[bb[d] + atomicAdd(cnt + d, 1u)] = make_uint2(v[f], (uint32_t)(base + e + f));
        }
    }
}

__global__ __launch_bounds__(kP2Blk) void k_p2_buckets(const uint2* __restrict__ tmp,
                                                      const uint32_t* __restrict__ pstart, uint32_t b1,
                                                      uint32_t b2, uint32_t perm_cap, uint32_t* __restrict__ dir,
                                                      uint2* __restrict__ pairs, uint64_t n) {
    extern __shared__ uint32_t sh[];   // [cnt 2^b2 | offsets 2^b2 | scan scratch 1024 | perm]
    const uint32_t p = blockIdx.x;
    const uint32_t nsub = 1u << b2, shift = 32 - b1 - b2, mask = nsub - 1u;
    uint32_t* cnt = sh;
    uint32_t* off = sh + nsub;
    uint32_t* scr = sh + 2 * nsub;
    uint32_t* perm = scr + 1024;
    const uint32_t lo = pstart[p], hi = pstart[p + 1], m = hi - lo;
    for (uint32_t i = threadIdx.x; i < nsub; i += kP2Blk) cnt[i] = 0;
    __syncthreads();
    for (uint32_t i = lo + threadIdx.x; i < hi; i += kP2Blk) atomicAdd(cnt + ((tmp[i].x >> shift) & mask), 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nsub; i += kP2Blk) off[i] = cnt[i];
    __syncthreads();
    block_scan_inplace(off, nsub, scr);
    for (uint32_t i = threadIdx.x; i < nsub; i += kP2Blk) {
        dir[((uint64_t)p << b2) + i] = lo + off[i];
        cnt[i] = 0;
    }
    if (p == gridDim.x - 1 && threadIdx.x == 0) dir[(uint64_t)gridDim.x << b2] = (uint32_t)n;
    __syncthreads();
    if (m <= perm_cap) {
        // bucket permutation in LDS, then a gather (reads inside the partition's L2-resident
        // slice) with coalesced writes
        for (uint32_t j = threadIdx.x; j < m; j += kP2Blk) {
            const uint32_t s = (tmp[lo + j].x >> shift) & mask;
            perm[off[s] + atomicAdd(cnt + s, 1u)] = j;
        }
        __syncthreads();
        for (uint32_t j = threadIdx.x; j < m; j += kP2Blk) pairs[lo + j] = tmp[lo + perm[j]];
    } else {
        for (uint32_t i = lo + threadIdx.x; i < hi; i += kP2Blk) {
            const uint2 a = tmp[i];
            const uint32_t s = (a.x >> shift) & mask;
            pairs[lo + off[s] + atomicAdd(cnt + s, 1u)] = a;
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
// lane-distributed result list at slots [base, base + take).
__device__ void select_range(const uint2* __restrict__ pairs, uint32_t lo, uint32_t hi,
                             const uint32_t* __restrict__ planes, uint64_t stride, const uint32_t* t,
                             uint32_t take, uint32_t base, uint32_t lane, uint32_t& res) {
    const uint32_t m = hi - lo;
    if (m <= 64) {
        const Cand mine = lane < m ? load_cand(pairs, lo + lane, t[0]) : cand_none();
        uint32_t rank = 0;
        for (uint32_t o = 0; o < m; ++o) {
            const Cand other = cand_readlane(mine, o);
            if (other.d0 < mine.d0) ++rank;
            else if (other.d0 == mine.d0 && o != lane && lane < m) rank += cand_less(other, mine, planes, stride, t);
        }
        const bool keep = lane < m && rank < take;
        uint64_t km = __ballot(keep);
        while (km) {
            const uint32_t l = (uint32_t)__ffsll((long long)km) - 1;
            km &= km - 1;
            const uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)rank, l);
            const uint32_t id = (uint32_t)__builtin_amdgcn_readlane((int)mine.idx, l);
            if (lane == base + r) res = id;
        }
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
    const uint32_t lane = lane_id();
    const uint32_t qi = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
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
            select_range(pairs, tlo, thi, planes, stride, t, need, got, lane, res);
            got += need;
            break;
        }
        // subtree big but its t-side child (level lp + 1) holds < need ids: take the child
        // whole (every id in it is closer than the rest), continue in the sibling subtree
        const uint32_t clo = (uint32_t)__builtin_amdgcn_readlane((int)lo, x);
        const uint32_t chi = (uint32_t)__builtin_amdgcn_readlane((int)hi, x);
        if (chi > clo) select_range(pairs, clo, chi, planes, stride, t, chi - clo, got, lane, res);
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
    // partitions of ~2^14 ids so that a partition's bucket permutation fits LDS
    uint32_t lg = 0;
    while (lg < 63 && (1ull << lg) < n) ++lg;
    int x = (int)lg - 14;
    if (x < (int)B - 12) x = (int)B - 12;   // b2 <= 12
    if (x > 12) x = 12;
    if (x < 1) x = 1;
    if (x > (int)B) x = (int)B;
    b1 = (uint32_t)x;
    b2 = B - b1;
}

static uint32_t p1_blocks(uint64_t n) { return (uint32_t)((n + kP1Tile - 1) / kP1Tile); }

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
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)k_p2_buckets, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax);
        attr_set = true;
    }
    if (ev) (void)hipEventRecord(ev[0], s);
    if (n) {
        k_p0_hist<<<nblk, kBlk, np * 4, s>>>(planes, n, b1, nblk, H);
        if (ev) (void)hipEventRecord(ev[1], s);
        k_p0_rowscan<<<(uint32_t)np, 1024, 0, s>>>(H, nblk, pcount);
    } else {
        if (ev) (void)hipEventRecord(ev[1], s);
        hipError_t e = hipMemsetAsync(pcount, 0, np * 4, s);
        if (e != hipSuccess) return e;
    }
    k_p0_scan<<<1, 1024, 0, s>>>(pcount, (uint32_t)np, pstart, n);
    if (ev) (void)hipEventRecord(ev[2], s);
    if (n) k_p1_scatter<<<nblk, kBlk, np * 8, s>>>(planes, n, b1, nblk, H, pstart, tmp);
    if (ev) (void)hipEventRecord(ev[3], s);
    // LDS: fixed part + a permutation sized ~3x the average partition (cap: 160 KB)
    const uint32_t fixed = ((2u << b2) + 1024) * 4;
    uint64_t cap = 3 * ((n >> b1) + 1) + 1024;
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
