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
// K4 (index build) is a counting sort of the ids by their top B bits into 32-byte records
// {w0..w4, index, pad} plus the 2^B + 1 entry prefix directory (two LDS-histogram passes,
// see below).  Order inside a bucket is irrelevant: candidates are ranked by (distance,
// index).
#include "dhtgpu_dev.h"
#include "dhtgpu_internal.h"

namespace dhtgpu {
namespace {

constexpr int kBlk = 256;

// Two-pass partition by the top B = b1 + b2 bits (b1, b2 <= 12), all histograms in LDS:
//   P0  histogram of the top b1 bits (LDS per block, one global add per bin per block)
//   P0s exclusive scan of the 2^b1 partition counts (one block)
//   P1  scatter every id into its b1-partition: tmp record {w0..w4, idx, 0, 0} + tmp w0
//   P2  one block per partition: LDS histogram of the next b2 bits, directory entries for
//       the partition's 2^b2 buckets, scatter of the records into bucket order.
// Positions inside a (block, bin) come from LDS atomics, so order inside a bucket is
// arbitrary; queries rank candidates by (distance, index), so results do not depend on it.
constexpr uint32_t kP1Tile = 4096;   // ids per P0/P1 block (256 threads x 16)

__global__ __launch_bounds__(kBlk) void k_p0_hist(const uint32_t* __restrict__ w0, uint64_t n, uint32_t b1,
                                                 uint32_t* __restrict__ pcount) {
    extern __shared__ uint32_t sh[];
    const uint32_t nbin = 1u << b1, shift = 32 - b1;
    for (uint32_t i = threadIdx.x; i < nbin; i += kBlk) sh[i] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kP1Tile;
    for (uint32_t e = threadIdx.x; e < kP1Tile; e += kBlk)
        if (base + e < n) atomicAdd(sh + (w0[base + e] >> shift), 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nbin; i += kBlk)
        if (sh[i]) atomicAdd(pcount + i, sh[i]);
}

__global__ __launch_bounds__(1024) void k_p0_scan(const uint32_t* __restrict__ pcount, uint32_t nbin,
                                                 uint32_t* __restrict__ pstart, uint32_t* __restrict__ pcursor,
                                                 uint64_t n) {
    __shared__ uint32_t sh[1024];
    uint32_t carry = 0;
    for (uint32_t b = 0; b < nbin; b += 1024) {
        const uint32_t i = b + threadIdx.x;
        const uint32_t v = i < nbin ? pcount[i] : 0;
        sh[threadIdx.x] = v;
        __syncthreads();
        for (uint32_t off = 1; off < 1024; off <<= 1) {
            const uint32_t x = threadIdx.x >= off ? sh[threadIdx.x - off] : 0;
            __syncthreads();
            sh[threadIdx.x] += x;
            __syncthreads();
        }
        if (i < nbin) {
            pstart[i] = carry + sh[threadIdx.x] - v;
            pcursor[i] = carry + sh[threadIdx.x] - v;
        }
        carry += sh[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) pstart[nbin] = (uint32_t)n;
}

__global__ __launch_bounds__(kBlk) void k_p1_scatter(const uint32_t* __restrict__ planes, uint64_t stride,
                                                    uint64_t n, uint32_t b1, uint32_t* __restrict__ pcursor,
                                                    uint4* __restrict__ tmp, uint32_t* __restrict__ tmpw0) {
    extern __shared__ uint32_t sh[];   // [cnt 2^b1 | base 2^b1]
    const uint32_t nbin = 1u << b1, shift = 32 - b1;
    uint32_t* cnt = sh;
    uint32_t* bb = sh + nbin;
    for (uint32_t i = threadIdx.x; i < nbin; i += kBlk) cnt[i] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kP1Tile;
    constexpr uint32_t PER = kP1Tile / kBlk;
    uint32_t d[PER];
#pragma unroll
    for (uint32_t e = 0; e < PER; ++e) {
        const uint64_t i = base + e * kBlk + threadIdx.x;
        d[e] = i < n ? planes[i] >> shift : DHT_NONE;
        if (i < n) atomicAdd(cnt + d[e], 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nbin; i += kBlk) {
        const uint32_t c = cnt[i];
        bb[i] = c ? atomicAdd(pcursor + i, c) : 0;
        cnt[i] = 0;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t e = 0; e < PER; ++e) {
        const uint64_t i = base + e * kBlk + threadIdx.x;
        if (i >= n) continue;
        const uint32_t pos = bb[d[e]] + atomicAdd(cnt + d[e], 1u);
        uint32_t w[DHT_W];
        load_id(planes, stride, i, w);
        tmp[2 * (uint64_t)pos] = make_uint4(w[0], w[1], w[2], w[3]);
        tmp[2 * (uint64_t)pos + 1] = make_uint4(w[4], (uint32_t)i, 0u, 0u);
        tmpw0[pos] = w[0];
    }
}

constexpr int kP2Blk = 1024;

__global__ __launch_bounds__(kP2Blk) void k_p2_buckets(const uint4* __restrict__ tmp,
                                                      const uint32_t* __restrict__ tmpw0,
                                                      const uint32_t* __restrict__ pstart, uint32_t b1,
                                                      uint32_t b2, uint32_t* __restrict__ dir,
                                                      uint4* __restrict__ rec, uint64_t n) {
    extern __shared__ uint32_t sh[];   // [cnt 2^b2 | offsets 2^b2 | scan scratch 1024]
    const uint32_t p = blockIdx.x;
    const uint32_t nsub = 1u << b2, shift = 32 - b1 - b2, mask = nsub - 1u;
    uint32_t* cnt = sh;
    uint32_t* off = sh + nsub;
    uint32_t* scr = sh + 2 * nsub;
    const uint32_t lo = pstart[p], hi = pstart[p + 1];
    for (uint32_t i = threadIdx.x; i < nsub; i += kP2Blk) cnt[i] = 0;
    __syncthreads();
    for (uint32_t i = lo + threadIdx.x; i < hi; i += kP2Blk) atomicAdd(cnt + ((tmpw0[i] >> shift) & mask), 1u);
    __syncthreads();
    // exclusive scan of cnt -> off (chunks of 1024 with carry)
    uint32_t carry = 0;
    for (uint32_t b = 0; b < nsub; b += kP2Blk) {
        const uint32_t i = b + threadIdx.x;
        const uint32_t v = i < nsub ? cnt[i] : 0;
        scr[threadIdx.x] = v;
        __syncthreads();
        for (uint32_t o = 1; o < kP2Blk; o <<= 1) {
            const uint32_t x = threadIdx.x >= o ? scr[threadIdx.x - o] : 0;
            __syncthreads();
            scr[threadIdx.x] += x;
            __syncthreads();
        }
        if (i < nsub) {
            off[i] = carry + scr[threadIdx.x] - v;
            dir[((uint64_t)p << b2) + i] = lo + carry + scr[threadIdx.x] - v;
            cnt[i] = 0;
        }
        carry += scr[kP2Blk - 1];
        __syncthreads();
    }
    if (p == gridDim.x - 1 && threadIdx.x == 0) dir[(uint64_t)gridDim.x << b2] = (uint32_t)n;
    for (uint32_t i = lo + threadIdx.x; i < hi; i += kP2Blk) {
        const uint4 a = tmp[2 * (uint64_t)i], b = tmp[2 * (uint64_t)i + 1];
        const uint32_t s = (a.x >> shift) & mask;
        const uint32_t pos = lo + off[s] + atomicAdd(cnt + s, 1u);
        rec[2 * (uint64_t)pos] = a;
        rec[2 * (uint64_t)pos + 1] = b;
    }
}

// ---------------------------------------------------------------------------------
// K5: one wave per target.
// Candidate key = (w0^t0, .., w4^t4, idx); lexicographic; strict total order.
// ---------------------------------------------------------------------------------
struct Key {
    uint32_t d[5];
    uint32_t idx;
};

__device__ __forceinline__ bool key_less(const Key& a, const Key& b) {
#pragma unroll
    for (int j = 0; j < 5; ++j)
        if (a.d[j] != b.d[j]) return a.d[j] < b.d[j];
    return a.idx < b.idx;
}

__device__ __forceinline__ Key key_none() {
    Key k;
#pragma unroll
    for (int j = 0; j < 5; ++j) k.d[j] = DHT_NONE;
    k.idx = DHT_NONE;
    return k;
}

__device__ __forceinline__ Key key_readlane(const Key& a, uint32_t l) {
    Key k;
#pragma unroll
    for (int j = 0; j < 5; ++j) k.d[j] = (uint32_t)__builtin_amdgcn_readlane((int)a.d[j], l);
    k.idx = (uint32_t)__builtin_amdgcn_readlane((int)a.idx, l);
    return k;
}

__device__ __forceinline__ Key load_key(const uint4* __restrict__ rec, uint32_t pos, const uint32_t* t) {
    const uint4 a = rec[2 * (uint64_t)pos], b = rec[2 * (uint64_t)pos + 1];
    Key k;
    k.d[0] = a.x ^ t[0];
    k.d[1] = a.y ^ t[1];
    k.d[2] = a.z ^ t[2];
    k.d[3] = a.w ^ t[3];
    k.d[4] = b.x ^ t[4];
    k.idx = b.y;
    return k;
}

// Append the `take` closest ids of records [lo, hi) (ascending) to the lane-distributed
// result list at slots [base, base + take).  Exact: ranks among the range by key.
__device__ void select_range(const uint4* __restrict__ rec, uint32_t lo, uint32_t hi, const uint32_t* t,
                             uint32_t take, uint32_t base, uint32_t lane, uint32_t& res) {
    const uint32_t m = hi - lo;
    if (m <= 64) {
        const Key mine = lane < m ? load_key(rec, lo + lane, t) : key_none();
        uint32_t rank = 0;
        for (uint32_t o = 0; o < m; ++o) {
            const Key other = key_readlane(mine, o);
            rank += key_less(other, mine);
        }
        // lane with rank r (< take) owns result slot base + r: route its idx there
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
    // large range (clustered inputs): running lane-distributed top-`take` list, filled by
    // serial insertion of the candidates that beat the current take-th key
    Key ent = key_none();
    uint32_t cnt = 0;
    for (uint32_t c = lo; c < hi; c += 64) {
        const bool v = c + lane < hi;
        const Key mine = v ? load_key(rec, c + lane, t) : key_none();
        Key worst = cnt == take ? key_readlane(ent, take - 1) : key_none();
        uint64_t cm = __ballot(v && (cnt < take || key_less(mine, worst)));
        while (cm) {
            const uint32_t l = (uint32_t)__ffsll((long long)cm) - 1;
            cm &= cm - 1;
            const Key cand = key_readlane(mine, l);
            if (cnt == take && !key_less(cand, worst)) continue;
            const bool closer = lane < cnt && key_less(ent, cand);
            const uint32_t pos = (uint32_t)__popcll(__ballot(closer));
            Key up;
#pragma unroll
            for (int j = 0; j < 5; ++j) up.d[j] = __shfl_up(ent.d[j], 1);
            up.idx = __shfl_up(ent.idx, 1);
            if (lane == pos) ent = cand;
            else if (lane > pos) ent = up;
            cnt = cnt + 1 < take ? cnt + 1 : take;
            worst = cnt == take ? key_readlane(ent, take - 1) : key_none();
        }
    }
    // move the list into result slots [base, base + cnt)
    const uint32_t idx_src = __shfl(ent.idx, (int)(lane >= base ? lane - base : 0));
    if (lane >= base && lane < base + cnt) res = idx_src;
}

__global__ __launch_bounds__(256) void k_query(const uint4* __restrict__ rec, const uint32_t* __restrict__ dir,
                                              uint32_t B, uint64_t n, const uint32_t* __restrict__ tp, uint64_t ts,
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
            select_range(rec, tlo, thi, t, need, got, lane, res);
            got += need;
            break;
        }
        // subtree big but its t-side child (level lp + 1) holds < need ids: take the child
        // whole (every id in it is closer than the rest), continue in the sibling subtree
        const uint32_t clo = (uint32_t)__builtin_amdgcn_readlane((int)lo, x);
        const uint32_t chi = (uint32_t)__builtin_amdgcn_readlane((int)hi, x);
        if (chi > clo) select_range(rec, clo, chi, t, chi - clo, got, lane, res);
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

static void index_split(uint32_t B, uint32_t& b1, uint32_t& b2) {
    b2 = B / 2 < 12 ? B / 2 : 12;
    b1 = B - b2;   // index_bits() caps B at 24, so b1 <= 12 and every LDS histogram fits 64 KB
}

// workspace: rec (n x 32 B) | dir (2^B + 1) | tmp (n x 32 B) | tmpw0 (n) | pcount | pstart | pcursor
size_t index_bytes(uint64_t n, uint32_t B) {
    uint32_t b1, b2;
    index_split(B, b1, b2);
    const uint64_t nb = 1ull << B, np = 1ull << b1;
    return (size_t)n * 32 * 2 + (size_t)n * 4 + (nb + 1) * 4 + (3 * np + 1) * 4 + 1024;
}

hipError_t launch_index_build(const uint32_t* planes, uint64_t stride, uint64_t n, uint32_t B, void* ws,
                              hipStream_t s) {
    uint32_t b1, b2;
    index_split(B, b1, b2);
    const uint64_t nb = 1ull << B, np = 1ull << b1;
    uint8_t* base = static_cast<uint8_t*>(ws);
    uint4* rec = reinterpret_cast<uint4*>(base);
    uint32_t* dir = reinterpret_cast<uint32_t*>(base + (size_t)n * 32);
    uint4* tmp = reinterpret_cast<uint4*>(base + (((size_t)n * 32 + (nb + 1) * 4 + 15) & ~size_t(15)));
    uint32_t* tmpw0 = reinterpret_cast<uint32_t*>(tmp + 2 * n);
    uint32_t* pcount = tmpw0 + n;
    uint32_t* pstart = pcount + np;
    uint32_t* pcursor = pstart + np + 1;
    hipError_t e = hipMemsetAsync(pcount, 0, np * 4, s);
    if (e != hipSuccess) return e;
    const uint32_t tiles = (uint32_t)((n + kP1Tile - 1) / kP1Tile);
    if (n) k_p0_hist<<<tiles, kBlk, np * 4, s>>>(planes, n, b1, pcount);
    k_p0_scan<<<1, 1024, 0, s>>>(pcount, (uint32_t)np, pstart, pcursor, n);
    if (n) k_p1_scatter<<<tiles, kBlk, np * 8, s>>>(planes, stride, n, b1, pcursor, tmp, tmpw0);
    k_p2_buckets<<<(uint32_t)np, kP2Blk, ((2u << b2) + kP2Blk) * 4, s>>>(tmp, tmpw0, pstart, b1, b2, dir, rec, n);
    return hipGetLastError();
}

hipError_t launch_index_query(const void* ws, uint64_t n, uint32_t B, const uint32_t* tp, uint64_t ts,
                              uint32_t q, uint32_t k, uint32_t* out_idx, uint32_t* out_cnt, hipStream_t s) {
    if (!q) return hipSuccess;
    const uint8_t* base = static_cast<const uint8_t*>(ws);
    const uint4* rec = reinterpret_cast<const uint4*>(base);
    const uint32_t* dir = reinterpret_cast<const uint32_t*>(base + (size_t)n * 32);
    k_query<<<(q + 3) / 4, 256, 0, s>>>(rec, dir, B, n, tp, ts, q, k, out_idx, out_cnt);
    return hipGetLastError();
}

}  // namespace dhtgpu
