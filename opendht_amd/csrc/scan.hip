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
            // two lists' heads agree on both distance words (the same index or not: lists built
            // with colliding indices must not be taken for duplicates without the full key)
            tie = tie || (p0 == m0 && p1 == m1 && pi != DHT_NONE && mi != DHT_NONE);
            const bool less = p0 < m0 || (p0 == m0 && (p1 < m1 || (p1 == m1 && pi < mi)));
            if (less) { m0 = p0; m1 = p1; mi = pi; }
        }
        const uint64_t gmask = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << (g * G);
        bool adv = h0 == m0 && h1 == m1 && hi == mi;
        if (__ballot(tie) & gmask) {
            // the group minimum by the full key (words 2..4 from the records), then by index
            uint32_t f[DHT_W + 1], own[DHT_W + 1];
            own[0] = h0; own[1] = h1; own[DHT_W] = hi;
            for (int w = 2; w < DHT_W; ++w)
                own[w] = hi == DHT_NONE ? DHT_NONE : src[p * 6 + w] ^ tp[(uint64_t)w * ts + qc];
            for (int w = 0; w <= DHT_W; ++w) f[w] = own[w];
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
            adv = true;   // advance every list whose head IS the winner: the same id and index
            for (int w = 0; w <= DHT_W; ++w) adv = adv && own[w] == f[w];
        }
        if (mi == DHT_NONE) continue;   // this target's lists are exhausted (group-uniform)
        if (tv && j == 0) out_idx[(uint64_t)qi * k + r] = mi;
        ++cnt;
        if (adv && lv) {   // the winning list advances (and every list holding the same record)
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

// ---- compact candidate records (the public record form, include/dhtgpu.h) --------------------
// rec[i] = {w0, w1, global idx} of local index idx[i] (12 B; all DHT_NONE for an empty slot): two
// 4-B reads per candidate from the w0 / w1 planes, which a cfg-2-sized set keeps in the Infinity
// Cache (the 24-B form's words 2..4 came from a 400 MB copy of the set, i.e. from HBM: 17 us per
// 65,536 x 8 records).  The global index is gidx[x] (nullable map) or x + base.
__global__ __launch_bounds__(256) void k_rec3(const uint32_t* __restrict__ idx, uint64_t m,
                                              const uint32_t* __restrict__ planes, uint64_t stride, uint32_t base,
                                              const uint32_t* __restrict__ gidx, uint32_t* __restrict__ rec) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    const uint32_t x = idx[i];
    const bool none = x == DHT_NONE;
    const uint32_t xc = none ? 0u : x;
    const uint32_t w0 = planes[xc], w1 = planes[stride + xc];
    rec[i * 3] = none ? DHT_NONE : w0;
    rec[i * 3 + 1] = none ? DHT_NONE : w1;
    rec[i * 3 + 2] = none ? DHT_NONE : (gidx ? gidx[xc] : x + base);
}

// K3 over compact records: the heads merge of k_merge_heads on (w0 ^ t0, w1 ^ t1, idx).  When two
// lists' heads agree on both distance words -- two different ids sharing their first 64 bits, or
// the same id sent by two lists -- the records cannot order them: the row's answer (ordered by
// index there) is provisional, and the row is appended to ties = {count, rows[cap]} (nullable when
// lists == 1: one list is already in order) for the second exchange (words 2..4) and
// k_merge_full.  Hash-distributed ids never share 64 bits among one target's candidates.
template <uint32_t G>
__global__ __launch_bounds__(kMergeThreads) void k_merge3(const uint32_t* __restrict__ rec, uint32_t lists, uint32_t q,
                                                          uint32_t kin, const uint32_t* __restrict__ tp, uint64_t ts,
                                                          uint32_t k, uint32_t* __restrict__ out_idx,
                                                          uint32_t* __restrict__ out_cnt, uint32_t* __restrict__ ties,
                                                          uint32_t tie_cap) {
    extern __shared__ uint32_t sm[];   // [list][block target][kin][3]: the block's records as stored
    constexpr uint32_t TPW = 64 / G, T = (kMergeThreads / 64) * TPW;   // targets per block
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    const uint32_t g = lane / G, j = lane % G;
    const uint32_t qb = blockIdx.x * T, tl = wv * TPW + g;
    const uint32_t qi = qb + tl;
    const bool tv = qi < q, lv = tv && j < lists;
    const uint32_t qc = tv ? qi : 0u;
    const uint32_t t0 = tp[qc], t1 = tp[ts + qc];
    // the block's targets' records are one contiguous run per list: copied by all threads with
    // consecutive lanes on consecutive words (a thread reading its own 12-B records strode 96 B
    // across the wave), then read from LDS
    const uint32_t nt = q - qb < T ? q - qb : T, run = nt * kin * 3;
    for (uint32_t l = 0; l < lists; ++l) {
        const uint32_t* src = rec + ((uint64_t)l * q + qb) * kin * 3;
        uint32_t* dst = sm + l * T * kin * 3;
        for (uint32_t w = threadIdx.x; w < run; w += kMergeThreads) dst[w] = src[w];
    }
    __syncthreads();
    const uint32_t* my = sm + ((lv ? j : 0u) * T + (tv ? tl : 0u)) * kin * 3;
    auto head = [&](uint32_t p, uint32_t& a, uint32_t& b, uint32_t& ix) {
        ix = lv && p < kin ? my[3 * p + 2] : DHT_NONE;
        const bool none = ix == DHT_NONE;
        a = none ? DHT_NONE : my[3 * p] ^ t0;
        b = none ? DHT_NONE : my[3 * p + 1] ^ t1;
    };
    if (G == 1 && k == 8 && ((uintptr_t)out_idx & 15) == 0) {
        // one list (G = 1): the list is the answer, in order up to its first empty slot -- the row
        // as two 16-B stores (the merge loop's eight dword stores per lane strode 32 B across the
        // wave: 30 us for 2^20 rows at the cfg-3 broadcast rank)
        if (!tv) return;
        uint32_t row[8], cnt = 0;
        bool stop = false;
#pragma unroll
        for (uint32_t r = 0; r < 8; ++r) {
            const uint32_t ix = r < kin && lv ? my[3 * r + 2] : DHT_NONE;
            stop = stop || ix == DHT_NONE;
            row[r] = stop ? DHT_NONE : ix;
            cnt += stop ? 0u : 1u;
        }
        uint4* o = reinterpret_cast<uint4*>(out_idx + (uint64_t)qi * 8);
        o[0] = make_uint4(row[0], row[1], row[2], row[3]);
        o[1] = make_uint4(row[4], row[5], row[6], row[7]);
        out_cnt[qi] = cnt;
        return;
    }
    const uint64_t gmask = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << (g * G);
    uint32_t p = 0, cnt = 0;
    uint32_t h0, h1, hi;
    head(0, h0, h1, hi);
    bool row_tie = false;
    if (k == 8 && ((uintptr_t)out_idx & 15) == 0) {
        // k = 8: the row kept in registers and stored as two 16-B stores by the group's lane 0
        // (the loop below stores one dword per place: a 32-B stride across the wave)
        uint32_t row[8];
#pragma unroll
        for (uint32_t r = 0; r < 8; ++r) {
            uint32_t m0 = h0, m1 = h1, mi = hi;
            bool tie = false;
#pragma unroll
            for (uint32_t o = 1; o < G; o <<= 1) {
                const uint32_t p0 = (uint32_t)__shfl_xor((int)m0, (int)o), p1 = (uint32_t)__shfl_xor((int)m1, (int)o);
                const uint32_t pi = (uint32_t)__shfl_xor((int)mi, (int)o);
                tie = tie || (p0 == m0 && p1 == m1 && pi != DHT_NONE && mi != DHT_NONE);
                const bool less = p0 < m0 || (p0 == m0 && (p1 < m1 || (p1 == m1 && pi < mi)));
                if (less) { m0 = p0; m1 = p1; mi = pi; }
            }
            row_tie = row_tie || (__ballot(tie) & gmask) != 0;
            row[r] = mi;   // DHT_NONE once the target's lists are exhausted (then every later place)
            cnt += mi != DHT_NONE ? 1u : 0u;
            if (mi != DHT_NONE && lv && h0 == m0 && h1 == m1 && hi == mi) head(++p, h0, h1, hi);
        }
        if (tv && j == 0) {
            uint4* o = reinterpret_cast<uint4*>(out_idx + (uint64_t)qi * 8);
            o[0] = make_uint4(row[0], row[1], row[2], row[3]);
            o[1] = make_uint4(row[4], row[5], row[6], row[7]);
            out_cnt[qi] = cnt;
            if (row_tie && ties) {
                const uint32_t s = atomicAdd(ties, 1u);
                if (s < tie_cap) ties[1 + s] = qi;
            }
        }
        return;
    }
    for (uint32_t r = 0; r < k; ++r) {   // wave-uniform
        uint32_t m0 = h0, m1 = h1, mi = hi;
        bool tie = false;
#pragma unroll
        for (uint32_t o = 1; o < G; o <<= 1) {
            const uint32_t p0 = (uint32_t)__shfl_xor((int)m0, (int)o), p1 = (uint32_t)__shfl_xor((int)m1, (int)o);
            const uint32_t pi = (uint32_t)__shfl_xor((int)mi, (int)o);
            tie = tie || (p0 == m0 && p1 == m1 && pi != DHT_NONE && mi != DHT_NONE);
            const bool less = p0 < m0 || (p0 == m0 && (p1 < m1 || (p1 == m1 && pi < mi)));
            if (less) { m0 = p0; m1 = p1; mi = pi; }
        }
        row_tie = row_tie || (__ballot(tie) & gmask) != 0;
        if (mi == DHT_NONE) continue;   // this target's lists are exhausted (group-uniform)
        if (tv && j == 0) out_idx[(uint64_t)qi * k + r] = mi;
        ++cnt;
        if (lv && h0 == m0 && h1 == m1 && hi == mi) head(++p, h0, h1, hi);
    }
    if (tv && j == 0) {
        for (uint32_t r = cnt; r < k; ++r) out_idx[(uint64_t)qi * k + r] = DHT_NONE;
        out_cnt[qi] = cnt;
        if (row_tie && ties) {
            const uint32_t s = atomicAdd(ties, 1u);
            if (s < tie_cap) ties[1 + s] = qi;
        }
    }
}

// words 2..4 of this rank's candidates in the rows listed by ties = {count, rows[cap]} (rows offset
// by row_base: an all-to-all slice), or of every row when ties == nullptr: words[(slot * k + r) * 3
// + {0, 1, 2}].  A record's global index maps back to the set's local index through the sorted
// index map gmap (prefix shards; nullable) or by subtracting base.
__global__ __launch_bounds__(256) void k_tie_words(const uint32_t* __restrict__ rec, uint32_t q, uint32_t k,
                                                   const uint32_t* __restrict__ ties, uint32_t tie_cap,
                                                   uint32_t row_base, const uint32_t* __restrict__ planes,
                                                   uint64_t stride, uint64_t n, const uint32_t* __restrict__ gmap,
                                                   uint32_t base, uint32_t* __restrict__ words) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t slot = i / k, r = i % k;
    const uint64_t nrows = ties ? (ties[0] < tie_cap ? ties[0] : tie_cap) : q;
    if (slot >= nrows) return;
    const uint64_t row = ties ? (uint64_t)ties[1 + slot] + row_base : slot;
    const uint32_t gi = row < q ? rec[(row * k + r) * 3 + 2] : DHT_NONE;
    uint32_t* o = words + (slot * k + r) * 3;
    uint64_t x = n;
    if (gi != DHT_NONE) {
        if (gmap) {   // lower_bound in the ascending map
            uint64_t lo = 0, hi = n;
            while (lo < hi) {
                const uint64_t mid = (lo + hi) >> 1;
                if (gmap[mid] < gi) lo = mid + 1; else hi = mid;
            }
            x = lo < n && gmap[lo] == gi ? lo : n;
        } else if (gi >= base) {
            x = gi - base;
        }
    }
    const bool ok = x < n;
#pragma unroll
    for (int w = 0; w < 3; ++w) o[w] = ok ? planes[(uint64_t)(2 + w) * stride + x] : DHT_NONE;
}

// The listed rows (or every row when ties == nullptr) merged again by the full key: list j's
// candidate r of the row is {rec: w0, w1, idx} + {words: w2, w3, w4} (words rows: the tie slots,
// wrows per list), each list already ascending by the full distance.  Lanes whose head equals the
// winner in all five words and the index advance together (the same id sent twice); different ids
// with colliding indices are both kept, ordered by distance.
template <uint32_t G>
__global__ __launch_bounds__(256) void k_merge_full(const uint32_t* __restrict__ rec, const uint32_t* __restrict__ words,
                                                    uint32_t lists, uint32_t q, uint32_t kin, uint32_t wrows,
                                                    const uint32_t* __restrict__ tp, uint64_t ts, uint32_t k,
                                                    const uint32_t* __restrict__ ties, uint32_t tie_cap,
                                                    uint32_t* __restrict__ out_idx, uint32_t* __restrict__ out_cnt) {
    constexpr uint32_t TPW = 64 / G;
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    const uint32_t g = lane / G, j = lane % G;
    const uint32_t slot = (blockIdx.x * 4 + wv) * TPW + g;
    const uint32_t nrows = ties ? (ties[0] < tie_cap ? ties[0] : tie_cap) : q;
    const bool tv = slot < nrows;
    const uint32_t row = tv ? (ties ? ties[1 + slot] : slot) : 0u;
    const bool lv = tv && j < lists && row < q;
    uint32_t t[DHT_W];
    for (int w = 0; w < DHT_W; ++w) t[w] = tp[(uint64_t)w * ts + row];
    auto head = [&](uint32_t p, uint32_t* f) {
        const bool in = lv && p < kin;   // every address below stays inside the buffers
        const uint64_t jc = in ? j : 0u, rc = in ? row : 0u, sc = in ? slot : 0u, pc = in ? p : 0u;
        const uint32_t* r3 = rec + ((jc * q + rc) * kin + pc) * 3;
        const uint32_t* w3 = words + ((jc * wrows + sc) * kin + pc) * 3;
        uint32_t v[DHT_W + 1] = {r3[0], r3[1], w3[0], w3[1], w3[2], r3[2]};
        const bool none = !in || v[DHT_W] == DHT_NONE;
        for (int w = 0; w < DHT_W; ++w) f[w] = none ? DHT_NONE : v[w] ^ t[w];
        f[DHT_W] = none ? DHT_NONE : v[DHT_W];
    };
    uint32_t h[DHT_W + 1], p = 0, cnt = 0;
    head(0, h);
    for (uint32_t r = 0; r < k; ++r) {
        uint32_t f[DHT_W + 1];
        for (int w = 0; w <= DHT_W; ++w) f[w] = h[w];
#pragma unroll
        for (uint32_t o = 1; o < G; o <<= 1) {
            uint32_t pf[DHT_W + 1];
            for (int w = 0; w <= DHT_W; ++w) pf[w] = (uint32_t)__shfl_xor((int)f[w], (int)o);
            bool less = false, decided = false;
            for (int w = 0; w <= DHT_W; ++w)
                if (!decided && pf[w] != f[w]) { less = pf[w] < f[w]; decided = true; }
            if (less)
                for (int w = 0; w <= DHT_W; ++w) f[w] = pf[w];
        }
        if (f[DHT_W] == DHT_NONE) continue;   // group-uniform
        if (tv && j == 0) out_idx[(uint64_t)row * k + r] = f[DHT_W];
        ++cnt;
        bool adv = lv;
        for (int w = 0; w <= DHT_W; ++w) adv = adv && h[w] == f[w];
        if (adv) head(++p, h);
    }
    if (tv && j == 0) {
        for (uint32_t r = cnt; r < k; ++r) out_idx[(uint64_t)row * k + r] = DHT_NONE;
        out_cnt[row] = cnt;
    }
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

hipError_t launch_rec3(const uint32_t* idx, uint64_t m, const uint32_t* planes, uint64_t stride, uint32_t base,
                       const uint32_t* gidx, uint32_t* rec, hipStream_t s) {
    if (!m) return hipSuccess;
    k_rec3<<<(uint32_t)((m + 255) / 256), 256, 0, s>>>(idx, m, planes, stride, base, gidx, rec);
    return hipGetLastError();
}

hipError_t launch_merge3(const uint32_t* rec, uint32_t lists, uint32_t q, uint32_t kin, const uint32_t* tp,
                         uint64_t ts, uint32_t k, uint32_t* out_idx, uint32_t* out_cnt, uint32_t* ties,
                         uint32_t tie_cap, hipStream_t s) {
    if (lists > 64 || kin > 32) return hipErrorInvalidValue;
    uint32_t G = 1;
    while (G < lists) G <<= 1;
    const uint32_t tpb = (kMergeThreads / 64) * (64 / G);
    const dim3 grid((q + tpb - 1) / tpb), blk(kMergeThreads);
    const size_t lds = (size_t)kMergeThreads * kin * 3 * sizeof(uint32_t);
    static std::once_flag once[kMaxDevices];
    const hipError_t e = per_device_once(once, [] {
        const void* fs[] = {(const void*)k_merge3<1>, (const void*)k_merge3<2>, (const void*)k_merge3<4>,
                            (const void*)k_merge3<8>, (const void*)k_merge3<16>, (const void*)k_merge3<32>,
                            (const void*)k_merge3<64>};
        for (const void* f : fs) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
    });
    if (e != hipSuccess) return e;
    if (ties) {   // the tie count starts at zero for every merge
        const hipError_t z = hipMemsetAsync(ties, 0, sizeof(uint32_t), s);
        if (z != hipSuccess) return z;
    }
#define DHT_M3(GG) k_merge3<GG><<<grid, blk, lds, s>>>(rec, lists, q, kin, tp, ts, k, out_idx, out_cnt, ties, tie_cap)
    switch (G) {
        case 1: DHT_M3(1); break;
        case 2: DHT_M3(2); break;
        case 4: DHT_M3(4); break;
        case 8: DHT_M3(8); break;
        case 16: DHT_M3(16); break;
        case 32: DHT_M3(32); break;
        default: DHT_M3(64); break;
    }
#undef DHT_M3
    return hipGetLastError();
}

hipError_t launch_tie_words(const uint32_t* rec, uint32_t q, uint32_t k, const uint32_t* ties, uint32_t tie_cap,
                            uint32_t row_base, const uint32_t* planes, uint64_t stride, uint64_t n,
                            const uint32_t* gmap, uint32_t base, uint32_t* words, hipStream_t s) {
    const uint64_t m = (uint64_t)(ties ? tie_cap : q) * k;
    if (!m) return hipSuccess;
    k_tie_words<<<(uint32_t)((m + 255) / 256), 256, 0, s>>>(rec, q, k, ties, tie_cap, row_base, planes, stride, n,
                                                            gmap, base, words);
    return hipGetLastError();
}

hipError_t launch_merge_full(const uint32_t* rec, const uint32_t* words, uint32_t lists, uint32_t q, uint32_t kin,
                             const uint32_t* tp, uint64_t ts, uint32_t k, const uint32_t* ties, uint32_t tie_cap,
                             uint32_t* out_idx, uint32_t* out_cnt, hipStream_t s) {
    if (lists > 64 || kin > 32) return hipErrorInvalidValue;
    uint32_t G = 1;
    while (G < lists) G <<= 1;
    const uint32_t rows = ties ? tie_cap : q, wrows = rows;
    if (!rows) return hipSuccess;
    const uint32_t tpb = 4 * (64 / G);
    const dim3 grid((rows + tpb - 1) / tpb), blk(256);
#define DHT_MF(GG) k_merge_full<GG><<<grid, blk, 0, s>>>(rec, words, lists, q, kin, wrows, tp, ts, k, ties, tie_cap, \
                                                         out_idx, out_cnt)
    switch (G) {
        case 1: DHT_MF(1); break;
        case 2: DHT_MF(2); break;
        case 4: DHT_MF(4); break;
        case 8: DHT_MF(8); break;
        case 16: DHT_MF(16); break;
        case 32: DHT_MF(32); break;
        default: DHT_MF(64); break;
    }
#undef DHT_MF
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
