// table.hip -- routing-table kernels for gfx950.
//   K1r k_find_closest : RoutingTable::findClosestNodes (src/routing_table.cpp:110-150)
//   K2  k_classify     : RoutingTable::findBucket (:153-166) + InfoHash::commonBits
//                        (include/opendht/infohash.h:154-176) histogram
//   a8  k_cached       : NodeCache::getCachedNodes (src/node_cache.cpp:42-74)
#include "dhtgpu_dev.h"
#include "dhtgpu_internal.h"

#include <type_traits>

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
// K2.  findBucket + commonBits of every id against one table snapshot, streaming word 0
// only.  An id's bucket and its commonBits with myid follow from its word 0 alone unless
// that word equals a bucket first's word 0 or myid's; only then are words 1..4 of the id
// loaded (rare on hash-distributed ids).  Algorithmic bytes: 4 B/id read + the 1-B bucket
// written (round 3 streamed all five planes: 21 B/id).  Two ways to the bucket, chosen per
// workgroup from the firsts (block-uniform):
//   register path  (routing tables) the ids with commonBits c < kRegT form one key range per c
//               (myid's top c bits, bit c flipped); when no first lies inside such a range --
//               a first with commonBits c < kRegT sits at its range's start (the reference's
//               splits along myid's prefix, src/routing_table.cpp RoutingTable::split, put them
//               there) -- the bucket is a function of c alone: 15 bytes in four registers,
//               looked up four ids at a time with v_perm.  f = clz((w0 ^ myid w0) | 2^16)
//               gives c and the histogram field in two instructions; f = kRegT (commonBits
//               >= 15, one id in 32,768 on hashes) takes the exact path.  No table read: the
//               cell table's random LDS reads (bank conflicts) were ~0.035 of its 0.12 ms.
//   cell table  (any other sorted firsts) built in LDS by every workgroup: for each value of
//               the top kClsT bits of word 0, the bucket of the cell's first key and
//               commonBits with myid (both constant over the cell), or a flag sending the
//               cell's ids to the exact path: a bucket boundary inside the cell (the binary
//               search over the firsts' word 0, the full key on a word-0 tie -- the bucket the
//               reference's linear walk, src/routing_table.cpp:153-166, stops at), or myid's
//               own cell (commonBits >= kClsT: clz of the word-0 xor, infohash.h:154-176, all
//               five words when word 0 equals myid's).
//   histogram   per-lane 4-bit counters of bins 0..14 packed in one 64-bit word (one 64-bit
//               add per id; an exact-path id adds to field 15, discarded), spread into byte
//               counters (two 64-bit words) after every chunk (<= 4 kClsU ids per lane: no
//               overflow) and wave-reduced into the block's LDS bins every kClsFlush chunks;
//               the exact path counts with LDS atomics; one global atomic per bin per workgroup.
// Layout: a wave handles chunks of 64 x kClsU uint4 of word 0 (256 x kClsU ids), lane l the
// uint4s chunk * 64 kClsU + u * 64 + l, so every load and every 4-B bucket store of a wave is
// one contiguous 1-KB / 256-B run; the chunk index is wave-uniform (scalar address math).  The
// next two chunks' loads are issued before this chunk's work (three chunks in flight per lane).
// ---------------------------------------------------------------------------------
// one 1,024-thread workgroup per CU (16 waves, 4 per SIMD): every workgroup ends with one global
// atomic per histogram bin it touched, and the 1,024 workgroups of 256 threads ended together with
// 1,024 atomics on bin 0's address, serialised at the memory side (0.0926 -> 0.088 ms without them,
// 0.0935 -> 0.0897-0.092 with 256 workgroups of 1,024: profiles/r05/experiments/k2_blocks.txt)
constexpr int kClsBlock = 1024;
constexpr int kClsPerCu = 1;                     // workgroups per CU (16 waves per CU: 0.105 -> 0.096 ms against 32 in r04)
constexpr uint32_t kClsU = 3;                    // uint4 of word 0 per lane per chunk
static_assert(4 * kClsU <= 15, "4-bit histogram fields flushed once per chunk");
constexpr uint32_t kClsT = 10, kClsCells = 1u << kClsT;
constexpr uint32_t kClsExact = 0x8000u;          // table flag: the cell's ids take the exact path
constexpr uint32_t kClsSkip = 15u;               // histogram field an exact-path id adds to (discarded)
constexpr uint32_t kRegT = 15u;                  // register path: commonBits below this from word 0
constexpr uint32_t kClsFlush = 255u / (4 * kClsU);   // chunks per byte-counter flush
constexpr uint32_t kClsQCap = 1024;              // queued exact-path ids per wave (> one chunk's 4 * 64 * kClsU)
// k_classify's static LDS (sf, sh, lut, s_bad, s_map, s_q, s_qn below): 73 KB with the exact-path
// queues -- more than the 64 KB per workgroup of earlier CDNA parts; gfx950 gives a workgroup the
// CU's 160 KB (the Makefile builds gfx950 only)
constexpr size_t kClsLds = (size_t)DHT_W * 256 * 4 + 161 * 4 + (size_t)(1u << 10) * 2 + 4 + 16 +
                           (size_t)(kClsBlock / 64) * kClsQCap * 4 + (kClsBlock / 64) * 4;
static_assert(kClsLds <= kLdsBytes, "k_classify's LDS exceeds gfx950's 160 KB per workgroup");

// the reference's findBucket over the firsts in LDS (sf: plane-major, nb entries per plane):
// the last bucket whose first <= id, bucket 0 when none (a linear walk from the front stops
// at the same bucket); word 0 decides unless it ties
__device__ __forceinline__ uint32_t cls_find_bucket(const uint32_t* sf, uint32_t nb, const uint32_t* id) {
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
    return j;
}

// the exact path for id i (word 0 = x): {bucket, commonBits}.  Words 1..4 are loaded only when
// word 0 cannot decide.  One out-of-line copy (inlined at every unrolled id it bloated the
// loop's code ~10x).
__device__ __noinline__ uint2 cls_exact(const uint32_t* __restrict__ planes, uint64_t stride, uint64_t i, uint32_t x,
                                        const uint32_t* sf, uint32_t nb, uint32_t m0, uint32_t m1, uint32_t m2,
                                        uint32_t m3, uint32_t m4) {
    uint32_t id[DHT_W] = {x, 0u, 0u, 0u, 0u};
    bool tie = x == m0;
    for (uint32_t c = 0; c < nb && !tie; ++c) tie = sf[c] == x;
    if (tie) {
#pragma unroll
        for (int w = 1; w < DHT_W; ++w) id[w] = planes[(uint64_t)w * stride + i];
    }
    const uint32_t my[DHT_W] = {m0, m1, m2, m3, m4};
    return make_uint2(cls_find_bucket(sf, nb, id), tie ? common_bits(id, my) : (uint32_t)__clz(x ^ m0));
}

__global__ __launch_bounds__(kClsBlock) void k_classify(
    const uint32_t* __restrict__ planes, uint64_t stride, uint64_t n, uint32_t nb,
    const uint32_t* __restrict__ fp, uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3,
    uint32_t m4, uint8_t* __restrict__ out_bucket, unsigned long long* __restrict__ hist) {
    __shared__ uint32_t sf[DHT_W * 256];
    __shared__ uint32_t sh[161];
    __shared__ uint16_t lut[kClsCells];   // bucket | commonBits << 8 | kClsExact
    __shared__ uint32_t s_bad;            // a first inside a commonBits range: no register path
    __shared__ uint32_t s_map[4];         // register path: bucket of commonBits c in byte c
    // the exact path, deferred: each wave queues its exact-path ids (index) here during the
    // stream and answers them between chunks once the queue could not take another chunk's worth,
    // and at the end -- a call inside the chunk kept the chunk's ids and keys live across it (117
    // VGPRs, 4 waves per SIMD; without it 95)
    __shared__ uint32_t s_q[kClsBlock / 64][kClsQCap];
    __shared__ uint32_t s_qn[kClsBlock / 64];
    constexpr uint32_t CH = 64 * kClsU;   // uint4 per wave chunk
    constexpr uint32_t NE = 4 * kClsU;    // ids per lane per chunk
    const uint64_t n4 = (n + 3) / 4;
    const uint64_t nch = (n4 + CH - 1) / CH;
    const uint64_t nfull = n / (4 * CH);  // chunks with every id valid
    const uint32_t lane = lane_id();
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t W = (uint64_t)gridDim.x * (kClsBlock / 64);
    uint64_t c = (uint64_t)blockIdx.x * (kClsBlock / 64) + wv;
    const uint4* __restrict__ w04 = reinterpret_cast<const uint4*>(planes);
    // unconditional loads (an address past the set is clamped to its last uint4, whose ids are
    // masked): a conditional load made the compiler wait for the look-ahead chunk too (vmcnt(0)
    // at the branch join)
    // (32-bit index math: the host keeps n < 2^32, so every uint4 index, the two-chunk look-ahead included, < 2^32)
    const uint32_t last4 = (uint32_t)(n4 - 1);
    auto load = [&](uint64_t ch, uint4* v) {
        const uint32_t cb = (uint32_t)(ch * CH) + lane;
#pragma unroll
        for (uint32_t u = 0; u < kClsU; ++u) {
            const uint32_t i4 = min(cb + u * 64, last4);
            typedef unsigned int u4v __attribute__((ext_vector_type(4)));
            const u4v t = __builtin_nontemporal_load(reinterpret_cast<const u4v*>(w04) + i4);
            v[u] = make_uint4(t[0], t[1], t[2], t[3]);
        }
    };
    // the first chunk's loads ahead of the setup
    uint4 v[kClsU];
    load(c, v);
    // three chunks in flight per wave: the next two issued ahead (0.0900-0.0920 -> 0.0893-0.0896
    // ms against one ahead, profiles/r05/experiments/k2_depth.txt; 6 of the 128 VGPRs the 16 waves per CU allow)
    uint4 v2[kClsU];
    load(c + W, v2);
    for (uint32_t i = threadIdx.x; i < DHT_W * nb; i += kClsBlock) sf[i] = fp[i];
    for (uint32_t i = threadIdx.x; i < 161; i += kClsBlock) sh[i] = 0;
    if (threadIdx.x < 4) s_map[threadIdx.x] = 0u;
    if (threadIdx.x < kClsBlock / 64) s_qn[threadIdx.x] = 0u;
    if (threadIdx.x == 0) s_bad = 0u;
    __syncthreads();
    // register path test: every first with commonBits c < kRegT starts its range (the bits
    // below the flipped one, and words 1..4, zero)
    for (uint32_t j = threadIdx.x; j < nb; j += kClsBlock) {
        const uint32_t f0 = sf[j], cb = (uint32_t)__clz((f0 ^ m0) | (1u << (31 - kRegT)));
        if (cb < kRegT) {
            bool start = (f0 & ((0x80000000u >> cb) - 1u)) == 0u;
#pragma unroll
            for (int w = 1; w < DHT_W; ++w) start = start && sf[w * nb + j] == 0u;
            if (!start) s_bad = 1u;
        }
    }
    if (threadIdx.x < kRegT) {   // the bucket of each commonBits range's first key
        const uint32_t b = 0x80000000u >> threadIdx.x;
        const uint32_t key[DHT_W] = {(m0 ^ b) & ~(b - 1u), 0u, 0u, 0u, 0u};
        atomicOr(&s_map[threadIdx.x >> 2], cls_find_bucket(sf, nb, key) << (8 * (threadIdx.x & 3u)));
    }
    __syncthreads();
    const bool regs = s_bad == 0u;   // block-uniform
    const uint32_t ma = s_map[0], mb = s_map[1], mc = s_map[2], md = s_map[3];
    if (!regs) {
        const uint32_t mycell = m0 >> (32 - kClsT);
        for (uint32_t cell = threadIdx.x; cell < kClsCells; cell += kClsBlock) {
            const uint32_t key[DHT_W] = {cell << (32 - kClsT), 0u, 0u, 0u, 0u};
            const uint32_t j = cls_find_bucket(sf, nb, key);
            // the smallest first above the cell's first key decides whether the bucket changes inside it
            const bool inside = j + 1 < nb && (sf[j + 1] >> (32 - kClsT)) == cell;
            const uint32_t cb = (uint32_t)__clz((cell ^ mycell) << (32 - kClsT));   // < kClsT off myid's cell
            lut[cell] = (uint16_t)(inside || cell == mycell ? kClsExact | (kClsSkip << 8) : j | (cb << 8));
        }
        __syncthreads();
    }
    // per-lane bin counts in bytes: acc_e bins 0, 2, .., 14, acc_o bins 1, 3, .., 15 (<= 12 per
    // chunk: flushed to the block's LDS bins every kClsFlush chunks, before a byte can wrap)
    unsigned long long acc_e = 0, acc_o = 0;
    uint32_t nacc = 0;
    auto flush_acc = [&]() {   // wave-uniform
#pragma unroll
        for (uint32_t b = 0; b < kRegT; ++b) {
            uint32_t x = (uint32_t)(((b & 1u) ? acc_o : acc_e) >> (8 * (b >> 1))) & 0xFFu;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) x += (uint32_t)__shfl_xor((int)x, o);
            if (lane == 0 && x) atomicAdd(&sh[b], x);
        }
        acc_e = acc_o = 0;
        nacc = 0;
    };
    // one chunk; FULL: every id of the chunk is < n (no per-id bounds test); REGS: the register path
    auto chunk = [&](auto full_c, auto regs_c) {
        constexpr bool FULL = decltype(full_c)::value, REGS = decltype(regs_c)::value;
        uint32_t x[NE];
#pragma unroll
        for (uint32_t u = 0; u < kClsU; ++u) {
            x[4 * u] = v[u].x;
            x[4 * u + 1] = v[u].y;
            x[4 * u + 2] = v[u].z;
            x[4 * u + 3] = v[u].w;
        }
        unsigned long long pk = 0;   // 4-bit counts of bins 0..14 (field kClsSkip: exact-path ids)
        uint32_t packed[kClsU], exact = 0;
        if constexpr (REGS) {
            uint32_t fk[NE];
#pragma unroll
            for (uint32_t u = 0; u < kClsU; ++u) {
                uint32_t* f = fk + 4 * u;
#pragma unroll
                for (uint32_t e = 0; e < 4; ++e) f[e] = (uint32_t)__clz((x[4 * u + e] ^ m0) | (1u << (31 - kRegT)));
                // four byte lookups at once: v_perm over {mb:ma} (c = 0..7) and {md:mc} (8..15)
                const uint32_t sel = f[0] | f[1] << 8 | f[2] << 16 | f[3] << 24, s7 = sel & 0x07070707u;
                const uint32_t lo = __builtin_amdgcn_perm(mb, ma, s7), hi = __builtin_amdgcn_perm(md, mc, s7);
                const uint32_t m = ((sel >> 3) & 0x01010101u) * 0xFFu;
                packed[u] = (hi & m) | (lo & ~m);
#pragma unroll
                for (uint32_t e = 0; e < 4; ++e) {
                    const bool valid = FULL || 4 * (c * CH + u * 64 + lane) + e < n;
                    pk += (unsigned long long)valid << (4 * f[e]);
                }
            }
            if (pk >> (4 * kClsSkip)) {   // field 15: this lane holds an id with commonBits >= 15
#pragma unroll
                for (uint32_t k = 0; k < NE; ++k) {
                    const bool valid = FULL || 4 * (c * CH + (k >> 2) * 64 + lane) + (k & 3u) < n;
                    exact |= (uint32_t)(valid && fk[k] == kRegT) << k;
                }
            }
        } else {
            uint32_t ent[NE];
#pragma unroll
            for (uint32_t e = 0; e < NE; ++e) ent[e] = lut[x[e] >> (32 - kClsT)];
#pragma unroll
            for (uint32_t u = 0; u < kClsU; ++u) {
                packed[u] = 0;
#pragma unroll
                for (uint32_t e = 0; e < 4; ++e) {
                    const uint32_t k = 4 * u + e, en = ent[k];
                    const bool valid = FULL || 4 * (c * CH + u * 64 + lane) + e < n;
                    packed[u] |= (en & 0xFFu) << (8 * e);
                    pk += (unsigned long long)valid << (4 * ((en >> 8) & 0xFu));
                    exact |= (uint32_t)(valid && en >= kClsExact) << k;
                }
            }
        }
        // the exact path's ids (rare) join the wave's queue; their bucket bytes are stored below
        // as placeholders and rewritten when the queue is answered, their bins are field 15's
        while (exact) {
            const uint32_t k = (uint32_t)__ffs(exact) - 1;
            exact &= exact - 1;
            const uint32_t i = 4 * ((uint32_t)(c * CH) + (k >> 2) * 64 + lane) + (k & 3u);
            s_q[wv][atomicAdd(&s_qn[wv], 1u)] = i;
        }
        acc_e += pk & 0x0F0F0F0F0F0F0F0Full;
        acc_o += (pk >> 4) & 0x0F0F0F0F0F0F0F0Full;
        if (++nacc == kClsFlush) flush_acc();
        if (out_bucket) {
#pragma unroll
            for (uint32_t u = 0; u < kClsU; ++u) {
                const uint64_t i4 = c * CH + u * 64 + lane;
                if (FULL || 4 * i4 + 3 < n) {
                    *reinterpret_cast<uint32_t*>(out_bucket + 4 * i4) = packed[u];
                } else {
                    for (uint32_t e = 0; e < 4; ++e)
                        if (4 * i4 + e < n) out_bucket[4 * i4 + e] = (uint8_t)(packed[u] >> (8 * e));
                }
            }
        }
    };
    // answer the wave's queued exact-path ids, one per lane: bucket byte (after this wave's
    // earlier stores of the same words have completed) and commonBits bin
    auto answer_queue = [&]() {   // wave-uniform
        const uint32_t nq = __builtin_amdgcn_readfirstlane(s_qn[wv]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        for (uint32_t b = 0; b < nq; b += 64) {
            if (b + lane < nq) {
                const uint32_t i = s_q[wv][b + lane];
                const uint2 r = cls_exact(planes, stride, i, planes[i], sf, nb, m0, m1, m2, m3, m4);
                if (out_bucket) out_bucket[i] = (uint8_t)r.x;
                atomicAdd(&sh[r.y], 1u);
            }
        }
        if (lane == 0) s_qn[wv] = 0u;
    };
    auto stream = [&](auto regs_c) {
        for (; c < nch; c += W) {   // wave-uniform
            uint4 nx[kClsU];
            load(c + 2 * W, nx);
            if (c < nfull) chunk(std::true_type{}, regs_c);
            else chunk(std::false_type{}, regs_c);
            // room for the next chunk's ids in the queue (wave-uniform)
            if (__builtin_amdgcn_readfirstlane(s_qn[wv]) > kClsQCap - 4 * CH) answer_queue();
#pragma unroll
            for (uint32_t u = 0; u < kClsU; ++u) { v[u] = v2[u]; v2[u] = nx[u]; }
        }
    };
    if (regs) stream(std::true_type{});
    else stream(std::false_type{});
    answer_queue();
    flush_acc();
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
    if (n >= (1ull << 32)) return hipErrorInvalidValue;   // k_classify's 32-bit id indices (queued exact-path ids)
    const uint64_t n4 = (n + 3) / 4;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint64_t nch = (n4 + 64 * kClsU - 1) / (64 * kClsU);   // wave chunks
    uint64_t grid = (nch + kClsBlock / 64 - 1) / (kClsBlock / 64);
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
