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
//   F4  answers the fallback list with the K1 streaming scan (scan_dev.h) over all ids,
//       its roles sized at run time from the list's device-side count (target groups of
//       128 x id-range splits, split lists merged by the last split of each group), and
//       the ties F3 deferred (one wave each).  On uniform ids the list is empty and the
//       scan roles exit at once.
// F3 also clears the bitmap words it owns, so the bitmap is all-zero between calls.
//
// Algorithmic bytes per call: n * 4 (w0) + q * 4 (target w0) + survivors * 16 (written
// and re-read as {w0, idx}) + q * k * 4 (results).  On uniform ids the survivor fraction
// is 1 - exp(-q / 2^Lm) (12 % at the cfg-2 batch).
#include "scan_dev.h"
#include <hip/hip_ext.h>

#include <mutex>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <string>
#include <vector>

namespace dhtgpu {
namespace {

constexpr int kF1Threads = 256;                      // one thread per target
constexpr int kF3Threads = 256;
constexpr uint32_t kF3Cap = 4096;                    // survivors per partition staged in LDS
constexpr uint32_t kF3Per = kF3Cap / kF3Threads;
constexpr uint32_t kMaxLm = 19;                      // 2^19-bit bitmap = 64 KB of LDS in F2
constexpr uint32_t kMaxSubBits = 11;                 // F3 sub-prefix histogram <= 2048 bins
constexpr uint32_t kMaxQ = 1u << 22;                 // targets per call
constexpr uint32_t kTieSlots = 8;                    // deferred-tie slots per F3 partition
// F1's per-target bucket counters tcount[p] sit 256 B apart: their returning atomics execute
// at the memory side, one request per lane (random partitions), and counters packed into one
// 4 KB run would all queue on the same channel.  F2's pcount stays packed: its flush reserves
// consecutive partitions from consecutive lanes, which coalesce into one request per line.
// F2's survivor buckets come in kSets sets, one per XCD (block b uses set b % 8: blocks b and
// b + 8 share an XCD): a counter then takes 32 blocks' reservations instead of 256 (one
// address completes about 88 returning atomics per µs), and a bucket's partial-line runs are
// all written through one XCD's L2, which merges them into whole lines.  F3 gathers a
// partition from its kSets contiguous buckets.
constexpr uint32_t kSets = 8;
constexpr uint32_t kCtrStride = 64;
constexpr uint32_t kLdsMax = 160 * 1024;

__device__ __forceinline__ uint32_t top_bits(uint32_t w, uint32_t b) { return b ? w >> (32 - b) : 0u; }

// Workgroup barrier that orders LDS only.  __syncthreads() also drains this wave's
// outstanding global stores (vmcnt) -- a full memory round trip after every burst of
// result/bucket stores -- while nothing in these kernels reads another wave's global
// stores before the kernel ends.
__device__ __forceinline__ void sync_lds() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Inclusive scan over the 64 lanes of a wave with DPP (no LDS): row_shr 1/2/4/8 inside each
// 16-lane row, then row_bcast 15 / 31 across rows.  Lanes whose DPP source is out of range
// take `old` = 0.  Needs the whole wave active.
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);   // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);   // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);   // row_bcast:31
    return x;
}

// Exclusive scan of a[0, len) in LDS by a block of NT threads; returns the total.  Every
// thread must call it.  wsum: NT / 64 + 1 words of LDS scratch.  Wave w owns a contiguous
// run of rows; a row is 4 consecutive entries per lane (one 16-B LDS access each, 256 entries
// at consecutive addresses: no bank conflicts -- one thread per contiguous run of len / NT
// entries was a stride-(len / NT) pattern, 7 us for 4096 bins) scanned with DPP, carrying
// the row total.  Unaligned or ragged arrays take rows of one entry per lane.
template <int NT>
__device__ uint32_t scan_lds(uint32_t* a, uint32_t len, uint32_t* wsum) {
    constexpr int NW = NT / 64;
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    const bool vec = (len & 3u) == 0 && ((uintptr_t)a & 15u) == 0;
    const uint32_t per = vec ? 4u : 1u, rl = 64u * per;
    const uint32_t rows = (len + rl - 1) / rl, rpw = (rows + NW - 1) / NW;
    const uint32_t r0 = w * rpw < rows ? w * rpw : rows, r1 = r0 + rpw < rows ? r0 + rpw : rows;
    auto ld = [&](uint32_t r) {
        const uint32_t i = r * rl + lane * per;
        if (vec) return i < len ? *reinterpret_cast<const uint4*>(a + i) : make_uint4(0u, 0u, 0u, 0u);
        return make_uint4(i < len ? a[i] : 0u, 0u, 0u, 0u);
    };
    uint32_t s = 0;
    for (uint32_t r = r0; r < r1; ++r) {
        const uint4 v = ld(r);
        s += v.x + v.y + v.z + v.w;
    }
    const uint32_t ws = (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_incl(s), 63);
    if (lane == 0) wsum[w] = ws;
    sync_lds();
    if (threadIdx.x < 64) {
        const uint32_t v = lane < (uint32_t)NW ? wsum[lane] : 0u;
        const uint32_t xv = wave_scan_incl(v);
        if (lane < (uint32_t)NW) wsum[lane] = xv - v;
        if (lane == (uint32_t)NW - 1) wsum[NW] = xv;
    }
    sync_lds();
    uint32_t carry = wsum[w];
    for (uint32_t r = r0; r < r1; ++r) {
        const uint4 v = ld(r);
        const uint32_t t = v.x + v.y + v.z + v.w;
        const uint32_t x = wave_scan_incl(t);
        const uint32_t e0 = carry + x - t, i = r * rl + lane * per;
        if (i < len) {
            if (vec) *reinterpret_cast<uint4*>(a + i) = make_uint4(e0, e0 + v.x, e0 + v.x + v.y, e0 + v.x + v.y + v.z);
            else a[i] = e0;
        }
        carry += (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
    }
    const uint32_t total = wsum[NW];
    sync_lds();
    return total;
}

// median of three: with a <= b it is max(a, min(b, c)), the sorted-insertion step
__device__ __forceinline__ uint32_t med3_u32(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// ---- F1: mark target prefixes, bucket the targets by partition ----------------------------
// One thread per target: it sets the target's level-Lm prefix bit in the bitmap and appends
// {w0, index} to its partition's bucket tbuf[p][...] (slot from a returning atomic on
// tcount[p]; F3 reads the bucket as one coalesced run).  Prefix-shard contexts
// (dhtgpu_gen_ids_prefix: every id shares its top `shift` bits) keep a second word-0 plane
// shifted left by `shift` (the next bits of word 1 shifted in), and the targets' word 0 is
// shifted the same way here: inside the shard the dropped bits XOR to one constant for every
// id, so the order is unchanged -- for targets of other prefixes too -- and word 0 keeps 32
// distinguishing bits.  A target whose bucket is full goes to the spill list (count
// ctr[kSpill]); F3 moves the spill list to the F4 fallback list.
constexpr uint32_t kSpill = 8;   // ctr word: spilled targets (all-zero between calls)

// Prefix sub-partitions (dhtgpu_ctx: a set too large for one plan is split by the next
// sub_bits id bits after its shard prefix, each part compacted with its own shifted word-0
// plane): ONE launch sequence serves all of them.  A target's sub-partition is its bits
// [sub_shift, sub_shift + sub_bits); every sub-partition has its own bitmap and its own np
// partitions (global partition = sub * np + p); F2's workgroups are dealt to the
// sub-partitions in proportion to their ids; F3 / F4 read the tie words and map the results
// through the target's sub-partition.  A set that needs no split is the one sub-partition.
struct SubDesc {
    const uint32_t* w0;       // streamed word-0 plane (shifted for shards / sub-partitions)
    const uint32_t* planes;   // unshifted word planes (tie words)
    uint64_t stride, n;
    const uint32_t* gidx;     // result index map (nullable) ...
    uint32_t base;            // ... or offset
    uint32_t lim;             // last 16-B aligned word offset loadable inside w0's allocation
    uint32_t blk0, nblk;      // its F2 workgroups
    uint64_t per_blk;         // F2 ids per workgroup
};

struct F1Args {
    const uint32_t* tw0; const uint32_t* tw1;
    uint32_t q, Lm, b1, shift;
    uint32_t sub_shift, sub_bits;   // a target's sub-partition: its bits [sub_shift, sub_shift + sub_bits)
    uint32_t np, nwords;            // partitions and bitmap words per sub-partition
    uint32_t* bitmap;
    uint32_t* tcount; uint2* tbuf; uint32_t tcap;
    uint32_t* ctr; uint32_t* tspill;
    const uint8_t* cells; uint32_t k;   // nullable: per sub-partition level-Lm cell counts (sibling marking)
};

__global__ __launch_bounds__(kF1Threads) void k_f1_targets(F1Args a) {
    if (blockIdx.x == 0 && threadIdx.x < 4) a.ctr[threadIdx.x] = 0;   // fallback, survivors, wave path, -
    const uint32_t i = blockIdx.x * kF1Threads + threadIdx.x;
    if (i >= a.q) return;
    const uint32_t w = a.tw0[i];
    const uint32_t sub = a.sub_bits ? (w << a.sub_shift) >> (32 - a.sub_bits) : 0u;
    const uint32_t v = a.shift ? (w << a.shift) | (a.tw1[i] >> (32 - a.shift)) : w;
    const uint32_t pre = top_bits(v, a.Lm);
    // sibling marking (plans with cells): a level-Lm cell holding < k ids marks its sibling too, so
    // the target's level-(Lm - 1) subtree is complete among the survivors
    const bool sib = a.cells && a.cells[((uint64_t)sub << a.Lm) + pre] < a.k;
    atomicOr(a.bitmap + sub * a.nwords + (pre >> 5), (1u << (pre & 31)) | (sib ? 1u << ((pre ^ 1u) & 31) : 0u));
    const uint32_t p = sub * a.np + top_bits(v, a.b1);
    const uint32_t slot = atomicAdd(a.tcount + p * kCtrStride, 1u);
    if (slot < a.tcap) {
        a.tbuf[(uint64_t)p * a.tcap + slot] = make_uint2(v, i);
        return;
    }
    // spill: one atomic per wave (a single counter would serialise every lane's add)
    const uint64_t sp = __ballot(1);   // the lanes still here (the others returned)
    const uint32_t lane = lane_id();
    uint32_t base = 0;
    if (lane == (uint32_t)__ffsll((long long)sp) - 1) base = atomicAdd(a.ctr + kSpill, (uint32_t)__popcll(sp));
    base = __shfl((int)base, __ffsll((long long)sp) - 1);
    a.tspill[base + (uint32_t)__popcll(sp & ((1ull << lane) - 1ull))] = i;
}

// ---- F1 for large batches: the same marks and buckets with no per-target global atomic --------
// k_f1_targets costs two memory-side atomics per target on distinct lines (bitmap OR, bucket
// counter): at 2^20 targets that is 2.1 M atomic requests, 95 us at the chip's atomic rate
// (DESIGN 5d).  Large batches take two passes instead:
//   F1a k_f1_coarse  groups the targets by a coarse bin = (sub-partition, top c bits): an LDS
//                    histogram per workgroup of 4,096 targets, ONE returning global atomic per
//                    (workgroup, bin) reserving the workgroup's run in the bin's bucket cbuf[bin];
//   F1b k_f1_fine    one workgroup per bin owns the bin's bitmap words and its 2^(b1 - c)
//                    partitions outright: it marks the bitmap in LDS (sibling marks as F1) and
//                    ranks the targets per partition with LDS atomics, stores each target at
//                    tbuf[p][rank], then writes its bitmap words and partition counts with plain
//                    stores (every word and count of the bin, zeros included).
// A bin or bucket past its capacity spills the target to the F4 fallback list, as F1 does.
constexpr uint32_t kF1aThreads = 1024, kF1aPer = 4, kF1aTargets = kF1aThreads * kF1aPer;
constexpr uint32_t kF1bThreads = 1024, kF1bPer = 4;
constexpr uint32_t kMaxCoarse = 4096;             // bins (the coarse counters live in the clean head)
constexpr uint32_t kF1bLdsWords = 16384;          // F1b's bitmap words + partition counts (64 KB)
constexpr uint32_t kF1CoarseMinQ = 1u << 17;      // smaller batches: k_f1_targets (at 2^17 F1 is as fast either
                                                  // way, 13.1-13.4 us, and the two-pass form leaves the other call
                                                  // in flight the atomics: prefix rank 0.130-0.135 -> 0.127-0.128 ms)

struct F1cArgs {
    const uint32_t* tw0; const uint32_t* tw1;
    uint32_t q, shift, sub_shift, sub_bits;
    uint32_t c, ccap;                  // coarse bin = sub << c | top c bits; bin bucket capacity
    uint32_t* ccount; uint2* cbuf;     // [nbins] (all-zero between calls: F1b resets), [nbins][ccap]
    uint32_t Lm, b1, np, nwords;
    uint32_t* bitmap;
    uint32_t* tcount; uint2* tbuf; uint32_t tcap;
    uint32_t* ctr; uint32_t* tspill;
    const uint8_t* cells; uint32_t k;
};

// the lanes with `sp` set append `val` to the spill list (one atomic per wave)
__device__ __forceinline__ void f1_spill(bool sp, uint32_t val, uint32_t* ctr, uint32_t* tspill) {
    const uint64_t m = __ballot(sp);
    if (!m) return;
    const uint32_t lane = lane_id(), lead = (uint32_t)__ffsll((long long)m) - 1;
    uint32_t base = 0;
    if (lane == lead) base = atomicAdd(ctr + kSpill, (uint32_t)__popcll(m));
    base = (uint32_t)__shfl((int)base, (int)lead);
    if (sp) tspill[base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = val;
}

__global__ __launch_bounds__(kF1aThreads) void k_f1_coarse(F1cArgs a) {
    __shared__ uint32_t hist[kMaxCoarse];
    const uint32_t nbins = (1u << a.sub_bits) << a.c;
    if (blockIdx.x == 0 && threadIdx.x < 4) a.ctr[threadIdx.x] = 0;   // fallback, survivors, wave path, -
    for (uint32_t b = threadIdx.x; b < nbins; b += kF1aThreads) hist[b] = 0;
    __syncthreads();
    const uint32_t i0 = blockIdx.x * kF1aTargets + threadIdx.x;
    uint32_t v[kF1aPer], bin[kF1aPer], r[kF1aPer];
#pragma unroll
    for (uint32_t u = 0; u < kF1aPer; ++u) {
        const uint32_t i = i0 + u * kF1aThreads;
        if (i < a.q) {
            const uint32_t w = a.tw0[i];
            const uint32_t sub = a.sub_bits ? (w << a.sub_shift) >> (32 - a.sub_bits) : 0u;
            v[u] = a.shift ? (w << a.shift) | (a.tw1[i] >> (32 - a.shift)) : w;
            bin[u] = (sub << a.c) | top_bits(v[u], a.c);
            r[u] = atomicAdd(hist + bin[u], 1u);
        }
    }
    __syncthreads();
    // one reservation per (workgroup, bin): consecutive lanes on consecutive counters
    for (uint32_t b = threadIdx.x; b < nbins; b += kF1aThreads) {
        const uint32_t h = hist[b];
        if (h) hist[b] = atomicAdd(a.ccount + b, h);
    }
    __syncthreads();
#pragma unroll
    for (uint32_t u = 0; u < kF1aPer; ++u) {
        const uint32_t i = i0 + u * kF1aThreads;
        const uint32_t pos = i < a.q ? hist[bin[u]] + r[u] : 0u;
        if (i < a.q && pos < a.ccap) a.cbuf[(uint64_t)bin[u] * a.ccap + pos] = make_uint2(v[u], i);
        f1_spill(i < a.q && pos >= a.ccap, i, a.ctr, a.tspill);
    }
}

__global__ __launch_bounds__(kF1bThreads) void k_f1_fine(F1cArgs a) {
    extern __shared__ uint32_t sh1[];
    const uint32_t b = blockIdx.x, sub = b >> a.c, hi = b & ((1u << a.c) - 1u);
    const uint32_t lw = a.Lm - a.c - 5, nw = 1u << lw;          // the bin's bitmap words
    const uint32_t lp = a.b1 - a.c, nps = 1u << lp;             // the bin's partitions
    uint32_t* bm = sh1;
    uint32_t* fc = sh1 + nw;
    for (uint32_t j = threadIdx.x; j < nw + nps; j += kF1bThreads) sh1[j] = 0;
    const uint32_t m0 = a.ccount[b];
    __syncthreads();   // (every thread has read the count)
    if (threadIdx.x == 0) a.ccount[b] = 0;   // all-zero again for the next call
    const uint32_t m = m0 < a.ccap ? m0 : a.ccap;
    const uint32_t pbase = sub * a.np + (hi << lp);
    const uint2* src = a.cbuf + (uint64_t)b * a.ccap;
    const uint8_t* cells = a.cells ? a.cells + ((uint64_t)sub << a.Lm) : nullptr;
    // kF1bPer entries per thread loaded at once (one round trip per kF1bPer * kF1bThreads entries:
    // a loop of one load per thread at a time made F1 34 us at 2^20 targets)
    for (uint32_t j0 = 0; j0 < m; j0 += kF1bPer * kF1bThreads) {   // block-uniform
        uint2 e[kF1bPer];
        uint8_t cl[kF1bPer];
#pragma unroll
        for (uint32_t u = 0; u < kF1bPer; ++u) {
            const uint32_t j = j0 + u * kF1bThreads + threadIdx.x;
            e[u] = j < m ? src[j] : make_uint2(0u, 0u);
        }
#pragma unroll
        for (uint32_t u = 0; u < kF1bPer; ++u) {
            const uint32_t j = j0 + u * kF1bThreads + threadIdx.x;
            cl[u] = (cells && j < m) ? cells[top_bits(e[u].x, a.Lm)] : (uint8_t)255;
        }
#pragma unroll
        for (uint32_t u = 0; u < kF1bPer; ++u) {
            const uint32_t j = j0 + u * kF1bThreads + threadIdx.x;
            bool sp = false;
            if (j < m) {
                const uint32_t pre = top_bits(e[u].x, a.Lm);
                const bool sib = cl[u] < a.k;
                atomicOr(bm + ((pre >> 5) & (nw - 1u)), (1u << (pre & 31)) | (sib ? 1u << ((pre ^ 1u) & 31) : 0u));
                const uint32_t pl = top_bits(e[u].x, a.b1) & (nps - 1u);
                const uint32_t rk = atomicAdd(fc + pl, 1u);
                if (rk < a.tcap) a.tbuf[(uint64_t)(pbase + pl) * a.tcap + rk] = e[u];
                else sp = true;
            }
            f1_spill(sp, e[u].y, a.ctr, a.tspill);
        }
    }
    __syncthreads();
    uint32_t* gbm = a.bitmap + (uint64_t)sub * a.nwords + ((uint64_t)hi << lw);
    for (uint32_t j = threadIdx.x; j < nw; j += kF1bThreads) gbm[j] = bm[j];
    for (uint32_t j = threadIdx.x; j < nps; j += kF1bThreads) a.tcount[(uint64_t)(pbase + j) * kCtrStride] = fc[j];
}

// ---- F2: stream w0, keep ids in marked subtrees, partition them ----------------------
// Persistent: one workgroup per CU, each owning a contiguous id range streamed through
// a ring of kF2Ring 16-B loads per lane (32 KB in flight per CU).  Survivors are appended
// to an LDS stage; when the stage could overflow (and at the end) it is flushed into the
// partition-major survivor buckets pbuf[p][...] (see f2_flush).
constexpr int kF2Threads = 1024;
constexpr uint32_t kF2Sub = 4 * kF2Threads;          // ids per sub-step (one uint4 per thread)
constexpr uint32_t kF2Step = 4 * kF2Sub;             // ids per chunk
constexpr uint32_t kStage = 11264;                   // LDS stage entries (88 KB)
// window mode (prefix-sorted sub-partitions: a workgroup's bitmap is the window of words its
// sorted range spans, a few KB instead of 64): the stage takes the freed LDS when one final flush
// then holds the workgroup's survivors (the cfg-3 shard: 16.2 K per workgroup, two flushes before)
constexpr uint32_t kStageWin = 25600;

__host__ __device__ inline uint32_t f2_fixed_words(uint32_t nwords, uint32_t np) {
    return (36 + nwords + np + 1 + 17 + np / 32 + 1 + 3) & ~3u;
}

struct F2Args {
    const SubDesc* subs; const uint8_t* blk_sub;   // sub-partitions; workgroup -> sub-partition
    SubDesc one; uint32_t nsub;                    // nsub == 1: the one sub-partition (no table loads)
    uint32_t np_all;                               // partitions over all sub-partitions
    uint32_t Lm, b1;
    const uint32_t* bitmap; uint32_t nwords;
    uint32_t* pcount;             // [kSets][np_all] survivors per set and partition (all-zero between calls)
    uint2* pbuf;                  // [np_all][nsets][pcap] survivors, partition- and set-major
    uint32_t pcap;
    uint32_t* ctr;                // shared counters (F2 writes none; the survivor total is sum(pcount))
    uint32_t stage;               // LDS stage capacity (entries, <= kStage)
    uint32_t dbg;                 // diagnostics: bit 256 = phase stamps (results unchanged)
    uint32_t sparse;              // 1: no per-sub-step barrier (plan: the stage holds a segment's survivors)
    uint32_t seg;                 // sparse mode: ids per segment (the stage is flushed after each)
    unsigned long long* stamps;   // dbg & 256: per-block phase timestamps [nblk2][16]
    uint32_t nsets;               // kSets, or 1 over prefix-sorted sub-partitions (a partition's survivors come from one or two workgroups)
    uint32_t wwords;              // window mode: bitmap words in LDS (the window from the range's first word)
    uint32_t pk_ob;               // window + Sparse: index-offset bits of the packed stage (StagePk)
};
#define F2_STAMP(i) \
    do { if ((a.dbg & 256) && threadIdx.x == 0) a.stamps[(uint64_t)blockIdx.x * 16 + (i)] = __builtin_amdgcn_s_memrealtime(); } while (0)


// Flush the stage: the entries move to registers, are counting-sorted by partition back
// into the stage, and every partition's run is then written with consecutive lanes on
// consecutive addresses of its bucket pbuf[p][...], whose slots one returning global
// atomic per partition reserved.  A partition that outgrows pcap keeps counting (F3 then
// sends its targets to the fallback).
// Narrow stage (kF2Narrow: a workgroup's ids span < 2^16): the stage is two arrays, word 0
// [a.stage] u32 then the id's offset from the workgroup's first id [a.stage] u16 -- 6 B per
// entry instead of 8, so F2's LDS leaves room for an F3 workgroup of another batch on its CU.
constexpr uint32_t kStagePer = (kStage + 1023) / 1024;
constexpr uint32_t kStagePerWin = (kStageWin + 1023) / 1024;
// Packed stage (window mode, Sparse): the same two arrays, holding the 48-bit value
// (w0 - wb0) << ob | (index - the workgroup's first id): a sorted workgroup range spans a few
// thousand bitmap words, so its word 0 minus the window's first word fits 48 - ob bits (the host
// checks) -- the stage of the cfg-3 shard's 16 K-survivor ranges then fits one final flush.
struct StagePk { uint32_t wb0, ob; };
template <int Fmt>   // 0: 8-B {w0, index}; 1: narrow (u32 w0, u16 offset); 2: packed
__device__ __forceinline__ uint2 stage_get(const uint2* stage, uint32_t cap, uint32_t ibase, uint32_t j, StagePk pk) {
    if (Fmt == 0) return stage[j];
    const uint32_t* sw = reinterpret_cast<const uint32_t*>(stage);
    const uint16_t* si = reinterpret_cast<const uint16_t*>(sw + cap);
    if (Fmt == 1) return make_uint2(sw[j], ibase + si[j]);
    const uint64_t v = (uint64_t)si[j] << 32 | sw[j];
    return make_uint2(pk.wb0 + (uint32_t)(v >> pk.ob), ibase + (uint32_t)(v & ((1ull << pk.ob) - 1ull)));
}
template <int Fmt>
__device__ __forceinline__ void stage_put(uint2* stage, uint32_t cap, uint32_t ibase, uint32_t j, uint32_t w, uint32_t i,
                                          StagePk pk) {
    if (Fmt == 0) { stage[j] = make_uint2(w, i); return; }
    uint32_t* sw = reinterpret_cast<uint32_t*>(stage);
    uint16_t* si = reinterpret_cast<uint16_t*>(sw + cap);
    if (Fmt == 1) {
        sw[j] = w;
        si[j] = (uint16_t)(i - ibase);
        return;
    }
    const uint64_t v = (uint64_t)(w - pk.wb0) << pk.ob | (i - ibase);
    sw[j] = (uint32_t)v;
    si[j] = (uint16_t)(v >> 32);
}
// Agg (window mode): a sorted range's survivors sit in the stage in stream order, so wave w's
// contiguous chunk [w C, (w + 1) C) of it holds one or two partitions.  No stage sort: the wave
// ranks its entries per partition in registers (up to 4 partitions a round), reserves each
// partition's share of its bucket with one returning atomic per (wave, partition) -- all of a
// round's in one instruction -- and stores the entries there itself.  (Sorting a sorted stage by
// per-entry LDS atomics on one or two addresses serialised: the window's single flush of 15 K
// entries spent 6 us ranking them.)
template <int Fmt, uint32_t Per = kStagePer, bool Agg = false>
__device__ void f2_flush(const F2Args& a, uint32_t cnt, uint2* stage, uint32_t* hist, uint32_t* wsum, uint32_t poff,
                         uint32_t ibase, StagePk pk = StagePk{0u, 0u}) {
    const uint32_t np = 1u << a.b1;
    uint2 e[Per];
    uint32_t rk[Per];
    const uint32_t lane = lane_id();
    if (Agg) {
        const uint32_t w = threadIdx.x >> 6;
        const uint32_t C = (cnt + kF2Threads - 1) / kF2Threads * 64;   // entries per wave (<= Per * 64)
        uint32_t valid = 0;   // bit r: slice r holds an entry for this lane
#pragma unroll
        for (uint32_t r = 0; r < Per; ++r) {
            const uint32_t j = w * C + r * 64 + lane;
            if (r * 64 < C && j < cnt) {
                e[r] = stage_get<Fmt>(stage, a.stage, ibase, j, pk);
                valid |= 1u << r;
            }
        }
        F2_STAMP(6);
        sync_lds();   // every entry is in registers: the caller may refill the stage after this flush
        const uint32_t set = a.nsets == 1 ? 0u : blockIdx.x % kSets, set_off = set * a.np_all + poff;
        for (;;) {   // wave-uniform rounds of up to 4 partitions (one round on sorted uniform ids)
            uint32_t tk[4] = {DHT_NONE, DHT_NONE, DHT_NONE, DHT_NONE}, tc[4] = {0u, 0u, 0u, 0u}, nt = 0, pend = 0;
#pragma unroll
            for (uint32_t r = 0; r < Per; ++r) {
                const bool v = (valid >> r) & 1u;
                const uint32_t key = v ? top_bits(e[r].x, a.b1) : DHT_NONE;
                uint64_t act = __ballot(v);
                while (act) {
                    const uint32_t kk = (uint32_t)__builtin_amdgcn_readlane((int)key, __ffsll((long long)act) - 1);
                    const uint64_t m = __ballot(key == kk) & act;
                    act &= ~m;
                    uint32_t q = 4;
#pragma unroll
                    for (uint32_t x = 0; x < 4; ++x) q = (x < nt && tk[x] == kk) ? x : q;
                    if (q == 4 && nt < 4) { q = nt++; tk[q] = kk; }
                    if (q == 4) continue;   // a fifth partition: the next round
                    if ((m >> lane) & 1ull) {
                        rk[r] = (tc[q] + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))) | (q << 28);
                        pend |= 1u << r;
                    }
                    tc[q] += (uint32_t)__popcll(m);
                }
            }
            if (nt == 0) break;
            uint32_t res = 0;
            if (lane < nt) {
                const uint32_t kq = lane == 0 ? tk[0] : lane == 1 ? tk[1] : lane == 2 ? tk[2] : tk[3];
                const uint32_t cq = lane == 0 ? tc[0] : lane == 1 ? tc[1] : lane == 2 ? tc[2] : tc[3];
                res = atomicAdd(a.pcount + set_off + kq, cq);
            }
            const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)res, 0), b1 = (uint32_t)__builtin_amdgcn_readlane((int)res, 1);
            const uint32_t b2 = (uint32_t)__builtin_amdgcn_readlane((int)res, 2), b3 = (uint32_t)__builtin_amdgcn_readlane((int)res, 3);
#pragma unroll
            for (uint32_t r = 0; r < Per; ++r) {
                if (!((pend >> r) & 1u)) continue;
                const uint32_t q = rk[r] >> 28;
                const uint32_t pos = (q == 0 ? b0 : q == 1 ? b1 : q == 2 ? b2 : b3) + (rk[r] & 0x0FFFFFFFu);
                const uint32_t p = q == 0 ? tk[0] : q == 1 ? tk[1] : q == 2 ? tk[2] : tk[3];
                if (pos < a.pcap) a.pbuf[(uint64_t)((poff + p) * a.nsets + set) * a.pcap + pos] = e[r];
            }
            valid &= ~pend;
        }
        F2_STAMP(7);
        return;
    }
    for (uint32_t i = threadIdx.x; i <= np; i += kF2Threads) hist[i] = 0;
    sync_lds();
#pragma unroll
    for (uint32_t r = 0; r < Per; ++r) {
        const uint32_t j = r * kF2Threads + threadIdx.x;
        if (j < cnt) {
            e[r] = stage_get<Fmt>(stage, a.stage, ibase, j, pk);
            rk[r] = atomicAdd(hist + top_bits(e[r].x, a.b1), 1u);
        }
    }
    sync_lds();
    // reserve the partitions' slots (before the scan overwrites the counts)
    uint32_t res[8];
    const uint32_t set = a.nsets == 1 ? 0u : blockIdx.x % kSets, set_off = set * a.np_all + poff;   // this block's bucket set
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) {
        const uint32_t p = i * kF2Threads + threadIdx.x;
        const uint32_t c = p < np ? hist[p] : 0u;
        res[i] = c ? atomicAdd(a.pcount + set_off + p, c) : 0u;
    }
    F2_STAMP(3);
    scan_lds<kF2Threads>(hist, np, wsum);   // hist = partition starts inside the stage
    if (threadIdx.x == 0) hist[np] = cnt;
#pragma unroll
    for (uint32_t r = 0; r < Per; ++r) {
        const uint32_t j = r * kF2Threads + threadIdx.x;
        if (j < cnt) stage_put<Fmt>(stage, a.stage, ibase, hist[top_bits(e[r].x, a.b1)] + rk[r], e[r].x, e[r].y, pk);
    }
    // wsum is free again: reuse the stage-local starts to turn reservations into deltas
    // (bucket offset of stage position j = res[p] - start[p] + j)
    sync_lds();
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) {
        const uint32_t p = i * kF2Threads + threadIdx.x;
        if (p < np) res[i] -= hist[p];
    }
    sync_lds();
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) {
        const uint32_t p = i * kF2Threads + threadIdx.x;
        if (p < np) hist[p] = res[i];
    }
    sync_lds();
    F2_STAMP(4);
    for (uint32_t j = threadIdx.x; j < cnt; j += kF2Threads) {
        const uint2 x = stage_get<Fmt>(stage, a.stage, ibase, j, pk);
        const uint32_t p = top_bits(x.x, a.b1);
        const uint32_t pos = hist[p] + j;
        if (pos < a.pcap) a.pbuf[(uint64_t)((poff + p) * a.nsets + set) * a.pcap + pos] = x;
    }
    sync_lds();
}

// Loads are unconditional 16-B loads (no data-dependent branches, so every load of the
// ring stays in flight): addresses past the id range are clamped into the plane
// allocation and their words are masked by the caller's range test.
constexpr uint32_t kRing = 8;    // S1's ring (two 512-thread workgroups per CU: 64 KB each)
// F2's ring: 2 sub-steps = 32 KB in flight per CU.  A pure 64 MB stream by one 1024-thread
// workgroup per CU (tools/experiments/stream_probe.hip, profiles/r03/experiments) takes
// 13.3 us with 8 (128 KB in flight), 11.7 with 4, 11.1 with 3, 10.3 with 2: a deeper ring only
// queues longer.  F2 at cfg 2: 21.9 us with 4, 21.3 with 3, 20.7 with 2 (round 2: 8, 24.1 us)
constexpr uint32_t kF2Ring = 2;
// The ring loads are buffer loads through a descriptor based at the workgroup's first id
// (f2_rsrc): the plane pointers come from sub-partition descriptors in memory, whose address
// space the compiler cannot infer -- plain loads through them are FLAT loads, which also count
// on lgkmcnt, so every LDS wait in the loop would wait for the ring.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t f2_rsrc(const uint32_t* w0, uint32_t lo, uint32_t lim) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)(w0 + lo), (short)0, (int)((lim - lo + 4u) * 4u), 0x00020000);
}
__device__ __forceinline__ uint4 f2_load1g(const uint32_t* __restrict__ w0, uint32_t c, uint32_t lim) {
    uint32_t j = c + 4 * threadIdx.x;
    j = j < lim ? j : lim;
    return *reinterpret_cast<const uint4*>(w0 + j);
}
template <bool NT>
__device__ __forceinline__ uint4 f2_load1(__amdgpu_buffer_rsrc_t rs, uint32_t lo, uint32_t c, uint32_t lim) {
    uint32_t j = c + 4 * threadIdx.x;
    j = j < lim ? j : lim;
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)((j - lo) * 4u), 0, NT ? 2 : 0);   // 2: nt
    return make_uint4(v[0], v[1], v[2], v[3]);
}

// Modes: kF2Dense flushes the stage whenever a sub-step could overflow it (one barrier
// per sub-step); kF2Sparse (the plan proved a block's survivors fit the stage) has no
// barrier in the loop and flushes once at the end; kF2Seg is kF2Sparse with a flush every
// a.seg ids (ranges longer than one stage-full: large sub-partitioned sets) -- its own
// instantiation, because the flush inlined in the loop keeps the ring live across it (128
// VGPRs, the whole register file at 16 waves per CU, where kF2Sparse needs 68 and leaves
// room for the other stream's F1 / F4 waves).
// kF2Narrow is kF2Sparse over the 6-B narrow stage (a workgroup's range < 2^16 ids).
constexpr uint32_t kF2Dense = 0, kF2Sparse = 1, kF2Seg = 3, kF2Narrow = 4;

// Src: kF2One -- one set: its descriptor from the kernel arguments, the ring through plain
// global loads; kF2Subs -- several sub-partitions (descriptors read from memory, the ring
// through buffer loads); kF2SubsNT -- the same with non-temporal ring loads, for sets whose w0
// planes exceed the Infinity Cache (kNtBytes): the stream then no longer evicts the survivor
// and target buckets F3 / F4 read next (cfg-3 shard: F2 118 -> 103 us, F3 43 -> 38, F4 19 ->
// 17, profiles/r03/experiments/stream_nt_ab.txt).  A set the cache holds keeps cached loads:
// non-temporal ones re-read it from HBM every call (cfg 2: F2 20.5 -> 22.9 us).
constexpr uint32_t kF2One = 0, kF2Subs = 1, kF2SubsNT = 2;
constexpr uint64_t kNtBytes = 192ull << 20;   // 3/4 of the 256 MB Infinity Cache
// Win (Subs only): the sub-partitions are sorted by prefix, so a workgroup's contiguous id range
// spans a narrow run of bitmap words, starting at its first id's: only that window (a.wwords words,
// which the host bounded from the sub-partitions' span table) is copied to LDS, and the stage
// takes the rest (Sparse: one final flush of up to kStageWin entries)
template <uint32_t Mode, uint32_t Src, bool Win = false>
__global__ __launch_bounds__(kF2Threads) void k_f2_filter(F2Args a) {
    constexpr bool Subs = Src != kF2One, NT = Src == kF2SubsNT;
    constexpr bool Narrow = Mode == kF2Narrow;
    constexpr bool Sparse = Mode == kF2Sparse || Mode == kF2Seg || Narrow;
    constexpr bool Pack = Win && Mode == kF2Sparse;   // window + one final flush: the packed stage
    constexpr int Fmt = Pack ? 2 : Narrow ? 1 : 0;
    constexpr uint32_t Per = Pack ? kStagePerWin : kStagePer;
    static_assert(!Win || (Subs && !Narrow), "window mode: sorted sub-partitions, 8-B stage");
    extern __shared__ uint32_t sh[];   // (32 spare) | misc[8] | bm[bmw] | hist[np + 1] | wsum[17] | lost[np/32 + 1] | stage
    const uint32_t np = 1u << a.b1;
    const uint32_t bmw = Win ? a.wwords : a.nwords;
    uint32_t* misc = sh + 28;
    uint32_t* bm = sh + 36;
    uint32_t* hist = bm + bmw;
    uint32_t* wsum = hist + np + 1;
    uint32_t* lost = wsum + 17;   // sparse mode: partitions that lost survivors past a full stage
    uint2* stage = reinterpret_cast<uint2*>(sh + f2_fixed_words(bmw, np));
    const uint32_t sub = Subs ? (uint32_t)a.blk_sub[blockIdx.x] : 0u;
    const SubDesc d = Subs ? a.subs[sub] : a.one;
    const uint64_t lo64 = (uint64_t)(blockIdx.x - d.blk0) * d.per_blk;
    if (lo64 >= d.n) return;
    F2_STAMP(0);
    const uint32_t* const w0 = d.w0;
    const uint32_t poff = sub * np;   // this sub-partition's first partition
    const uint32_t lo = (uint32_t)lo64;
    const uint32_t hi = (uint32_t)(lo64 + d.per_blk < d.n ? lo64 + d.per_blk : d.n);
    const uint32_t lane = lane_id();
    // level-Lm prefix = bits [32 - Lm, 32) of w0: one v_bfe
    const uint32_t pre_off = 32 - a.Lm;
    const uint32_t lm5 = a.Lm > 5 ? a.Lm - 5 : 0u;   // word index width
    const uint32_t tid4 = 4 * threadIdx.x;
    // the prefix bitmap first (ahead of the ring, its loads land first: measured 1 µs better
    // per block than ring-first; per-XCD copies stored by F1 -- L2-resident on paper -- did not
    // shorten this phase either: it is the fabric, not the source); indices past the end are
    // clamped, so a clamped lane rewrites a word with its own value
    const uint32_t* bsrc = a.bitmap + sub * a.nwords;
    // window mode: the bitmap word of the range's first (smallest) id -- the first load of the
    // workgroup, waited for alone; the window's words (<= 2 per thread) are loaded before the ring
    // is issued and stored to LDS after it, so their round trip overlaps the ring's
    uint32_t wbase = 0, wv0 = 0, wv1 = 0;
    if (Win) {
        const uint32_t flim = min(d.lim, ((hi + 3u) & ~3u) - 4u);
        const uint32_t f0 = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(f2_rsrc(w0, lo, flim), 0, 0, 0);
        wbase = a.Lm > 5 ? __builtin_amdgcn_readfirstlane(f0 >> (pre_off + 5)) : 0u;
        const uint32_t i0 = wbase + threadIdx.x, i1 = i0 + kF2Threads;
        wv0 = threadIdx.x < a.wwords && i0 < a.nwords ? bsrc[i0] : 0u;
        wv1 = threadIdx.x + kF2Threads < a.wwords && i1 < a.nwords ? bsrc[i1] : 0u;
    }
    const StagePk pk{Win && a.Lm > 5 ? wbase << (pre_off + 5) : 0u, a.pk_ob};
    if (Win) {
    } else if ((a.nwords & 3) == 0) {
        for (uint32_t i0 = 0; i0 < a.nwords; i0 += kF2Threads * 16) {
            uint4 t[4];
            uint32_t ic[4];
#pragma unroll
            for (uint32_t r = 0; r < 4; ++r) {
                uint32_t i = i0 + (r * kF2Threads + threadIdx.x) * 4;
                ic[r] = i < a.nwords ? i : a.nwords - 4;
                t[r] = *reinterpret_cast<const uint4*>(bsrc + ic[r]);
            }
#pragma unroll
            for (uint32_t r = 0; r < 4; ++r) *reinterpret_cast<uint4*>(bm + ic[r]) = t[r];
        }
    } else {
        for (uint32_t i = threadIdx.x; i < a.nwords; i += kF2Threads) bm[i] = bsrc[i];
    }
    // ring of kF2Ring sub-steps (one 16-B load per lane each) in flight: 32 KB per CU.
    // Loads past the block's range are clamped to its last 16 B (cache hits, masked).
    // (the ring's first loads take most of this phase's ~4 µs: all CUs start their streams at
    // once; the 64 KB bitmap copy alone is ~1 µs)
    const uint32_t lim = min(d.lim, ((hi + 3u) & ~3u) - 4u);
    const __amdgpu_buffer_rsrc_t rs = f2_rsrc(w0, lo, lim);
    uint4 ring[kF2Ring];
#pragma unroll
    for (uint32_t r = 0; r < kF2Ring; ++r)
        ring[r] = Subs ? f2_load1<NT>(rs, lo, lo + r * kF2Sub, lim) : f2_load1g(w0, lo + r * kF2Sub, lim);
    if (Win) {
        if (threadIdx.x < a.wwords) bm[threadIdx.x] = wv0;
        if (threadIdx.x + kF2Threads < a.wwords) bm[threadIdx.x + kF2Threads] = wv1;
    }
    if (threadIdx.x < 3) misc[threadIdx.x] = 0;
    for (uint32_t i = threadIdx.x; i <= np / 32; i += kF2Threads) lost[i] = 0;
    sync_lds();
    F2_STAMP(1);
    // Dense mode: stage fill `cnt` is block-uniform.  Sub-step s reserves slots with one
    // LDS atomic per wave on counter misc[s % 3]; after the sub-step's barrier every wave
    // adds that counter to cnt.  The counter of sub-step s + 1 is zeroed during sub-step s
    // (before its barrier), when every read of its previous use (sub-step s - 2) is complete.
    // Sparse mode: one counter misc[0] for the whole block, read after the final barrier.
    uint32_t cnt = 0, s3 = 0;
    for (uint32_t c0 = lo; c0 < hi; c0 += kF2Ring * kF2Sub) {
        if (Mode == kF2Seg && c0 != lo && (c0 - lo) % a.seg == 0) {
            // segment boundary (block-uniform): flush while the ring's next loads are in flight
            sync_lds();
            f2_flush<0, Per, Win>(a, misc[0] < a.stage ? misc[0] : a.stage, stage, hist, wsum, poff, 0u);
            if (threadIdx.x == 0) misc[0] = 0;
            sync_lds();
        }
#pragma unroll
        for (uint32_t r = 0; r < kF2Ring; ++r) {
            const uint32_t sb = c0 + r * kF2Sub;
            if (sb < hi) {   // block-uniform
                if (Mode == kF2Dense && cnt > a.stage - kF2Sub) {
                    f2_flush<0, Per, Win>(a, cnt, stage, hist, wsum, poff, 0u);
                    cnt = 0;
                }
                const uint32_t j0 = sb + 4 * threadIdx.x;
                const uint32_t v4[4] = {ring[r].x, ring[r].y, ring[r].z, ring[r].w};
                // lanes past hi (the block's last sub-step only) are masked by one compare
                // against the sub-step's remaining length (block-uniform)
                const uint32_t rem = hi - sb;
                bool sv[4];
                uint64_t bal[4];
                // the four bitmap words first (one LDS wait for all four: read one at a time, each
                // read waited before the next issued)
                uint32_t bw[4];
#pragma unroll
                for (uint32_t f = 0; f < 4; ++f) bw[f] = bm[__builtin_amdgcn_ubfe(v4[f], pre_off + 5, lm5) - wbase];
#pragma unroll
                for (uint32_t f = 0; f < 4; ++f) {
                    // prefix bit: word pre >> 5 of the bitmap, bit pre & 31 (v_bfe masks it)
                    const uint32_t pre = __builtin_amdgcn_ubfe(v4[f], pre_off, a.Lm);
                    const bool hit = __builtin_amdgcn_ubfe(bw[f], pre, 1) != 0, in = tid4 + f < rem;
                    sv[f] = hit && in;
                    bal[f] = __builtin_amdgcn_ballot_w64(hit) & __builtin_amdgcn_ballot_w64(in);
                }
                const uint32_t tot = (uint32_t)(__popcll(bal[0]) + __popcll(bal[1]) + __popcll(bal[2]) +
                                                __popcll(bal[3]));
                uint32_t base = 0;
                const uint32_t ctr_i = Mode == kF2Dense ? s3 : 0u;
                if (lane == 0 && tot) base = atomicAdd(misc + ctr_i, tot);
                uint32_t pos = __builtin_amdgcn_readfirstlane(base);
                if (Mode == kF2Dense) {
                    pos += cnt;
                    const uint32_t s3n = s3 == 2 ? 0u : s3 + 1;
                    if (threadIdx.x == 0) misc[s3n] = 0;
                    s3 = s3n;
                }
                if (Mode == kF2Dense || pos + tot <= a.stage) {   // wave-uniform
#pragma unroll
                    for (uint32_t f = 0; f < 4; ++f) {
                        if (sv[f]) {
                            const uint32_t at = __builtin_amdgcn_mbcnt_hi(
                                (uint32_t)(bal[f] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal[f], pos));
                            stage_put<Fmt>(stage, a.stage, lo, at, v4[f], j0 + f, pk);
                        }
                        pos += (uint32_t)__popcll(bal[f]);
                    }
                } else {
                    // sparse-mode overflow (never on uniform ids; clustered ids): an entry past
                    // the stage is dropped and its partition marked lost -- the block then
                    // pushes that partition's count past the F3 stage, so F3 sends its targets
                    // to the exact fallback scan (no per-entry global atomics on a hot counter)
#pragma unroll
                    for (uint32_t f = 0; f < 4; ++f) {
                        if (sv[f]) {
                            const uint32_t at = __builtin_amdgcn_mbcnt_hi(
                                (uint32_t)(bal[f] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal[f], pos));
                            if (at < a.stage) {
                                stage_put<Fmt>(stage, a.stage, lo, at, v4[f], j0 + f, pk);
                            } else {
                                const uint32_t p = top_bits(v4[f], a.b1);
                                atomicOr(lost + (p >> 5), 1u << (p & 31));
                            }
                        }
                        pos += (uint32_t)__popcll(bal[f]);
                    }
                }
                if (Mode == kF2Dense) {
                    sync_lds();
                    cnt += misc[s3 == 0 ? 2u : s3 - 1];
                }
            }
            ring[r] = Subs ? f2_load1<NT>(rs, lo, sb + kF2Ring * kF2Sub, lim) : f2_load1g(w0, sb + kF2Ring * kF2Sub, lim);
        }
    }
    if (Sparse) {
        sync_lds();
        cnt = misc[0] < a.stage ? misc[0] : a.stage;
    }
    F2_STAMP(2);
    if (cnt) f2_flush<Fmt, Per, Win>(a, cnt, stage, hist, wsum, poff, lo, pk);
    if (Sparse) {   // partitions that lost entries: count past any stage (F3 -> fallback)
        for (uint32_t i = threadIdx.x; i <= np / 32; i += kF2Threads) {
            uint32_t m = lost[i];
            while (m) {
                const uint32_t b = (uint32_t)__ffs(m) - 1;
                m &= m - 1;
                atomicAdd(a.pcount + (a.nsets == 1 ? 0u : blockIdx.x % kSets) * a.np_all + poff + 32 * i + b, a.pcap + 1u);
            }
        }
    }
    F2_STAMP(5);
}

// ---- F2 direct (prefix-sorted sub-partitions): no stage, no flush ------------------------
// Over sorted sub-partitions a workgroup's contiguous id range is a contiguous run of partitions,
// and every partition strictly inside the range belongs to this workgroup alone.  So each wave
// writes its survivors straight to their partition's bucket: per sub-step it ranks its survivors
// (ballot + mbcnt; the 256 ids of a wave's sub-step are consecutive in sorted order, so they meet
// one partition, rarely two) and reserves the run with ONE LDS atomic on the partition's counter
// -- a returning global atomic only for the range's first and last partitions when a neighbouring
// workgroup shares them.  At the end the owned partitions' counts are stored plainly.  The LDS
// holds the bitmap window and the counters only (a few KB, where the staged forms filled the CU's
// 160 KB), so F3 workgroups of another call in flight fit beside it, and the stream never stops
// for a flush (the segmented window stage flushed ~6 times per workgroup at the cfg-3 broadcast
// rank).  A partition past its bucket capacity keeps counting (F3 sends its targets to the
// fallback), as in the staged forms.
constexpr uint32_t kDirParts = 4096;   // LDS counters: partitions a range may own (more: global atomics)

template <uint32_t Src>
__global__ __launch_bounds__(kF2Threads) void k_f2_direct(F2Args a) {
    constexpr bool NT = Src == kF2SubsNT;
    extern __shared__ uint32_t sh[];   // misc[8] | bm[wwords] | cnt[kDirParts]
    uint32_t* misc = sh;
    uint32_t* bm = sh + 8;
    uint32_t* cnt = bm + a.wwords;
    const uint32_t sub = (uint32_t)a.blk_sub[blockIdx.x];
    const SubDesc d = a.subs[sub];
    const uint64_t lo64 = (uint64_t)(blockIdx.x - d.blk0) * d.per_blk;
    if (lo64 >= d.n) return;
    F2_STAMP(0);
    const uint32_t* const w0 = d.w0;
    const uint32_t np = 1u << a.b1, poff = sub * np;
    const uint32_t lo = (uint32_t)lo64;
    const uint32_t hi = (uint32_t)(lo64 + d.per_blk < d.n ? lo64 + d.per_blk : d.n);
    const uint32_t lane = lane_id();
    const uint32_t pre_off = 32 - a.Lm;
    const uint32_t lm5 = a.Lm > 5 ? a.Lm - 5 : 0u;
    const uint32_t tid4 = 4 * threadIdx.x;
    const uint32_t lim = min(d.lim, ((hi + 3u) & ~3u) - 4u);
    const __amdgpu_buffer_rsrc_t rs = f2_rsrc(w0, lo, lim);
    // the range's first and last words (sorted: its smallest and largest prefixes) and their
    // neighbours outside the range, in one round trip: the bitmap window's base and the partitions
    // a neighbouring workgroup shares
    const uint32_t f0 = __builtin_amdgcn_readfirstlane(w0[lo]);
    const uint32_t fl = __builtin_amdgcn_readfirstlane(w0[hi - 1]);
    const uint32_t fp = lo > 0 ? __builtin_amdgcn_readfirstlane(w0[lo - 1]) : 0u;
    const uint32_t fn = hi < d.n ? __builtin_amdgcn_readfirstlane(w0[hi]) : 0u;
    const uint32_t wbase = a.Lm > 5 ? f0 >> (pre_off + 5) : 0u;
    const uint32_t p_first = top_bits(f0, a.b1), p_last = top_bits(fl, a.b1);
    const bool sh_first = lo > 0 && top_bits(fp, a.b1) == p_first;
    const bool sh_last = hi < d.n && top_bits(fn, a.b1) == p_last;
    const uint32_t* bsrc = a.bitmap + sub * a.nwords;
    const uint32_t i0 = wbase + threadIdx.x, i1 = i0 + kF2Threads;
    const uint32_t wv0 = threadIdx.x < a.wwords && i0 < a.nwords ? bsrc[i0] : 0u;
    const uint32_t wv1 = threadIdx.x + kF2Threads < a.wwords && i1 < a.nwords ? bsrc[i1] : 0u;
    uint4 ring[kF2Ring];
#pragma unroll
    for (uint32_t r = 0; r < kF2Ring; ++r) ring[r] = f2_load1<NT>(rs, lo, lo + r * kF2Sub, lim);
    if (threadIdx.x < a.wwords) bm[threadIdx.x] = wv0;
    if (threadIdx.x + kF2Threads < a.wwords) bm[threadIdx.x + kF2Threads] = wv1;
    for (uint32_t i = threadIdx.x; i < kDirParts; i += kF2Threads) cnt[i] = 0;
    sync_lds();
    F2_STAMP(1);
    uint32_t* const pc = a.pcount + poff;   // one bucket set (nsets == 1)
    uint2* const pb = a.pbuf + (uint64_t)poff * a.pcap;
    for (uint32_t c0 = lo; c0 < hi; c0 += kF2Ring * kF2Sub) {
#pragma unroll
        for (uint32_t r = 0; r < kF2Ring; ++r) {
            const uint32_t sb = c0 + r * kF2Sub;
            if (sb < hi) {   // block-uniform
                const uint32_t j0 = sb + tid4;
                const uint32_t v4[4] = {ring[r].x, ring[r].y, ring[r].z, ring[r].w};
                const uint32_t rem = hi - sb;
                uint32_t bw[4];
#pragma unroll
                for (uint32_t f = 0; f < 4; ++f) bw[f] = bm[__builtin_amdgcn_ubfe(v4[f], pre_off + 5, lm5) - wbase];
                bool sv[4];
                uint64_t bal[4], any = 0;
#pragma unroll
                for (uint32_t f = 0; f < 4; ++f) {
                    const uint32_t pre = __builtin_amdgcn_ubfe(v4[f], pre_off, a.Lm);
                    sv[f] = __builtin_amdgcn_ubfe(bw[f], pre, 1) != 0 && tid4 + f < rem;
                    bal[f] = __builtin_amdgcn_ballot_w64(sv[f]);
                    any |= bal[f];
                }
                if (any) {   // wave-uniform
                    // the wave's survivors meet partitions [plo, phi] (ascending with the lane)
                    const uint32_t l0 = (uint32_t)__ffsll((long long)any) - 1, l1 = 63u - (uint32_t)__clzll(any);
                    const uint32_t mylo = sv[0] ? v4[0] : sv[1] ? v4[1] : sv[2] ? v4[2] : v4[3];
                    const uint32_t myhi = sv[3] ? v4[3] : sv[2] ? v4[2] : sv[1] ? v4[1] : v4[0];
                    const uint32_t plo = top_bits((uint32_t)__builtin_amdgcn_readlane((int)mylo, (int)l0), a.b1);
                    const uint32_t phi = top_bits((uint32_t)__builtin_amdgcn_readlane((int)myhi, (int)l1), a.b1);
                    for (uint32_t p = plo; p <= phi; ++p) {   // wave-uniform, usually one pass
                        uint64_t bp[4];
                        uint32_t tot = 0;
#pragma unroll
                        for (uint32_t f = 0; f < 4; ++f) {
                            bp[f] = plo == phi ? bal[f] : bal[f] & __builtin_amdgcn_ballot_w64(top_bits(v4[f], a.b1) == p);
                            tot += (uint32_t)__popcll(bp[f]);
                        }
                        if (!tot) continue;
                        const uint32_t pl = p - p_first;
                        const bool glob = (p == p_first && sh_first) || (p == p_last && sh_last) || pl >= kDirParts;
                        uint32_t base = 0;
                        if (lane == 0) base = glob ? atomicAdd(pc + p, tot) : atomicAdd(cnt + pl, tot);
                        uint32_t pos = __builtin_amdgcn_readfirstlane(base);
#pragma unroll
                        for (uint32_t f = 0; f < 4; ++f) {
                            if ((bp[f] >> lane) & 1ull) {
                                const uint32_t at = __builtin_amdgcn_mbcnt_hi(
                                    (uint32_t)(bp[f] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bp[f], pos));
                                if (at < a.pcap) pb[(uint64_t)p * a.pcap + at] = make_uint2(v4[f], j0 + f);
                            }
                            pos += (uint32_t)__popcll(bp[f]);
                        }
                    }
                }
            }
            ring[r] = f2_load1<NT>(rs, lo, sb + kF2Ring * kF2Sub, lim);
        }
    }
    sync_lds();
    F2_STAMP(2);
    // the owned partitions' counts (shared ones were counted in place)
    const uint32_t nown = min(p_last - p_first + 1u, kDirParts);
    for (uint32_t i = threadIdx.x; i < nown; i += kF2Threads) {
        const uint32_t p = p_first + i;
        if (!((p == p_first && sh_first) || (p == p_last && sh_last))) pc[p] = cnt[i];
    }
    (void)misc;
    F2_STAMP(5);
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
// Setup: the partition's survivors (F2 bucket) and targets (F1 bucket) are loaded together;
// the survivors are counting-sorted into LDS by their prefix bits [b1, Lq).  Queries, per
// chunk of kF3Threads targets:
//   A  G lanes per target (G = 4, 2 or 1 as the chunk fills the block): each lane keeps a
//      register-resident sorted top-K of its share of the subtree's candidates keyed by
//      (w0 distance, LDS position), the group merges them (DPP butterflies) -- exact
//      unless two candidates' w0 words tie at or above the k-th place, which the group
//      detects (adjacent equal distances, or an evicted distance equal to the k-th);
//      such a target's candidates are handed to F4 (a wave per target, off this block's
//      critical path) while one of the partition's kTieSlots slots is free;
//   B  the remaining ties and large subtrees: one WAVE per target here, exact order by
//      the full 160-bit key (words 1..4 read from the id planes).
// Targets whose subtree holds fewer than min(k, n) ids go to the F4 fallback list.
constexpr uint32_t kLaneMax = 256;   // largest subtree a lane scans alone

__host__ __device__ inline uint32_t f3_words(uint32_t nsub) {
    return (nsub + 1 + 17 + kF3Threads + 1 + 2 + 1) & ~1u;
}

// Record form (dhtgpu_batch_topk_dev with out_rec): every K6 writer of a result row -- F3's fast
// path, the wave paths of F3 and F4 (ties, large subtrees), F4's fallback scan and its split merge
// -- stores the row's compact records {w0, w1, global idx} itself, from the words it already holds
// (word 0 from the LDS stage when the stage holds unshifted words, word 1 where the wave paths
// loaded it) and a gather from the planes otherwise.  No conversion pass follows K6: the 65,536 x 8
// gathers of a separate pass cost 23 us on the chain at cfg 2, the pass over the rows F3 left 2 us
// (profiles/r05/b, r05/g/ablation_f).
struct RecOut {
    uint32_t* out;            // nullable: q * k * 3 words
    const uint32_t* planes;   // the context's (unshifted) planes; record words of context-local indices
    uint64_t stride;
    const uint32_t* gidx;     // context-local -> global index (nullable) ...
    uint32_t base;            // ... or offset
    uint32_t w0_direct;       // the F3 stage holds unshifted word 0 (one set, no shard shift)
    // else F3's fast path rebuilds word 0 from the stage's shifted word: every id of the set (of a
    // sub-partition: w0_pre | its index) shares its top w0_shift bits (no plane read per result: at
    // the cfg-3 broadcast rank the results touch every line of the planes they are read from)
    uint32_t w0_shift, w0_pre;
};

// place r of target qi's records: the id at index x of the writer's set (a.planes: the context's,
// or a sub-partition's with a.gidx mapping x to the context-local index); w0 when the caller holds
// the unshifted word (w0_ok), else read; w1 as loaded by the caller.  x == DHT_NONE: an empty place.
__device__ __forceinline__ void rec_place(const RecOut& o, const uint32_t* __restrict__ planes, const uint32_t* gidx,
                                          uint32_t base, uint32_t k, uint32_t qi, uint32_t r, uint32_t x, uint32_t w0,
                                          bool w0_ok, uint32_t w1) {
    uint32_t* ro = o.out + ((uint64_t)qi * k + r) * 3;
    if (x == DHT_NONE) {
        ro[0] = DHT_NONE;
        ro[1] = DHT_NONE;
        ro[2] = DHT_NONE;
        return;
    }
    const uint32_t cl = gidx ? gidx[x] : x + base;   // context-local
    ro[0] = w0_ok ? w0 : planes[x];
    ro[1] = w1;
    ro[2] = o.gidx ? o.gidx[cl] : cl + o.base;
}

struct F3Args {
    const uint2* pbuf; uint32_t* pcount; uint32_t pcap;
    const uint2* tbuf; uint32_t* tcount; uint32_t tcap;   // F1 target buckets (tcount all-zero between calls)
    const uint32_t* tspill;
    uint32_t Lm, b1, Lq;
    uint32_t* bitmap; uint32_t nwords;
    const uint32_t* planes; uint64_t stride; uint64_t n;
    const uint32_t* tp; uint64_t ts; uint32_t k;
    const uint32_t* gidx; uint32_t base;
    uint32_t* out_idx; uint32_t* out_cnt;
    uint32_t* ctr; uint32_t* fb_list;   // ctr[0] = fallback targets
    uint8_t* fb_sub;                     // [q] the listed target's sub-partition (255: scan the whole set)
    uint32_t* pstat;                     // [np] survivors per partition (statistics; plain stores)
    uint4* tie_hdr;                      // [np][kTieSlots] deferred ties {qi, t0, count, 0}
    uint2* tie_cand;                     // [np][kTieSlots][64] their candidates {w0, idx}
    uint32_t* tie_cnt;                   // [np] deferred-tie slots in use per partition (all-zero between calls)
    const SubDesc* subs; uint32_t np_sub;   // sub-partitions, partitions per sub-partition
    uint32_t dbg;
    unsigned long long* stamps;          // dbg & 256: per-block phase timestamps [np][16]
    uint32_t cap;                        // LDS stage entries (the plan's, <= kF3Cap)
    RecOut rec;                          // record form: F3's fast path writes compact records itself
    uint32_t Lmin;                       // coarsest complete level: Lm, or Lm - 1 with sibling marking (F1)
    uint32_t nsets;                      // F2's bucket sets per partition (pbuf stride): kSets or 1
};

// [lo, hi) of the deepest level L in [Lmin, Lq] whose subtree sub(t, L) holds >= want survivors
// (survivors sorted by their prefix bits [b1, Lq); sq = t's bits [b1, Lq)).  Every level in
// [Lmin, Lq] that the loop can stop at is complete among the survivors: a target's level-Lm subtree
// is marked whole, and with sibling marking its level-(Lm - 1) subtree too whenever the level-Lm one
// holds fewer than k ids -- the loop only reaches Lm - 1 for such a target.
__device__ __forceinline__ void level_range(const uint32_t* sofs, uint32_t sq, uint32_t Lq, uint32_t Lmin, uint32_t want,
                                            uint32_t& lo, uint32_t& hi) {
    uint32_t L = Lq + 1;
    do {
        --L;
        const uint32_t sh_l = Lq - L;
        lo = sofs[(sq >> sh_l) << sh_l];
        hi = sofs[((sq >> sh_l) + 1) << sh_l];
    } while (hi - lo < want && L > Lmin);
}

// (w0 distance, w1 distance, index) order; words 2..4 are read only when both distances tie
__device__ __forceinline__ bool key2_less(uint32_t da, uint32_t a1, uint32_t ia, uint32_t db, uint32_t b1, uint32_t ib,
                                          const uint32_t* __restrict__ planes, uint64_t stride, const uint32_t* t) {
    if (da != db) return da < db;
    if (a1 != b1) return a1 < b1;
    return id_less(da, ia, db, ib, planes, stride, t);
}

// rank of this lane's candidate by (w0 distance md, w1 distance m1) among the mm candidates of
// lanes [0, mm) (mm wave-uniform): a branch-free count over readlanes.  *tie: another candidate
// has the same 64-bit distance (only then does the order need words 2..4 and the index).  The
// branchy form (full-key compare inside the loop) ran ~135 ns per candidate: exec-mask saves and
// scalar branches around every readlane (S2 stamps, profiles/r04/experiments/s2_stamps.txt).
__device__ __forceinline__ uint32_t wave_rank64(uint32_t md, uint32_t m1, uint32_t mm, uint32_t lane, bool* tie) {
    uint32_t rank = 0, eq = 0;
    for (uint32_t o = 0; o < mm; ++o) {
        const uint32_t xd = (uint32_t)__builtin_amdgcn_readlane((int)md, (int)o);
        const uint32_t x1 = (uint32_t)__builtin_amdgcn_readlane((int)m1, (int)o);
        rank += (uint32_t)(xd < md) | ((uint32_t)(xd == md) & (uint32_t)(x1 < m1));
        eq |= (uint32_t)(xd == md) & (uint32_t)(x1 == m1) & (uint32_t)(o != lane);
    }
    *tie = eq != 0;
    return rank;
}

// exact answer for one target from <= 64 candidates, one per lane (lane < mm): its rank is
// the number of candidates strictly closer by (w0, w1) distance (full key on a double tie).
// Word 1 and the target are loaded unconditionally (clamped), in one round trip.
// (the ranking itself, once word 1 of this lane's candidate and the target's words are loaded)
__device__ void wave_rank_loaded(const F3Args& a, uint2 me, uint32_t mm, uint32_t qi, uint32_t t0, uint32_t want,
                                 uint32_t lane, uint32_t w1, const uint32_t* t) {
    const bool act = lane < mm;
    const uint32_t md = me.x ^ t0;
    const uint32_t m1 = act ? w1 ^ t[1] : DHT_NONE;
    bool tie;
    uint32_t rank = wave_rank64(md, m1, mm, lane, &tie);
    if (__ballot(act && tie)) {   // a 64-bit distance tie (duplicate ids): the full key decides
        rank = 0;
        for (uint32_t o = 0; o < mm; ++o) {
            const uint32_t xd = __builtin_amdgcn_readlane((int)md, (int)o);
            const uint32_t x1 = __builtin_amdgcn_readlane((int)m1, (int)o);
            const uint32_t xi = __builtin_amdgcn_readlane((int)me.y, (int)o);
            if (xd < md || (xd == md && x1 < m1)) ++rank;
            else if (xd == md && x1 == m1 && act && o != lane && id_less(xd, xi, md, me.y, a.planes, a.stride, t)) ++rank;
        }
    }
    if (a.rec.out) {   // record form (the candidates' word 0 as staged)
        if (act && rank < want) rec_place(a.rec, a.planes, a.gidx, a.base, a.k, qi, rank, me.y, me.x, a.rec.w0_direct, w1);
        if (lane >= want && lane < a.k) rec_place(a.rec, a.planes, a.gidx, a.base, a.k, qi, lane, DHT_NONE, 0u, true, 0u);
        return;
    }
    uint32_t* orow = a.out_idx + (uint64_t)qi * a.k;
    if (act && rank < want) orow[rank] = map_out(me.y, a.gidx, a.base);
    if (lane >= want && lane < a.k) orow[lane] = DHT_NONE;
    if (lane == 0) a.out_cnt[qi] = want;
}

__device__ void wave_rank_answer(const F3Args& a, uint2 me, uint32_t mm, uint32_t qi, uint32_t t0, uint32_t want,
                                 uint32_t lane) {
    const uint32_t w1 = a.planes[a.stride + (lane < mm ? me.y : 0u)];
    uint32_t t[DHT_W];
    load_target(a.tp, a.ts, qi, t);
    wave_rank_loaded(a, me, mm, qi, t0, want, lane, w1, t);
}

// exact wave-cooperative answer for one target (ties on w0, large subtrees).  Every lane
// gathers word 1 of its candidate up front (one round trip for the whole wave), so the
// ordering loops below compare (w0, w1) distances in registers.
__device__ void f3_wave_answer(const F3Args& a, const uint2* S, uint32_t lo, uint32_t hi, uint32_t qi,
                               uint32_t t0, uint32_t want, uint32_t lane) {
    const uint32_t mm = hi - lo;
    if (mm <= 64) {
        wave_rank_answer(a, S[lo + (lane < mm ? lane : 0u)], mm, qi, t0, want, lane);
        return;
    }
    uint32_t t[DHT_W];
    load_target(a.tp, a.ts, qi, t);
    uint32_t* orow = a.out_idx + (uint64_t)qi * a.k;
    {
        // running lane-distributed top-`want` list of (w0 distance, w1 distance, index)
        uint32_t ed = DHT_NONE, e1 = DHT_NONE, ei = DHT_NONE, cnt = 0;
        for (uint32_t c = lo; c < hi; c += 64) {
            const bool v = c + lane < hi;
            const uint2 x = v ? S[c + lane] : make_uint2(0u, DHT_NONE);
            const uint32_t xd = x.x ^ t0, xi = x.y;
            const uint32_t x1 = v ? a.planes[a.stride + xi] ^ t[1] : DHT_NONE;
            uint32_t wd = cnt == want ? __builtin_amdgcn_readlane((int)ed, want - 1) : DHT_NONE;
            uint32_t w1 = cnt == want ? __builtin_amdgcn_readlane((int)e1, want - 1) : DHT_NONE;
            uint32_t wi = cnt == want ? __builtin_amdgcn_readlane((int)ei, want - 1) : DHT_NONE;
            uint64_t cm = __ballot(v && (cnt < want || key2_less(xd, x1, xi, wd, w1, wi, a.planes, a.stride, t)));
            while (cm) {
                const uint32_t l = (uint32_t)__ffsll((long long)cm) - 1;
                cm &= cm - 1;
                const uint32_t cd = __builtin_amdgcn_readlane((int)xd, l), c1 = __builtin_amdgcn_readlane((int)x1, l);
                const uint32_t ci = __builtin_amdgcn_readlane((int)xi, l);
                if (cnt == want && !key2_less(cd, c1, ci, wd, w1, wi, a.planes, a.stride, t)) continue;
                const bool closer = lane < cnt && key2_less(ed, e1, ei, cd, c1, ci, a.planes, a.stride, t);
                const uint32_t pos = (uint32_t)__popcll(__ballot(closer));
                const uint32_t ud = __shfl_up(ed, 1), u1 = __shfl_up(e1, 1), ui = __shfl_up(ei, 1);
                if (lane == pos) { ed = cd; e1 = c1; ei = ci; }
                else if (lane > pos) { ed = ud; e1 = u1; ei = ui; }
                cnt = cnt + 1 < want ? cnt + 1 : want;
                wd = cnt == want ? __builtin_amdgcn_readlane((int)ed, want - 1) : DHT_NONE;
                w1 = cnt == want ? __builtin_amdgcn_readlane((int)e1, want - 1) : DHT_NONE;
                wi = cnt == want ? __builtin_amdgcn_readlane((int)ei, want - 1) : DHT_NONE;
            }
        }
        if (a.rec.out) {   // record form: word 0 / word 1 back from the distances
            if (lane < a.k)
                rec_place(a.rec, a.planes, a.gidx, a.base, a.k, qi, lane, lane < want ? ei : DHT_NONE, ed ^ t0,
                          a.rec.w0_direct, e1 ^ t[1]);
            return;
        }
        if (lane < want) orow[lane] = map_out(ei, a.gidx, a.base);
    }
    if (lane >= want && lane < a.k) orow[lane] = DHT_NONE;
    if (lane == 0) a.out_cnt[qi] = want;
}

// Merge the top-K list of this lane with its DPP partner's (CTRL: quad_perm lane ^ 1 or ^ 2):
// both lists ascending, so min(mine[r], partner[K-1-r]) holds the K smallest of the union as a
// bitonic sequence (the max side -- the K that leave -- lowers lmin); a half-cleaner network
// then sorts it.  Both partners end with the same list.
template <int K, int CTRL>
__device__ __forceinline__ void f3_merge(uint32_t (&key)[K], uint32_t& lmin) {
    uint32_t b[K];
#pragma unroll
    for (int r = 0; r < K; ++r) b[r] = (uint32_t)__builtin_amdgcn_mov_dpp((int)key[K - 1 - r], CTRL, 0xF, 0xF, true);
    lmin = min(lmin, (uint32_t)__builtin_amdgcn_mov_dpp((int)lmin, CTRL, 0xF, 0xF, true));
#pragma unroll
    for (int r = 0; r < K; ++r) {
        lmin = min(lmin, max(key[r], b[r]));
        key[r] = min(key[r], b[r]);
    }
#pragma unroll
    for (int d = K / 2; d >= 1; d >>= 1) {
#pragma unroll
        for (int r = 0; r < K; ++r) {
            if (r & d) continue;
            const uint32_t x = min(key[r], key[r + d]), y = max(key[r], key[r + d]);
            key[r] = x;
            key[r + d] = y;
        }
    }
}

#define F3_STAMP(i) \
    do { if (Diag && (a.dbg & 256) && threadIdx.x == 0) a.stamps[(uint64_t)blockIdx.x * 16 + (i)] = __builtin_amdgcn_s_memrealtime(); } while (0)

// Diag: the DHTGPU_DBG build (phase stamps and ablation exits); production launches Diag = false.
// Exact: k == K and n >= k, so want == K is a compile-time constant (no per-place masks).
// Subs: the call serves several prefix sub-partitions (tie words and result maps per partition);
// the one-set instantiation keeps every pointer a kernel argument, so the compiler emits global
// (not flat) loads through them
template <int K, bool Diag, bool Exact, bool Subs>
__global__ __launch_bounds__(kF3Threads) void k_f3_answer(F3Args a) {
    extern __shared__ uint32_t sh[];
    const uint32_t p = blockIdx.x, np = gridDim.x;   // partition over all sub-partitions
    const uint32_t sub = p / a.np_sub, pl = p - sub * a.np_sub;
    if (Subs && a.np_sub != np) {   // tie words and result maps of the partition's sub-partition (a.n stays the set's)
        const SubDesc d = a.subs[sub];
        a.planes = d.planes;
        a.stride = d.stride;
        a.gidx = d.gidx;
        a.base = d.base;
    }
    F3_STAMP(0);
    // survivors are sorted by their prefix bits [b1, Lq); a target answers from the deepest
    // level L in [Lm, Lq] whose subtree sub(t, L) holds >= want ids (a contiguous range)
    const uint32_t nsub = 1u << (a.Lq - a.b1);
    uint32_t* sofs = sh;                      // [nsub + 1]
    uint32_t* wsum = sofs + nsub + 1;         // [17]
    uint32_t* slow = wsum + 17;               // [kF3Threads + 1] slow-path target slots, count last
    uint32_t* ntie = slow + kF3Threads + 1;   // [0] deferred-tie slots taken, [1] wave-path targets (stat)
    uint2* S = reinterpret_cast<uint2*>(sh + f3_words(nsub));
    uint2* T = S + a.cap;
    // the bitmap is no longer read in this call: clear this block's share of its sub-partition's
    for (uint32_t i = pl + a.np_sub * threadIdx.x; i < a.nwords; i += a.np_sub * kF3Threads)
        a.bitmap[sub * a.nwords + i] = 0;
    for (uint32_t i = threadIdx.x; i <= nsub; i += kF3Threads) sofs[i] = 0;
    if (threadIdx.x == 0) ntie[0] = ntie[1] = 0;
    // survivors of this partition in each of the kSets bucket sets (F2) and its targets (F1) --
    // the counts and the first chunk of targets in one round trip; the survivors themselves are
    // gathered exactly once the counts are known (a speculative gather of fixed slots with the
    // counts fetched 2x the algorithmic bytes at cfg 2 for no measured gain)
    static_assert(kF3Cap / kSets == 2 * kF3Threads && kF3Per == 2 * kSets, "gather layout");
    uint32_t ms[kSets];
#pragma unroll
    for (uint32_t x = 0; x < kSets; ++x) ms[x] = a.pcount[x * np + p];
    const uint32_t mt0 = a.tcount[p * kCtrStride];   // targets of this partition (F1)
    const uint2* tsrc = a.tbuf + (uint64_t)p * a.tcap;
    const uint2 tfirst = tsrc[threadIdx.x < a.tcap ? threadIdx.x : 0u];
    uint2 e[kF3Per];
    const uint2* pb = a.pbuf + (uint64_t)p * a.nsets * a.pcap;
#pragma unroll
    for (uint32_t u = 0; u < kF3Per; ++u) e[u] = make_uint2(0u, 0u);
    const uint32_t mt = mt0 < a.tcap ? mt0 : a.tcap;
    if (p == 0) {   // spilled targets (foreign, or a full bucket) join the fallback list
        const uint32_t nsp = a.ctr[kSpill];
        if (nsp) {   // one reservation for the block
            if (threadIdx.x == 0) ntie[2] = atomicAdd(a.ctr, nsp);
            sync_lds();
            for (uint32_t j = threadIdx.x; j < nsp; j += kF3Threads) {
                a.fb_list[ntie[2] + j] = a.tspill[j];
                a.fb_sub[ntie[2] + j] = 255;
            }
        }
    }
    sync_lds();   // every thread has read the counts
    // set offsets inside the partition (soff[x] = entries of sets < x); over = a set overflowed
    uint32_t soff[kSets + 1];
    bool over = false;
    soff[0] = 0;
#pragma unroll
    for (uint32_t x = 0; x < kSets; ++x) {
        over = over || ms[x] > a.pcap;
        soff[x + 1] = soff[x] + (ms[x] < a.pcap ? ms[x] : a.pcap);
    }
    const uint32_t m = soff[kSets];
    if (threadIdx.x < kSets) a.pcount[threadIdx.x * np + p] = 0;   // all-zero again for the next call
    if (threadIdx.x == 0) {
        a.pstat[p] = m;
        a.tcount[p * kCtrStride] = 0;
        if (p == 0) a.ctr[kSpill] = 0;
    }
    if (mt == 0) return;   // no targets in this partition (block-uniform)
    F3_STAMP(1);
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    constexpr uint32_t NWV = kF3Threads / 64;
    if (m > a.cap || over) {
        // strongly clustered ids: this partition's targets take the exact brute-force path
        if (threadIdx.x == 0) ntie[2] = atomicAdd(a.ctr, mt);   // one reservation for the block
        sync_lds();
        for (uint32_t j = threadIdx.x; j < mt; j += kF3Threads) {
            a.fb_list[ntie[2] + j] = tsrc[j].y;
            a.fb_sub[ntie[2] + j] = (uint8_t)sub;
        }
        return;
    }
    const uint32_t smask = nsub - 1u;
    uint32_t rk[kF3Per];
    const uint32_t sq_sh = 32 - a.Lq;                            // sub-prefix = bfe(w, 32 - Lq, Lq - b1)
    // valid[u]: slot u holds one of the partition's entries
    uint32_t valid = 0;
    {
        // gather the partition exactly, entry j from set x (soff[x] <= j < soff[x + 1]) at slot
        // j - soff[x] -- only the m entries are loaded
#pragma unroll
        for (uint32_t u = 0; u < kF3Per; ++u) {
            const uint32_t j = u * kF3Threads + threadIdx.x;
            uint32_t x = 0, base = 0;
#pragma unroll
            for (uint32_t y = 1; y < kSets; ++y)
                if (j >= soff[y]) { x = y; base = soff[y]; }
            if (j < m) e[u] = pb[x * a.pcap + j - base];
            valid |= (uint32_t)(j < m) << u;
        }
    }
    // counting sort by sub-prefix: LDS histogram (ranks from the atomics), scan, placement
    // rk[u] = NONE marks an empty slot (the scatter tests the value: no exec masks kept live)
#pragma unroll
    for (uint32_t u = 0; u < kF3Per; ++u) {
        rk[u] = DHT_NONE;
        if ((valid >> u) & 1u) rk[u] = atomicAdd(sofs + __builtin_amdgcn_ubfe(e[u].x, sq_sh, a.Lq - a.b1), 1u);
    }
    sync_lds();
    F3_STAMP(2);
    scan_lds<kF3Threads>(sofs, nsub, wsum);
    if (threadIdx.x == 0) sofs[nsub] = m;
    sync_lds();
#pragma unroll
    for (uint32_t u = 0; u < kF3Per; ++u)
        if (rk[u] != DHT_NONE) S[sofs[__builtin_amdgcn_ubfe(e[u].x, sq_sh, a.Lq - a.b1)] + rk[u]] = e[u];
    F3_STAMP(3);
    const uint32_t want = Exact ? (uint32_t)K : (a.n < a.k ? (uint32_t)a.n : a.k);
    const bool full_row = Exact && ((uintptr_t)a.out_idx & 15) == 0;
    for (uint32_t t0i = 0; t0i < mt; t0i += kF3Threads) {
        const uint32_t mtr = mt - t0i < kF3Threads ? mt - t0i : kF3Threads;
        if (threadIdx.x < mtr) T[threadIdx.x] = t0i ? tsrc[t0i + threadIdx.x] : tfirst;
        if (threadIdx.x == 0) slow[kF3Threads] = 0;
        sync_lds();
        if (t0i == 0) F3_STAMP(4);
        // A: G lanes per target (G = 4 / 2 / 1 as the chunk's targets fill the block).  Lane
        // j of a group scans candidates lo + j, lo + j + G, ... into its own top-K and the
        // group merges its lists with DPP butterflies (f3_merge).  G = 1 deals the targets
        // round-robin over the waves so that every SIMD runs a share of the candidate loops.
        const uint32_t G = a.Lmin >= 12 ? (mtr <= kF3Threads / 4 ? 4u : mtr <= kF3Threads / 2 ? 2u : 1u) : 1u;
        const uint32_t slot = G == 4 ? threadIdx.x >> 2 : G == 2 ? threadIdx.x >> 1 : lane * NWV + wv;
        const uint32_t gj = threadIdx.x & (G - 1);
        // one set (no sub-partitions): a group leader's tied target, answered inline by its wave
        uint32_t tq = 0, tt0 = 0, tlo = 0, thi = 0;
        bool tinl = false;
        if (slot < mtr) {   // group-uniform from here on
            const uint2 te = T[slot];
            const uint32_t t0 = te.x, qi = te.y;
            // deepest level L in [Lmin, Lq] with >= want ids in sub(t, L)
            uint32_t lo = 0, hi = 0;
            level_range(sofs, top_bits(t0, a.Lq) & smask, a.Lq, a.Lmin, want, lo, hi);
            const uint32_t mm = hi - lo;
            if (t0i == 0) F3_STAMP(8);
            if (mm < want) {
                if (gj == 0) {
                    const uint32_t at = atomicAdd(a.ctr, 1u);
                    a.fb_list[at] = qi;
                    a.fb_sub[at] = (uint8_t)sub;
                }
            } else if (mm > kLaneMax || a.Lm == 0) {
                if (gj == 0) {
                    slow[atomicAdd(slow + kF3Threads, 1u)] = slot;
                    atomicAdd(ntie + 1, 1u);
                }
            } else {
                uint32_t dk[K], ok[K];
                uint32_t rmin = DHT_NONE;   // smallest distance that left (or never entered) the list
                if (a.Lmin >= 12) {
                    // packed keys (w0 distance << 12 | LDS position): distances are below
                    // 2^(32 - Lmin) <= 2^20 and positions below kF3Cap = 2^12, so the key order
                    // is the (distance, position) order; one v_med3 per slot inserts
                    uint32_t key[K];
#pragma unroll
                    for (int r = 0; r < K; ++r) key[r] = DHT_NONE;
                    uint32_t lmin = DHT_NONE;   // smallest key that left the list
                    uint32_t o = lo + gj;
                    uint32_t nxt = S[o < hi ? o : lo].x;   // next candidate's word, read ahead
                    for (; o < hi; o += G) {
                        const uint32_t c = ((nxt ^ t0) << 12) | o;
                        nxt = S[o + G < hi ? o + G : o].x;
                        lmin = min(lmin, max(c, key[K - 1]));
#pragma unroll
                        for (int r = K - 1; r > 0; --r) key[r] = med3_u32(key[r - 1], key[r], c);
                        key[0] = min(key[0], c);
                    }
                    if (t0i == 0) F3_STAMP(9);
                    if (G >= 2) f3_merge<K, 0xB1>(key, lmin);   // quad_perm [1,0,3,2]: lane ^ 1
                    if (G == 4) f3_merge<K, 0x4E>(key, lmin);   // quad_perm [2,3,0,1]: lane ^ 2
#pragma unroll
                    for (int r = 0; r < K; ++r) {
                        dk[r] = key[r] == DHT_NONE ? DHT_NONE : key[r] >> 12;
                        ok[r] = key[r] & 0xFFFu;
                    }
                    rmin = lmin == DHT_NONE ? DHT_NONE : lmin >> 12;
                } else {
#pragma unroll
                    for (int r = 0; r < K; ++r) { dk[r] = DHT_NONE; ok[r] = DHT_NONE; }
                    uint32_t nxt = S[lo].x;
                    for (uint32_t o = lo; o < hi; ++o) {
                        const uint32_t d = nxt ^ t0;   // < 2^(32 - Lm) <= 2^31 < NONE
                        nxt = S[o + 1 < hi ? o + 1 : o].x;
                        const bool ins = d < dk[K - 1];
                        rmin = min(rmin, ins ? dk[K - 1] : d);
                        if (ins) {
#pragma unroll
                            for (int r = K - 1; r > 0; --r) {
                                const bool up = d < dk[r - 1];
                                const bool here = d < dk[r];
                                ok[r] = up ? ok[r - 1] : (here ? o : ok[r]);
                                dk[r] = up ? dk[r - 1] : (here ? d : dk[r]);
                            }
                            if (d < dk[0]) { dk[0] = d; ok[0] = o; }
                        }
                    }
                }
                // ties on w0 at or above the want-th place need the full key: equal
                // neighbours among places [0, want], or a distance that left the list
                // equal to the want-th
                if (t0i == 0) F3_STAMP(10);
                bool tie = rmin == dk[want - 1];
#pragma unroll
                for (int r = 0; r + 1 < K; ++r) tie = tie || ((uint32_t)r + 1 <= want && dk[r] == dk[r + 1]);
                if (tie && !Subs) {
                    if (gj == 0) {   // answered by the wave below, after the groups' results
                        tinl = true;
                        tq = qi;
                        tt0 = t0;
                        tlo = lo;
                        thi = hi;
                        atomicAdd(ntie + 1, 1u);
                    }
                } else if (tie) {
                    // sub-partitioned calls: hand the candidates to F4 (one wave per tie, off this
                    // block's critical path) while a slot is free and they fit a wave; else phase B
                    uint32_t tsl = kTieSlots;
                    {   // slots for the wave's tied groups at once: one LDS atomic, ranks by ballot
                        const uint64_t want_slot = __ballot(gj == 0 && mm <= 64), leaders = __ballot(gj == 0);
                        const uint32_t first = (uint32_t)__ffsll((long long)leaders) - 1;
                        uint32_t base = 0;
                        if (lane == first) {
                            atomicAdd(ntie + 1, (uint32_t)__popcll(leaders));
                            if (want_slot) base = atomicAdd(ntie, (uint32_t)__popcll(want_slot));
                        }
                        base = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)first);
                        const uint32_t leader = lane & ~(G - 1);
                        if (mm <= 64) tsl = base + (uint32_t)__popcll(want_slot & ((1ull << leader) - 1ull));
                    }
                    if (tsl < kTieSlots) {
                        const uint32_t g = p * kTieSlots + tsl;
                        uint2* dst = a.tie_cand + (uint64_t)g * 64;
                        for (uint32_t o = gj; o < mm; o += G) dst[o] = S[lo + o];
                        if (gj == 0) a.tie_hdr[g] = make_uint4(qi, t0, mm, 0u);
                    } else if (gj == 0) {
                        slow[atomicAdd(slow + kF3Threads, 1u)] = slot;
                    }
                } else if (gj == 0 || (K == 8 && a.rec.out && full_row && G > 1 && ((uintptr_t)a.rec.out & 15) == 0)) {
                    // (record form, k = 8, whole 16-B aligned rows: the group's G lanes all gather
                    // the row -- their loads hit the same addresses -- and store its six 16-B
                    // chunks together, below)
                    uint32_t* orow = a.out_idx + (uint64_t)qi * a.k;
                    // LDS reads first, then (shards) all gidx loads together: one wait before
                    // the stores instead of one per place
                    uint32_t res[K];
                    if (a.rec.out) {   // record form (block-uniform): the target's records here
                        uint32_t w0[K], w1[K], gi[K];
#pragma unroll
                        for (int r = 0; r < K; ++r) {
                            const uint2 e = S[(uint32_t)r < want && ok[r] < a.cap ? ok[r] : 0u];
                            res[r] = e.y;
                            w0[r] = e.x;
                        }
                        // words 0 / 1 from the planes the stage indexes (a sub-partition's own: its
                        // local index) together with the index map: one round trip, not two
                        // dependent ones (the map first, then the context's planes)
#pragma unroll
                        for (int r = 0; r < K; ++r) {
                            if (!a.rec.w0_direct)
                                w0[r] = a.rec.w0_shift ? ((a.rec.w0_pre | (Subs ? sub : 0u)) << (32 - a.rec.w0_shift)) |
                                                             (w0[r] >> a.rec.w0_shift)
                                                       : a.planes[res[r]];
                            w1[r] = a.planes[a.stride + res[r]];
                            res[r] = map_out(res[r], a.gidx, a.base);   // context-local
                        }
#pragma unroll
                        for (int r = 0; r < K; ++r) gi[r] = a.rec.gidx ? a.rec.gidx[res[r]] : res[r] + a.rec.base;
                        uint32_t* ro = a.rec.out + (uint64_t)qi * a.k * 3;
                        if (full_row && ((uintptr_t)a.rec.out & 15) == 0) {
                            // k == K == want: the row is 3K words from a 16-B boundary (K % 4 == 0),
                            // 3K / 4 vector stores instead of 3K dword stores
                            uint32_t wds[3 * K];
#pragma unroll
                            for (int r = 0; r < K; ++r) {
                                wds[3 * r] = w0[r];
                                wds[3 * r + 1] = w1[r];
                                wds[3 * r + 2] = gi[r];
                            }
                            if (K == 8 && G > 1) {
                                // lane gj of the group stores chunks gj, gj + G, ..: one store
                                // instruction covers G adjacent chunks of the row (one or two
                                // lines) instead of one lane issuing all six
                                // (straight-line: chunk gj in [0, 4), gj + G in [2, 8), gj + 2G in [4, 6) for G = 2)
                                auto put = [&](uint32_t c, uint32_t c_lo, uint32_t c_hi) {
                                    uint32_t x[4];
#pragma unroll
                                    for (int i = 0; i < 4; ++i) {
                                        x[i] = 0u;
#pragma unroll
                                        for (uint32_t cc = 0; cc < 6; ++cc)
                                            if (cc >= c_lo && cc < c_hi) x[i] = c == cc ? wds[(4 * cc + i) % (3 * K)] : x[i];
                                    }
                                    *reinterpret_cast<uint4*>(ro + 4 * c) = make_uint4(x[0], x[1], x[2], x[3]);
                                };
                                put(gj, 0u, 4u);
                                if (gj + G < 6) put(gj + G, 2u, 6u);
                                if (gj + 2 * G < 6) put(gj + 2 * G, 4u, 6u);
                            } else {
#pragma unroll
                                for (int r = 0; r < 3 * K; r += 4)
                                    *reinterpret_cast<uint4*>(ro + r) = make_uint4(wds[r], wds[r + 1], wds[r + 2], wds[r + 3]);
                            }
                        } else {
#pragma unroll
                            for (int r = 0; r < K; ++r) {
                                if ((uint32_t)r >= a.k) continue;
                                const bool v = (uint32_t)r < want;
                                ro[3 * r] = v ? w0[r] : DHT_NONE;
                                ro[3 * r + 1] = v ? w1[r] : DHT_NONE;
                                ro[3 * r + 2] = v ? gi[r] : DHT_NONE;
                            }
                        }
                    } else if (full_row) {   // k == K == want, 16-B aligned rows (block-uniform)
#pragma unroll
                        for (int r = 0; r < K; ++r) res[r] = S[ok[r]].y;
                        if (a.gidx) {
#pragma unroll
                            for (int r = 0; r < K; ++r) res[r] = a.gidx[res[r]];
                        } else {
#pragma unroll
                            for (int r = 0; r < K; ++r) res[r] += a.base;
                        }
#pragma unroll
                        for (int r = 0; r < K; r += 4)
                            *reinterpret_cast<uint4*>(orow + r) = make_uint4(res[r], res[r + 1], res[r + 2], res[r + 3]);
                        a.out_cnt[qi] = want;
                    } else {
#pragma unroll
                        for (int r = 0; r < K; ++r) res[r] = (uint32_t)r < want ? S[ok[r] < a.cap ? ok[r] : 0u].y : 0u;
                        if (a.gidx) {
#pragma unroll
                            for (int r = 0; r < K; ++r) res[r] = a.gidx[res[r]];
                        } else {
#pragma unroll
                            for (int r = 0; r < K; ++r) res[r] += a.base;
                        }
#pragma unroll
                        for (int r = 0; r < K; ++r)
                            if ((uint32_t)r < a.k) orow[r] = (uint32_t)r < want ? res[r] : DHT_NONE;
                        a.out_cnt[qi] = want;
                    }
                }
            }
        }
        // One set: the wave's tied targets, answered by the whole wave right away (one round trip
        // each: word 1 of the candidates and the target's words) while the block's other waves
        // finish; ties whose subtrees fit a wave go two at a time (both round trips in flight).
        // cfg 2: F3 + F4 15.5 + 7.3 -> 18.2 + 4.2 us serial, step 33.9 -> 33.4 us, latency 54 ->
        // 52 us; the cfg-3 shard keeps the F4 hand-off (F3 38 -> 48 us inline: 0.153 -> 0.162 ms
        // at two in flight; profiles/r05/experiments/f3_tie_inline*.txt, cfg3_tie_inline.txt)
        if (!Subs) {
            uint64_t tb = __ballot(tinl);
            while (tb) {
                const int L0 = __ffsll((long long)tb) - 1;
                tb &= tb - 1;
                const uint32_t lo0 = (uint32_t)__builtin_amdgcn_readlane((int)tlo, L0);
                const uint32_t mm0 = (uint32_t)__builtin_amdgcn_readlane((int)thi, L0) - lo0;
                const uint32_t q0 = (uint32_t)__builtin_amdgcn_readlane((int)tq, L0);
                const uint32_t t00 = (uint32_t)__builtin_amdgcn_readlane((int)tt0, L0);
                if (mm0 > 64 || !tb) {
                    f3_wave_answer(a, S, lo0, lo0 + mm0, q0, t00, want, lane);
                    continue;
                }
                const int L1 = __ffsll((long long)tb) - 1;
                const uint32_t lo1 = (uint32_t)__builtin_amdgcn_readlane((int)tlo, L1);
                const uint32_t mm1 = (uint32_t)__builtin_amdgcn_readlane((int)thi, L1) - lo1;
                if (mm1 > 64) {   // the second one alone, later
                    f3_wave_answer(a, S, lo0, lo0 + mm0, q0, t00, want, lane);
                    continue;
                }
                tb &= tb - 1;
                const uint32_t q1 = (uint32_t)__builtin_amdgcn_readlane((int)tq, L1);
                const uint32_t t01 = (uint32_t)__builtin_amdgcn_readlane((int)tt0, L1);
                const uint2 c0 = S[lo0 + (lane < mm0 ? lane : 0u)], c1 = S[lo1 + (lane < mm1 ? lane : 0u)];
                const uint32_t w10 = a.planes[a.stride + (lane < mm0 ? c0.y : 0u)];
                const uint32_t w11 = a.planes[a.stride + (lane < mm1 ? c1.y : 0u)];
                uint32_t tw0[DHT_W], tw1[DHT_W];
                load_target(a.tp, a.ts, q0, tw0);
                load_target(a.tp, a.ts, q1, tw1);
                wave_rank_loaded(a, c0, mm0, q0, t00, want, lane, w10, tw0);
                wave_rank_loaded(a, c1, mm1, q1, t01, want, lane, w11, tw1);
            }
        }
        if (Diag && (a.dbg & 256) && t0i == 0) {   // per wave: the end of its phase-A work
            if (lane == 0) a.stamps[2ull * 8192 * 16 + (uint64_t)blockIdx.x * 16 + wv] = __builtin_amdgcn_s_memrealtime();
        }
        sync_lds();
        if (t0i == 0) F3_STAMP(5);
        if (Diag && (a.dbg & 256) && threadIdx.x == 0 && t0i == 0) {
            a.stamps[(uint64_t)blockIdx.x * 16 + 11] = __builtin_amdgcn_s_memrealtime();
            a.stamps[(uint64_t)blockIdx.x * 16 + 13] = mt;
            a.stamps[(uint64_t)blockIdx.x * 16 + 12] =
                (__builtin_amdgcn_s_getreg((31 << 11) | 4) >> 8 & 0xFFu) | (__builtin_amdgcn_s_getreg((31 << 11) | 20) & 0xFu) << 8;
            a.stamps[(uint64_t)blockIdx.x * 16 + 14] = ntie[0];
        }
        // B: one wave per target for ties and large subtrees (phase A's range: complete, >= want ids)
        const uint32_t ns = slow[kF3Threads];
        for (uint32_t i = wv; i < ns; i += NWV) {
            const uint2 te = T[slow[i]];
            const uint32_t t0 = __builtin_amdgcn_readfirstlane(te.x);
            const uint32_t qi = __builtin_amdgcn_readfirstlane(te.y);
            uint32_t lo = 0, hi = 0;
            level_range(sofs, top_bits(t0, a.Lq) & smask, a.Lq, a.Lmin, want, lo, hi);
            f3_wave_answer(a, S, __builtin_amdgcn_readfirstlane(lo), __builtin_amdgcn_readfirstlane(hi), qi, t0, want,
                           lane);
        }
        if (ns || t0i + kF3Threads < mt) sync_lds();   // T / slow are reused by the next chunk
        if (t0i == 0) F3_STAMP(6);
    }
    // the wave-path statistic: one global atomic per block (a per-target atomic on one
    // address serialises at the memory side: 1,000 of them held this kernel ~10 µs)
    sync_lds();
    if (threadIdx.x == 0 && ntie[1]) atomicAdd(a.ctr + 2, ntie[1]);
    // this partition's deferred ties for F4 (a plain store: no shared counter to serialise on)
    if (threadIdx.x == 0 && ntie[0]) a.tie_cnt[p] = ntie[0] < kTieSlots ? ntie[0] : kTieSlots;
    F3_STAMP(7);
}

// ---- F4: the fallback targets (K1 scan, run-time roles) and the deferred ties -------------
// Every block first answers the ties F3 deferred in its share of the partitions (one wave per
// slot: wave_rank_answer on the copied candidates), then the fallback list (count ctr[0],
// known only on the device) is answered by
// the K1 streaming scan over all ids: target groups of 128 (8 waves x 16) x id-range splits,
// S = min(nfb / groups, 256 / k) so that the chip fills however short the list is; with
// S > 1 every split writes its sorted candidate records and the last split of a group to
// finish (agent-scope counter, sc1 records: MI355X_MICROARCH inter-workgroup hand-off)
// merges the group's S lists per target (a k-way merge over the list heads, one wave per
// target).
constexpr uint32_t kF4Threads = scan::WAVES * 64;                 // 512
constexpr uint32_t kFbGroup = scan::WAVES * kScanTargets;          // targets per scan role
constexpr uint32_t kFbBlocks = 256;                                // fallback-scan workgroups
constexpr uint32_t kFbCands = 256;                                 // merge: splits * k <= 256, splits <= 64
constexpr uint32_t kFbSingle = 64;                                 // per-target groups up to this many listed

struct FbArgs {
    uint32_t* rec;      // [kFbBlocks * kFbGroup * k * 6] split lists (S > 1 only)
    uint32_t* done;     // [kFbBlocks] per-group split completion counters (all-zero between calls)
    uint32_t nfb;       // fallback-scan workgroups (the grid)
    uint32_t np_ties;   // partitions whose deferred ties F4 answers (0: a list scan)
    uint32_t* hint;     // nullable: F4 stores the list length here (mapped host memory)
};

__device__ __forceinline__ uint32_t ld_sc1(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x = min(x, (uint32_t)__shfl_xor((int)x, o));
    return x;
}

// merge the S sorted split lists of every target of group g (one wave per target); gsize:
// targets per group (kFbGroup, or 1 for the per-target groups of short sub-partitioned lists)
__device__ void fb_merge(const F3Args& a, const FbArgs& f, uint32_t g, uint32_t S, uint32_t cnt, uint32_t* lds,
                         uint32_t gsize = kFbGroup) {
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    const uint32_t k = a.k, nt = cnt - g * gsize < gsize ? cnt - g * gsize : gsize;
    uint32_t* buf = lds + wv * 2 * kFbCands;   // this wave's candidates: {w0 distance, local index}
    for (uint32_t j = wv; j < nt; j += scan::WAVES) {
        const uint32_t qr = __builtin_amdgcn_readfirstlane(a.fb_list[g * gsize + j]);
        uint32_t t[DHT_W];
        load_target(a.tp, a.ts, qr, t);
        for (uint32_t c = lane; c < S * k; c += 64) {
            const uint32_t l = c / k, r = c - l * k;
            const uint32_t* src = f.rec + ((((uint64_t)g * S + l) * kFbGroup + j) * k + r) * 6;
            const uint32_t w0 = ld_sc1(src), ix = ld_sc1(src + 5);
            buf[2 * c] = ix == DHT_NONE ? DHT_NONE : w0 ^ t[0];
            buf[2 * c + 1] = ix;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // lane l < S walks list l; each round takes the closest head (full key on a w0 tie)
        uint32_t p = 0, hd = DHT_NONE, hi = DHT_NONE;
        if (lane < S) {
            hd = buf[2 * lane * k];
            hi = buf[2 * lane * k + 1];
        }
        uint32_t* orow = a.out_idx + (uint64_t)qr * k;
        uint32_t r = 0;
        for (; r < k; ++r) {
            const bool valid = hi != DHT_NONE;
            const uint32_t m = wave_min_u32(valid ? hd : DHT_NONE);
            const uint64_t cand = __ballot(valid && hd == m);
            if (!cand) break;
            uint32_t win = (uint32_t)__ffsll((long long)cand) - 1;
            if (__popcll(cand) > 1) {
                uint64_t rest = cand & (cand - 1);
                while (rest) {
                    const uint32_t l2 = (uint32_t)__ffsll((long long)rest) - 1;
                    rest &= rest - 1;
                    const uint32_t ib = __builtin_amdgcn_readlane((int)hi, (int)win);
                    const uint32_t i2 = __builtin_amdgcn_readlane((int)hi, (int)l2);
                    if (id_less(m, i2, m, ib, a.planes, a.stride, t)) win = l2;
                }
            }
            const uint32_t wi = __builtin_amdgcn_readlane((int)hi, (int)win);
            if (lane == 0) {
                if (a.rec.out)   // record form: word 0 back from the distance, word 1 read
                    rec_place(a.rec, a.planes, a.gidx, a.base, k, qr, r, wi, m ^ t[0], true, a.planes[a.stride + wi]);
                else
                    orow[r] = map_out(wi, a.gidx, a.base);
            }
            if (lane == win) {
                ++p;
                hd = p < k ? buf[2 * (lane * k + p)] : DHT_NONE;
                hi = p < k ? buf[2 * (lane * k + p) + 1] : DHT_NONE;
            }
        }
        for (uint32_t x = r + lane; x < k; x += 64) {
            if (a.rec.out) rec_place(a.rec, a.planes, a.gidx, a.base, k, qr, x, DHT_NONE, 0u, true, 0u);
            else orow[x] = DHT_NONE;
        }
        if (lane == 0) a.out_cnt[qr] = r;
    }
}

// Record form after a one-split scan role: the wave converts the rows its role just wrote
// (context-local indices; its own stores, drained, read back at agent scope past the L1) into
// records from the context's planes.  Writing the records inside the scan's unrolled result loop
// took F4 from 135 VGPRs to 221 + 752 B of scratch per lane (F4 7.5 -> 25 us, profiles/r05/g/probe_scan_rec_stores_221vgpr.json).
__device__ void fb_rows_to_records(const F3Args& a, uint32_t qb, uint32_t qend) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t lane = lane_id(), k = a.k;
    const uint32_t nt = qend > qb ? (qend - qb < kScanTargets ? qend - qb : kScanTargets) : 0u;
    for (uint32_t c = lane; c < nt * k; c += 64) {
        const uint32_t j = c / k, r = c - j * k;
        const uint32_t qr = a.fb_list[qb + j];
        const uint32_t x = ld_sc1(a.out_idx + (uint64_t)qr * k + r);
        rec_place(a.rec, a.rec.planes, nullptr, 0u, k, qr, r, x, 0u, false, x == DHT_NONE ? 0u : a.rec.planes[a.rec.stride + x]);
    }
}

// The fallback list's K1 scan (a.fb_list[0, cnt)): roles of target groups x id-range splits over
// f.nfb workgroups, this one being workgroup `blk` of them (k_f4, and KS's scan-role workgroups)
template <int K>
__device__ __forceinline__ void fb_list_scan(const F3Args& a, const FbArgs& f, uint32_t cnt, uint32_t blk, uint32_t* lds,
                             uint32_t* last) {
    const uint32_t wv = threadIdx.x >> 6;
    // Sub-partitioned call with a short list (on uniform ids: the rare target whose level-Lm
    // subtree holds < k ids): every target is its own group and scans only its own
    // sub-partition -- which holds its top-k when it holds >= k ids -- over S splits (a scan of
    // the whole set cost a single target ~3 ms at 2^28 ids).  Up to one target per
    // sub-partition: past that, one scan of the whole set for all of them reads less.  (One
    // scan_run call site for both forms: a second inlined copy doubled this kernel's VGPRs.)
    const bool single = a.np_sub != f.np_ties && cnt <= min(kFbSingle, f.np_ties / a.np_sub);
    const uint32_t gsize = single ? 1u : kFbGroup;
    const uint32_t groups = (cnt + gsize - 1) / gsize;
    // splits: S * k candidates fit the merge buffer, and one list head per lane (S <= 64; at
    // k < 4 the buffer alone allowed up to 256 splits, whose lists past lane 63 were dropped)
    const uint32_t smax = kFbCands / a.k < 64u ? kFbCands / a.k : 64u;
    uint32_t S = f.nfb / groups;
    S = S < 1 ? 1u : S > smax ? smax : S;
    if (!single) {
        const uint64_t ntiles = (a.n + scan::TILE - 1) / scan::TILE;
        if ((uint64_t)S > ntiles) S = ntiles ? (uint32_t)ntiles : 1u;
        const uint64_t sl = (ntiles ? (ntiles + S - 1) / S : 1) * scan::TILE;
        if (ntiles) S = (uint32_t)((a.n + sl - 1) / sl);
    }
    const uint32_t roles = groups * S;
    for (uint32_t role = blk; role < roles; role += f.nfb) {
        const uint32_t g = role / S, sp = role - g * S;
        F3Args as = a;   // single: the target's sub-partition (or the whole set)
        if (single) {
            const uint32_t sb = __builtin_amdgcn_readfirstlane((uint32_t)a.fb_sub[g]);
            if (sb != 255u) {
                const SubDesc d = a.subs[sb];
                if (d.n >= a.k) {
                    as.planes = d.planes;
                    as.stride = d.stride;
                    as.n = d.n;
                    as.gidx = d.gidx;
                    as.base = d.base;
                }
            }
        }
        const uint64_t nt = (as.n + scan::TILE - 1) / scan::TILE;
        const uint64_t split_len = (nt ? (nt + S - 1) / S : 1) * scan::TILE;
        const uint64_t lo = (uint64_t)sp * split_len < as.n ? (uint64_t)sp * split_len : as.n;
        const uint64_t hi = lo + split_len < as.n ? lo + split_len : as.n;
        // split lists at record slot (g * S + sp) * kFbGroup + target-in-group (fb_merge's layout)
        const uint64_t rb = single ? ((uint64_t)g * S + sp) * kFbGroup - g
                                   : (uint64_t)g * kFbGroup * (S - 1) + (uint64_t)sp * kFbGroup;
        const scan::ScanOut o{as.out_idx, as.out_cnt, as.gidx, as.base, S > 1 ? f.rec : nullptr, rb, 0u};
        const uint32_t qb = single ? (wv == 0 ? g : g + 1) : g * kFbGroup + wv * kScanTargets;
        scan::scan_run<K, kScanTargets>(lds, as.planes, as.stride, lo, hi, as.tp, as.ts, as.fb_list, qb,
                                        single ? g + 1 : cnt, as.k, o);
        if (S == 1) {
            if (a.rec.out) fb_rows_to_records(a, qb, single ? g + 1 : cnt);
            continue;
        }
        // hand-off: every wave's sc1 record stores drained, then one agent-scope add per block;
        // the block whose add completes the group merges it (its waves load after the barrier)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) *last = atomicAdd(f.done + g, 1u) == S - 1 ? 1u : 0u;
        __syncthreads();
        if (!*last) continue;
        fb_merge(as, f, g, S, cnt, lds, gsize);
        if (threadIdx.x == 0) f.done[g] = 0;   // all-zero again for the next call
        __syncthreads();                       // lds is reused by this block's next role
    }
}

template <int K>
__global__ __launch_bounds__(kF4Threads) void k_f4(F3Args a, FbArgs f) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[scan::lds_words<kScanTargets>()];
    __shared__ uint32_t last;
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    // deferred ties of the block's partitions p = blockIdx + j * gridDim, 64 at a time (j0 + lane
    // = j < ppb): lane j loads partition j's count, a wave scan numbers the round's ties, and
    // the waves take them round-robin -- every tie in flight at once (one round trip for the
    // counts; one round unless np_ties > 64 * gridDim)
    const uint32_t ppb = f.np_ties ? (f.np_ties + gridDim.x - 1) / gridDim.x : 0u;
    for (uint32_t j0 = 0; j0 < ppb; j0 += 64) {
        const uint32_t want = a.n < a.k ? (uint32_t)a.n : a.k;
        const uint32_t pj = blockIdx.x + (j0 + lane) * gridDim.x;
        const bool mine = j0 + lane < ppb && pj < f.np_ties;
        const uint32_t myc = mine ? a.tie_cnt[pj] : 0u;
        uint32_t inc = myc;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)inc, o);
            if (lane >= (uint32_t)o) inc += y;
        }
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        // two ties per wave in flight: both ties' loads (header, candidates, sub-partition
        // descriptor; then word 1 and the target) are issued before either is ranked, so a wave
        // holding two ties pays two round trips, not four (the cfg-3 shard defers ~1.5 per wave)
        for (uint32_t t = wv; t < total; t += 2 * scan::WAVES) {
            const bool two = t + scan::WAVES < total;   // wave-uniform
            uint32_t g[2], part[2];
#pragma unroll
            for (int x = 0; x < 2; ++x) {
                const uint32_t tt = x ? (two ? t + scan::WAVES : t) : t;
                const uint32_t j = (uint32_t)__popcll(__ballot(inc <= tt));   // partition j holds tie tt
                const uint32_t before = j ? (uint32_t)__builtin_amdgcn_readlane((int)inc, (int)j - 1) : 0u;
                part[x] = blockIdx.x + (j0 + j) * gridDim.x;
                g[x] = part[x] * kTieSlots + (tt - before);
            }
            uint4 h[2];
            uint2 c[2];
            F3Args as[2] = {a, a};   // each partition's sub-partition: tie words and result map
#pragma unroll
            for (int x = 0; x < 2; ++x) {
                h[x] = a.tie_hdr[g[x]];
                c[x] = a.tie_cand[(uint64_t)g[x] * 64 + lane];
                if (a.np_sub != f.np_ties) {
                    const SubDesc d = a.subs[__builtin_amdgcn_readfirstlane(part[x] / a.np_sub)];
                    as[x].planes = d.planes;
                    as[x].stride = d.stride;
                    as[x].gidx = d.gidx;
                    as[x].base = d.base;
                }
            }
            uint32_t mm[2], qi[2], t0[2], w1[2], tw[2][DHT_W];
#pragma unroll
            for (int x = 0; x < 2; ++x) {
                mm[x] = __builtin_amdgcn_readfirstlane(h[x].z);
                qi[x] = __builtin_amdgcn_readfirstlane(h[x].x);
                t0[x] = __builtin_amdgcn_readfirstlane(h[x].y);
                w1[x] = as[x].planes[as[x].stride + (lane < mm[x] ? c[x].y : 0u)];
                load_target(a.tp, a.ts, qi[x], tw[x]);
            }
            wave_rank_loaded(as[0], c[0], mm[0], qi[0], t0[0], want, lane, w1[0], tw[0]);
            if (two) wave_rank_loaded(as[1], c[1], mm[1], qi[1], t0[1], want, lane, w1[1], tw[1]);
        }
        if (total) {   // block-uniform: every wave has read the counts before they are cleared
            __syncthreads();
            if (threadIdx.x < 64 && mine && myc) a.tie_cnt[pj] = 0;   // all-zero again for the next call
        }
    }
    if (f.hint && blockIdx.x == 0 && threadIdx.x == 0)   // sizes a later call's grid (mapped host memory)
        __hip_atomic_store(f.hint, a.ctr[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint32_t cnt = a.ctr[0];
    if (cnt == 0) return;
    fb_list_scan<K>(a, f, cnt, blockIdx.x, lds, &last);
}

struct BatchPlan {
    uint32_t Lm, b1, Lq, nwords, nblk1, nblk2, stage, sparse, tcap;
    uint32_t sib;    // 1: sibling marking from the set's level-Lm cell counts (Lmin = Lm - 1)
    uint32_t nstage; // F2's narrow stage entries (6 B each; 0: none) -- F2 then leaves room for an F3 workgroup
    uint32_t f3cap;  // F3's LDS stage entries (kF3Cap, or the 6-sigma bound when that buys a 4th workgroup per CU)
    uint32_t scap;   // survivors per (bucket set, partition)
    uint32_t f3cap_wide;   // F3's LDS stage entries when F2 runs its 8-B stage (no narrow stage)
    uint32_t cap6;         // the plan's 6-sigma partition bound (F3 stage entries, <= kF3Cap)
    uint32_t wwords;       // F2 window mode: bitmap words in LDS per workgroup (0: the whole bitmap)
    bool wpack;            // window mode's stage is packed (6 B; one final flush) -- else 8 B, segments
    uint32_t nsets;        // F2 bucket sets per partition: kSets, or 1 over prefix-sorted sub-partitions
    // variance of an F2 range's survivor count per expected survivor: ids of a range are a random
    // sample (1 - f), or -- prefix-sorted sub-partitions -- whole level-Lm cells of mu ids each,
    // marked with probability f ((1 - f) mu + 1: ~30x the binomial at the cfg-3 shard)
    double clump;
    bool fits;   // partitions' survivors fit the F3 stage on uniform ids
    uint64_t per_blk;
};



uint32_t floor_log2(uint64_t x) {
    uint32_t r = 0;
    while (x > 1) { x >>= 1; ++r; }
    return r;
}

// P(X < k) for X ~ Poisson(m)
double poisson_below(double m, uint32_t k) {
    double term = std::exp(-m), sum = 0.0;
    for (uint32_t j = 0; j < k; ++j) {
        sum += term;
        term *= m / (double)(j + 1);
    }
    return sum;
}

BatchPlan plan_batch_compute(uint64_t n, uint32_t q, uint32_t k, int num_cus, uint32_t pf, uint32_t wwords);

// plan_batch is a pure function of (n, q, k, CUs, plan flags, window), asked three times per call
// (workspace size, clean head, the launch): the last few plans are kept per host thread
BatchPlan plan_batch(uint64_t n, uint32_t q, uint32_t k, int num_cus, uint32_t pf = 0, uint32_t wwords = 0) {
    struct Entry { uint64_t n; uint32_t q, k; int cus; uint32_t pf; uint32_t ww; BatchPlan P; bool used; };
    thread_local Entry cache[6] = {};
    thread_local uint32_t next = 0;
    for (const Entry& e : cache)
        if (e.used && e.n == n && e.q == q && e.k == k && e.cus == num_cus && e.pf == pf && e.ww == wwords)
            return e.P;
    Entry& e = cache[next++ % 6u];
    e = Entry{n, q, k, num_cus, pf, wwords, plan_batch_compute(n, q, k, num_cus, pf, wwords), true};
    return e.P;
}

BatchPlan plan_batch_compute(uint64_t n, uint32_t q, uint32_t k, int num_cus, uint32_t pf, uint32_t wwords) {
    BatchPlan P;
    const bool cells = (pf & kPlanCells) != 0, sorted = (pf & kPlanSorted) != 0;
    P.wwords = wwords;
    // mark level: 4k or more ids per level-Lm subtree -- or one level finer (2k..4k) when, on
    // uniform ids, fewer than 0.01 of the q targets are expected to land in a subtree with
    // under k ids (those go to the F4 brute force).  Without the finer step a prefix shard
    // just under a power of two (n = 2^24 - few) would mark at half the resolution and
    // double the survivors.
    const uint64_t per = 4ull * k;
    P.Lm = n >= per ? floor_log2(n / per) : 0;
    P.sib = 0;
    if (n >= per && P.Lm < kMaxLm) {
        if (poisson_below((double)n / (double)(1ull << (P.Lm + 1)), k) * q <= 0.01) {
            ++P.Lm;
        } else if (cells && P.Lm + 1 == kMaxLm && poisson_below((double)n / (double)(1ull << P.Lm), k) * q <= 0.01) {
            // sibling marking (the set's level-kMaxLm cell counts, kept with its sub-partitions):
            // a target whose level-Lm cell holds < k ids marks the sibling cell too, so it answers
            // from its complete level-(Lm - 1) subtree; only a short PAIR falls back.  One level
            // finer than the rule above allows: the survivors drop from 1 - exp(-q / 2^(Lm-1)) to
            // about 1 - exp(-q / 2^Lm) (cfg 3's broadcast rank: 39 % -> 22 %)
            ++P.Lm;
            P.sib = 1;
        }
    }
    if (P.Lm > kMaxLm) P.Lm = kMaxLm;
    // survivors on uniform ids: n (1 - exp(-q (1 + p) / 2^Lm)), p = the fraction of targets that
    // mark a sibling too; partitions of about kF3Cap / 2
    const double psib = P.sib ? poisson_below((double)n / (double)(1ull << P.Lm), k) : 0.0;
    const double f = 1.0 - std::exp(-(double)q * (1.0 + psib) / (double)(1ull << P.Lm));
    const double surv = (double)n * f + 1.0;
    uint32_t b1 = 0;
    while (b1 + P.sib < P.Lm && surv / (double)(1ull << b1) > kF3Cap / 2) ++b1;   // F3 sorts level Lm - sib
    if (P.Lm > kMaxSubBits && b1 < P.Lm - kMaxSubBits) b1 = P.Lm - kMaxSubBits;
    if (b1 > 13) b1 = 13;   // kMaxParts
    // a partition's survivors come in whole level-Lm subtrees (n / 2^Lm ids each, marked
    // with probability f): on uniform ids mean s f mu, variance s f (1 - f) mu^2 + s f mu
    // over its s = 2^(Lm - b1) subtrees.  Split further until mean + 6 sigma fits the F3
    // stage (an overflowing partition sends its targets to the brute force); plans that
    // cannot are refused (batch_supported), e.g. n >> 2^24 with its 256-id subtrees.
    P.fits = false;
    double need = (double)kF3Cap;   // the partition bound the plan was accepted with
    for (;; ++b1) {
        const double sub = (double)(1ull << (P.Lm - b1)), mu = (double)n / (double)(1ull << P.Lm);
        const double mean = sub * f * mu, var = sub * f * (1.0 - f) * mu * mu + sub * f * mu;
        need = mean + 6.0 * std::sqrt(var) + 64.0;
        if (need <= (double)kF3Cap) { P.fits = true; break; }
        if (b1 >= 13 || b1 + P.sib >= P.Lm) break;
    }
    P.b1 = b1;
    // prefix-sorted sub-partitions (the plans with cell counts): an F2 workgroup's range is a
    // narrow prefix range, so a partition's survivors come from one or two workgroups -- one
    // bucket set, sized for the whole partition (with 8 sets planned for an eighth each, every
    // partition overflowed its set)
    P.nsets = sorted ? 1u : kSets;
    P.clump = sorted ? (1.0 - f) * (double)n / (double)(1ull << P.Lm) + 1.0 : 1.0 - f;
    {   // a set holds each id with probability 1 / kSets (ids are spread over the blocks by
        // index, independently of their prefix): mean + 8 sigma + 64 of one set's share
        const double sub = (double)(1ull << (P.Lm - b1)), mu = (double)n / (double)(1ull << P.Lm) / P.nsets;
        const double mean = sub * f * mu, var = sub * f * (1.0 - f) * mu * mu + sub * f * mu;
        const double cap = mean + 8.0 * std::sqrt(var) + 64.0;
        P.scap = cap >= (double)kF3Cap ? kF3Cap : ((uint32_t)cap + 63u) & ~63u;
        // F3 gathers exactly after the counts: the survivors' bytes only (PMC at cfg 2: 18.5 MB
        // against 19.7 MB algorithmic; round 2's fixed speculative slots fetched 40 MB) and no
        // slower (cfg-2 step 37.7-38.1 us against 38.3-38.4 with a planned mean + 5 sigma)
    }
    // F3 sorts by up to 1 bit below the mark level (finer candidate ranges), <= 4096 bins
    P.Lq = P.Lm + 1 < 32 ? P.Lm + 1 : 32;
    while (P.Lq > P.Lm && P.Lq - P.b1 > 12) --P.Lq;
    // F3's LDS: four workgroups per CU (40 KB each) where the plan allows -- sort one bit less
    // finely, and stage the plan's own 6-sigma bound instead of kF3Cap entries (a partition past
    // it sends its targets to the exact fallback, as one past kF3Cap always did).  The cfg-3
    // shard's plan (b1 = 8, 4096 sort bins: 52 KB) ran three per CU, 2.7 rounds of 2,048 blocks.
    P.f3cap = kF3Cap;
    auto lds3 = [&](uint32_t Lq, uint32_t cap) {
        return (size_t)f3_words(1u << (Lq - P.b1)) * 4 + (size_t)(cap + kF3Threads) * 8;
    };
    constexpr size_t kF3Lds4 = kLdsMax / 4;
    const uint32_t cap6 = std::min<uint32_t>(kF3Cap, ((uint32_t)need + 63u) & ~63u);
    P.cap6 = cap6;
    if (P.fits && lds3(P.Lq, P.f3cap) > kF3Lds4) {
        for (uint32_t lq = P.Lq; lq >= P.Lm && lq > P.b1; --lq) {
            if (lds3(lq, kF3Cap) <= kF3Lds4) { P.Lq = lq; break; }
            if (lds3(lq, cap6) <= kF3Lds4) { P.Lq = lq; P.f3cap = cap6; break; }
            if (lq == P.Lm) break;
        }
    }
    P.nwords = P.Lm >= 5 ? (1u << (P.Lm - 5)) : 1u;
    P.nblk1 = (q + kF1Threads - 1) / kF1Threads;
    // target buckets: mean + 6 sigma + 64 (uniform targets); overflow spills to F4
    const double mu = (double)q / (double)(1u << P.b1);
    P.tcap = ((uint32_t)(mu + 6.0 * std::sqrt(mu) + 64.0) + 63u) & ~63u;
    // F2: one persistent workgroup per CU, ranges in whole chunks
    const uint64_t chunks = (n + kF2Step - 1) / kF2Step;
    const uint64_t g = num_cus > 0 ? (uint64_t)num_cus : 256;
    const uint64_t cpb = (chunks + g - 1) / g;
    P.per_blk = (cpb ? cpb : 1) * kF2Step;
    P.nblk2 = (uint32_t)((n + P.per_blk - 1) / P.per_blk);
    // F2 LDS stage: what is left of the LDS next to the bitmap (or its window) and histogram
    const size_t fixed = (size_t)f2_fixed_words(wwords ? wwords : P.nwords, 1u << P.b1) * 4;
    // (window mode: a packed 6-B stage while one final flush holds the range's survivors)
    const size_t room = fixed < kLdsMax ? (kLdsMax - fixed) / 8 : 0;
    const size_t room6 = fixed + 1024 < kLdsMax ? (kLdsMax - fixed - 1024) / 6 : 0;
    P.stage = wwords ? (uint32_t)std::min<size_t>(room6, kStageWin) : (uint32_t)(room < kStage ? room : kStage);
    P.wpack = wwords != 0;
    // sparse mode when a block's survivors (mean + 8 sigma on uniform ids) fit the stage,
    // with ranges shrunk (more blocks) while that helps
    P.sparse = 0;
    for (uint64_t pb = P.per_blk; pb >= kF2Step; pb /= 2) {
        const double mean = (double)pb * f, sd = std::sqrt(mean * P.clump);
        if (mean + 8.0 * sd + 256.0 <= (double)P.stage) {
            P.sparse = 1;
            P.per_blk = (pb / kF2Step) * kF2Step;
            P.nblk2 = (uint32_t)((n + P.per_blk - 1) / P.per_blk);
            break;
        }
        if (pb == kF2Step) break;
    }
    // window mode past one stage-full: the segmented instantiation's flush holds kStagePer entries
    // per thread in registers (its ring stays live across the flush: 128 VGPRs at most)
    if (wwords && !P.sparse) {
        P.stage = (uint32_t)(room < kStage ? room : kStage);
        P.wpack = false;
    }
    // F2's narrow stage (6 B per entry: ranges < 2^16 ids, the cfg-2 shape): sized so that F2
    // plus one F3 workgroup fit a CU's LDS -- the F2 of one batch in flight and the F3 of another
    // then share CUs instead of waiting for each other's workgroups to drain.  F3 stages its
    // plan's own 6-sigma bound where that is what makes the pair fit (a partition past it sends
    // its targets to the exact fallback, as one past kF3Cap does).  1 KB of margin per kernel
    // for the LDS allocation granule.
    P.nstage = 0;
    P.f3cap_wide = P.f3cap;
    if (P.sparse && P.per_blk <= 65536 && !wwords) {
        const double mean = (double)P.per_blk * f, sd = std::sqrt(mean * (1.0 - f));
        const double need2 = mean + 8.0 * sd + 256.0;
        for (int pass = 0; pass < 2 && !P.nstage; ++pass) {
            uint32_t cap3 = P.f3cap_wide;   // pass 1: F3 stages the 6-sigma bound to make room
            if (pass == 1) {
                if (!P.fits || cap6 >= cap3) break;
                cap3 = cap6;
            }
            const size_t f3l = (lds3(P.Lq, cap3) + 1023) & ~(size_t)1023;
            if (fixed + f3l + 1024 >= kLdsMax) continue;
            const size_t room6 = (kLdsMax - f3l - fixed - 1024) / 6;
            if ((double)room6 >= need2) {
                P.nstage = (uint32_t)std::min<size_t>(room6, kStage) & ~1u;
                P.f3cap = cap3;   // committed only with the narrow stage it makes room for
            }
        }
    }
    return P;
}

size_t f2_lds(const BatchPlan& P, bool narrow = false) {
    const size_t fixed = (size_t)f2_fixed_words(P.wwords ? P.wwords : P.nwords, 1u << P.b1) * 4;
    if (P.wpack) return fixed + (size_t)P.stage * 6;   // window mode's packed stage
    return fixed + (narrow ? (size_t)P.nstage * 6 : (size_t)P.stage * 8);
}

size_t f3_lds(const BatchPlan& P, uint32_t cap) {
    const uint32_t nsub = 1u << (P.Lq - P.b1);
    return (size_t)f3_words(nsub) * 4 + (size_t)(cap + kF3Threads) * 8;
}

// DHTGPU_DBG=256: per-block phase profiles of F2 and F3 from their s_memrealtime stamps
// (100 MHz real-time counter: 10 ns ticks), printed to stderr (synchronises s)
void print_phase_profile(const BatchPlan& P, uint32_t nblk2, uint32_t np, unsigned long long* stamps, hipStream_t s) {
    if (!stamps) return;
    const uint32_t dbg = 256;
    if (dbg & 256) {   // phase profile of F2 (100 MHz real-time stamps: 10 ns ticks)
        std::vector<unsigned long long> h((size_t)nblk2 * 16);
        (void)hipMemcpyAsync(h.data(), stamps + 8192 * 16, h.size() * 8, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        unsigned long long t0 = ~0ull;
        for (uint32_t b = 0; b < nblk2; ++b) t0 = h[b * 16] && h[b * 16] < t0 ? h[b * 16] : t0;
        auto pct2 = [](std::vector<double> d) {
            std::sort(d.begin(), d.end());
            const size_t m = d.size();
            char buf[96];
            snprintf(buf, sizeof buf, "p10 %.2f p50 %.2f p90 %.2f max %.2f", d[m / 10], d[m / 2], d[m * 9 / 10], d[m - 1]);
            return std::string(buf);
        };
        const char* nm[] = {"", "bitmap+ring", "stream+filter", "flush hist", "flush reserve+scan", "flush writes"};
        for (int i = 1; i <= 5; ++i) {
            std::vector<double> d;
            for (uint32_t b = 0; b < nblk2; ++b)
                if (h[b * 16 + 5]) d.push_back((double)(h[b * 16 + i] - h[b * 16 + i - 1]) / 100.0);
            if (!d.empty()) fprintf(stderr, "  F2 %-20s %s\n", nm[i], pct2(d).c_str());
        }
        {   // window flushes (the last one's sub-phases): ranks in registers, table, offsets; spill flag
            const char* nw[] = {"win load", "win reserve+write"};
            const int from[] = {2, 6}, to[] = {6, 7};
            for (int i = 0; i < 2; ++i) {
                std::vector<double> d;
                for (uint32_t b = 0; b < nblk2; ++b)
                    if (h[b * 16 + 5] && h[b * 16 + to[i]] > h[b * 16 + from[i]])
                        d.push_back((double)(h[b * 16 + to[i]] - h[b * 16 + from[i]]) / 100.0);
                if (!d.empty()) fprintf(stderr, "  F2 %-20s %s\n", nw[i], pct2(d).c_str());
            }
        }
        std::vector<double> st, en;
        for (uint32_t b = 0; b < nblk2; ++b)
            if (h[b * 16 + 5]) { st.push_back((double)(h[b * 16] - t0) / 100.0); en.push_back((double)(h[b * 16 + 5] - t0) / 100.0); }
        if (!st.empty()) fprintf(stderr, "  F2 start %s\n  F2 end   %s\n", pct2(st).c_str(), pct2(en).c_str());
    }
    if (dbg & 256) {   // phase profile of F3 (100 MHz real-time stamps: 10 ns ticks)
        std::vector<unsigned long long> h((size_t)np * 16);
        (void)hipMemcpyAsync(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        unsigned long long t0min = ~0ull;
        for (uint32_t b = 0; b < np; ++b) t0min = h[b * 16] && h[b * 16] < t0min ? h[b * 16] : t0min;
        std::vector<uint32_t> live;
        for (uint32_t b = 0; b < np; ++b)
            if (h[b * 16 + 7]) live.push_back(b);
        const size_t nb = live.size();
        auto pct = [](std::vector<double> d) {
            std::sort(d.begin(), d.end());
            const size_t m = d.size();
            char buf[96];
            snprintf(buf, sizeof buf, "p10 %.2f p50 %.2f p90 %.2f max %.2f", d[m / 10], d[m / 2], d[m * 9 / 10], d[m - 1]);
            return std::string(buf);
        };
        if (nb) {
            for (int i = 1; i < 8; ++i) {
                std::vector<double> d;
                for (uint32_t b : live) d.push_back((double)(h[b * 16 + i] - h[b * 16 + i - 1]) / 100.0);
                fprintf(stderr, "  phase %d %s\n", i, pct(d).c_str());
            }
            {   // phase A split by group size (G = 4 for <= 64 targets) and by deferred ties
                std::vector<double> d[2][2];
                for (uint32_t b : live)
                    d[h[b * 16 + 13] > 64][h[b * 16 + 14] > 0].push_back((double)(h[b * 16 + 5] - h[b * 16 + 4]) / 100.0);
                for (int g = 0; g < 2; ++g)
                    for (int t = 0; t < 2; ++t)
                        if (!d[g][t].empty())
                            fprintf(stderr, "  phase A %s %s (%zu blocks): %s\n", g ? "G<=2" : "G=4 ", t ? "ties" : "none",
                                    d[g][t].size(), pct(d[g][t]).c_str());
            }
            {   // the slowest blocks, phase by phase
                std::vector<std::pair<unsigned long long, uint32_t>> ord;
                for (uint32_t b : live) ord.push_back({h[b * 16 + 7] - t0min, b});
                std::sort(ord.rbegin(), ord.rend());
                for (size_t ii = 0; ii < ord.size() && ii < 3; ++ii) {   // CU-mates of the slowest blocks
                    const uint32_t b = ord[ii].second;
                    fprintf(stderr, "  CU of block %u:\n", b);
                    for (uint32_t c : live) {
                        if (h[c * 16 + 12] != h[b * 16 + 12]) continue;
                        fprintf(stderr, "     block %4u ends of phases:", c);
                        for (int j = 0; j < 8; ++j) fprintf(stderr, " %.2f", (double)(h[c * 16 + j] - t0min) / 100.0);
                        fprintf(stderr, "  loop %.2f-%.2f\n", (double)(h[c * 16 + 8] - t0min) / 100.0, (double)(h[c * 16 + 9] - t0min) / 100.0);
                    }
                }
                for (size_t ii = 0; ii < ord.size() && ii < 10; ++ii) {
                    const size_t i = ii < 5 ? ii : ord.size() - 10 + ii;
                    const uint32_t b = ord[i].second;
                    fprintf(stderr, "  slow block %u (mt %llu, ties %llu): start %.2f phases", b, h[b * 16 + 13], h[b * 16 + 14],
                            (double)(h[b * 16] - t0min) / 100.0);
                    for (int j = 1; j < 8; ++j) fprintf(stderr, " %.2f", (double)(h[b * 16 + j] - h[b * 16 + j - 1]) / 100.0);
                    fprintf(stderr, "  A: level %.2f loop %.2f merge %.2f out %.2f",
                            (double)(h[b * 16 + 8] - h[b * 16 + 4]) / 100.0, (double)(h[b * 16 + 9] - h[b * 16 + 8]) / 100.0,
                            (double)(h[b * 16 + 10] - h[b * 16 + 9]) / 100.0, (double)(h[b * 16 + 5] - h[b * 16 + 10]) / 100.0);
                    std::vector<unsigned long long> hw(16);
                    (void)hipMemcpy(hw.data(), stamps + 2ull * 8192 * 16 + (uint64_t)b * 16, 16 * 8, hipMemcpyDeviceToHost);
                    fprintf(stderr, "  waves end");
                    for (int w = 0; w < 4; ++w) fprintf(stderr, " %.2f", hw[w] ? (double)(hw[w] - t0min) / 100.0 : -1.0);
                    fprintf(stderr, "\n");
                }
            }
            std::vector<double> en, st;
            for (uint32_t b : live) {
                en.push_back((double)(h[b * 16 + 7] - t0min) / 100.0);
                st.push_back((double)(h[b * 16] - t0min) / 100.0);
            }
            fprintf(stderr, "  start %s\n  end   %s\n", pct(st).c_str(), pct(en).c_str());
        }
    }
}

std::once_flag g_attr_once[kMaxDevices];   // set_lds_attributes, per device (per_device_once)

void set_lds_attributes() {
    const void* fs[] = {(const void*)k_f2_filter<kF2Dense, kF2One>, (const void*)k_f2_filter<kF2Sparse, kF2One>,
                        (const void*)k_f2_filter<kF2Seg, kF2One>,
                        (const void*)k_f2_filter<kF2Dense, kF2Subs>, (const void*)k_f2_filter<kF2Sparse, kF2Subs>,
                        (const void*)k_f2_filter<kF2Seg, kF2Subs>,
                        (const void*)k_f2_filter<kF2Narrow, kF2One>, (const void*)k_f2_filter<kF2Narrow, kF2Subs>,
                        (const void*)k_f2_filter<kF2Dense, kF2SubsNT>, (const void*)k_f2_filter<kF2Sparse, kF2SubsNT>,
                        (const void*)k_f2_filter<kF2Seg, kF2SubsNT>,
                        (const void*)k_f2_filter<kF2Narrow, kF2SubsNT>,
                        (const void*)k_f2_filter<kF2Sparse, kF2Subs, true>, (const void*)k_f2_filter<kF2Seg, kF2Subs, true>,
                        (const void*)k_f2_filter<kF2Sparse, kF2SubsNT, true>, (const void*)k_f2_filter<kF2Seg, kF2SubsNT, true>,
                        (const void*)k_f3_answer<8, false, true, false>,  (const void*)k_f3_answer<16, false, true, false>,
                        (const void*)k_f3_answer<32, false, true, false>, (const void*)k_f3_answer<8, true, true, false>,
                        (const void*)k_f3_answer<16, true, true, false>,  (const void*)k_f3_answer<32, true, true, false>,
                        (const void*)k_f3_answer<8, false, false, false>, (const void*)k_f3_answer<16, false, false, false>,
                        (const void*)k_f3_answer<32, false, false, false>, (const void*)k_f3_answer<8, true, false, false>,
                        (const void*)k_f3_answer<16, true, false, false>, (const void*)k_f3_answer<32, true, false, false>,
                        (const void*)k_f3_answer<8, false, true, true>,  (const void*)k_f3_answer<16, false, true, true>,
                        (const void*)k_f3_answer<32, false, true, true>, (const void*)k_f3_answer<8, false, false, true>,
                        (const void*)k_f3_answer<16, false, false, true>, (const void*)k_f3_answer<32, false, false, true>};
    for (const void* f : fs) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax);
}

// workspace: bitmap[nsub][nwords] | ctr[64] | pcount[kSets][NP] | tcount[kMaxParts * kCtrStride] |
// tie_hdr[NP * kTieSlots] | fb done[kFbBlocks] | tie_cnt[NP] -- all-zero between calls -- |
// fb_list[q] | tspill[q] | pstat[NP] | tbuf[NP * tcap] | tie_cand[NP * kTieSlots * 64] |
// pbuf[NP * kSets * scap] | fb rec[kFbBlocks * kFbGroup * k * 6] | sub descriptors | F2 map
// (NP = nsub * np partitions over all sub-partitions)
constexpr uint32_t kMaxParts = 1u << 15;
constexpr uint32_t kMaxSubs = 256;            // F2's workgroup -> sub-partition map is u8
constexpr uint32_t kMaxF2Blocks = 65536;
inline size_t al256(size_t b) { return (b + 255) & ~size_t(255); }

struct WsLayout {
    size_t ctr, bitmap, pcount, tcount, tie_hdr, fb_done, tie_cnt, ccount, clean;
    size_t fb_list, fb_sub, tspill, pstat, tbuf, tie_cand, pbuf, fb_rec, desc, blk_sub, cbuf, total;
};

// F1's two-pass form (k_f1_coarse + k_f1_fine) for batches of >= kF1CoarseMinQ targets: the
// coarse bins are the finest split (<= b1 and Lm - 5 bits per sub-partition) that keeps >= 512
// targets per bin and >= 16 per (F1a workgroup, bin) -- each reservation a run of >= 128 B (2,048
// bins at 2^20 targets left 2 per run: F1a 34 us, 524 K reservations) -- with F1b's LDS within
// kF1bLdsWords.  c = ~0u: one pass.
struct F1Coarse { uint32_t c, nbins, ccap; };
F1Coarse f1_coarse(const BatchPlan& P, uint32_t nsub, uint32_t q) {
    F1Coarse f{~0u, 0, 0};
    if (q < kF1CoarseMinQ || P.Lm < 5) return f;
    auto lds_ok = [&](uint32_t c) { return (1u << (P.Lm - c - 5)) + (1u << (P.b1 - c)) <= kF1bLdsWords; };
    uint32_t c = 0;
    while (c < P.b1 && c + 5 < P.Lm && ((uint64_t)nsub << (c + 1)) <= kF1aTargets / 16 &&
           ((uint64_t)nsub << (c + 1)) * 512 <= q)
        ++c;
    while (c < P.b1 && c + 5 < P.Lm && !lds_ok(c)) ++c;
    if (!lds_ok(c) || ((uint64_t)nsub << c) > kMaxCoarse) return f;
    f.c = c;
    f.nbins = nsub << c;
    const double M = (double)q / (double)f.nbins;
    f.ccap = ((uint32_t)(M + 8.0 * std::sqrt(M) + 64.0) + 63u) & ~63u;
    return f;
}

WsLayout ws_layout(const BatchPlan& P, uint32_t nsub, uint32_t q, uint32_t k) {
    const size_t NP = (size_t)nsub << P.b1;
    WsLayout L{};
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t r = off;
        off += al256(bytes);
        return r;
    };
    // bitmap first and the counter arrays sized for kMaxParts partitions: the compact layout
    // (counters right behind one another) cost F1 0.5 us and the pipelined cfg-2 step 0.3 us
    // (measured); the clean head is memset once per workspace
    L.bitmap = take(std::max<size_t>(65536, (size_t)nsub * P.nwords * 4));
    L.ctr = take(256);
    L.pcount = take((size_t)kSets * NP * 4);
    L.tcount = take((size_t)kMaxParts * kCtrStride * 4);
    L.tie_hdr = take((size_t)kMaxParts * kTieSlots * 16);
    L.fb_done = take((size_t)kFbBlocks * 4);
    L.tie_cnt = take((size_t)kMaxParts * 4);
    L.ccount = take((size_t)kMaxCoarse * 4);
    L.clean = off;
    L.fb_list = take((size_t)q * 4);
    L.fb_sub = take((size_t)q);
    L.tspill = take((size_t)q * 4);
    L.pstat = take(NP * 4);
    L.tbuf = take(NP * P.tcap * 8);
    L.tie_cand = take(NP * kTieSlots * 64 * 8);
    L.pbuf = take(NP * P.nsets * P.scap * 8);
    L.fb_rec = take((size_t)kFbBlocks * kFbGroup * k * 24);
    L.desc = take((size_t)kMaxSubs * sizeof(SubDesc));
    L.blk_sub = take(kMaxF2Blocks);
    const F1Coarse fc = f1_coarse(P, nsub, q);
    L.cbuf = take((size_t)fc.nbins * fc.ccap * 8);
    L.total = off;
    return L;
}

// F2's workgroups over the sub-partitions: whole rounds of num_cus workgroups, each
// sub-partition's share in proportion to its ids.  Sparse mode: the stage is flushed every
// *seg ids, the most it holds on uniform ids (mean + 8 sigma + 256 survivors) in whole ring
// turns -- one round of workgroups however large the set; when not even one ring turn fits, no
// workgroup gets more ids than that bound.
uint32_t deal_f2_blocks(const BatchPlan& P, const SubSpec* subs, uint32_t nsub, uint32_t q_plan, int num_cus,
                        SubDesc* d, uint32_t* seg) {
    const double f = 1.0 - std::exp(-(double)q_plan / (double)(1ull << P.Lm));
    uint64_t pb_cap = 1ull << 40;   // dense mode: no cap
    if (P.sparse) {
        pb_cap = kF2Step;
        for (uint64_t pb = kF2Step; pb <= (1ull << 31); pb += kF2Step) {
            const double mean = (double)pb * f, sd = std::sqrt(mean * P.clump);
            if (mean + 8.0 * sd + 256.0 > (double)P.stage) break;
            pb_cap = pb;
        }
    }
    *seg = 0xFFFFFFFFu;
    constexpr uint64_t turn = (uint64_t)kF2Ring * kF2Sub;
    if (P.sparse && pb_cap >= turn) {
        *seg = (uint32_t)std::min<uint64_t>(pb_cap / turn * turn, 0x80000000ull);
        pb_cap = 1ull << 40;
    }
    const uint64_t g = num_cus > 0 ? (uint64_t)num_cus : 256;
    uint64_t n_tot = 0, need = 0;
    for (uint32_t i = 0; i < nsub; ++i) {
        n_tot += subs[i].n;
        need += (subs[i].n + pb_cap - 1) / pb_cap;
    }
    const uint64_t total = std::max<uint64_t>(1, (need + g - 1) / g) * g;
    uint32_t blk = 0;
    for (uint32_t i = 0; i < nsub; ++i) {
        const uint64_t n = subs[i].n;
        uint64_t want = n_tot ? (uint64_t)std::llround((double)total * (double)n / (double)n_tot) : 0;
        want = std::max<uint64_t>(want, (n + pb_cap - 1) / pb_cap);
        if (n && !want) want = 1;
        // whole groups of kSets workgroups: block b writes bucket set b % kSets, and scap plans
        // every set for 1 / kSets of a partition's survivors (a sub-partition dealt 4 workgroups
        // would fill only 4 sets, each twice over: overflowing partitions, fallback scans)
        want = (want + kSets - 1) / kSets * kSets;
        uint64_t per = want ? (n + want - 1) / want : kF2Step;
        per = (per + kF2Step - 1) / kF2Step * kF2Step;
        if (per > pb_cap) per = pb_cap;
        const uint64_t nb = n ? (n + per - 1) / per : 0;
        const uint64_t lim = (subs[i].w0s ? subs[i].stride : 5 * subs[i].stride) - 4;
        d[i] = SubDesc{subs[i].w0s ? subs[i].w0s : subs[i].planes, subs[i].planes, subs[i].stride, n, subs[i].gidx,
                       subs[i].base, (uint32_t)(lim < 0xFFFFFFF0ull ? lim : 0xFFFFFFF0ull), blk, (uint32_t)nb, per};
        blk += (uint32_t)nb;
    }
    return blk;
}

}  // namespace

bool batch_supported(uint64_t n, uint32_t q, uint32_t k, int num_cus, uint32_t nsub, uint32_t pf) {
    if (k == 0 || k > DHTGPU_MAX_K_DEV || n >= (1ull << 31) || nsub == 0 || nsub > kMaxSubs) return false;
    const BatchPlan P = plan_batch(n, q, k, num_cus, pf);
    if ((uint64_t)q * nsub > kMaxQ) return false;
    if (((uint64_t)nsub << P.b1) > kMaxParts) return false;
    // dense mode flushes whenever less than one sub-step of room is left
    if (!P.fits || P.Lm - P.b1 > 13 || (!P.sparse && P.stage < kF2Sub + 1024)) return false;
    return f3_lds(P, P.f3cap_wide) <= kLdsMax && f2_lds(P) <= kLdsMax;
}

size_t batch_ctr_offset(uint64_t n, uint32_t q_plan, uint32_t k, int num_cus, uint32_t nsub, uint32_t pf) {
    return ws_layout(plan_batch(n, q_plan, k, num_cus, pf), nsub, 0, k).ctr;
}

size_t batch_clean_bytes(uint64_t n, uint32_t q_plan, uint32_t k, int num_cus, uint32_t nsub, uint32_t pf) {
    return ws_layout(plan_batch(n, q_plan, k, num_cus, pf), nsub, 0, k).clean;
}

size_t batch_bytes(uint64_t n, uint32_t q, uint32_t q_plan, uint32_t k, int num_cus, uint32_t nsub, uint32_t pf) {
    return ws_layout(plan_batch(n, q_plan, k, num_cus, pf), nsub, q, k).total;
}

hipError_t batch_read_stats(const void* ws, uint64_t n, uint32_t q, uint32_t q_plan, uint32_t k, int num_cus,
                            uint32_t* stats4, hipStream_t s, uint32_t nsub, uint32_t pf) {
    const BatchPlan P = plan_batch(n, q_plan, k, num_cus, pf);
    const WsLayout Ly = ws_layout(P, nsub, q, k);
    const size_t NP = (size_t)nsub << P.b1;
    const uint8_t* w = static_cast<const uint8_t*>(ws);
    std::vector<uint32_t> ps(NP);
    hipError_t e = hipMemcpyAsync(stats4, w + Ly.ctr, 16, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipMemcpyAsync(ps.data(), w + Ly.pstat, NP * 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    uint64_t tot = 0;
    for (uint32_t v : ps) tot += v;
    stats4[1] = (uint32_t)tot;   // survivors = sum over partitions
    return e;
}

__global__ void k_shift_w0(const uint32_t* __restrict__ planes, uint64_t stride, uint32_t shift,
                           uint32_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < stride) out[i] = (planes[i] << shift) | (planes[stride + i] >> (32 - shift));
}

// Level-kMaxLm cell counts of a sub-partition (its shifted word-0 plane): u32 counters, then
// saturated to u8 (F1's sibling rule only compares them with k <= DHTGPU_MAX_K_DEV < 255).
// Persistent with the sub-partitions (2^kMaxLm B each), rebuilt when the set changes.
__global__ void k_cell_count(const uint32_t* __restrict__ w0s, uint64_t n, uint32_t* __restrict__ cnt) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        atomicAdd(cnt + (w0s[i] >> (32 - kMaxLm)), 1u);
}
__global__ void k_cell_pack(const uint32_t* __restrict__ cnt, uint8_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < (1u << kMaxLm)) out[i] = (uint8_t)(cnt[i] < 255u ? cnt[i] : 255u);
}

uint32_t cell_level() { return kMaxLm; }

// spans[j] = max over i of cell(i + 2^j - 1) - cell(i) (level-kMaxLm cells of a prefix-sorted
// shifted word-0 plane; the last id when 2^j > n - i): the most cells (hence bitmap words) any
// 2^j consecutive ids of the sub-partition span -- F2's window bound (j < 32)
__global__ void k_cell_spans(const uint32_t* __restrict__ w0s, uint64_t n, uint32_t* __restrict__ spans) {
    __shared__ uint32_t smax[32];
    if (threadIdx.x < 32) smax[threadIdx.x] = 0;
    __syncthreads();
    uint32_t mx[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) mx[j] = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint32_t c0 = w0s[i] >> (32 - kMaxLm);
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            const uint64_t e = i + (1ull << j) - 1;
            const uint32_t c1 = w0s[e < n ? e : n - 1] >> (32 - kMaxLm);
            mx[j] = max(mx[j], c1 - c0);
        }
    }
#pragma unroll
    for (int j = 0; j < 32; ++j) atomicMax(&smax[j], mx[j]);
    __syncthreads();
    if (threadIdx.x < 32) atomicMax(spans + threadIdx.x, smax[threadIdx.x]);
}

hipError_t launch_cell_spans(const uint32_t* w0s, uint64_t n, uint32_t* spans, hipStream_t s) {
    hipError_t e = hipMemsetAsync(spans, 0, 32 * 4, s);
    if (e != hipSuccess || !n) return e;
    k_cell_spans<<<dim3(1024), dim3(256), 0, s>>>(w0s, n, spans);
    return hipGetLastError();
}

hipError_t launch_cell_counts(const uint32_t* w0s, uint64_t n, uint32_t* scratch, uint8_t* out, hipStream_t s) {
    hipError_t e = hipMemsetAsync(scratch, 0, ((size_t)1 << kMaxLm) * 4, s);
    if (e != hipSuccess) return e;
    if (n) k_cell_count<<<dim3(2048), dim3(256), 0, s>>>(w0s, n, scratch);
    k_cell_pack<<<dim3((1u << kMaxLm) / 256), dim3(256), 0, s>>>(scratch, out);
    return hipGetLastError();
}

hipError_t launch_shift_w0(const uint32_t* planes, uint64_t stride, uint32_t shift, uint32_t* out, hipStream_t s) {
    if (shift == 0 || shift >= 32) return hipErrorInvalidValue;
    k_shift_w0<<<dim3((uint32_t)((stride + 255) / 256)), dim3(256), 0, s>>>(planes, stride, shift, out);
    return hipGetLastError();
}

// Sub-partition handles <-> indices (dhtgpu_handles_to_indices_dev; the K1 route of a
// sub-partitioned call under handles).  tab: the context's sub-partitions, offsets ascending.
__global__ void k_handles_to_idx(const HandleSub* __restrict__ tab, uint32_t nsub, const uint32_t* __restrict__ h,
                                 uint64_t m, uint32_t* __restrict__ out, uint32_t global, uint32_t base) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    const uint32_t x = h[i];
    uint32_t r = DHT_NONE;
    if (x != DHT_NONE) {
        uint32_t lo = 0, hi = nsub;   // the last sub-partition whose offset <= x
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (tab[mid].off <= x) lo = mid; else hi = mid;
        }
        const HandleSub t = tab[lo];
        const uint64_t j = x - t.off;
        if (j < t.n) r = global ? t.gmap[j] : t.map[j] + base;
    }
    out[i] = r;
}

__global__ void k_idx_to_handles(const uint32_t* __restrict__ hinv, uint32_t* __restrict__ idx, uint64_t m) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    const uint32_t x = idx[i];
    if (x != DHT_NONE) idx[i] = hinv[x];
}

__global__ void k_handle_inverse(const uint32_t* __restrict__ map, uint64_t m, uint32_t off, uint32_t* __restrict__ hinv) {
    for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < m; j += (uint64_t)gridDim.x * 256)
        hinv[map[j]] = off + (uint32_t)j;
}

// Sub-partition handles: the rows F4 answered from the whole set (targets whose own sub-partition
// holds fewer than k ids, long fallback lists) hold context-local index | kHandleMark (the
// whole-set roles' result offset); this pass, after F4 and only under handles, turns them into
// handles.  The fallback list and its count (ctr[0]) are the call's own, F1 of the next call
// resets them.
__global__ void k_fb_handles(uint32_t* __restrict__ out_idx, uint32_t k, const uint32_t* __restrict__ fb_list,
                             const uint32_t* __restrict__ ctr, const uint32_t* __restrict__ hinv) {
    const uint64_t m = (uint64_t)ctr[0] * k;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (uint64_t)gridDim.x * 256) {
        uint32_t* p = out_idx + (uint64_t)fb_list[i / k] * k + i % k;
        const uint32_t x = *p;
        if (x == DHT_NONE || !(x & kHandleMark)) continue;
        *p = hinv[x & ~kHandleMark];
    }
}

hipError_t launch_handles_to_idx(const HandleSub* tab, uint32_t nsub, const uint32_t* h, uint64_t m, uint32_t* out,
                                 bool global, uint32_t base, hipStream_t s) {
    if (!m) return hipSuccess;
    k_handles_to_idx<<<dim3((uint32_t)((m + 255) / 256)), dim3(256), 0, s>>>(tab, nsub, h, m, out, global ? 1u : 0u, base);
    return hipGetLastError();
}

hipError_t launch_idx_to_handles(const uint32_t* hinv, uint32_t* idx, uint64_t m, hipStream_t s) {
    if (!m) return hipSuccess;
    k_idx_to_handles<<<dim3((uint32_t)((m + 255) / 256)), dim3(256), 0, s>>>(hinv, idx, m);
    return hipGetLastError();
}

hipError_t launch_handle_inverse(const uint32_t* map, uint64_t m, uint32_t off, uint32_t* hinv, hipStream_t s) {
    if (!m) return hipSuccess;
    k_handle_inverse<<<dim3(2048), dim3(256), 0, s>>>(map, m, off, hinv);
    return hipGetLastError();
}

hipError_t launch_batch_topk(const BatchCall& c, hipStream_t s) {
    if (c.skip && !c.w0s && !c.nsub) return hipErrorInvalidValue;
    if (c.nsub > kMaxSubs) return hipErrorInvalidValue;
    if (!c.q) return hipSuccess;
    {
        const hipError_t e = per_device_once(g_attr_once, set_lds_attributes);
        if (e != hipSuccess) return e;
    }
    const uint32_t q = c.q, k = c.k;
    // the sub-partitions (a set that needs no split is its own one sub-partition); the plan is
    // the largest one's
    const SubSpec one{c.planes, c.w0s, c.stride, c.n, c.gidx, c.base};
    const SubSpec* subs = c.nsub ? c.subs : &one;
    const uint32_t nsub = c.nsub ? c.nsub : 1u;
    uint64_t n_max = 0, n_all = 0;
    for (uint32_t i = 0; i < nsub; ++i) {
        n_max = std::max<uint64_t>(n_max, subs[i].n);
        n_all += subs[i].n;
    }
    const bool nt = 4 * n_all > kNtBytes;   // F2's ring: non-temporal past the Infinity Cache
    const uint32_t pf = (c.cells ? kPlanCells : 0u) | (c.sorted ? kPlanSorted : 0u);
    BatchPlan P = plan_batch(n_max, c.q_plan, k, c.num_cus, pf);
    const BatchPlan P0 = P;   // the workspace layout's plan (window mode may refine P below)
    const uint32_t np = 1u << P.b1, NP = nsub * np;
    uint32_t dbg = c.dbg & 256u;   // the only diagnostics bit: phase stamps (results unchanged)
    hipEvent_t* ev = c.ev;
    const WsLayout Ly = ws_layout(P, nsub, q, k);
    uint8_t* const w = static_cast<uint8_t*>(c.ws);
    uint32_t* bitmap = reinterpret_cast<uint32_t*>(w + Ly.bitmap);
    uint32_t* ctr = reinterpret_cast<uint32_t*>(w + Ly.ctr);
    uint32_t* pcount = reinterpret_cast<uint32_t*>(w + Ly.pcount);
    uint32_t* tcount = reinterpret_cast<uint32_t*>(w + Ly.tcount);
    uint4* tie_hdr = reinterpret_cast<uint4*>(w + Ly.tie_hdr);
    uint32_t* fb_done = reinterpret_cast<uint32_t*>(w + Ly.fb_done);
    uint32_t* tie_cnt = reinterpret_cast<uint32_t*>(w + Ly.tie_cnt);
    uint32_t* fb_list = reinterpret_cast<uint32_t*>(w + Ly.fb_list);
    uint8_t* fb_sub = w + Ly.fb_sub;
    uint32_t* tspill = reinterpret_cast<uint32_t*>(w + Ly.tspill);
    uint32_t* pstat = reinterpret_cast<uint32_t*>(w + Ly.pstat);
    uint2* tbuf = reinterpret_cast<uint2*>(w + Ly.tbuf);
    uint2* tie_cand = reinterpret_cast<uint2*>(w + Ly.tie_cand);
    uint2* pbuf = reinterpret_cast<uint2*>(w + Ly.pbuf);
    uint32_t* fb_rec = reinterpret_cast<uint32_t*>(w + Ly.fb_rec);
    SubDesc* d_desc = reinterpret_cast<SubDesc*>(w + Ly.desc);
    uint8_t* d_blk = w + Ly.blk_sub;
    // sub-partition descriptors and F2's workgroup map: one sub-partition travels in the kernel
    // arguments; several are uploaded when they differ from what this workspace holds
    // (steady-state calls upload nothing)
    SubDesc hd[kMaxSubs];
    uint32_t seg = 0, pk_ob = 0;
    uint32_t nblk2 = deal_f2_blocks(P, subs, nsub, c.q_plan, c.num_cus, hd, &seg);
    // window mode (prefix-sorted sub-partitions with span tables): every workgroup's bitmap window
    // is bounded by its sub-partition's largest cell span over as many consecutive ids as the
    // workgroup holds; taken when that bound is small (the cfg-3 shard: ~520 words of 16,384)
    bool direct = false;   // k_f2_direct (sorted sub-partitions: no stage)
    if (c.spans && c.sorted && nsub > 1 && P.Lm >= 6 && P.Lm <= kMaxLm) {
        auto need = [&](const SubDesc* dd) {
            uint32_t w = 0;
            for (uint32_t i = 0; i < nsub; ++i) {
                if (!dd[i].nblk) continue;
                uint32_t j = 0;
                while (j < 31 && (1ull << j) < dd[i].per_blk) ++j;
                const uint32_t span19 = c.spans[i * 32 + j];   // level-kMaxLm cells
                w = std::max<uint32_t>(w, (span19 >> (kMaxLm - P.Lm + 5)) + 3u);
            }
            return w;
        };
        if (P.nsets == 1) {   // direct: one persistent workgroup per CU (no stage bounds a range)
            BatchPlan Pd = P;
            Pd.sparse = 0;
            SubDesc hw[kMaxSubs];
            uint32_t segw = 0;
            const uint32_t nbw = deal_f2_blocks(Pd, subs, nsub, c.q_plan, c.num_cus, hw, &segw);
            uint32_t wd = 64;
            while (wd < need(hw)) wd <<= 1;
            if (wd <= 2 * kF2Threads && 2 * wd <= P.nwords && nbw <= kMaxF2Blocks) {
                direct = true;
                P.wwords = wd;
                nblk2 = nbw;
                std::copy(hw, hw + nsub, hd);
            }
        }
        uint32_t ww = 64;
        while (ww < need(hd)) ww <<= 1;
        if (!direct && P.sparse && ww <= 2 * kF2Threads && 2 * ww <= P.nwords) {
            BatchPlan Pw = plan_batch(n_max, c.q_plan, k, c.num_cus, pf, ww);
            SubDesc hw[kMaxSubs];
            uint32_t segw = 0;
            uint32_t nbw = deal_f2_blocks(Pw, subs, nsub, c.q_plan, c.num_cus, hw, &segw);
            bool segd = false;
            for (uint32_t i = 0; i < nsub; ++i) segd = segd || (hw[i].nblk && hw[i].per_blk > segw);
            // ranges past one packed stage-full: 8-B segments (kStagePer entries in registers) in the
            // LDS the window leaves.  (Sizing the segmented stage so that two F3 workgroups of the
            // other call in flight fit beside F2 measured equal at the cfg-3 prefix rank, 0.148 ms
            // both, and slower at the broadcast rank, 0.558 -> 0.593 ms: profiles/r06/window_ab.txt)
            if (Pw.sparse && segd) {
                const size_t fx = (size_t)f2_fixed_words(ww, 1u << Pw.b1) * 4;
                Pw.stage = (uint32_t)std::min<size_t>(fx < kLdsMax ? (kLdsMax - fx) / 8 : 0, kStage);
                Pw.wpack = false;
                nbw = deal_f2_blocks(Pw, subs, nsub, c.q_plan, c.num_cus, hw, &segw);
            }
            // the packed stage's index offsets take ob bits, word 0 above the window's first word
            // log2(ww) + 37 - Lm bits: 48 in all
            uint64_t pbmax = 1;
            for (uint32_t i = 0; i < nsub; ++i) pbmax = std::max<uint64_t>(pbmax, hw[i].nblk ? hw[i].per_blk : 1);
            uint32_t ob = 0, lw = 0;
            while ((1ull << ob) < pbmax) ++ob;
            while ((1u << lw) < ww) ++lw;
            bool ok = Pw.sparse && need(hw) <= ww && nbw <= kMaxF2Blocks;
            bool segw_used = false;
            for (uint32_t i = 0; i < nsub; ++i) segw_used = segw_used || (hw[i].nblk && hw[i].per_blk > segw);
            if (Pw.wpack) ok = ok && !segw_used && lw + 37 - Pw.Lm + ob <= 48;
            else ok = ok && segw_used;   // (8-B window stage: the segmented instantiation only)
            if (ok) {
                P = Pw;
                nblk2 = nbw;
                seg = segw;
                pk_ob = ob;
                std::copy(hw, hw + nsub, hd);
            }
        }
    }
    const bool win = P.wwords != 0;
    bool seg_used = false;   // some workgroup's range spans more than one segment
    for (uint32_t i = 0; i < nsub; ++i) seg_used = seg_used || (hd[i].nblk && hd[i].per_blk > seg);
    if (nblk2 > kMaxF2Blocks) return hipErrorInvalidValue;
    // the narrow stage: every workgroup's range under 2^16 ids and its survivors (mean + 8 sigma
    // + 256 on uniform ids) within the narrow stage; no segments
    bool narrow = !direct && P.nstage && P.sparse && !seg_used;
    {
        const double f = 1.0 - std::exp(-(double)c.q_plan / (double)(1ull << P.Lm));
        for (uint32_t i = 0; i < nsub && narrow; ++i) {
            const double mean = (double)hd[i].per_blk * f, sd = std::sqrt(mean * P.clump);
            if (hd[i].nblk && (hd[i].per_blk > 65536 || mean + 8.0 * sd + 256.0 > (double)P.nstage)) narrow = false;
        }
    }
    if (NP > 8192 || nblk2 > 8192) dbg &= ~256u;   // phase stamps hold 8192 workgroups per kernel
    if (nsub > 1) {
        uint64_t sig = 1469598103934665603ull;
        auto mix = [&](const void* p, size_t b) {
            const uint8_t* x = static_cast<const uint8_t*>(p);
            for (size_t i = 0; i < b; ++i) sig = (sig ^ x[i]) * 1099511628211ull;
        };
        mix(hd, nsub * sizeof(SubDesc));
        mix(&nsub, 4);
        mix(&nblk2, 4);   // (seg travels in the kernel arguments)
        // where the tables live: their offsets depend on k and q (the layout puts them after
        // the k-sized fallback records), so a call with another k on the same workspace must
        // upload them again
        const uint8_t* wd = reinterpret_cast<const uint8_t*>(d_desc);
        const uint8_t* wb = d_blk;
        mix(&wd, sizeof wd);
        mix(&wb, sizeof wb);
        if (sig == 0) sig = 1;
        if (!c.desc_sig || *c.desc_sig != sig) {
            std::vector<uint8_t> bs(nblk2);
            for (uint32_t i = 0; i < nsub; ++i)
                for (uint32_t b = 0; b < hd[i].nblk; ++b) bs[hd[i].blk0 + b] = (uint8_t)i;
            hipError_t e = hipMemcpyAsync(d_desc, hd, nsub * sizeof(SubDesc), hipMemcpyHostToDevice, s);
            if (e == hipSuccess && nblk2) e = hipMemcpyAsync(d_blk, bs.data(), nblk2, hipMemcpyHostToDevice, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);   // the host copies are released below
            if (e != hipSuccess) return e;
            if (c.desc_sig) *c.desc_sig = sig;
        }
    }
    // ev (diagnostics): 8 events, a start/stop pair per kernel recorded by the kernel's own
    // dispatch (hipExtLaunchKernel), so the pairs time the kernels themselves
    auto go = [&](int i, auto kern, dim3 g, dim3 b, size_t lds, auto... args) {
        if (ev) hipExtLaunchKernelGGL(kern, g, b, (uint32_t)lds, s, ev[2 * i], ev[2 * i + 1], 0, args...);
        else kern<<<g, b, lds, s>>>(args...);
    };
    unsigned long long* stamps = (dbg & 256u) ? c.stamps : nullptr;   // F3 [8192][16] then F2 [8192][16]
    if (dbg & 256) (void)hipMemsetAsync(stamps, 0, (size_t)3 * 8192 * 16 * 8, s);
    const F1Args a1{c.tp, c.tp + c.ts, q, P.Lm, P.b1, c.skip, c.sub_shift, c.nsub ? c.sub_bits : 0u, np, P.nwords,
                    bitmap, tcount, tbuf, P.tcap, ctr, tspill, P.sib ? c.cells : nullptr, k};
    const F1Coarse f1c = f1_coarse(P0, nsub, q);
    if (f1c.nbins && P.Lm == P0.Lm && P.b1 == P0.b1) {
        F1cArgs ac{c.tp, c.tp + c.ts, q, c.skip, c.sub_shift, c.nsub ? c.sub_bits : 0u, f1c.c, f1c.ccap,
                   reinterpret_cast<uint32_t*>(w + Ly.ccount), reinterpret_cast<uint2*>(w + Ly.cbuf),
                   P.Lm, P.b1, np, P.nwords, bitmap, tcount, tbuf, P.tcap, ctr, tspill,
                   P.sib ? c.cells : nullptr, k};
        const dim3 ga((q + kF1aTargets - 1) / kF1aTargets), gb(f1c.nbins);
        const size_t lb = (size_t)((1u << (P.Lm - f1c.c - 5)) + (1u << (P.b1 - f1c.c))) * 4;
        if (ev) {   // pair 0 brackets both passes
            hipExtLaunchKernelGGL(k_f1_coarse, ga, dim3(kF1aThreads), 0, s, ev[0], nullptr, 0, ac);
            hipExtLaunchKernelGGL(k_f1_fine, gb, dim3(kF1bThreads), (uint32_t)lb, s, nullptr, ev[1], 0, ac);
        } else {
            k_f1_coarse<<<ga, dim3(kF1aThreads), 0, s>>>(ac);
            k_f1_fine<<<gb, dim3(kF1bThreads), lb, s>>>(ac);
        }
    } else {
        go(0, k_f1_targets, dim3((q + kF1Threads - 1) / kF1Threads), dim3(kF1Threads), 0, a1);
    }
    if (nblk2) {
        F2Args a2{d_desc, d_blk, hd[0], nsub, NP, P.Lm, P.b1, bitmap, P.nwords, pcount, pbuf, P.scap, ctr,
                  narrow ? P.nstage : P.stage, dbg, P.sparse, seg, (dbg & 256) ? stamps + 8192 * 16 : stamps};
        a2.nsets = P.nsets;
        a2.wwords = P.wwords;
        a2.pk_ob = pk_ob;
        const dim3 g2(nblk2), b2(kF2Threads);
        const size_t l2 = f2_lds(P, narrow);
#define F2_GO(MM)                                                    \
    do {                                                             \
        if (nsub > 1 && nt) go(1, k_f2_filter<MM, kF2SubsNT>, g2, b2, l2, a2); \
        else if (nsub > 1) go(1, k_f2_filter<MM, kF2Subs>, g2, b2, l2, a2);   \
        else go(1, k_f2_filter<MM, kF2One>, g2, b2, l2, a2);                  \
    } while (0)
        // window mode: no stage (direct), the packed stage with one final flush (P.wpack), or 8-B segments
        if (direct && nt) go(1, k_f2_direct<kF2SubsNT>, g2, b2, (size_t)(8 + P.wwords + kDirParts) * 4, a2);
        else if (direct) go(1, k_f2_direct<kF2Subs>, g2, b2, (size_t)(8 + P.wwords + kDirParts) * 4, a2);
        else if (win && nt && !P.wpack) go(1, k_f2_filter<kF2Seg, kF2SubsNT, true>, g2, b2, l2, a2);
        else if (win && nt) go(1, k_f2_filter<kF2Sparse, kF2SubsNT, true>, g2, b2, l2, a2);
        else if (win && !P.wpack) go(1, k_f2_filter<kF2Seg, kF2Subs, true>, g2, b2, l2, a2);
        else if (win) go(1, k_f2_filter<kF2Sparse, kF2Subs, true>, g2, b2, l2, a2);
        else if (narrow) F2_GO(kF2Narrow);
        else if (P.sparse && seg_used) F2_GO(kF2Seg);
        else if (P.sparse) F2_GO(kF2Sparse);
        else F2_GO(kF2Dense);
#undef F2_GO
    } else if (ev) {
        (void)hipEventRecord(ev[2], s);
        (void)hipEventRecord(ev[3], s);
    }
    // the base arguments are the whole set's: F4's scan (fallback targets) runs over all its ids
    F3Args a{pbuf, pcount, P.scap, tbuf, tcount, P.tcap, tspill, P.Lm, P.b1, P.Lq, bitmap, P.nwords, c.planes, c.stride,
             c.n, c.tp, c.ts, k, c.gidx, c.base, c.out_idx, c.out_cnt, ctr, fb_list, fb_sub, pstat, tie_hdr, tie_cand, tie_cnt,
             d_desc, np, dbg, stamps, narrow ? P.f3cap : P.f3cap_wide, RecOut{}, P.Lm - P.sib, P.nsets};
    if (c.out_rec)
        a.rec = RecOut{c.out_rec, c.planes, c.stride, c.rec_gidx, c.rec_base, (nsub == 1 && !c.w0s && !c.skip) ? 1u : 0u,
                       c.skip && c.skip < 32 ? c.skip : 0u, c.nsub ? c.pval << c.sub_bits : c.pval};

    // F3 stages the plan's 6-sigma bound beside F2's narrow stage (which it makes room for), and on
    // sub-partitioned calls whose partitions run in several rounds of workgroups when that lets 5 or
    // 6 of them share a CU instead of 4 (F3<8> holds 78 VGPRs: 6 waves per SIMD); F3 is a chain of
    // round trips per workgroup, so a round of more workgroups shortens the launch (a partition past
    // the bound sends its targets to the exact fallback, as one past kF3Cap does)
    if (!narrow && nsub > 1 && k <= 8 && P.fits && P.cap6 < a.cap && NP >= 8u * (uint32_t)std::max(c.num_cus, 1)) {
        auto per_cu = [](size_t l) { return std::min<size_t>(6, kLdsMax / ((l + 1023) & ~(size_t)1023)); };
        if (per_cu(f3_lds(P, P.cap6)) > per_cu(f3_lds(P, a.cap))) a.cap = P.cap6;
    }
    size_t l3 = f3_lds(P, a.cap);
    const dim3 g3(NP), b3(kF3Threads);
    const bool ex = c.n >= k && (k == 8 || k == 16 || k == 32);
#define F3_GO(KK, DD, SS)                                                     \
    do {                                                                      \
        if (ex) go(2, k_f3_answer<KK, DD, true, SS>, g3, b3, l3, a);        \
        else go(2, k_f3_answer<KK, DD, false, SS>, g3, b3, l3, a);          \
    } while (0)
    if (nsub > 1) {   // (no phase-stamp build for sub-partitioned calls)
        if (k <= 8) F3_GO(8, false, true);
        else if (k <= 16) F3_GO(16, false, true);
        else F3_GO(32, false, true);
    } else if (dbg) {
        if (k <= 8) F3_GO(8, true, false);
        else if (k <= 16) F3_GO(16, true, false);
        else F3_GO(32, true, false);
    } else {
        if (k <= 8) F3_GO(8, false, false);
        else if (k <= 16) F3_GO(16, false, false);
        else F3_GO(32, false, false);
    }
#undef F3_GO
    if (dbg & 256) print_phase_profile(P, nblk2, NP, stamps, s);
    // F4's grid: its workgroups (50 KB of LDS each) hold CUs the other batches' F2 / F3 want,
    // and on one set (ties answered inline by F3) an empty fallback list leaves them nothing to
    // do -- 32 workgroups when the context's last completed call listed no target (a hint F4
    // leaves in mapped host memory; read without a sync, so possibly a call or two old; a list
    // that appears then is scanned by those 32, still exactly), the full grid otherwise (the
    // fallback scan's parallelism).  Round 5: 128 -> 32 with the tie-count reads gone, cfg-2 step
    // 33.6 -> 31.7-31.9 us (profiles/r05/experiments/f4_idle_ab.txt, f4_idle_grid_ab.txt; 16 and
    // 8 equal).  (a sub-partitioned call fills the chip alone and defers ~1 tie per partition over
    // 2,048+ partitions: the full grid keeps them at about one per wave)
    constexpr uint32_t kF4IdleGrid = 32;
    const uint32_t nfb = (c.fb_hint && *c.fb_hint == 0u && nsub == 1) ? kF4IdleGrid : kFbBlocks;
    // one set: F3 answers its ties inline, so F4 reads no deferred-tie counts (np_ties 0)
    const FbArgs fa{fb_rec, fb_done, nfb, nsub > 1 ? NP : 0u, c.fb_hint_dev};
    const dim3 g4(nfb), b4(kF4Threads);
    if (k <= 8) go(3, k_f4<8>, g4, b4, 0, a, fa);
    else if (k <= 16) go(3, k_f4<16>, g4, b4, 0, a, fa);
    else go(3, k_f4<32>, g4, b4, 0, a, fa);
    if (c.handles && nsub > 1 && !c.out_rec)   // the whole-set fallback rows -> handles
        k_fb_handles<<<dim3(64), dim3(256), 0, s>>>(c.out_idx, k, fb_list, ctr, c.hinv);
    return hipGetLastError();
}


// ---- KS: small batches (q <= kSmallQ) --------------------------------------------------------
// K6's four kernels cost ~30 µs whatever q is; a handful of targets needs one pass over w0 and
// little else.  S1 streams w0 once on every CU: each id's top hb = min(16, Ls) bits are tested
// against an LDS bitmap of the targets' (at most 64 set bits of 2^16), and the rare hits are
// matched exactly against the sorted distinct level-Ls prefixes of the targets; a match is
// appended, with its word 1 (loaded after the stream, with the append), to that prefix's
// candidate bucket.  S2, one launch: one workgroup per distinct prefix answers the prefix's
// targets from its bucket -- every id of sub(t, Ls), complete, so the exact top-k when it holds
// >= k ids (the candidates' (w0, w1) distance order in registers, the full key only on a double
// tie) -- and kSmallFbBlocks scan-role workgroups beside them read the final bucket counts (S1
// has completed), list the targets whose bucket is short of k ids or overflowed, and answer
// them with the K1 scan over all ids (F4's list scan); on uniform ids the list is empty and the
// role workgroups exit after one round trip (round 2 launched a separate F4 for it: an empty
// kernel of ~4 µs on every call).  The bucket counters come in two sets used by alternate calls:
// S2's workgroups read this call's while S2 zeroes the other's for the next call.  Prefix
// shards stream their shifted word-0 plane, as K6 does.
namespace {
constexpr uint32_t kSmallQ = 64;
constexpr uint32_t kSmallCap = 512;                   // candidates per prefix bucket
constexpr uint32_t kS1Queue = 512;                    // matched ids queued in LDS per block
constexpr uint32_t kSmallFbBlocks = 32;               // K1 fallback scan workgroups (S2's scan roles)
constexpr int kS2Threads = scan::WAVES * 64;
static_assert(kSmallCap <= (uint32_t)kS2Threads, "one bucket slot per S2 thread");

struct SmallArgs {
    const uint32_t* w0; uint64_t n; uint64_t per_blk; uint32_t lim;
    const uint32_t* w1;         // the ids' word-1 plane (unshifted): carried with every candidate
    const uint32_t* tp; uint64_t ts; uint32_t q, shift, Ls;
    uint32_t* cnt;              // [kSmallQ] this call's bucket fills (all-zero before S1)
    uint32_t* cnt_next;         // [kSmallQ] the next call's (S2 zeroes them)
    uint4* cand;                // [kSmallQ][kSmallCap] {shifted w0, index, word 1, 0}
    uint32_t* tab;              // [kSmallQ + 1] the sorted distinct prefixes (S1 block 0), their number last
    uint32_t* fb;               // [kSmallFbBlocks][kSmallQ] each scan role's copy of the fallback list
};

// target qi's word 0 as the streamed plane holds it (shifted for a prefix shard)
__device__ __forceinline__ uint32_t small_tw0(const SmallArgs& a, uint32_t qi) {
    const uint32_t w = a.tp[qi];
    return a.shift ? (w << a.shift) | (a.tp[a.ts + qi] >> (32 - a.shift)) : w;
}

// NQ > 0 (q <= NQ targets, so at most NQ distinct prefixes): an id's level-Ls prefix is compared
// in registers with the NQ sorted prefixes (wave-uniform, unused slots past any prefix) and the
// match is its bucket slot -- one v_bfe + NQ compares per id instead of the LDS bitmap read and
// the binary search of a hit.  The filter cost 2.4 us of S1 at q = 1 over the bare stream
// (profiles/r03/experiments/s1_measure.txt); NQ = 1 (q = 1): S1 13.0 -> 11.8 us.  NQ = 8 for
// q <= 8 measured slower than the bitmap (20.3 against 13.9 us at q = 8): q > 1 takes NQ = 0,
// the bitmap.
template <int NT, int NQ>
__global__ __launch_bounds__(NT) void k_s1_filter(SmallArgs a) {
    constexpr uint32_t kS1Sub = 4 * NT;
    __shared__ uint32_t b16[2048];      // 2^16 bits: the targets' top hb prefix bits
    __shared__ uint32_t tab[kSmallQ];   // sorted distinct level-Ls prefixes
    __shared__ uint4 hitq[kS1Queue];    // matched ids {w0, index, prefix slot}, appended after the stream
    __shared__ uint32_t ntab_s, nhit;
    const uint32_t lane = lane_id();
    const uint32_t hb = a.Ls < 16 ? a.Ls : 16u;
    const uint64_t lo64 = (uint64_t)blockIdx.x * a.per_blk;
    const uint32_t lo = (uint32_t)(lo64 < a.n ? lo64 : a.n);
    const uint32_t hi = (uint32_t)(lo64 + a.per_blk < a.n ? lo64 + a.per_blk : a.n);
    const uint32_t lim = min(a.lim, ((hi + 3u) & ~3u) - 4u);
    // non-temporal ring loads: q = 1 11.9 -> 10.9 us, q = 8 13.9 -> 12.5 us on the cfg-2 set
    // (profiles/r03/experiments/stream_nt_ab.txt)
    typedef unsigned int u4v __attribute__((ext_vector_type(4)));
    auto load = [&](uint32_t c) {
        uint32_t j = c + 4 * threadIdx.x;
        j = j < lim ? j : lim;
        const u4v x = __builtin_nontemporal_load(reinterpret_cast<const u4v*>(a.w0 + j));
        return make_uint4(x[0], x[1], x[2], x[3]);
    };
    // the id ring first: the setup below runs while its loads are in flight
    uint4 ring[kRing];
#pragma unroll
    for (uint32_t r = 0; r < kRing; ++r) ring[r] = load(lo + r * kS1Sub);
    for (uint32_t i = threadIdx.x; i < 2048; i += NT) b16[i] = 0;
    if (threadIdx.x == 0) nhit = 0;
    if (threadIdx.x < 64) {   // wave 0: the distinct prefixes, ranked (q <= 64: one per lane)
        const bool v = lane < a.q;
        const uint32_t pre = v ? top_bits(small_tw0(a, lane), a.Ls) : DHT_NONE;
        bool first = v;
        uint32_t rank = 0;
        for (uint32_t o = 0; o < 64; ++o) {
            const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)pre, (int)o);
            if (o < lane && x == pre) first = false;
        }
        const uint64_t fm = __ballot(first);
        for (uint32_t o = 0; o < 64; ++o) {
            const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)pre, (int)o);
            if (((fm >> o) & 1ull) && x < pre) ++rank;
        }
        if (first) tab[rank] = pre;
        if (lane == 0) ntab_s = (uint32_t)__popcll(fm);
        if (blockIdx.x == 0) {
            if (first) a.tab[rank] = pre;
            if (lane == 0) a.tab[kSmallQ] = (uint32_t)__popcll(fm);
        }
    }
    __syncthreads();
    const uint32_t ntab = ntab_s;
    if (threadIdx.x < ntab) {
        const uint32_t h = tab[threadIdx.x] >> (a.Ls - hb);
        atomicOr(b16 + (h >> 5), 1u << (h & 31));
    }
    __syncthreads();
    // a matched id goes to the block's LDS queue (a returning global atomic inside the loop
    // would wait for the whole ring: vmcnt is in order); past the queue, straight to its bucket
    auto emit = [&](uint32_t w, uint32_t j, uint32_t slot) {
        const uint32_t qi = atomicAdd(&nhit, 1u);
        if (qi < kS1Queue) {
            hitq[qi] = make_uint4(w, j, slot, 0u);
        } else {
            const uint32_t pos = atomicAdd(a.cnt + slot, 1u);
            if (pos < kSmallCap) a.cand[slot * kSmallCap + pos] = make_uint4(w, j, a.w1[j], 0u);
        }
    };
    // the level-Ls match of an id the 16-bit filter passed: binary search over the sorted distinct
    // prefixes (NONE: no target prefix)
    auto match = [&](uint32_t w) {
        const uint32_t pre = top_bits(w, a.Ls);
        uint32_t lo_s = 0, n_s = ntab;   // the first entry >= pre
        while (n_s) {
            const uint32_t half = n_s >> 1;
            if (tab[lo_s + half] < pre) { lo_s += half + 1; n_s -= half + 1; }
            else n_s = half;
        }
        return lo_s < ntab && tab[lo_s] == pre ? lo_s : DHT_NONE;
    };
    const uint32_t h_off = 32 - hb, tid4 = 4 * threadIdx.x;
    uint32_t tq[NQ > 0 ? NQ : 1];
#pragma unroll
    for (int i = 0; i < (NQ > 0 ? NQ : 1); ++i)
        tq[i] = (uint32_t)i < ntab ? __builtin_amdgcn_readfirstlane(tab[i]) : DHT_NONE;   // prefixes < 2^31
    for (uint32_t c0 = lo; c0 < hi; c0 += kRing * kS1Sub) {
#pragma unroll
        for (uint32_t r = 0; r < kRing; ++r) {
            const uint32_t sb = c0 + r * kS1Sub;
            if (sb < hi) {   // block-uniform
                const uint32_t v4[4] = {ring[r].x, ring[r].y, ring[r].z, ring[r].w};
                const uint32_t rem = hi - sb;
                if (NQ > 0) {
                    uint32_t m[4];
#pragma unroll
                    for (uint32_t f = 0; f < 4; ++f) {
                        const uint32_t pre = top_bits(v4[f], a.Ls);
                        m[f] = 0;
#pragma unroll
                        for (int i = 0; i < NQ; ++i) m[f] |= (uint32_t)(pre == tq[i]) << i;
                        m[f] = tid4 + f < rem ? m[f] : 0u;
                    }
                    if (__ballot((m[0] | m[1] | m[2] | m[3]) != 0)) {   // rare
#pragma unroll
                        for (uint32_t f = 0; f < 4; ++f) {
                            if (m[f]) emit(v4[f], sb + tid4 + f, (uint32_t)__ffs(m[f]) - 1);
                        }
                    }
                    ring[r] = load(sb + kRing * kS1Sub);
                    continue;
                }
                bool hit[4];
#pragma unroll
                for (uint32_t f = 0; f < 4; ++f) {
                    const uint32_t h = __builtin_amdgcn_ubfe(v4[f], h_off, hb);
                    hit[f] = ((b16[h >> 5] >> (h & 31)) & 1u) && tid4 + f < rem;
                }
                if (__ballot(hit[0] || hit[1] || hit[2] || hit[3])) {   // rare
                    // the 16-bit hits go to the LDS queue as they are (one LDS atomic per wave, no
                    // search in the stream: the dependent binary search per hit held the whole wave
                    // at q = 64, S1 18.6 us against 10.6 for the bare stream); the level-Ls match
                    // runs on the queue after the stream
#pragma unroll
                    for (uint32_t f = 0; f < 4; ++f) {
                        const uint64_t bal = __ballot(hit[f]);
                        if (!bal) continue;   // wave-uniform
                        uint32_t base = 0;
                        if (lane_id() == (uint32_t)__ffsll((long long)bal) - 1) base = atomicAdd(&nhit, (uint32_t)__popcll(bal));
                        base = __shfl((int)base, __ffsll((long long)bal) - 1);
                        if (hit[f]) {
                            const uint32_t qi = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)bal, base));
                            if (qi < kS1Queue) {
                                hitq[qi] = make_uint4(v4[f], sb + tid4 + f, DHT_NONE, 0u);
                            } else {   // past the queue (strongly clustered ids): matched and appended here
                                const uint32_t sl = match(v4[f]);
                                if (sl != DHT_NONE) {
                                    const uint32_t j = sb + tid4 + f;
                                    const uint32_t pos = atomicAdd(a.cnt + sl, 1u);
                                    if (pos < kSmallCap) a.cand[sl * kSmallCap + pos] = make_uint4(v4[f], j, a.w1[j], 0u);
                                }
                            }
                        }
                    }
                }
            }
            ring[r] = load(sb + kRing * kS1Sub);
        }
    }
    __syncthreads();
    // the queue to the buckets (the level-Ls match of a 16-bit hit first): word 1 and the slot
    // reservation in one round trip
    const uint32_t nq = nhit < kS1Queue ? nhit : kS1Queue;
    for (uint32_t i = threadIdx.x; i < nq; i += NT) {
        const uint4 e = hitq[i];
        const uint32_t sl = e.z != DHT_NONE ? e.z : match(e.x);
        if (sl == DHT_NONE) continue;
        const uint32_t w1 = a.w1[e.y];
        const uint32_t pos = atomicAdd(a.cnt + sl, 1u);
        if (pos < kSmallCap) a.cand[sl * kSmallCap + pos] = make_uint4(e.x, e.y, w1, 0u);
    }
}

// exact top-`want` of target qi (word 0 as streamed: t0; all five words: t) from the c
// candidates S[0, c) of one bucket, {w0, index, w1}: order by (w0 distance, w1 distance), the
// full key (planes) only on a double tie.  c <= 64: one candidate per lane, its rank counted
// against all of them; else a lane-distributed running list over chunks of 64.
__device__ void ks_answer(const F3Args& a, const uint4* S, uint32_t c, uint32_t qi, uint32_t t0, const uint32_t* t,
                          uint32_t want, uint32_t lane) {
    uint32_t* orow = a.out_idx + (uint64_t)qi * a.k;
    if (c <= 64) {
        const bool act = lane < c;
        const uint4 me = S[act ? lane : 0u];
        const uint32_t md = act ? me.x ^ t0 : DHT_NONE, m1 = act ? me.z ^ t[1] : DHT_NONE;
        bool tie;
        uint32_t rank = wave_rank64(md, m1, __builtin_amdgcn_readfirstlane(c), lane, &tie);
        if (__ballot(act && tie)) {   // a 64-bit distance tie (duplicate ids): the full key decides
            rank = 0;
            for (uint32_t o = 0; o < c; ++o) {
                const uint32_t xd = __builtin_amdgcn_readlane((int)md, (int)o);
                const uint32_t x1 = __builtin_amdgcn_readlane((int)m1, (int)o);
                const uint32_t xi = __builtin_amdgcn_readlane((int)me.y, (int)o);
                if (xd < md || (xd == md && x1 < m1)) ++rank;
                else if (xd == md && x1 == m1 && act && o != lane && id_less(xd, xi, md, me.y, a.planes, a.stride, t)) ++rank;
            }
        }
        if (act && rank < want) orow[rank] = map_out(me.y, a.gidx, a.base);
    } else {
        uint32_t ed = DHT_NONE, e1 = DHT_NONE, ei = DHT_NONE, cnt = 0;
        for (uint32_t c0 = 0; c0 < c; c0 += 64) {
            const bool v = c0 + lane < c;
            const uint4 x = v ? S[c0 + lane] : make_uint4(0u, DHT_NONE, 0u, 0u);
            const uint32_t xd = x.x ^ t0, xi = x.y, x1 = v ? x.z ^ t[1] : DHT_NONE;
            uint32_t wd = cnt == want ? __builtin_amdgcn_readlane((int)ed, want - 1) : DHT_NONE;
            uint32_t w1 = cnt == want ? __builtin_amdgcn_readlane((int)e1, want - 1) : DHT_NONE;
            uint32_t wi = cnt == want ? __builtin_amdgcn_readlane((int)ei, want - 1) : DHT_NONE;
            uint64_t cm = __ballot(v && (cnt < want || key2_less(xd, x1, xi, wd, w1, wi, a.planes, a.stride, t)));
            while (cm) {
                const uint32_t l = (uint32_t)__ffsll((long long)cm) - 1;
                cm &= cm - 1;
                const uint32_t cd = __builtin_amdgcn_readlane((int)xd, l), c1 = __builtin_amdgcn_readlane((int)x1, l);
                const uint32_t ci = __builtin_amdgcn_readlane((int)xi, l);
                if (cnt == want && !key2_less(cd, c1, ci, wd, w1, wi, a.planes, a.stride, t)) continue;
                const bool closer = lane < cnt && key2_less(ed, e1, ei, cd, c1, ci, a.planes, a.stride, t);
                const uint32_t pos = (uint32_t)__popcll(__ballot(closer));
                const uint32_t ud = __shfl_up(ed, 1), u1 = __shfl_up(e1, 1), ui = __shfl_up(ei, 1);
                if (lane == pos) { ed = cd; e1 = c1; ei = ci; }
                else if (lane > pos) { ed = ud; e1 = u1; ei = ui; }
                cnt = cnt + 1 < want ? cnt + 1 : want;
                wd = cnt == want ? __builtin_amdgcn_readlane((int)ed, want - 1) : DHT_NONE;
                w1 = cnt == want ? __builtin_amdgcn_readlane((int)e1, want - 1) : DHT_NONE;
                wi = cnt == want ? __builtin_amdgcn_readlane((int)ei, want - 1) : DHT_NONE;
            }
        }
        if (lane < want) orow[lane] = map_out(ei, a.gidx, a.base);
    }
    if (lane >= want && lane < a.k) orow[lane] = DHT_NONE;
    if (lane == 0) a.out_cnt[qi] = want;
}

// S2: workgroups [0, q) answer the distinct prefixes (workgroup s: prefix s, if s < ntab), the
// kSmallFbBlocks after them are the fallback list's scan roles
template <int K>
__global__ __launch_bounds__(kS2Threads) void k_s2_answer(F3Args a, SmallArgs sa, FbArgs f) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[scan::lds_words<kScanTargets>()];
    __shared__ uint32_t misc[4];
    __shared__ uint32_t s2_last;
    static_assert(scan::lds_words<kScanTargets>() >= 4 * kSmallCap + kSmallQ * (1 + DHT_W), "S2 LDS image");
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    const uint32_t want = a.n < a.k ? (uint32_t)a.n : a.k;
    if (blockIdx.x == 0 && threadIdx.x < kSmallQ) sa.cnt_next[threadIdx.x] = 0;   // the next call's counters
    if (blockIdx.x >= sa.q) {
        // ---- scan role r: the fallback list, from the final bucket counts (one round trip) ----
        const uint32_t r = blockIdx.x - sa.q;
        uint32_t* list = sa.fb + r * kSmallQ;   // this role's own copy (every role builds the same)
        if (threadIdx.x < 64) {
            const uint32_t ntab = sa.tab[kSmallQ];
            const uint32_t tb = sa.tab[lane], cb = sa.cnt[lane];
            const uint32_t pre = lane < sa.q ? top_bits(small_tw0(sa, lane), sa.Ls) : DHT_NONE;
            const bool short_b = lane < ntab && (cb < want || cb > kSmallCap);
            bool mine = false;   // my target's prefix is one of the short buckets
            for (uint64_t m = __ballot(short_b); m; m &= m - 1) {
                const uint32_t b = (uint32_t)__ffsll((long long)m) - 1;
                mine = mine || pre == (uint32_t)__builtin_amdgcn_readlane((int)tb, (int)b);
            }
            mine = mine && lane < sa.q;
            const uint64_t lm = __ballot(mine);
            if (mine) list[__popcll(lm & ((1ull << lane) - 1ull))] = lane;
            if (lane == 0) misc[0] = (uint32_t)__popcll(lm);
        }
        __syncthreads();   // wave 0's list stores are visible to the workgroup
        const uint32_t nfl = __builtin_amdgcn_readfirstlane(misc[0]);
        if (!nfl) return;   // uniform ids: nothing to scan (block-uniform)
        F3Args as = a;
        as.fb_list = list;
        fb_list_scan<K>(as, f, nfl, r, lds, &s2_last);
        return;
    }
    // ---- prefix workgroup s: one round trip for the table, the count, the targets' words and
    // the bucket (one slot per thread) ----
    const uint32_t s = blockIdx.x;
    uint4* S = reinterpret_cast<uint4*>(lds);
    uint32_t* tl = lds + 4 * kSmallCap;   // this prefix's targets
    uint32_t* tw = tl + kSmallQ;          // [DHT_W][kSmallQ] target words
    const uint32_t ntab = sa.tab[kSmallQ];
    const uint32_t pre_s = sa.tab[s < kSmallQ ? s : 0u];
    const uint32_t c = sa.cnt[s < kSmallQ ? s : 0u];
    const uint32_t t0s = threadIdx.x < 64 && lane < sa.q ? small_tw0(sa, lane) : 0u;
    const uint4 e = sa.cand[(s < kSmallQ ? s : 0u) * kSmallCap + (threadIdx.x < kSmallCap ? threadIdx.x : 0u)];
    const uint32_t tj = threadIdx.x / kSmallQ, tq = threadIdx.x % kSmallQ;
    const uint32_t twv = tj < DHT_W && tq < sa.q ? sa.tp[(uint64_t)tj * sa.ts + tq] : 0u;
    if (s >= ntab) return;   // block-uniform
    if (threadIdx.x < 64) {   // this prefix's targets
        const bool v = lane < sa.q && top_bits(t0s, sa.Ls) == pre_s;
        const uint64_t m = __ballot(v);
        if (v) tl[__popcll(m & ((1ull << lane) - 1ull))] = lane;
        if (lane == 0) misc[0] = (uint32_t)__popcll(m);
    }
    if (threadIdx.x < c && threadIdx.x < kSmallCap) S[threadIdx.x] = e;
    if (tj < DHT_W) tw[tj * kSmallQ + tq] = twv;
    __syncthreads();
    if (c < want || c > kSmallCap) return;   // the scan roles answer this prefix's targets
    const uint32_t ntl = misc[0];
    for (uint32_t i = wv; i < ntl; i += scan::WAVES) {
        const uint32_t qi = __builtin_amdgcn_readfirstlane(tl[i]);
        uint32_t t[DHT_W];
#pragma unroll
        for (int j = 0; j < DHT_W; ++j) t[j] = __builtin_amdgcn_readfirstlane(tw[j * kSmallQ + qi]);
        const uint32_t t0 = sa.shift ? (t[0] << sa.shift) | (t[1] >> (32 - sa.shift)) : t[0];
        ks_answer(a, S, c, qi, t0, t, want, lane);
    }
}

}  // namespace

// F4 scratch for a list scan: done counters | split records
static size_t list_scan_bytes(uint32_t k) { return al256((size_t)kFbBlocks * 4) + al256((size_t)kFbBlocks * kFbGroup * k * 24); }

bool small_supported(uint64_t n, uint32_t q, uint32_t k) {
    return q >= 1 && q <= kSmallQ && k >= 1 && k <= DHTGPU_MAX_K_DEV && n >= 1 && n < (1ull << 31);
}

// cnt[2][kSmallQ] | tab | fb[kSmallFbBlocks][kSmallQ] | F4 scratch (list_scan_bytes(32): done
// counters first) | cand
size_t small_bytes() {
    return al256((size_t)2 * kSmallQ * 4) + al256((size_t)(kSmallQ + 1) * 4) + al256((size_t)kSmallFbBlocks * kSmallQ * 4) +
           list_scan_bytes(DHTGPU_MAX_K_DEV) + (size_t)kSmallQ * kSmallCap * 16;
}

hipError_t launch_small_topk(const BatchCall& c, void* sws, uint32_t parity, hipStream_t s) {
    uint8_t* w = static_cast<uint8_t*>(sws);
    SmallArgs a{};
    a.cnt = reinterpret_cast<uint32_t*>(w) + (parity & 1u) * kSmallQ;
    a.cnt_next = reinterpret_cast<uint32_t*>(w) + ((parity & 1u) ^ 1u) * kSmallQ;
    uint8_t* x = w + al256((size_t)2 * kSmallQ * 4);
    a.tab = reinterpret_cast<uint32_t*>(x);
    x += al256((size_t)(kSmallQ + 1) * 4);
    a.fb = reinterpret_cast<uint32_t*>(x);
    x += al256((size_t)kSmallFbBlocks * kSmallQ * 4);
    void* fb_scratch = x;
    x += list_scan_bytes(DHTGPU_MAX_K_DEV);
    a.cand = reinterpret_cast<uint4*>(x);
    const uint64_t n = c.n;
    // level: the deepest with >= 4k ids per subtree on uniform ids (K6's rule), at most 31
    a.Ls = 0;
    while (a.Ls < 31 && (n >> (a.Ls + 1)) >= 4ull * c.k) ++a.Ls;
    a.w0 = c.w0s ? c.w0s : c.planes;
    a.w1 = c.planes + c.stride;
    a.n = n;
    const uint64_t lim = (c.w0s ? c.stride : 5 * c.stride) - 4;
    a.lim = (uint32_t)(lim < 0xFFFFFFF0ull ? lim : 0xFFFFFFF0ull);
    a.tp = c.tp;
    a.ts = c.ts;
    a.q = c.q;
    a.shift = c.w0s ? c.skip : 0u;
    // S1: two 512-thread workgroups per CU (measured against 1 x 1024, 2 x 1024 and 4 x 256:
    // 2 x 1024 -- twice the loads in flight -- is 35 % slower, the others equal or slower),
    // ranges in whole sub-steps
    constexpr uint32_t nt = 512, bpc = 2;
    const uint64_t g = (uint64_t)(c.num_cus > 0 ? c.num_cus : 256) * bpc;
    const uint64_t sub = 4ull * nt;
    const uint64_t subs = (n + sub - 1) / sub;
    a.per_blk = ((subs + g - 1) / g) * sub;
    const uint32_t nblk = (uint32_t)((n + a.per_blk - 1) / a.per_blk);
    F3Args f{};
    f.planes = c.planes;
    f.stride = c.stride;
    f.n = n;
    f.tp = c.tp;
    f.ts = c.ts;
    f.k = c.k;
    f.gidx = c.gidx;
    f.base = c.base;
    f.out_idx = c.out_idx;
    f.out_cnt = c.out_cnt;
    hipEvent_t* ev = c.ev;
    auto go = [&](int i, auto kern, dim3 gr, dim3 b, size_t l, auto... args) {
        if (ev) hipExtLaunchKernelGGL(kern, gr, b, (uint32_t)l, s, ev[2 * i], ev[2 * i + 1], 0, args...);
        else kern<<<gr, b, l, s>>>(args...);
    };
    if (ev) {   // no F1 here: an empty pair
        (void)hipEventRecord(ev[0], s);
        (void)hipEventRecord(ev[1], s);
    }
    if (c.q == 1) go(1, k_s1_filter<nt, 1>, dim3(nblk), dim3(nt), 0, a);
    else go(1, k_s1_filter<nt, 0>, dim3(nblk), dim3(nt), 0, a);
    // S2: the prefix workgroups and the fallback list's scan roles in one launch
    const FbArgs fa{reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(fb_scratch) + al256((size_t)kFbBlocks * 4)),
                    static_cast<uint32_t*>(fb_scratch), kSmallFbBlocks, 0u, nullptr};
    const dim3 g2(c.q + kSmallFbBlocks), b2(kS2Threads);
    if (c.k <= 8) go(2, k_s2_answer<8>, g2, b2, 0, f, a, fa);
    else if (c.k <= 16) go(2, k_s2_answer<16>, g2, b2, 0, f, a, fa);
    else go(2, k_s2_answer<32>, g2, b2, 0, f, a, fa);
    if (ev) {   // no separate fallback kernel: an empty pair
        (void)hipEventRecord(ev[6], s);
        (void)hipEventRecord(ev[7], s);
    }
    return hipGetLastError();
}

}  // namespace dhtgpu
