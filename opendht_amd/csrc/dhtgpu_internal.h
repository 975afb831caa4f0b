// dhtgpu_internal.h -- host-side launch entry points shared between the kernel
// translation units and the C ABI (api.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

namespace dhtgpu {

// hipFuncSetAttribute (e.g. MaxDynamicSharedMemorySize) applies to the device current on the
// calling thread: set() runs once per device id below kMaxDevices, from whichever thread gets
// there first, and on every call for a device id past the table.  Returns hipGetDevice's error.
constexpr int kMaxDevices = 64;
inline hipError_t per_device_once(std::once_flag* flags, void (*set)()) {
    int dev = 0;
    const hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev >= 0 && dev < kMaxDevices) std::call_once(flags[dev], set);
    else set();
    return hipSuccess;
}

// ID-plane geometry: planes are padded to a multiple of kTile ids so that the scan
// kernel can stream whole tiles without bounds checks.
constexpr uint32_t kTile = 4096;
constexpr uint32_t kScanWaves = 8;       // waves per scan workgroup
constexpr uint32_t kScanTargets = 16;    // targets held (wave-uniform) per wave
constexpr uint32_t kLdsBytes = 160 * 1024;   // LDS per CU (gfx950)

inline uint64_t pad_ids(uint64_t n) { return ((n + kTile - 1) / kTile) * kTile; }

// keys.hip
hipError_t launch_gen(uint64_t seed, uint64_t start, uint64_t n, uint32_t* planes,
                      uint64_t stride, hipStream_t s);
hipError_t launch_pack(const uint8_t* ids20, uint64_t n, uint32_t* planes, uint64_t stride,
                       hipStream_t s);
hipError_t launch_unpack(const uint32_t* planes, uint64_t stride, uint64_t first, uint64_t n,
                         uint8_t* out20, hipStream_t s);
hipError_t launch_fill(uint32_t* p, uint64_t n, uint32_t v, hipStream_t s);
// sets *d_flag to 1 if ids are NOT strictly ascending (unsorted or duplicated)
hipError_t launch_check_sorted(const uint32_t* planes, uint64_t stride, uint64_t n,
                               uint32_t* d_flag, hipStream_t s);

// ids whose top pbits bits equal pval, compacted in index order (out == nullptr: count
// only).  scratch: select_scratch_words(n) u32; *d_total = number selected; gidx[j] =
// gbase + original index of the j-th selected id (nullable).
hipError_t launch_select_prefix(const uint32_t* planes, uint64_t stride, uint64_t n, uint32_t pbits,
                                uint32_t pval, uint32_t* scratch, unsigned long long* d_total,
                                uint32_t* out, uint64_t out_stride, uint32_t* gidx, uint64_t gbase,
                                hipStream_t s);
uint64_t select_scratch_words(uint64_t n);

// scan.hip
struct ScanPlan {
    uint32_t blocks_x;   // target groups
    uint32_t splits;     // id-range splits
    uint64_t split_len;  // ids per split (multiple of kTile)
};
// splits are capped so that K3 can stage splits * k records (24 B) of a target in LDS
ScanPlan plan_scan(uint64_t n, uint32_t q, uint32_t k, int num_cus);
// final form: out_idx/out_cnt mapped through gidx (nullable) or offset by idx_base;
// split record form (out_rec != nullptr, internal to the K1 split merge): full 24-B records
// rec[((split * q) + qi) * k + r] * 6 = {w0..w4, idx + idx_base}
hipError_t launch_scan(const uint32_t* ids, uint64_t is, uint64_t n, const ScanPlan& p,
                       const uint32_t* tp, uint64_t ts, uint32_t q, uint32_t k,
                       uint32_t* out_idx, uint32_t* out_cnt, uint32_t* out_rec,
                       const uint32_t* gidx, uint32_t idx_base, hipStream_t s);
hipError_t launch_merge(const uint32_t* rec, uint32_t lists, uint32_t q, uint32_t kin,
                        const uint32_t* tp, uint64_t ts, uint32_t k, uint32_t* out_idx,
                        uint32_t* out_cnt, hipStream_t s);

// valid idx[i] -> gidx ? gidx[idx[i]] : idx[i] + base
hipError_t launch_map_idx(uint32_t* idx, uint64_t m, const uint32_t* gidx, uint32_t base, hipStream_t s);
// compact candidate records (the public record form): rec[i * 3 ..] = {w0, w1, global index} of
// local index idx[i] (all DHT_NONE for DHT_NONE); the global index is gidx[idx[i]] when gidx !=
// nullptr, else idx[i] + base
hipError_t launch_rec3(const uint32_t* idx, uint64_t m, const uint32_t* planes, uint64_t stride, uint32_t base,
                       const uint32_t* gidx, uint32_t* rec, hipStream_t s);
// K3 over compact records (lists <= 64, kin <= 32): rows whose candidates tie on their first 64
// bits across lists are appended to ties = {count, rows[tie_cap]} (zeroed here; nullable)
hipError_t launch_merge3(const uint32_t* rec, uint32_t lists, uint32_t q, uint32_t kin, const uint32_t* tp,
                         uint64_t ts, uint32_t k, uint32_t* out_idx, uint32_t* out_cnt, uint32_t* ties,
                         uint32_t tie_cap, hipStream_t s);
// words 2..4 of this set's candidates (rec: its own compact records, q x k) in the listed rows
// (+ row_base) or every row (ties == nullptr); gmap (nullable, ascending) maps global -> local
hipError_t launch_tie_words(const uint32_t* rec, uint32_t q, uint32_t k, const uint32_t* ties, uint32_t tie_cap,
                            uint32_t row_base, const uint32_t* planes, uint64_t stride, uint64_t n,
                            const uint32_t* gmap, uint32_t base, uint32_t* words, hipStream_t s);
// the listed rows (every row when ties == nullptr) merged again on the full keys
hipError_t launch_merge_full(const uint32_t* rec, const uint32_t* words, uint32_t lists, uint32_t q, uint32_t kin,
                             const uint32_t* tp, uint64_t ts, uint32_t k, const uint32_t* ties, uint32_t tie_cap,
                             uint32_t* out_idx, uint32_t* out_cnt, hipStream_t s);

// table.hip
hipError_t launch_find_closest(uint32_t nb, const uint32_t* fp, const uint32_t* off,
                               const uint32_t* gcnt, const uint32_t* np, uint64_t ns,
                               const uint8_t* good, const uint32_t* tp, uint64_t ts, uint32_t q,
                               uint32_t count, uint32_t* out_idx, uint32_t* out_cnt,
                               hipStream_t s);
hipError_t launch_classify(const uint32_t* planes, uint64_t stride, uint64_t n, uint32_t nb,
                           const uint32_t* fp, const uint32_t* myid, uint8_t* out_bucket,
                           unsigned long long* hist, hipStream_t s);
// perm (nullable): sorted position -> caller index (accept and the output use caller indices)
hipError_t launch_cached(const uint32_t* planes, uint64_t stride, uint64_t n, const uint32_t* perm,
                         const uint8_t* accept, const uint32_t* tp, uint64_t ts, uint32_t q,
                         uint32_t count, uint32_t* out_idx, uint32_t* out_cnt, hipStream_t s);

// index.hip: K4 bucket index (counting sort by the top B bits) + K5 trie-descent k-NN
uint32_t index_bits(uint64_t n);
size_t index_bytes(uint64_t n, uint32_t B);
// ev (nullable): 5 events recorded before/between/after the build's kernels
hipError_t launch_index_build(const uint32_t* planes, uint64_t stride, uint64_t n, uint32_t B, void* ws,
                              hipStream_t s, hipEvent_t* ev = nullptr);
hipError_t launch_index_query(const void* ws, uint64_t n, uint32_t B, const uint32_t* planes, uint64_t stride,
                              const uint32_t* tp, uint64_t ts, uint32_t q, uint32_t k, uint32_t* out_idx,
                              uint32_t* out_cnt, hipStream_t s);

// batch.hip: K6 per-batch target-prefix filter + exact top-k (no persistent index).
// n: ids of the largest sub-partition (or of the set); q_plan: the targets one sub-partition
// is planned for (q / nsub); nsub: sub-partitions served by the call (1: the set itself).
bool batch_supported(uint64_t n, uint32_t q_plan, uint32_t k, int num_cus, uint32_t nsub = 1, uint32_t pf = 0);
size_t batch_bytes(uint64_t n, uint32_t q, uint32_t q_plan, uint32_t k, int num_cus, uint32_t nsub = 1, uint32_t pf = 0);
// leading workspace bytes that must be zero before a call (the call leaves them zero)
size_t batch_clean_bytes(uint64_t n, uint32_t q_plan, uint32_t k, int num_cus, uint32_t nsub = 1, uint32_t pf = 0);
// offset of the shared counters in the workspace head: their words 0..3 (the call's statistics, read by
// batch_read_stats) stay set after a call, so a head laid out with them elsewhere is zeroed again
size_t batch_ctr_offset(uint64_t n, uint32_t q_plan, uint32_t k, int num_cus, uint32_t nsub = 1, uint32_t pf = 0);
// stats4 = {fallback targets, survivors, wave-path targets, 0} of the last call on workspace ws
// (synchronises s)
hipError_t batch_read_stats(const void* ws, uint64_t n, uint32_t q, uint32_t q_plan, uint32_t k, int num_cus,
                            uint32_t* stats4, hipStream_t s, uint32_t nsub = 1, uint32_t pf = 0);
// pf (plan flags): kPlanCells -- the sub-partitions' level-cell_level() id counts (launch_cell_counts)
// are available, which lets the plan mark one level finer with sibling marking (BatchCall::cells);
// kPlanSorted -- the sub-partitions are sorted by prefix (one bucket set per partition, survivors
// of an F2 range clustered in whole cells; BatchCall::sorted)
constexpr uint32_t kPlanCells = 1u, kPlanSorted = 2u;
uint32_t cell_level();
// u8 counts (saturated) of the n ids of a shifted word-0 plane per top-cell_level()-bit prefix;
// scratch: 4 << cell_level() bytes
hipError_t launch_cell_counts(const uint32_t* w0s, uint64_t n, uint32_t* scratch, uint8_t* out, hipStream_t s);
// spans[j] (device, 32 words) = the most level-cell_level() cells that 2^j consecutive ids of a
// prefix-sorted shifted word-0 plane span (K6's F2 window bound)
hipError_t launch_cell_spans(const uint32_t* w0s, uint64_t n, uint32_t* spans, hipStream_t s);
// prefix shards: out[i] = planes word 0 << shift | word 1 >> (32 - shift), i < stride
hipError_t launch_shift_w0(const uint32_t* planes, uint64_t stride, uint32_t shift, uint32_t* out, hipStream_t s);
// One prefix sub-partition of a K6 call's id set (host view; see batch.hip SubDesc).
struct SubSpec {
    const uint32_t* planes; const uint32_t* w0s;   // unshifted planes; shifted word-0 plane (nullable)
    uint64_t stride, n;
    const uint32_t* gidx; uint32_t base;           // result index map (nullable) or offset
};

constexpr uint32_t kHandleMark = 0x80000000u;   // sets hold < 2^31 ids (batch_supported)
// DHTGPU_DBG bits the library honours (dhtgpu_ctx::dbg): 256 = phase stamps, 2^23 = K6 for
// small batches.  Diagnostics only -- no bit changes a result (tests/test_abi.py pins the mask).
constexpr uint32_t kDbgAllowed = 256u | (1u << 23);
// One sub-partition in handle space: handles [off, off + n) name its ids in its (prefix-sorted) order.
struct HandleSub {
    uint64_t n;
    const uint32_t* map;    // sub-local -> context-local
    const uint32_t* gmap;   // sub-local -> global stream index (nullable: no global map)
    uint32_t off, pad;
};
// out[i] = the index handle h[i] names: gmap (global) or map + base; DHT_NONE stays
hipError_t launch_handles_to_idx(const HandleSub* tab, uint32_t nsub, const uint32_t* h, uint64_t m, uint32_t* out,
                                 bool global, uint32_t base, hipStream_t s);
// idx[i] (context-local) -> its handle in place: hinv[idx[i]] (DHT_NONE stays)
hipError_t launch_idx_to_handles(const uint32_t* hinv, uint32_t* idx, uint64_t m, hipStream_t s);
// hinv[map[j]] = off + j, j < m: the context-local -> handle map of one sub-partition
hipError_t launch_handle_inverse(const uint32_t* map, uint64_t m, uint32_t off, uint32_t* hinv, hipStream_t s);

struct BatchCall {
    void* ws;                              // workspace (batch_bytes), head zero (batch_clean_bytes)
    const uint32_t* planes; uint64_t stride; uint64_t n;   // the id set (unshifted word planes)
    const uint32_t* tp; uint64_t ts;       // target planes
    uint32_t q;                            // targets F1 reads (the whole batch)
    uint32_t q_plan;                       // targets the plan is sized for
    uint32_t k;
    const SubSpec* subs; uint32_t nsub;    // prefix sub-partitions (nsub 0: the set planes/n/w0s/gidx/base)
    uint32_t sub_shift, sub_bits;          // a target's sub-partition: its bits [sub_shift, +sub_bits)
    uint64_t* desc_sig;                    // the workspace's uploaded sub-partition descriptors (signature)
    uint32_t skip; const uint32_t* w0s;    // w0s = 32 id bits from bit `skip` (every id shares its top skip bits)
    uint32_t pval;                         // skip > 0: the shared top bits' value (of the shard; sub-partitions
                                           // append their index: sub_bits more)
    const uint8_t* cells;                  // nullable: [nsub][1 << cell_level()] cell counts of the sub-partitions
    const uint32_t* spans;                 // nullable, HOST: [nsub][32] cell spans of the (prefix-sorted) sub-partitions
    uint32_t sorted;                       // the sub-partitions are sorted by prefix (spans then bound F2's windows)
    const uint32_t* gidx; uint32_t base;   // result index map (nullable) or offset
    uint32_t* out_idx; uint32_t* out_cnt;  // rows of the ORIGINAL target indices
    // record form (nullable): every writer of a result row (F3, the wave paths, F4's scan and
    // merge) stores the row's compact records instead of its indices; rec_gidx / rec_base map the
    // context-local index to the record's global index
    uint32_t* out_rec; const uint32_t* rec_gidx; uint32_t rec_base;
    // sub-partition handles (nsub > 1, dhtgpu_set_sub_handles): every sub-partition's results are
    // its base + sub-local index (SubSpec gidx null, base = the sub-partition's offset); rows F4
    // answers from the whole set carry context-local index | kHandleMark (gidx null, base =
    // kHandleMark) and a pass after F4 turns them into handles through htab
    uint32_t handles; const HandleSub* htab;
    const uint32_t* hinv;                  // handles: context-local index -> handle
    int num_cus;
    uint32_t dbg;                          // DHTGPU_DBG & kDbgAllowed (0 in production)
    const volatile uint32_t* fb_hint;      // nullable: the slot's last fallback-list length (mapped host memory)
    uint32_t* fb_hint_dev;                 // its device address (F4 writes it)
    unsigned long long* stamps;            // dbg & 256: phase stamps [2 * 8192 * 16]
    hipEvent_t* ev;                        // nullable: 8 events around F1..F4
};
hipError_t launch_batch_topk(const BatchCall& c, hipStream_t s);
// KS (batch.hip): batches of at most 64 targets -- one pass over word 0 and one workgroup per
// distinct target prefix (K6's results).  sws: small_bytes(), zero before its first use (left
// zero); parity: alternates between consecutive calls on one workspace (two counter sets);
// ev (nullable) gets S1 as F2's pair and S2 as F3's, F1 / F4 pairs empty.
bool small_supported(uint64_t n, uint32_t q, uint32_t k);
size_t small_bytes();
hipError_t launch_small_topk(const BatchCall& c, void* sws, uint32_t parity, hipStream_t s);

// sort.hip: lexicographic sort of an id set (stable LSD radix over the 160-bit keys).
// out_planes (out_stride >= n) = the ids in ascending InfoHash order, perm[j] = the input index
// of sorted id j; *unique = 0 when two ids are equal.  Synchronises s.
size_t sort_scratch_bytes(uint64_t n);
hipError_t launch_sort_ids(const uint32_t* planes, uint64_t stride, uint64_t n, uint32_t* out_planes, uint64_t out_stride,
                           uint32_t* perm, void* scratch, int* unique, hipStream_t s);

// search.hip: batched Dht::Search::insertNode; RoutingTable::depth + InfoHash::lowbit per bucket
hipError_t launch_search_insert(const uint32_t* planes, uint64_t stride, const uint8_t* st, const uint32_t* tp,
                                uint64_t ts, uint32_t q, uint32_t cap, uint32_t* list_node, uint8_t* list_flags,
                                uint32_t* list_len, uint8_t* expired, const uint64_t* ins_off, const uint32_t* ins_node,
                                const uint8_t* ins_token, uint8_t* ins_added, uint32_t* overflow, hipStream_t s);
hipError_t launch_table_stats(const uint32_t* fp, uint32_t nb, int32_t* out_lowbit, uint32_t* out_depth, hipStream_t s);

// wire.hip: NetworkEngine::bufferNodes / deserializeNodes (compact node records)
hipError_t launch_wire_encode(const uint32_t* planes, uint64_t stride, const uint8_t* tail, uint32_t alen,
                              const uint32_t* tp, uint64_t ts, uint32_t q, const uint32_t* cand, uint32_t c,
                              uint8_t* out, uint32_t* out_len, hipStream_t s);
hipError_t launch_wire_decode(const uint8_t* blob, const uint64_t* msg_off, const uint32_t* rec_start, uint32_t m,
                              uint32_t nrec, uint32_t af, const uint8_t* myid, const uint8_t* from_af,
                              const uint8_t* from_addr, uint8_t* out_ids, uint8_t* out_tail, uint8_t* out_status,
                              hipStream_t s);

// crawl.hip: crawl-replay model (iterative searches over implicit routing tables)
uint32_t search_list_cap();
// sorts the K4 index buckets (index workspace, n ids, B bits) by (w0, index) into out[n]
hipError_t launch_net_sort(const void* index_ws, uint64_t n, uint32_t B, uint2* out, hipStream_t s);
hipError_t launch_search(const uint32_t* planes, uint64_t stride, const uint2* sorted, const void* index_ws,
                         uint64_t n, uint32_t B, const uint8_t* dead, uint64_t seed, const uint32_t* tp, uint64_t ts,
                         uint32_t q, const uint32_t* searchers, uint32_t max_rounds, uint32_t alpha, uint32_t* out_idx,
                         uint8_t* out_flags, uint32_t* out_len, uint32_t* out_rounds, uint32_t* out_queries,
                         hipStream_t s);

}  // namespace dhtgpu
