/*
 * dhtgpu.h -- C ABI of libdhtgpu, the MI355X (gfx950) engine for OpenDHT's
 * XOR-closest-node lookup.
 *
 * Plain C: pointers and sizes only, integer status codes, no exceptions and no
 * callbacks cross this boundary.  Node IDs cross it as 20-byte big-endian
 * arrays, byte-for-byte dht::InfoHash::data() (include/opendht/infohash.h:263,
 * HASH_LEN = 20 at :267).  Results are INDICES into the ID array the caller
 * uploaded last; the caller maps them back to its Sp<Node>.
 *
 * Reference interfaces replaced (paths relative to the OpenDHT tree):
 *   dhtgpu_topk            std::partial_sort(ids, k, InfoHash::xorCmp)          (SURVEY §8 a12,
 *                          include/opendht/infohash.h:179-194) -- the flat exact k-NN
 *                          behind findClosestNodesBatch(targets[], k)
 *   dhtgpu_find_closest    RoutingTable::findClosestNodes(id, now, count)
 *                          (include/opendht/routing_table.h:56, src/routing_table.cpp:110-150)
 *   dhtgpu_cached_nodes    NodeCache::getCachedNodes(id, af, count)
 *                          (include/opendht/node_cache.h:31, src/node_cache.cpp:42-74)
 *   dhtgpu_classify        RoutingTable::findBucket (src/routing_table.cpp:153-166) +
 *                          InfoHash::commonBits (include/opendht/infohash.h:154-176)
 *   dhtgpu_table_depth     RoutingTable::depth (src/routing_table.cpp:100-107)
 *   dhtgpu_buffer_nodes    NetworkEngine::bufferNodes (src/network_engine.cpp:1003-1032)
 *   dhtgpu_deserialize_nodes  NetworkEngine::deserializeNodes (src/network_engine.cpp:849-887)
 *   dhtgpu_search_batch    Dht::Search node refresh: Search::insertNode (src/search.h:636-722)
 *                          driven by find_node rounds (crawl replay, tools/dhtscanner.cpp)
 *   dhtgpu_search_insert   Search::insertNode (src/search.h:636-722) itself, batched over searches
 *   dhtgpu_table_stats     InfoHash::lowbit + RoutingTable::depth of every bucket, on the device
 *   dhtgpu_cache_set/_nodes  NodeCache's map (node_cache.h:43) sorted on the device + getCachedNodes
 *
 * Threading (mirrors the reference, src/dhtrunner.cpp:115-150): one context per
 * thread, or external locking; every host-pointer call is synchronous.
 * The *_dev entry points take device pointers and a hipStream_t (void*), are
 * stream-ordered and do not synchronise (for batch/bench/multi-GPU use).  A stream passed
 * to a context must outlive it: a later call that moves a workspace slot to another stream
 * records an event on the slot's previous stream, and dhtgpu_ctx_destroy synchronises the
 * streams the slots last used.
 */
#ifndef DHTGPU_H
#define DHTGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DHTGPU_HASH_LEN 20u
#define DHTGPU_WORDS 5u              /* a 160-bit id = 5 big-endian u32 words */
#define DHTGPU_MAX_K 32u             /* largest k / count served */
#define DHTGPU_NONE 0xFFFFFFFFu      /* index padding for short results */
#define DHTGPU_REC_WORDS 3u          /* candidate record: {w0, w1, global index} (12 B) */
#define DHTGPU_MAX_LISTS 64u         /* candidate lists one merge takes (ranks of a sharded lookup) */

enum {
    DHTGPU_OK = 0,
    DHTGPU_EINVAL = -1,              /* bad argument (null pointer, k == 0 or > DHTGPU_MAX_K, ...) */
    DHTGPU_ENOMEM = -2,              /* device allocation failed */
    DHTGPU_EDEVICE = -3,             /* HIP runtime / kernel launch error */
    DHTGPU_ENOIDS = -4,              /* no id set uploaded */
    DHTGPU_EUNSORTED = -5,           /* cached_nodes / cache_set: the id set holds duplicate ids */
    DHTGPU_ERANGE = -6               /* size out of range (e.g. more than 2^32-1 ids) */
};

typedef struct dhtgpu_ctx dhtgpu_ctx;

/* ---- context ---------------------------------------------------------------- */
int dhtgpu_ctx_create(int device, dhtgpu_ctx** out);
void dhtgpu_ctx_destroy(dhtgpu_ctx* ctx);
const char* dhtgpu_strerror(int code);
int dhtgpu_device_count(int* out);
/* Device stream used by the synchronous calls (hipStream_t as void*). */
void* dhtgpu_ctx_stream(dhtgpu_ctx* ctx);

/* ---- the id set (the device mirror of the routing table / node cache) --------- */
/* Upload n ids (20-byte big-endian each).  The device keeps them as five u32
 * word planes (struct of arrays).  Also records whether the set is sorted and
 * unique (needed by dhtgpu_cached_nodes). */
int dhtgpu_set_ids(dhtgpu_ctx* ctx, const uint8_t* ids20_be, uint64_t n);
/* Generate n synthetic ids directly in HBM: splitmix64 stream,
 * id i = BE(x(3g)) || BE(x(3g+1)) || top4(BE(x(3g+2))), g = start + i. */
int dhtgpu_gen_ids(dhtgpu_ctx* ctx, uint64_t seed, uint64_t start, uint64_t n);
/* Multi-GPU prefix routing: generate the stream [start, start+n) and keep
 * only the ids whose top pbits bits equal pval, in stream order.  Every result index of
 * the context then refers to the GLOBAL stream (start + i); get_ids/classify use shard
 * order.  pbits <= 16. */
int dhtgpu_gen_ids_prefix(dhtgpu_ctx* ctx, uint64_t seed, uint64_t start, uint64_t n, uint32_t pbits,
                          uint32_t pval);
/* Prefix shard contexts (dhtgpu_gen_ids_prefix): on != 0 (the default) makes every
 * lookup return indices into the global stream; on == 0 returns shard-local indices
 * (positions in get_ids order) -- the handle a rank that owns its shard's node table
 * keeps, without the per-result gather through the index map. */
int dhtgpu_set_global_indices(dhtgpu_ctx* ctx, int on);
/* Sets too large for one K6 plan (e.g. a 2^27-id shard) are answered over prefix
 * sub-partitions, compacted copies in id order.  on != 0 makes such calls return
 * sub-partition handles instead of indices: handle = the sub-partition's offset + the id's
 * position in it (one handle per id, in [0, n)), saving the per-result read of the index map
 * (10 us of the cfg-3 shard's 0.15 ms).  Record form (out_rec) is unaffected.
 * dhtgpu_sub_handles_active tells whether a call of q targets at k returns handles (only
 * sub-partitioned calls do); dhtgpu_handles_to_indices_dev maps m handles to the indices the
 * call would have returned (global stream indices per dhtgpu_set_global_indices, else
 * context-local + idx_base); DHTGPU_NONE stays.  The handle space is the one the last
 * sub-partitioned call used (it changes with the id set). */
int dhtgpu_set_sub_handles(dhtgpu_ctx* ctx, int on);
int dhtgpu_sub_handles_active(dhtgpu_ctx* ctx, uint32_t q, uint32_t k);
int dhtgpu_handles_to_indices_dev(dhtgpu_ctx* ctx, const uint32_t* handles, uint64_t m, uint32_t* out_idx,
                                  uint32_t idx_base, void* stream);
uint64_t dhtgpu_num_ids(const dhtgpu_ctx* ctx);
/* Read back ids [first, first+n) as 20-byte big-endian. */
int dhtgpu_get_ids(dhtgpu_ctx* ctx, uint64_t first, uint64_t n, uint8_t* out20_be);
/* Device view of the planes: word j of id i is planes[j*stride + i]. */
int dhtgpu_ids_dev(dhtgpu_ctx* ctx, const uint32_t** planes, uint64_t* stride);

/* ---- K1: flat exact top-k (std::partial_sort over xorCmp) ------------------- */
/* For each of q targets, the k ids closest by XOR distance, ascending; equal ids
 * (not produced by OpenDHT) tie-break by lower index.  out_idx[q*k] (DHTGPU_NONE
 * padded), out_cnt[q] = min(k, n).  1 <= k <= DHTGPU_MAX_K. */
int dhtgpu_topk(dhtgpu_ctx* ctx, const uint8_t* targets20_be, uint32_t q, uint32_t k,
                uint32_t* out_idx, uint32_t* out_cnt);

/* Device form.  Targets as word planes (t_planes[j*t_stride + i]).  Writes either
 * the final indices (out_idx/out_cnt, offset by idx_base) or, if out_rec != NULL,
 * candidate records for a cross-shard merge: out_rec[(qi*k + r)*3 + {w0, w1, idx}] = the
 * first two words of the r-th closest id and its index offset by idx_base (global index
 * of a prefix shard context), ascending in XOR distance; all DHTGPU_NONE for empty slots. */
int dhtgpu_topk_dev(dhtgpu_ctx* ctx, const uint32_t* t_planes, uint64_t t_stride, uint32_t q,
                    uint32_t k, uint32_t* out_idx, uint32_t* out_cnt, uint32_t* out_rec,
                    uint32_t idx_base, void* stream);

/* K3: merge `lists` (<= DHTGPU_MAX_LISTS) candidate-record lists per target,
 * rec[((l*q + qi)*k_in + r)*3] as written by the record forms (each list ascending in XOR
 * distance, DHTGPU_NONE records after its valid ones), into the final top-k.  Used after the
 * RCCL all-gather of per-GPU shards.  The records carry 64 bits of each id: a row where two
 * lists' candidates agree on them (two ids sharing their first 64 bits -- never among the
 * candidates of hash-distributed ids -- or one id sent by two lists) is answered provisionally
 * and appended to ties = {count, rows[tie_cap]} (device, zeroed by this call; may be NULL only
 * when lists == 1); such rows are settled by the second exchange: dhtgpu_tie_words_dev on every
 * shard, then dhtgpu_merge_ties_dev.  Records equal in all five words and the index are one
 * candidate; different ids with equal indices are both kept. */
int dhtgpu_merge_dev(const uint32_t* rec, uint32_t lists, uint32_t q, uint32_t k_in,
                     const uint32_t* t_planes, uint64_t t_stride, uint32_t k,
                     uint32_t* out_idx, uint32_t* out_cnt, uint32_t* ties, uint32_t tie_cap, void* stream);
/* The second exchange's payload from one shard: words 2..4 of this context's candidates
 * (rec: its own q x k records from a record-form call with idx_base) in the rows listed by
 * ties (each row + row_base: the row's place in rec when the merge took a slice of the
 * targets), out_words[(slot*k + r)*3 + {w2, w3, w4}] for slot < min(count, tie_cap); ties ==
 * NULL: every row (slot = row), the fallback when count > tie_cap. */
int dhtgpu_tie_words_dev(dhtgpu_ctx* ctx, const uint32_t* rec, uint32_t q, uint32_t k, uint32_t idx_base,
                         const uint32_t* ties, uint32_t tie_cap, uint32_t row_base, uint32_t* out_words,
                         void* stream);
/* Settle the listed rows (every row when ties == NULL) of a dhtgpu_merge_dev by the full
 * 160-bit keys: words = the lists' tie-word payloads concatenated in list order (each
 * tie_cap x k_in x 3 words, or q x k_in x 3 when ties == NULL). */
int dhtgpu_merge_ties_dev(const uint32_t* rec, const uint32_t* words, uint32_t lists, uint32_t q, uint32_t k_in,
                          const uint32_t* t_planes, uint64_t t_stride, uint32_t k, const uint32_t* ties,
                          uint32_t tie_cap, uint32_t* out_idx, uint32_t* out_cnt, void* stream);

/* Device planes -> the ids whose top pbits bits equal pval, compacted in order into
 * out_planes (out_stride >= count) with out_gidx[j] = original index (nullable);
 * *out_count = number selected.  Synchronises (setup-time helper). */
int dhtgpu_select_prefix_dev(dhtgpu_ctx* ctx, const uint32_t* planes, uint64_t stride, uint64_t n,
                             uint32_t pbits, uint32_t pval, uint32_t* out_planes, uint64_t out_stride,
                             uint32_t* out_gidx, uint64_t* out_count, void* stream);

/* Convert 20-byte big-endian ids (device) into word planes (device). */
int dhtgpu_pack_dev(const uint8_t* ids20_be, uint64_t n, uint32_t* planes, uint64_t stride,
                    void* stream);
/* Generate synthetic ids (same stream as dhtgpu_gen_ids) into device planes. */
int dhtgpu_gen_dev(uint64_t seed, uint64_t start, uint64_t n, uint32_t* planes, uint64_t stride,
                   void* stream);

/* ---- K4/K5: bucket index + trie-descent exact top-k (same results as dhtgpu_topk) ---- */
/* Build (or rebuild) the index over the context's id set: a counting sort of the ids by
 * their top B = clamp(log2(n) - 4, 1, 24) bits into 32-byte records plus a 2^B + 1 entry
 * prefix directory.  Stream-ordered (NULL = the context stream); no host sync. */
int dhtgpu_index_build(dhtgpu_ctx* ctx, void* stream);
/* Diagnostics: the same build with HIP events between its kernels; synchronises and
 * returns per-phase device milliseconds ms4 = {P0 histogram, P0 scans, P1 partition
 * scatter, P2 bucket gather}. */
int dhtgpu_index_build_timed(dhtgpu_ctx* ctx, void* stream, float* ms4);
/* Exact top-k via the index: identical output to dhtgpu_topk_dev -- final indices +
 * counts, or (out_rec != NULL) candidate records for dhtgpu_merge_dev; idx offset by
 * idx_base.  Needs a built index (DHTGPU_ENOIDS otherwise). */
int dhtgpu_index_topk_dev(dhtgpu_ctx* ctx, const uint32_t* t_planes, uint64_t t_stride, uint32_t q,
                          uint32_t k, uint32_t* out_idx, uint32_t* out_cnt, uint32_t* out_rec,
                          uint32_t idx_base, void* stream);
/* Host form: builds the index if the id set changed since the last build, then queries. */
int dhtgpu_index_topk(dhtgpu_ctx* ctx, const uint8_t* targets20_be, uint32_t q, uint32_t k,
                      uint32_t* out_idx, uint32_t* out_cnt);

/* ---- K6: per-batch target-prefix filter + exact top-k (same results as dhtgpu_topk) ---- */
/* Nothing persists between calls: each call streams the id word plane w0 once, keeps only
 * the ids that share the batch targets' level-Lm prefixes (Lm ~ log2(n / 4k)), and answers
 * every target from its complete prefix subtree in LDS; targets whose subtree holds fewer
 * than min(k, n) ids, or whose partition overflows (clustered ids), are answered by the K1
 * scan over all ids inside the same call.  Same output forms as dhtgpu_topk_dev.
 * Large sets (n > 2^24 where one plan cannot cover the batch, e.g. the 2^27-id cfg-3 shard at
 * 131,072 targets): the set is split once into 2^s prefix sub-partitions of <= 2^24 ids (built
 * on the first such call, kept until the set changes: 28 B/id of extra HBM) and every call runs
 * ONE K6 launch sequence over all sub-partitions, each answering the targets of its prefix; a
 * sub-partition with fewer than k ids sends its targets to the K1 scan over the whole set.
 * DHTGPU_ERANGE only when q > 2^22 (or n >= 2^32).
 * Stream-ordered, no host sync (except the one-time sub-partition build).  A context keeps four
 * workspaces and gives each stream its own (the one it last used, else a free one), so calls
 * issued on up to four streams run concurrently (one batch's latency-bound answer phase
 * overlaps the other batches' HBM-bound id streams); a call that must take a workspace last
 * used on another stream (a fifth stream) first waits for that stream. */
int dhtgpu_batch_topk_dev(dhtgpu_ctx* ctx, const uint32_t* t_planes, uint64_t t_stride, uint32_t q,
                          uint32_t k, uint32_t* out_idx, uint32_t* out_cnt, uint32_t* out_rec,
                          uint32_t idx_base, void* stream);
/* Diagnostics: the same call with a start/stop HIP event pair recorded by each kernel's own
 * dispatch; synchronises and returns per-kernel device milliseconds ms4 = {F1 bucket
 * targets, F2 filter ids, F3 answer, F4 ties + fallback scan} and (nullable) stats4 =
 * {targets answered by the fallback scan, surviving ids, targets answered by an exact wave
 * (w0 ties, large subtrees), 0}.  Sub-partitioned calls: the one launch sequence over all
 * sub-partitions. */
int dhtgpu_batch_topk_timed(dhtgpu_ctx* ctx, const uint32_t* t_planes, uint64_t t_stride, uint32_t q,
                            uint32_t k, uint32_t* out_idx, uint32_t* out_cnt, void* stream, float* ms4,
                            uint32_t* stats4);
/* Arm per-kernel timing of the NEXT K6 call on this context without synchronising it:
 * its kernels' own dispatches record start/stop into ev8[0..7] (hipEvent_t as void*, created
 * by the caller with timing enabled) = {F1 start, F1 stop, F2 start, F2 stop, F3 .., F4 ..}
 * (sub-partitioned calls: sub-partition 0's kernels).  For timing kernels inside a timed loop. */
int dhtgpu_batch_events(dhtgpu_ctx* ctx, void** ev8);
/* Host form (synchronous). */
int dhtgpu_batch_topk(dhtgpu_ctx* ctx, const uint8_t* targets20_be, uint32_t q, uint32_t k,
                      uint32_t* out_idx, uint32_t* out_cnt);

/* ---- K1r: RoutingTable::findClosestNodes over a table snapshot ------------------ */
/* Snapshot: nb buckets in list order with firsts20[nb*20] (Bucket::first),
 * bucket_off[nb+1] (bucket b owns nodes [off[b], off[b+1]) of node_ids20), and
 * good[nn] = Node::isGood(now) (src/node.cpp:42-47).  For each target: the
 * min(count, C) XOR-closest good nodes of the contiguous bucket range visited by
 * the reference's outward walk, ascending.  out_idx[q*count] indexes node_ids20. */
int dhtgpu_find_closest(dhtgpu_ctx* ctx, uint32_t nb, const uint8_t* firsts20,
                        const uint32_t* bucket_off, const uint8_t* node_ids20,
                        const uint8_t* good, const uint8_t* targets20_be, uint32_t q,
                        uint32_t count, uint32_t* out_idx, uint32_t* out_cnt);

/* ---- K2: routing-bucket classification over the context's id set -------------- */
/* out_bucket[n] (nullable) = findBucket(id) index; hist161[161] = histogram of
 * commonBits(id, myid).  nb in [1, 256], firsts sorted ascending (as in the table). */
int dhtgpu_classify(dhtgpu_ctx* ctx, uint32_t nb, const uint8_t* firsts20,
                    const uint8_t* myid20, uint8_t* out_bucket, uint64_t* hist161);
int dhtgpu_classify_dev(const uint32_t* planes, uint64_t stride, uint64_t n, uint32_t nb,
                        const uint32_t* d_first_planes /* 5*nb, word-major */,
                        const uint32_t* myid_words /* host, 5 words */, uint8_t* out_bucket,
                        unsigned long long* d_hist161, void* stream);

/* ---- a8: NodeCache::getCachedNodes walk over the context's id set --------------------- */
/* accept[n] (nullable = all) = lock() && !isExpired() && !isClient().  Output in
 * the reference's walk order (not sorted), indices into the id set.  An id set uploaded
 * unsorted is sorted on the device on the first call (f2: LSD radix over the 160-bit keys,
 * kept until the set changes); DHTGPU_EUNSORTED if it holds duplicate ids. */
int dhtgpu_cached_nodes(dhtgpu_ctx* ctx, const uint8_t* accept, const uint8_t* targets20_be,
                        uint32_t q, uint32_t count, uint32_t* out_idx, uint32_t* out_cnt);

/* ---- f2: the NodeCache mirror (a second, context-private id set) ------------------------ */
/* NodeCache::NodeMap (include/opendht/node_cache.h:43: std::map<InfoHash, weak_ptr<Node>>,
 * src/node_cache.cpp:42-74) as n unique 20-byte keys in the CALLER's order (e.g. a walk of
 * the map, or any order): sorted lexicographically on the device; it does not touch the
 * context's k-NN id set.  version != 0 equal to the last upload's (same n) skips the upload:
 * the caller bumps it whenever the map changes.  DHTGPU_EUNSORTED on duplicate keys. */
int dhtgpu_cache_set(dhtgpu_ctx* ctx, const uint8_t* ids20, uint64_t n, uint64_t version);
/* getCachedNodes(target, af, count) for q targets over the mirror: accept[n] (nullable) and
 * the output indices are in the caller's order of the last dhtgpu_cache_set. */
int dhtgpu_cache_nodes(dhtgpu_ctx* ctx, const uint8_t* accept, const uint8_t* targets20_be, uint32_t q,
                       uint32_t count, uint32_t* out_idx, uint32_t* out_cnt);
/* The mirror's lexicographic order: perm[j] = caller index of the j-th smallest key. */
int dhtgpu_cache_sorted(dhtgpu_ctx* ctx, uint32_t* perm);

/* ---- a6: RoutingTable::depth (src/routing_table.cpp:100-107) over a table snapshot ---- */
/* *out_depth = max(lowbit(first[b]), lowbit(first[b+1])) + 1 (0 for an empty table);
 * table_depth of Dht::getNodesStats (src/dht.cpp:1425-1444) is depth(findBucket(myid)). */
int dhtgpu_table_depth(uint32_t nb, const uint8_t* firsts20, uint32_t b, uint32_t* out_depth);

/* ---- a11 / f4: compact node wire format ---------------------------------------------- */
/* NetworkEngine::bufferNodes(af, id, nodes) (src/network_engine.cpp:1003-1032), batched:
 * for each target, its candidates cand[qi*c .. +c) (indices into the context's id set,
 * DHTGPU_NONE = absent, c <= 64) are sorted by InfoHash::xorCmp to the target, the first
 * SEND_NODES = 8 are kept and written as 26-byte (af 4) / 38-byte (af 6) records
 * id || address || port to out[qi * 8 * rec ..]; out_len[qi] = bytes written.
 * node_tail[i*(alen+2)] = node i's address || port bytes as its sockaddr holds them
 * (network order), alen = 4 / 16.  Equal ids (never in OpenDHT) keep candidate order.
 * Every candidate must be DHTGPU_NONE or < the number of ids: the host form returns
 * DHTGPU_EINVAL otherwise; the _dev form does not check (device pointers). */
int dhtgpu_buffer_nodes_dev(dhtgpu_ctx* ctx, const uint8_t* node_tail, uint32_t af, const uint32_t* t_planes,
                            uint64_t t_stride, uint32_t q, const uint32_t* cand, uint32_t c, uint8_t* out,
                            uint32_t* out_len, void* stream);
int dhtgpu_buffer_nodes(dhtgpu_ctx* ctx, const uint8_t* node_tail, uint32_t af, const uint8_t* targets20,
                        uint32_t q, const uint32_t* cand, uint32_t c, uint8_t* out, uint32_t* out_len);
/* The same over the caller's own nodes: cand indexes node_ids20[nn * 20] / node_tail (the
 * context's id set is not used or changed). */
int dhtgpu_buffer_nodes_ids(dhtgpu_ctx* ctx, const uint8_t* node_ids20, const uint8_t* node_tail, uint32_t nn,
                            uint32_t af, const uint8_t* targets20, uint32_t q, const uint32_t* cand, uint32_t c,
                            uint8_t* out, uint32_t* out_len);
/* NetworkEngine::deserializeNodes (src/network_engine.cpp:849-887), batched over m received
 * n4 (af 4) / n6 (af 6) blobs: message i is blob[msg_off[i] .. msg_off[i+1]), received from
 * from_addr[i*16 ..] (family from_af[i]: 4, 6 or 0).  msg_status[i] = 1 when its length is
 * not a whole number of records (the reference's WRONG_NODE_INFO_BUF_LEN; none of its
 * records is decoded), else 0.  Every record of the other messages is decoded, in order,
 * into out_ids20 / out_tail (address || port after the loopback -> sender rewrite) and
 * out_status: 0 accepted, 1 own id (myid20), 2 martian (NetworkEngine::isMartian).
 * *out_nrec = records decoded (<= msg_off[m] / rec); isNodeBlacklisted stays with the
 * caller. */
int dhtgpu_deserialize_nodes(dhtgpu_ctx* ctx, uint32_t af, const uint8_t* myid20, const uint8_t* blob,
                             const uint64_t* msg_off, uint32_t m, const uint8_t* from_af, const uint8_t* from_addr,
                             uint8_t* out_ids20, uint8_t* out_tail, uint8_t* out_status, uint8_t* msg_status,
                             uint32_t* out_nrec);

/* ---- a10: Dht::Search::insertNode (src/search.h:636-722), batched ------------------------ */
/* q searches (targets20[q]): search s holds list_len[s] <= cap SearchNodes list_node[s*cap ..]
 * (indices into node_ids20[nn * 20], closest first) with list_flags (bit0 candidate, bit1
 * replied) and search_expired[s] (Search::expired).  Its insertions ins_node[ins_off[s] ..
 * ins_off[s+1]) (ins_token != 0: the node replied with a token) are applied in order with the
 * reference's ordering, trimming to SEARCH_NODES = 14 non-bad nodes (isBad = isExpired() ||
 * candidate, :352-354) and removeExpiredNode (:541-551); ins_added = insertNode's result.
 * node_state[nn]: bit0 Node::isExpired(), bit1 Node::isRemovable(now) (node.h:87-89), a
 * snapshot like the good mask of dhtgpu_find_closest.  Lists are updated in place;
 * DHTGPU_ERANGE if a list would outgrow cap (that insertion is dropped). */
int dhtgpu_search_insert(dhtgpu_ctx* ctx, const uint8_t* node_ids20, const uint8_t* node_state, uint32_t nn,
                         const uint8_t* targets20, uint32_t q, uint32_t cap, uint32_t* list_node, uint8_t* list_flags,
                         uint32_t* list_len, uint8_t* search_expired, const uint64_t* ins_off, const uint32_t* ins_node,
                         const uint8_t* ins_token, uint8_t* ins_added);

/* ---- a4 / a6: InfoHash::lowbit (infohash.h:132-143) + RoutingTable::depth per bucket ------ */
/* out_lowbit[b] = lowbit(first[b]) (-1 for the zero id), out_depth[b] = depth of bucket b
 * (src/routing_table.cpp:100-107) for every bucket of a table snapshot, on the device. */
int dhtgpu_table_stats(dhtgpu_ctx* ctx, uint32_t nb, const uint8_t* firsts20, int32_t* out_lowbit, uint32_t* out_depth);

/* ---- f3: crawl replay (BASELINE configs[4]) -------------------------------------------- */
/* The context's id set becomes a synthetic network (model: opendht_amd/csrc/crawl.hip and
 * oracle/crawl_oracle.cpp): node order by (first word, index), implicit k-bucket routing
 * tables sampled with table_seed, dead[n] (host, nullable) marks nodes that never answer.
 * Synchronous. */
int dhtgpu_net_prepare(dhtgpu_ctx* ctx, const uint8_t* dead, uint64_t table_seed);
/* One iterative search per target (Dht::Search, src/search.h: Search::insertNode :636-722,
 * SEARCH_NODES = 14, MAX_REQUESTED_SEARCH_NODES = 4 per round, isSynced :734-747), started
 * by node searchers[qi] from its own routing table.  Per search: the final SearchNode list
 * out_idx[qi*64 ..] (node indices, DHTGPU_NONE padded) with out_flags (bit0 asked, bit1
 * replied, bit2 bad), out_len, rounds run and find_node requests sent. */
int dhtgpu_search_batch(dhtgpu_ctx* ctx, const uint8_t* targets20, uint32_t q, const uint32_t* searchers,
                        uint32_t max_rounds, uint32_t* out_idx, uint8_t* out_flags, uint32_t* out_len,
                        uint32_t* out_rounds, uint32_t* out_queries);
/* Requests a search sends per round (alpha, 1..8) for the following search_batch calls on this
 * context: default 4 = MAX_REQUESTED_SEARCH_NODES (include/opendht/dht.h:321); BASELINE cfg 5
 * states a 3-way alpha. */
int dhtgpu_set_search_alpha(dhtgpu_ctx* ctx, uint32_t alpha);
int dhtgpu_search_batch_dev(dhtgpu_ctx* ctx, const uint32_t* t_planes, uint64_t t_stride, uint32_t q,
                            const uint32_t* searchers, uint32_t max_rounds, uint32_t* out_idx, uint8_t* out_flags,
                            uint32_t* out_len, uint32_t* out_rounds, uint32_t* out_queries, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DHTGPU_H */
