/*
 * dht_oracle.h -- CPU restatement of OpenDHT's XOR-closest-node path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for libdhtgpu.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it.  The product (libdhtgpu, opendht_amd) never links or calls it.
 *
 * Pinning: the reference C++ sources cannot be compiled in this image (every
 * translation unit on the path includes <msgpack.hpp>, which is absent, and a
 * stand-in header is not allowed), so there is no oracle/_ref build.  The
 * primitives are pinned by the known answers of the reference's own unit test
 * (tests/infohashtester.cpp:103-138, transcribed as data in
 * tests/golden/infohash_kat.json).  The composite walks (findClosestNodes,
 * getCachedNodes, findBucket) are restated line-by-line from the reference
 * source; the reference ships no tests or fixtures for them, so beyond the
 * primitive known answers their parity is "unpinned" (see DESIGN.md).
 *
 * IDs are 20-byte big-endian arrays, exactly dht::InfoHash's data_
 * (include/opendht/infohash.h:263, HASH_LEN = 20 at :267).
 */
#ifndef DHT_ORACLE_H
#define DHT_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* Synthetic ID generator shared by oracle, fixtures and the GPU generator:
 * splitmix64 counter stream; ID i = BE(x(3i)) || BE(x(3i+1)) || top4(BE(x(3i+2)))
 * with x(j) = mix(seed + (j+1)*0x9E3779B97F4A7C15).   */
void orc_gen_ids(uint64_t seed, uint64_t start, uint64_t n, uint8_t* out20);

/* InfoHash primitives. */
int orc_xor_cmp(const uint8_t* self, const uint8_t* id1, const uint8_t* id2); /* infohash.h:179-194 */
unsigned orc_common_bits(const uint8_t* a, const uint8_t* b);                 /* infohash.h:154-176 */
int orc_lowbit(const uint8_t* a);                                             /* infohash.h:132-143 */
int orc_cmp(const uint8_t* a, const uint8_t* b);                              /* infohash.h:149-151 */

/* Flat exact top-k: std::partial_sort over an index array with InfoHash::xorCmp
 * (SURVEY §8(a) a12); equal IDs break ties by lower index (documented extension).
 * out_idx[q*k] padded with UINT32_MAX, out_cnt[q] = min(k, n). */
void orc_topk(const uint8_t* ids20, uint64_t n, const uint8_t* targets20, uint32_t q,
              uint32_t k, uint32_t* out_idx, uint32_t* out_cnt, int threads);

/* orc_topk over the orc_gen_ids stream [start, start+n) generated on the fly (no id array held:
 * BASELINE cfg 3's 10^9 ids); out_idx are stream indices start + i (start + n <= 2^32). */
void orc_topk_gen(uint64_t seed, uint64_t start, uint64_t n, const uint8_t* targets20, uint32_t q, uint32_t k,
                  uint32_t* out_idx, uint32_t* out_cnt, int threads);

/* RoutingTable growth by onNewNode (src/routing_table.cpp:204-262), used to make
 * realistic table shapes.  All nodes are good when inserted. */
typedef struct orc_table orc_table;
orc_table* orc_table_new(const uint8_t* myid20, int is_client);
void orc_table_free(orc_table*);
/* returns 1 if the node was placed in a bucket, 0 if cached/dropped */
int orc_table_insert(orc_table*, const uint8_t* id20);
uint32_t orc_table_nbuckets(const orc_table*);
uint32_t orc_table_nnodes(const orc_table*);
/* Export: firsts[nb*20], off[nb+1], node ids[nn*20] grouped per bucket in list order. */
void orc_table_export(const orc_table*, uint8_t* firsts20, uint32_t* off, uint8_t* ids20);

/* RoutingTable::findBucket (src/routing_table.cpp:153-166) over a snapshot;
 * returns -1 for an empty table. */
int orc_find_bucket(uint32_t nb, const uint8_t* firsts20, const uint8_t* id20);
/* RoutingTable::depth (src/routing_table.cpp:100-107). */
unsigned orc_depth(uint32_t nb, const uint8_t* firsts20, uint32_t b);
/* RoutingTable::findClosestNodes (src/routing_table.cpp:110-150) over a snapshot
 * with a per-node good mask (Node::isGood(now), src/node.cpp:42-47).
 * out_idx[count] receives node indices (into the exported node array). */
uint32_t orc_find_closest(uint32_t nb, const uint8_t* firsts20, const uint32_t* off,
                          const uint8_t* ids20, const uint8_t* good, const uint8_t* target20,
                          uint32_t count, uint32_t* out_idx);
/* orc_find_closest for q targets (out_idx[q*count], out_cnt[q]) on `threads` threads. */
void orc_find_closest_batch(uint32_t nb, const uint8_t* firsts20, const uint32_t* off, const uint8_t* ids20,
                            const uint8_t* good, const uint8_t* targets20, uint32_t q, uint32_t count,
                            uint32_t* out_idx, uint32_t* out_cnt, int threads);
/* findBucket + commonBits classification (cfg 4). */
void orc_classify(uint32_t nb, const uint8_t* firsts20, const uint8_t* myid20,
                  const uint8_t* ids20, uint64_t n, uint8_t* out_bucket, uint64_t* hist161);
/* NodeCache::getCachedNodes (src/node_cache.cpp:42-74) over a lexicographically
 * sorted, unique id array with an accept mask (lock() && !isExpired() && !isClient()).
 * Output is in walk order (NOT sorted), indices into the sorted array. */
uint32_t orc_cached_nodes(const uint8_t* sorted_ids20, uint64_t n, const uint8_t* accept,
                          const uint8_t* target20, uint32_t count, uint32_t* out_idx);

/* orc_cached_nodes for q targets (out_idx[q*count], out_cnt[q]) on `threads` threads. */
void orc_cached_nodes_batch(const uint8_t* sorted_ids20, uint64_t n, const uint8_t* accept, const uint8_t* targets20,
                            uint32_t q, uint32_t count, uint32_t* out_idx, uint32_t* out_cnt, int threads);
/* Dht::Search::insertNode (src/search.h:636-722, + removeExpiredNode :541-551) batched over q
 * searches: search s holds list_len[s] entries list_node/list_flags[s*cap ..] (flags bit0
 * candidate, bit1 replied) and search_expired[s]; its insertions ins_node[ins_off[s] ..
 * ins_off[s+1]) (ins_token != 0: a reply with a token) are applied in order; ins_added =
 * insertNode's return value.  node_state[node]: bit0 isExpired(), bit1 isRemovable(now).
 * list_len may exceed cap (entries past cap are not stored). */
void orc_search_insert(const uint8_t* ids20, const uint8_t* node_state, const uint8_t* targets20, uint32_t q,
                       uint32_t cap, uint32_t* list_node, uint8_t* list_flags, uint32_t* list_len,
                       uint8_t* search_expired, const uint64_t* ins_off, const uint32_t* ins_node,
                       const uint8_t* ins_token, uint8_t* ins_added, int threads);
/* NetworkEngine::bufferNodes (src/network_engine.cpp:1003-1032): sort candidates by xorCmp
 * to the target, keep 8, pack 26 (IPv4, alen 4) / 38 (IPv6, alen 16) byte records.
 * tail[i] = node i's address || port bytes.  Returns the blob length. */
uint32_t orc_buffer_nodes(const uint8_t* ids20, const uint8_t* tail, uint32_t alen, const uint8_t* target20,
                          const uint32_t* cand, uint32_t c, uint8_t* out);
/* NetworkEngine::deserializeNodes (src/network_engine.cpp:849-887) for one record:
 * 0 = accepted, 1 = own id, 2 = martian; out_tail = address || port after the loopback
 * rewrite.  af / from_af: 4 or 6 (from_af 0 = unknown sender family). */
int orc_deserialize_node(const uint8_t* rec, uint32_t af, const uint8_t* myid20, uint32_t from_af,
                         const uint8_t* from_addr, uint8_t* out_tail);

/* orc_classify split over `threads` contiguous id ranges (cfg-4 CPU baseline). */
void orc_classify_mt(uint32_t nb, const uint8_t* firsts20, const uint8_t* myid20,
                     const uint8_t* ids20, uint64_t n, uint8_t* out_bucket, uint64_t* hist161, int threads);

/* Crawl-replay model (crawl_oracle.cpp header comment): one iterative search per target
 * over an n-node network with implicit k-bucket routing tables.  Outputs the final
 * SearchNode list (64 slots: index, flags bit0 asked / bit1 replied / bit2 bad), its
 * length, the rounds run and the find_node requests sent. */
void orc_search_batch(const uint8_t* ids20, uint64_t n, const uint8_t* dead, uint64_t table_seed,
                      const uint8_t* targets20, const uint32_t* searchers, uint32_t q, uint32_t max_rounds,
                      uint32_t* out_idx, uint8_t* out_flags, uint32_t* out_len, uint32_t* out_rounds,
                      uint32_t* out_queries, int threads, uint32_t alpha);

#ifdef __cplusplus
}
#endif
#endif
