/*
 * dht_oracle.cpp -- CPU restatement of OpenDHT's XOR-closest-node path.
 *
 * TEST INFRASTRUCTURE ONLY (see dht_oracle.h).  Never linked into libdhtgpu.
 *
 * Every function cites the reference file:line it restates.  Reference paths are
 * relative to the OpenDHT source tree (Dale-M/opendht @ v0).
 */
#include "dht_oracle.h"

#include <algorithm>
#include <array>
#include <cstring>
#include <iterator>
#include <list>
#include <stdexcept>
#include <thread>
#include <vector>

namespace {

constexpr unsigned HASH_LEN = 20;          /* include/opendht/infohash.h:267 */
constexpr unsigned TARGET_NODES = 8;       /* include/opendht/routing_table.h:26 */
constexpr size_t SEARCH_NODES = 14;        /* src/dht.h:308 */
using Id = std::array<uint8_t, HASH_LEN>;

inline Id load(const uint8_t* p) { Id r; std::memcpy(r.data(), p, HASH_LEN); return r; }

/* Hash<N>::xorCmp, include/opendht/infohash.h:179-194: at the first byte where id1
 * and id2 differ, compare id1^self with id2^self. */
inline int xor_cmp(const uint8_t* self, const uint8_t* a, const uint8_t* b) {
    for (unsigned i = 0; i < HASH_LEN; i++) {
        if (a[i] == b[i]) continue;
        uint8_t x1 = a[i] ^ self[i], x2 = b[i] ^ self[i];
        return x1 < x2 ? -1 : 1;
    }
    return 0;
}

/* Hash<N>::commonBits, include/opendht/infohash.h:154-176. */
inline unsigned common_bits(const uint8_t* a, const uint8_t* b) {
    unsigned i = 0;
    for (; i < HASH_LEN; i++)
        if (a[i] != b[i]) break;
    if (i == HASH_LEN) return 8 * HASH_LEN;
    uint8_t x = a[i] ^ b[i];
    unsigned j = 0;
    while ((x & 0x80) == 0) { x <<= 1; j++; }
    return 8 * i + j;
}

/* Hash<N>::lowbit, include/opendht/infohash.h:132-143. */
inline int lowbit(const uint8_t* a) {
    int i, j;
    for (i = HASH_LEN - 1; i >= 0; i--)
        if (a[i] != 0) break;
    if (i < 0) return -1;
    for (j = 7; j >= 0; j--)
        if ((a[i] & (0x80 >> j)) != 0) break;
    return 8 * i + j;
}

/* Hash<N>::cmp, include/opendht/infohash.h:149-151 (memcmp). */
inline int cmp(const uint8_t* a, const uint8_t* b) { return std::memcmp(a, b, HASH_LEN); }

/* Hash<N>::setBit, include/opendht/infohash.h:205-210. */
inline void set_bit(Id& id, unsigned nbit, bool b) {
    uint8_t& num = id[nbit / 8];
    unsigned bit = 7 - (nbit % 8);
    num ^= (-(int)b ^ num) & (1 << bit);
}

inline uint64_t splitmix(uint64_t seed, uint64_t j) {
    uint64_t z = seed + (j + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

inline void put_be64(uint8_t* p, uint64_t v, unsigned nbytes) {
    for (unsigned i = 0; i < nbytes; i++) p[i] = (uint8_t)(v >> (56 - 8 * i));
}

template <class F>
void parallel_for(uint64_t n, int threads, F f) {
    if (threads <= 1 || n < 2) { for (uint64_t i = 0; i < n; i++) f(i); return; }
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++)
        th.emplace_back([&, t] { for (uint64_t i = t; i < n; i += threads) f(i); });
    for (auto& x : th) x.join();
}

/* ---- RoutingTable restatement (src/routing_table.cpp, include/opendht/routing_table.h) ---- */
struct Bucket {
    Id first {};
    std::list<uint32_t> nodes;   /* node handles, list order as in Bucket::nodes (routing_table.h:38) */
};

} // namespace

struct orc_table {
    Id myid {};
    bool is_client {false};
    std::list<Bucket> buckets;
    std::vector<Id> ids;          /* node handle -> id */

    using It = std::list<Bucket>::iterator;

    /* RoutingTable::findBucket, src/routing_table.cpp:153-166 */
    It find_bucket(const Id& id) {
        if (buckets.empty()) return buckets.end();
        auto b = buckets.begin();
        while (true) {
            auto next = std::next(b);
            if (next == buckets.end()) return b;
            if (cmp(id.data(), next->first.data()) < 0) return b;
            b = next;
        }
    }
    /* RoutingTable::contains, include/opendht/routing_table.h:64-67 */
    bool contains(It b, const Id& id) {
        return cmp(b->first.data(), id.data()) <= 0 &&
               (std::next(b) == buckets.end() || cmp(id.data(), std::next(b)->first.data()) < 0);
    }
    /* RoutingTable::depth, src/routing_table.cpp:100-107 */
    unsigned depth(It b) {
        if (b == buckets.end()) return 0;
        int bit1 = lowbit(b->first.data());
        int bit2 = std::next(b) != buckets.end() ? lowbit(std::next(b)->first.data()) : -1;
        return std::max(bit1, bit2) + 1;
    }
    /* RoutingTable::split (+ middle, src/routing_table.cpp:87-97), :169-200 */
    bool split(It b) {
        unsigned bit = depth(b);
        if (bit >= 8 * HASH_LEN) return false;         /* middle() throws out_of_range */
        Id new_id = b->first;
        set_bit(new_id, bit, true);
        Bucket nb; nb.first = new_id;
        buckets.insert(std::next(b), nb);
        std::list<uint32_t> nodes;
        nodes.splice(nodes.begin(), b->nodes);
        while (!nodes.empty()) {
            auto n = nodes.begin();
            auto bb = find_bucket(ids[*n]);
            if (bb == buckets.end()) nodes.erase(n);
            else bb->nodes.splice(bb->nodes.begin(), nodes, n);
        }
        return true;
    }
    /* RoutingTable::onNewNode, src/routing_table.cpp:204-262, with every node good
     * (no expired node to replace, no dubious node, sendPing is a no-op). */
    int on_new_node(const Id& id) {
        for (int guard = 0; guard < 8 * (int)HASH_LEN + 2; guard++) {
            auto b = find_bucket(id);
            if (b == buckets.end()) return 0;
            for (auto n : b->nodes)
                if (ids[n] == id) return 0;          /* same node already there */
            bool mybucket = contains(b, myid);
            if (b->nodes.size() >= TARGET_NODES) {
                const bool dubious = false;
                if ((mybucket || (is_client && depth(b) < 6)) && (!dubious || buckets.size() == 1)) {
                    if (!split(b)) return 0;
                    continue;                        /* return onNewNode(node, ...) */
                }
                return 0;                            /* cached away */
            }
            ids.push_back(id);
            b->nodes.emplace_front((uint32_t)(ids.size() - 1));
            return 1;
        }
        return 0;
    }
};

extern "C" {

void orc_gen_ids(uint64_t seed, uint64_t start, uint64_t n, uint8_t* out20) {
    for (uint64_t i = 0; i < n; i++) {
        uint64_t g = start + i;
        uint8_t* p = out20 + 20 * i;
        put_be64(p, splitmix(seed, 3 * g), 8);
        put_be64(p + 8, splitmix(seed, 3 * g + 1), 8);
        put_be64(p + 16, splitmix(seed, 3 * g + 2), 4);
    }
}

int orc_xor_cmp(const uint8_t* self, const uint8_t* a, const uint8_t* b) { return xor_cmp(self, a, b); }
unsigned orc_common_bits(const uint8_t* a, const uint8_t* b) { return common_bits(a, b); }
int orc_lowbit(const uint8_t* a) { return lowbit(a); }
int orc_cmp(const uint8_t* a, const uint8_t* b) { int c = cmp(a, b); return (c > 0) - (c < 0); }

/* std::partial_sort(first, first+k, last, [t](a,b){ return t.xorCmp(a,b) < 0; })
 * over an index array; equal ids tie-break by lower index. */
void orc_topk(const uint8_t* ids20, uint64_t n, const uint8_t* targets20, uint32_t q,
              uint32_t k, uint32_t* out_idx, uint32_t* out_cnt, int threads) {
    parallel_for(q, threads, [&](uint64_t qi) {
        const uint8_t* t = targets20 + 20 * qi;
        std::vector<uint32_t> idx(n);
        for (uint64_t i = 0; i < n; i++) idx[i] = (uint32_t)i;
        uint64_t kk = std::min<uint64_t>(k, n);
        std::partial_sort(idx.begin(), idx.begin() + kk, idx.end(), [&](uint32_t a, uint32_t b) {
            int c = xor_cmp(t, ids20 + 20ull * a, ids20 + 20ull * b);
            return c < 0 || (c == 0 && a < b);
        });
        for (uint32_t i = 0; i < k; i++) out_idx[qi * k + i] = i < kk ? idx[i] : 0xFFFFFFFFu;
        out_cnt[qi] = (uint32_t)kk;
    });
}

/* The same top-k (std::partial_sort under xorCmp, equal ids by lower index) over the id stream
 * [start, start + n) of orc_gen_ids, generated on the fly: no 20-byte array of the whole set is
 * held (BASELINE cfg 3: 10^9 ids = 20 GB).  Threads take contiguous index ranges and keep, per
 * target, the k smallest (distance, index) pairs of their range in a sorted array; the per-thread
 * lists are then merged.  The 160-bit big-endian distance id ^ t compares as the word triple
 * (bytes 0..7, 8..15, 16..19), which is xorCmp's order (include/opendht/infohash.h:179-194: at the
 * first byte where two ids differ, the one whose byte XOR t is smaller is closer).  out_idx holds
 * stream indices (start + i); start + n <= 2^32. */
void orc_topk_gen(uint64_t seed, uint64_t start, uint64_t n, const uint8_t* targets20, uint32_t q, uint32_t k,
                  uint32_t* out_idx, uint32_t* out_cnt, int threads) {
    struct Cand { uint64_t d0, d1; uint32_t d2, idx; };
    auto less = [](const Cand& a, const Cand& b) {
        if (a.d0 != b.d0) return a.d0 < b.d0;
        if (a.d1 != b.d1) return a.d1 < b.d1;
        if (a.d2 != b.d2) return a.d2 < b.d2;
        return a.idx < b.idx;
    };
    auto be = [](const uint8_t* p, unsigned nb) {
        uint64_t v = 0;
        for (unsigned i = 0; i < nb; i++) v = v << 8 | p[i];
        return v;
    };
    std::vector<uint64_t> t0(q), t1(q), t2(q);
    for (uint32_t j = 0; j < q; j++) {
        t0[j] = be(targets20 + 20ull * j, 8);
        t1[j] = be(targets20 + 20ull * j + 8, 8);
        t2[j] = be(targets20 + 20ull * j + 16, 4);
    }
    if (threads < 1) threads = 1;
    const uint64_t kk = std::min<uint64_t>(k, n);
    std::vector<std::vector<Cand>> part((size_t)threads * q);
    parallel_for((uint64_t)threads, threads, [&](uint64_t th) {
        const uint64_t lo = n * th / threads, hi = n * (th + 1) / threads;
        std::vector<Cand>* lists = part.data() + th * q;
        for (uint32_t j = 0; j < q; j++) lists[j].reserve(kk + 1);
        std::vector<uint64_t> kth(q, ~0ull);   /* d0 of the list's k-th entry: a cheap reject */
        for (uint64_t i = lo; i < hi; i++) {
            const uint64_t g = start + i;
            const uint64_t x0 = splitmix(seed, 3 * g), x1 = splitmix(seed, 3 * g + 1);
            const uint32_t x2 = (uint32_t)(splitmix(seed, 3 * g + 2) >> 32);   /* top 4 bytes (orc_gen_ids) */
            for (uint32_t j = 0; j < q; j++) {
                const uint64_t d0 = x0 ^ t0[j];
                if (d0 > kth[j]) continue;
                const Cand c{d0, x1 ^ t1[j], x2 ^ (uint32_t)t2[j], (uint32_t)g};
                std::vector<Cand>& L = lists[j];
                if (L.size() == kk && !less(c, L.back())) continue;
                L.insert(std::upper_bound(L.begin(), L.end(), c, less), c);
                if (L.size() > kk) L.pop_back();
                if (L.size() == kk) kth[j] = L.back().d0;
            }
        }
    });
    for (uint32_t j = 0; j < q; j++) {
        std::vector<Cand> all;
        for (int th = 0; th < threads; th++) {
            const std::vector<Cand>& L = part[(size_t)th * q + j];
            all.insert(all.end(), L.begin(), L.end());
        }
        std::sort(all.begin(), all.end(), less);
        for (uint32_t i = 0; i < k; i++) out_idx[(uint64_t)j * k + i] = i < kk ? all[i].idx : 0xFFFFFFFFu;
        out_cnt[j] = (uint32_t)kk;
    }
}

orc_table* orc_table_new(const uint8_t* myid20, int is_client) {
    auto* t = new orc_table;
    t->myid = load(myid20);
    t->is_client = is_client != 0;
    t->buckets.emplace_back();                     /* Dht ctor: one bucket, first = zero hash */
    return t;
}
void orc_table_free(orc_table* t) { delete t; }
int orc_table_insert(orc_table* t, const uint8_t* id20) { return t->on_new_node(load(id20)); }
uint32_t orc_table_nbuckets(const orc_table* t) { return (uint32_t)t->buckets.size(); }
uint32_t orc_table_nnodes(const orc_table* t) {
    uint32_t c = 0;
    for (auto& b : t->buckets) c += (uint32_t)b.nodes.size();
    return c;
}
void orc_table_export(const orc_table* t, uint8_t* firsts20, uint32_t* off, uint8_t* ids20) {
    uint32_t bi = 0, ni = 0;
    for (auto& b : t->buckets) {
        std::memcpy(firsts20 + 20 * bi, b.first.data(), 20);
        off[bi] = ni;
        for (auto n : b.nodes) { std::memcpy(ids20 + 20ull * ni, t->ids[n].data(), 20); ni++; }
        bi++;
    }
    off[bi] = ni;
}

/* RoutingTable::findBucket, src/routing_table.cpp:153-166 (linear walk). */
int orc_find_bucket(uint32_t nb, const uint8_t* firsts20, const uint8_t* id20) {
    if (nb == 0) return -1;
    uint32_t b = 0;
    while (true) {
        uint32_t next = b + 1;
        if (next == nb) return (int)b;
        if (cmp(id20, firsts20 + 20 * next) < 0) return (int)b;
        b = next;
    }
}

unsigned orc_depth(uint32_t nb, const uint8_t* firsts20, uint32_t b) {
    if (b >= nb) return 0;
    int bit1 = lowbit(firsts20 + 20 * b);
    int bit2 = b + 1 < nb ? lowbit(firsts20 + 20 * (b + 1)) : -1;
    return (unsigned)(std::max(bit1, bit2) + 1);
}

/* RoutingTable::findClosestNodes, src/routing_table.cpp:110-150. */
uint32_t orc_find_closest(uint32_t nb, const uint8_t* firsts20, const uint32_t* off,
                          const uint8_t* ids20, const uint8_t* good, const uint8_t* target20,
                          uint32_t count, uint32_t* out_idx) {
    std::vector<uint32_t> nodes;
    nodes.reserve(count);
    int bucket = orc_find_bucket(nb, firsts20, target20);
    if (bucket < 0) return 0;
    auto sorted_bucket_insert = [&](int b) {
        for (uint32_t n = off[b]; n < off[b + 1]; n++) {
            if (!good[n]) continue;
            auto here = std::find_if(nodes.begin(), nodes.end(), [&](uint32_t node) {
                return xor_cmp(target20, ids20 + 20ull * n, ids20 + 20ull * node) < 0;
            });
            nodes.insert(here, n);
        }
    };
    int itn = bucket;                  /* end() == nb */
    int itp = bucket - 1;              /* end() == -1 */
    while (nodes.size() < count && (itn < (int)nb || itp >= 0)) {
        if (itn < (int)nb) { sorted_bucket_insert(itn); itn++; }
        if (itp >= 0) { sorted_bucket_insert(itp); itp--; }
    }
    if (nodes.size() > count) nodes.resize(count);
    for (size_t i = 0; i < nodes.size(); i++) out_idx[i] = nodes[i];
    return (uint32_t)nodes.size();
}

/* One findClosestNodes per target (the responder loop of Dht::onFindNode, src/dht.cpp:2128-2138,
 * over many requests); out_idx[q * count], out_cnt[q].  Threads split the targets. */
void orc_find_closest_batch(uint32_t nb, const uint8_t* firsts20, const uint32_t* off, const uint8_t* ids20,
                            const uint8_t* good, const uint8_t* targets20, uint32_t q, uint32_t count,
                            uint32_t* out_idx, uint32_t* out_cnt, int threads) {
    parallel_for(q, threads, [&](uint64_t i) {
        out_cnt[i] = orc_find_closest(nb, firsts20, off, ids20, good, targets20 + 20 * i, count, out_idx + i * count);
    });
}

void orc_classify(uint32_t nb, const uint8_t* firsts20, const uint8_t* myid20,
                  const uint8_t* ids20, uint64_t n, uint8_t* out_bucket, uint64_t* hist161) {
    for (unsigned i = 0; i <= 8 * HASH_LEN; i++) hist161[i] = 0;
    for (uint64_t i = 0; i < n; i++) {
        const uint8_t* id = ids20 + 20 * i;
        int b = orc_find_bucket(nb, firsts20, id);
        out_bucket[i] = (uint8_t)(b < 0 ? 0xFF : b);
        hist161[common_bits(id, myid20)]++;
    }
}

/* orc_classify over `threads` contiguous id ranges (the cfg-4 CPU baseline at every host core):
 * the same findBucket + commonBits per id, one 161-bin histogram per thread, summed. */
void orc_classify_mt(uint32_t nb, const uint8_t* firsts20, const uint8_t* myid20,
                     const uint8_t* ids20, uint64_t n, uint8_t* out_bucket, uint64_t* hist161, int threads) {
    if (threads < 1) threads = 1;
    std::vector<uint64_t> h((size_t)threads * 161, 0);
    parallel_for((uint64_t)threads, threads, [&](uint64_t t) {
        const uint64_t lo = n * t / threads, hi = n * (t + 1) / threads;
        orc_classify(nb, firsts20, myid20, ids20 + 20 * lo, hi - lo, out_bucket + lo, h.data() + 161 * t);
    });
    for (unsigned i = 0; i <= 8 * HASH_LEN; i++) {
        hist161[i] = 0;
        for (int t = 0; t < threads; t++) hist161[i] += h[161 * (size_t)t + i];
    }
}

/* NodeCache::getCachedNodes, src/node_cache.cpp:42-74. END plays the role of c.cend(). */
uint32_t orc_cached_nodes(const uint8_t* sorted_ids20, uint64_t n, const uint8_t* accept,
                          const uint8_t* target20, uint32_t count, uint32_t* out_idx) {
    const uint64_t END = n;
    uint64_t lo = 0, hi = n;                       /* c.lower_bound(id) */
    while (lo < hi) {
        uint64_t mid = (lo + hi) / 2;
        if (cmp(sorted_ids20 + 20 * mid, target20) < 0) lo = mid + 1; else hi = mid;
    }
    uint64_t it_p = lo, it_n = lo;
    auto dec_it = [&](uint64_t& it) {
        uint64_t ret = it;
        it = (it == 0) ? END : it - 1;             /* cbegin() -> cend(), else prev() */
        return ret;
    };
    if (n != 0) dec_it(it_p);
    uint32_t cnt = 0;
    while (cnt < count && (it_n != END || it_p != END)) {
        uint64_t it;
        if (it_p == END) it = it_n++;
        else if (it_n == END) it = dec_it(it_p);
        else it = xor_cmp(target20, sorted_ids20 + 20 * it_p, sorted_ids20 + 20 * it_n) < 0
                      ? dec_it(it_p) : it_n++;
        if (accept[it]) out_idx[cnt++] = (uint32_t)it;
    }
    return cnt;
}

/* One getCachedNodes per target (Dht::refill, src/dht.cpp:656-677, over many searches). */
void orc_cached_nodes_batch(const uint8_t* sorted_ids20, uint64_t n, const uint8_t* accept, const uint8_t* targets20,
                            uint32_t q, uint32_t count, uint32_t* out_idx, uint32_t* out_cnt, int threads) {
    parallel_for(q, threads, [&](uint64_t i) {
        out_cnt[i] = orc_cached_nodes(sorted_ids20, n, accept, targets20 + 20 * i, count, out_idx + i * count);
    });
}

/* ---- Dht::Search::insertNode, src/search.h:636-722 ------------------------------------------ */
/* One search's node list: entry = (node, candidate, replied); SearchNode::isBad (:352-354) =
 * node->isExpired() || candidate.  Node state comes from node_state[node]: bit0 isExpired(),
 * bit1 isRemovable(now) (include/opendht/node.h:87-89).  `expired` is Search::expired. */
struct OrcSearch {
    const uint8_t* ids;          /* node ids, 20 B each */
    const uint8_t* state;        /* per node: bit0 expired, bit1 removable */
    const uint8_t* target;
    std::vector<uint32_t> node;
    std::vector<uint8_t> fl;     /* bit0 candidate, bit1 replied */
    bool expired;
    bool is_bad(size_t i) const { return (state[node[i]] & 1) || (fl[i] & 1); }
    size_t bad_count() const {   /* Search::getNumberOfBadNodes */
        size_t b = 0;
        for (size_t i = 0; i < node.size(); i++) b += is_bad(i);
        return b;
    }
    /* Search::removeExpiredNode, src/search.h:541-551: erase the last removable node */
    void remove_expired_node() {
        for (size_t e = node.size(); e != 0;) {
            --e;
            if (state[node[e]] & 2) {
                node.erase(node.begin() + e);
                fl.erase(fl.begin() + e);
                return;
            }
        }
    }
    bool insert(uint32_t x, bool token) {
        const uint8_t* nid = ids + 20ull * x;
        bool found = false;
        size_t n = node.size();                  /* auto n = nodes.end() */
        while (n != 0) {
            --n;
            if (node[n] == x) { found = true; break; }
            if (xor_cmp(target, nid, ids + 20ull * node[n]) > 0) { ++n; break; }   /* insert after it */
        }
        bool new_search_node = false;
        if (!found) {
            size_t t = node.size();              /* auto t = nodes.cend() */
            size_t bad = 0;
            bool full = false;
            if (expired) {
                if (node.size() >= SEARCH_NODES) { full = true; t = SEARCH_NODES; }
            } else {
                bad = bad_count();
                full = node.size() - bad >= SEARCH_NODES;
                while (t - bad > SEARCH_NODES) {
                    --t;
                    if (is_bad(t)) bad--;
                }
            }
            if (full) {
                if (t != node.size()) { node.resize(t); fl.resize(t); }
                if (n >= t) return false;
            }
            node.insert(node.begin() + n, x);
            fl.insert(fl.begin() + n, (uint8_t)0);
            new_search_node = true;
            if (state[x] & 1) {
                if (!expired) bad++;
            } else if (expired) {
                bad = node.size() - 1;
                expired = false;
            }
            while (node.size() - bad > SEARCH_NODES) {
                if (!expired && is_bad(node.size() - 1)) bad--;
                node.pop_back();
                fl.pop_back();
            }
        }
        /* the token is recorded on the inserted node; when the trimming above popped it (it
         * was appended last) the reference's iterator would be dangling: skipped here */
        if (token && n < node.size() && node[n] == x) {
            fl[n] &= (uint8_t)~1u;   /* candidate = false */
            fl[n] |= 2;              /* last_get_reply = now */
            expired = false;
        }
        if (new_search_node) remove_expired_node();
        return new_search_node;
    }
};

/* Batched: search s applies insertions [ins_off[s], ins_off[s+1]) in order. */
void orc_search_insert(const uint8_t* ids20, const uint8_t* node_state, const uint8_t* targets20, uint32_t q,
                       uint32_t cap, uint32_t* list_node, uint8_t* list_flags, uint32_t* list_len,
                       uint8_t* search_expired, const uint64_t* ins_off, const uint32_t* ins_node,
                       const uint8_t* ins_token, uint8_t* ins_added, int threads) {
    parallel_for(q, threads, [&](uint64_t s) {
        OrcSearch sr;
        sr.ids = ids20;
        sr.state = node_state;
        sr.target = targets20 + 20 * s;
        sr.node.assign(list_node + s * cap, list_node + s * cap + list_len[s]);
        sr.fl.assign(list_flags + s * cap, list_flags + s * cap + list_len[s]);
        sr.expired = search_expired[s] != 0;
        for (uint64_t i = ins_off[s]; i < ins_off[s + 1]; i++)
            ins_added[i] = sr.insert(ins_node[i], ins_token[i] != 0) ? 1 : 0;
        const size_t len = sr.node.size() < cap ? sr.node.size() : cap;
        for (size_t i = 0; i < cap; i++) {
            list_node[s * cap + i] = i < len ? sr.node[i] : UINT32_MAX;
            list_flags[s * cap + i] = i < len ? sr.fl[i] : 0;
        }
        list_len[s] = (uint32_t)sr.node.size();
        search_expired[s] = sr.expired ? 1 : 0;
    });
}

/* ---- compact node wire format (src/network_engine.cpp) ------------------------------ */
/* NetworkEngine::bufferNodes, src/network_engine.cpp:1003-1032: std::sort by xorCmp to the
 * target, keep SEND_NODES = 8 (:62), emit id (20 B) || sin_addr (4 B) / sin6_addr (16 B) ||
 * port (2 B) exactly as stored in the sockaddr (network byte order): 26 / 38-byte records
 * (NODE4/6_INFO_BUF_LEN).  `tail[i]` holds node i's address || port bytes (alen + 2).
 * cand[c] are node indices (UINT32_MAX = absent).  std::sort is unstable; node ids are
 * unique in the reference, and equal ids here keep their candidate order (documented
 * extension, identical in the kernel).  Returns the blob length. */
uint32_t orc_buffer_nodes(const uint8_t* ids20, const uint8_t* tail, uint32_t alen, const uint8_t* target20,
                          const uint32_t* cand, uint32_t c, uint8_t* out) {
    std::vector<uint32_t> v;
    for (uint32_t j = 0; j < c; j++)
        if (cand[j] != 0xFFFFFFFFu) v.push_back(cand[j]);
    std::stable_sort(v.begin(), v.end(), [&](uint32_t a, uint32_t b) {
        return xor_cmp(target20, ids20 + 20 * (size_t)a, ids20 + 20 * (size_t)b) < 0;
    });
    const uint32_t nnode = (uint32_t)std::min<size_t>(8, v.size());
    const uint32_t rec = 20 + alen + 2;
    for (uint32_t i = 0; i < nnode; i++) {
        std::memcpy(out + rec * i, ids20 + 20 * (size_t)v[i], 20);
        std::memcpy(out + rec * i + 20, tail + (size_t)(alen + 2) * v[i], alen + 2);
    }
    return nnode * rec;
}

/* NetworkEngine::deserializeNodes, src/network_engine.cpp:849-887, for one record of a
 * message received from `from_addr` (family from_af: 4 or 6, 0 = none):
 * deserializeIPv4/6 (:831-846), self skip (:858-859), loopback -> sender address with the
 * record's port (:861-865, SockAddr::isLoopback src/utils.cpp:115-128), then
 * NetworkEngine::isMartian (:362-386).  Writes the (possibly rewritten) address || port to
 * out_tail; returns 0 = accepted, 1 = own id, 2 = martian.  (isNodeBlacklisted is host
 * policy state and stays with the caller.) */
int orc_deserialize_node(const uint8_t* rec, uint32_t af, const uint8_t* myid20, uint32_t from_af,
                         const uint8_t* from_addr, uint8_t* out_tail) {
    const uint32_t alen = af == 4 ? 4 : 16;
    if (std::memcmp(rec, myid20, 20) == 0) return 1;
    uint8_t a[16], port[2];
    std::memcpy(a, rec + 20, alen);
    std::memcpy(port, rec + 20 + alen, 2);
    bool loop;
    if (af == 4) {
        loop = a[0] == 127;
    } else {
        static const uint8_t lo6[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1};
        loop = std::memcmp(a, lo6, 16) == 0;
    }
    if (loop && from_af == af) std::memcpy(a, from_addr, alen);   /* addr = from; setPort(port) */
    std::memcpy(out_tail, a, alen);
    std::memcpy(out_tail + alen, port, 2);
    if (port[0] == 0 && port[1] == 0) return 2;
    if (af == 4) return (a[0] == 0 || (a[0] & 0xE0) == 0xE0) ? 2 : 0;
    static const uint8_t zeroes[16] = {0};
    static const uint8_t v4prefix[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xFF, 0xFF};
    const bool m = a[0] == 0xFF || (a[0] == 0xFE && (a[1] & 0xC0) == 0x80) || std::memcmp(a, zeroes, 16) == 0 ||
                   std::memcmp(a, v4prefix, 12) == 0;
    return m ? 2 : 0;
}

} // extern "C"
