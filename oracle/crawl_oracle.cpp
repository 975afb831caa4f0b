/*
 * crawl_oracle.cpp -- CPU restatement of the crawl-replay model.
 *
 * TEST INFRASTRUCTURE ONLY (see dht_oracle.h): the parity checker of libdhtgpu's
 * search-batch kernel (opendht_amd/csrc/crawl.hip), which follows the same model:
 *
 * Network: n node ids; dead[i] marks nodes that never answer.  Node order = ids sorted by
 * (w0, index), w0 = the id's first big-endian 32-bit word.
 *
 * Implicit routing table of node R: bucket i (0 <= i < 32) = up to 8 nodes of
 * S_i(R) = { x : the top i+1 bits of x are R's top i bits then NOT bit i of R } (the
 * nodes sharing exactly i bits with R), a contiguous range [a, b) of the node order.
 * If b - a <= 8 all of them, else positions a + (h + (j*(b-a) >> 3)) mod (b-a), j < 8,
 * h = splitmix(table_seed, 32*R + i) mod (b-a).  (Kademlia k-buckets of k = 8, as
 * RoutingTable's TARGET_NODES, include/opendht/routing_table.h:26.)
 *
 * find_node(R, t): d = commonBits of the w0 words (32 when equal); buckets visited in the
 * order d, d+1, ..., 31, d-1, ..., 0, stopping after the first bucket that brings the
 * collected count to >= 8; answer = the 8 XOR-closest collected nodes, ascending
 * (the responder's RoutingTable::findClosestNodes, src/routing_table.cpp:110-150,
 * over its implicit table).
 *
 * Search (Dht::Search, src/search.h): list of SearchNodes kept ascending by XOR distance
 * and trimmed by Search::insertNode (src/search.h:636-722: SEARCH_NODES = 14 non-bad
 * nodes, bad = expired).  Start: the searcher s0 inserts find_node(s0, t).  Each round:
 *   - if synced (Search::isSynced, src/search.h:734-747: the first TARGET_NODES = 8
 *     non-bad nodes all replied, and at least one) stop;
 *   - select, in list order, up to MAX_REQUESTED_SEARCH_NODES = 4 (src/dht.h:321) nodes
 *     that are not bad, not already asked and have not replied (Dht::searchSendGetValues,
 *     src/dht.cpp:313-378); none -> stop;
 *   - for each selected node R in that order: a dead R expires (its SearchNode turns bad;
 *     the search remembers it as expired); a live R answers find_node(R, t): the returned
 *     nodes (except s0, NetworkEngine::deserializeNodes skips its own id) are inserted in
 *     answer order (NetworkEngine -> onNewNode -> trySearchInsert, src/dht.cpp:118-150),
 *     then R itself with its token (Dht::searchNodeGetDone, src/dht.cpp:213-240).
 * Searches are independent (each with its own searcher); removeExpiredNode's 10-minute
 * rule never fires within a search; the list holds at most 64 nodes and the search
 * remembers at most 64 expired nodes (model limits).
 */
#include "dht_oracle.h"

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

inline uint64_t mix(uint64_t seed, uint64_t j) {
    uint64_t z = seed + (j + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

inline uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

// alpha (requests per round) is a parameter: the reference's MAX_REQUESTED_SEARCH_NODES = 4
// (include/opendht/dht.h:321) by default, BASELINE cfg 5's 3-way alpha on request
constexpr unsigned kSearchNodes = 14, kTargetNodes = 8, kBucket = 8, kLevels = 32;
constexpr unsigned kListCap = 64, kDeadCap = 64;
enum : uint8_t { Q = 1, REPLIED = 2, BAD = 4 };

struct Net {
    uint64_t n;
    const uint8_t* ids;
    const uint8_t* dead;
    uint64_t seed;
    std::vector<uint32_t> order, sw0;

    uint32_t w0(uint32_t i) const { return be32(ids + 20ull * i); }
    // XOR order of ids a, b relative to t; equal ids by index
    bool less(const uint8_t* t, uint32_t a, uint32_t b) const {
        const uint8_t* x = ids + 20ull * a;
        const uint8_t* y = ids + 20ull * b;
        for (int i = 0; i < 20; ++i) {
            const uint8_t dx = x[i] ^ t[i], dy = y[i] ^ t[i];
            if (dx != dy) return dx < dy;
        }
        return a < b;
    }
    uint64_t lb(uint64_t key) const {   // first position with w0 >= key
        return std::lower_bound(sw0.begin(), sw0.end(), key,
                                [](uint32_t v, uint64_t k) { return (uint64_t)v < k; }) - sw0.begin();
    }
    void bucket(uint32_t r, unsigned i, std::vector<uint32_t>& out) const {
        const uint32_t rw = w0(r);
        const uint64_t pre = ((uint64_t)(rw >> (31 - i)) ^ 1ull);   // level i+1 prefix of S_i(R)
        const unsigned sh = 31 - i;
        const uint64_t a = lb(pre << sh), b = lb((pre + 1) << sh);
        const uint64_t m = b - a;
        if (m <= kBucket) {
            for (uint64_t p = a; p < b; ++p) out.push_back(order[p]);
            return;
        }
        const uint64_t h = mix(seed, 32ull * r + i) % m;
        for (unsigned j = 0; j < kBucket; ++j) out.push_back(order[a + (h + ((j * m) >> 3)) % m]);
    }
    // find_node(R, t): up to 8 nodes, ascending XOR distance to t
    void answer(uint32_t r, const uint8_t* t, std::vector<uint32_t>& out) const {
        const uint32_t x = w0(r) ^ be32(t);
        const unsigned d = x ? (unsigned)__builtin_clz(x) : 32u;
        std::vector<uint32_t> c;
        for (unsigned i = d; i < kLevels && c.size() < kBucket; ++i) bucket(r, i, c);
        for (int i = (int)std::min(d, kLevels) - 1; i >= 0 && c.size() < kBucket; --i) bucket(r, (unsigned)i, c);
        std::sort(c.begin(), c.end(), [&](uint32_t a, uint32_t b) { return less(t, a, b); });
        out.assign(c.begin(), c.begin() + std::min<size_t>(kBucket, c.size()));
    }
};

struct Search {
    const Net* net;
    const uint8_t* t;
    std::vector<uint32_t> idx;
    std::vector<uint8_t> fl;
    std::vector<uint32_t> expired;   // nodes this search saw expire

    bool is_expired(uint32_t x) const { return std::find(expired.begin(), expired.end(), x) != expired.end(); }
    int find(uint32_t x) const {
        for (size_t i = 0; i < idx.size(); ++i)
            if (idx[i] == x) return (int)i;
        return -1;
    }
    // Search::insertNode, src/search.h:636-722 (search never "expired")
    bool insert(uint32_t x, bool token) {
        // backward walk: found, or position after the last closer node
        size_t n = idx.size();
        bool found = false;
        while (n > 0) {
            --n;
            if (idx[n] == x) { found = true; break; }
            if (net->less(t, idx[n], x)) { ++n; break; }
        }
        bool added = false;
        if (!found) {
            size_t bad = 0;
            for (uint8_t f : fl) bad += (f & BAD) != 0;
            const bool full = idx.size() - bad >= kSearchNodes;
            size_t tcut = idx.size();
            while (tcut - bad > kSearchNodes) {
                --tcut;
                if (fl[tcut] & BAD) bad--;
            }
            if (full) {
                if (tcut != idx.size()) { idx.resize(tcut); fl.resize(tcut); }
                if (n >= tcut) return false;
            }
            idx.insert(idx.begin() + n, x);
            fl.insert(fl.begin() + n, is_expired(x) ? (uint8_t)BAD : (uint8_t)0);
            if (fl[n] & BAD) bad++;
            added = true;
            while (idx.size() - bad > kSearchNodes) {
                if (fl.back() & BAD) bad--;
                idx.pop_back();
                fl.pop_back();
            }
            if (idx.size() > kListCap) { idx.resize(kListCap); fl.resize(kListCap); }   // model limit
            if (n >= idx.size()) return added;
        }
        if (token) fl[n] |= REPLIED;
        return added;
    }
    bool synced() const {   // Search::isSynced, src/search.h:734-747
        unsigned i = 0;
        for (size_t k = 0; k < idx.size(); ++k) {
            if (fl[k] & BAD) continue;
            if (!(fl[k] & REPLIED)) return false;
            if (++i == kTargetNodes) break;
        }
        return i > 0;
    }
};

}  // namespace

extern "C" {

/* One search per target.  out_idx[q*64] / out_flags[q*64] (bit0 queried, bit1 replied,
 * bit2 bad) hold the final list (out_len[q] entries), out_rounds[q] the rounds run,
 * out_queries[q] the find_node requests sent. */
void orc_search_batch(const uint8_t* ids20, uint64_t n, const uint8_t* dead, uint64_t table_seed,
                      const uint8_t* targets20, const uint32_t* searchers, uint32_t q, uint32_t max_rounds,
                      uint32_t* out_idx, uint8_t* out_flags, uint32_t* out_len, uint32_t* out_rounds,
                      uint32_t* out_queries, int threads, uint32_t alpha) {
    Net net;
    net.n = n;
    net.ids = ids20;
    net.dead = dead;
    net.seed = table_seed;
    net.order.resize(n);
    for (uint64_t i = 0; i < n; ++i) net.order[i] = (uint32_t)i;
    std::sort(net.order.begin(), net.order.end(), [&](uint32_t a, uint32_t b) {
        const uint32_t wa = net.w0(a), wb = net.w0(b);
        return wa != wb ? wa < wb : a < b;
    });
    net.sw0.resize(n);
    for (uint64_t i = 0; i < n; ++i) net.sw0[i] = net.w0(net.order[i]);
    auto run = [&](uint32_t s) {
        Search sr;
        sr.net = &net;
        sr.t = targets20 + 20ull * s;
        const uint32_t me = searchers[s];
        std::vector<uint32_t> ans;
        net.answer(me, sr.t, ans);
        for (uint32_t x : ans)
            if (x != me) sr.insert(x, false);
        uint32_t rounds = 0, queries = 0;
        for (; rounds < max_rounds; ++rounds) {
            if (sr.synced()) break;
            std::vector<uint32_t> sel;
            for (size_t k = 0; k < sr.idx.size() && sel.size() < alpha; ++k)
                if (!(sr.fl[k] & (BAD | Q | REPLIED))) {   // canGet: not bad, not asked, no reply yet
                    sr.fl[k] |= Q;
                    sel.push_back(sr.idx[k]);
                }
            if (sel.empty()) break;
            queries += (uint32_t)sel.size();
            for (uint32_t r : sel) {
                if (dead && dead[r]) {   // request expires: the node is expired (bad)
                    if (sr.expired.size() < kDeadCap) sr.expired.push_back(r);
                    const int k = sr.find(r);
                    if (k >= 0) sr.fl[k] |= BAD;
                    continue;
                }
                net.answer(r, sr.t, ans);
                for (uint32_t x : ans)
                    if (x != me) sr.insert(x, false);
                sr.insert(r, true);
            }
        }
        out_len[s] = (uint32_t)sr.idx.size();
        for (size_t k = 0; k < kListCap; ++k) {
            out_idx[(size_t)s * kListCap + k] = k < sr.idx.size() ? sr.idx[k] : 0xFFFFFFFFu;
            out_flags[(size_t)s * kListCap + k] = k < sr.idx.size() ? sr.fl[k] : 0;
        }
        out_rounds[s] = rounds;
        out_queries[s] = queries;
    };
    if (threads <= 1) {
        for (uint32_t s = 0; s < q; ++s) run(s);
        return;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
        th.emplace_back([&, t] { for (uint32_t s = t; s < q; s += threads) run(s); });
    for (auto& x : th) x.join();
}

}  // extern "C"
