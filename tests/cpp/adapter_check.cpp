// adapter_check.cpp -- exercises include/dhtgpu.hpp (C++11) against reference-shaped
// mock types (same member names as dht::Bucket / dht::Node / dht::InfoHash).
// Build-only on CPU (tests/test_abi.py); with --run on a GPU it compares the adapter
// against the oracle restatement (test infrastructure) and exits non-zero on mismatch.
#include <array>
#include <cstdio>
#include <cstring>
#include <list>
#include <map>
#include <memory>
#include <vector>

#include "dhtgpu.hpp"
#include "../../oracle/dht_oracle.h"

namespace mock {
struct InfoHash {
    std::array<uint8_t, 20> d;
    const uint8_t* data() const { return d.data(); }
    bool operator<(const InfoHash& o) const { return std::memcmp(d.data(), o.d.data(), 20) < 0; }
};
struct Node {
    InfoHash id;
    bool good, expired, client;
    bool isGood(long) const { return good; }
    bool isExpired() const { return expired; }
    bool isClient() const { return client; }
};
struct Bucket {
    InfoHash first;
    std::list<std::shared_ptr<Node>> nodes;
};
typedef std::list<Bucket> RoutingTable;
}  // namespace mock

static uint64_t rng_state = 88172645463325252ull;
static uint32_t rnd() { rng_state ^= rng_state << 13; rng_state ^= rng_state >> 7; rng_state ^= rng_state << 17; return (uint32_t)rng_state; }

int main(int argc, char** argv) {
    if (argc < 2 || std::strcmp(argv[1], "--run") != 0) { std::puts("built"); return 0; }
    // grow a table with the oracle's onNewNode restatement, then mirror it as mock types
    std::vector<uint8_t> myid(20), ids(20 * 20000);
    orc_gen_ids(99, 0, 1, myid.data());
    orc_gen_ids(100, 0, 20000, ids.data());
    orc_table* t = orc_table_new(myid.data(), 0);
    for (int i = 0; i < 20000; ++i) orc_table_insert(t, ids.data() + 20 * i);
    const uint32_t nb = orc_table_nbuckets(t), nn = orc_table_nnodes(t);
    std::vector<uint8_t> firsts(20 * nb), nodes(20 * nn), good(nn);
    std::vector<uint32_t> off(nb + 1);
    orc_table_export(t, firsts.data(), off.data(), nodes.data());
    orc_table_free(t);
    mock::RoutingTable table;
    for (uint32_t b = 0; b < nb; ++b) {
        mock::Bucket bk;
        std::memcpy(bk.first.d.data(), &firsts[20 * b], 20);
        for (uint32_t i = off[b]; i < off[b + 1]; ++i) {
            auto n = std::make_shared<mock::Node>();
            std::memcpy(n->id.d.data(), &nodes[20 * i], 20);
            good[i] = (rnd() % 10) >= 3;
            n->good = good[i] != 0;
            n->expired = !n->good && (rnd() & 1);
            n->client = false;
            bk.nodes.push_back(n);
        }
        table.push_back(bk);
    }
    dhtgpu::Context ctx(0);
    int bad = 0;
    std::vector<mock::InfoHash> targets(300);
    std::vector<uint8_t> tb(20 * 300);
    orc_gen_ids(101, 0, 300, tb.data());
    for (int i = 0; i < 300; ++i) std::memcpy(targets[i].d.data(), &tb[20 * i], 20);
    auto batch = dhtgpu::findClosestNodesBatch(ctx, table, targets.data(), targets.size(), 0L, 8);
    for (int i = 0; i < 300; ++i) {
        uint32_t want[32];
        uint32_t c = orc_find_closest(nb, firsts.data(), off.data(), nodes.data(), good.data(), &tb[20 * i], 8, want);
        auto one = dhtgpu::findClosestNodes(ctx, table, targets[i], 0L, 8);
        if (batch[i].size() != c || one.size() != c) { ++bad; continue; }
        for (uint32_t r = 0; r < c; ++r)
            if (std::memcmp(batch[i][r]->id.data(), &nodes[20 * want[r]], 20) || batch[i][r] != one[r]) ++bad;
    }
    // NodeCache-shaped map
    std::map<mock::InfoHash, std::weak_ptr<mock::Node>> cache;
    std::vector<std::shared_ptr<mock::Node>> keep;
    for (int i = 0; i < 5000; ++i) {
        auto n = std::make_shared<mock::Node>();
        std::memcpy(n->id.d.data(), &ids[20 * i], 20);
        n->expired = (rnd() % 4) == 0;
        n->client = (rnd() % 10) == 0;
        n->good = true;
        cache[n->id] = n;
        if (rnd() % 8) keep.push_back(n);   // the rest expire (weak_ptr lock fails)
    }
    std::vector<uint8_t> sorted, acc;
    for (const auto& kv : cache) {
        sorted.insert(sorted.end(), kv.first.d.begin(), kv.first.d.end());
        auto n = kv.second.lock();
        acc.push_back(n && !n->isExpired() && !n->isClient());
    }
    for (int i = 0; i < 300; ++i) {
        auto got = dhtgpu::getCachedNodes(ctx, cache, targets[i], 14);
        uint32_t want[32];
        uint32_t c = orc_cached_nodes(sorted.data(), cache.size(), acc.data(), &tb[20 * i], 14, want);
        if (got.size() != c) { ++bad; continue; }
        for (uint32_t r = 0; r < c; ++r)
            if (std::memcmp(got[r]->id.data(), &sorted[20 * want[r]], 20)) ++bad;
    }
    // the versioned form (upload skipped while the map is unchanged) gives the same nodes
    for (int i = 0; i < 50; ++i) {
        auto a = dhtgpu::getCachedNodes(ctx, cache, targets[i], 14, 7);
        auto b = dhtgpu::getCachedNodes(ctx, cache, targets[i], 14, 7);
        auto c0 = dhtgpu::getCachedNodes(ctx, cache, targets[i], 14);
        if (a != b || a != c0) ++bad;
    }
    // a ClosestIndex keeps answering over ITS id set across getCachedNodes / bufferNodesBatch
    // calls on the same Context (they use the context's NodeCache mirror / their own nodes)
    {
        const size_t nid = 30000, q = 200;
        std::vector<uint8_t> kb(20 * nid);
        orc_gen_ids(555, 0, nid, kb.data());
        std::vector<mock::InfoHash> kid(nid);
        for (size_t i = 0; i < nid; ++i) std::memcpy(kid[i].d.data(), &kb[20 * i], 20);
        dhtgpu::ClosestIndex index(ctx);
        index.assign(kid.data(), nid);
        std::vector<uint32_t> want(q * 8), wcnt(q);
        orc_topk(kb.data(), nid, tb.data(), q, 8, want.data(), wcnt.data(), 4);
        auto before = index.query(targets.data(), q, 8);
        auto unused = dhtgpu::getCachedNodes(ctx, cache, targets[0], 14);
        (void)unused;
        auto after = index.query(targets.data(), q, 8);
        for (size_t i = 0; i < q; ++i) {
            if (before[i] != after[i] || after[i].size() != wcnt[i]) { ++bad; continue; }
            for (uint32_t r = 0; r < wcnt[i]; ++r)
                if (after[i][r] != want[i * 8 + r]) ++bad;
        }
    }
    std::printf("adapter_check: %d mismatches\n", bad);
    return bad ? 1 : 0;
}
