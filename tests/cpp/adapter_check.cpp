// adapter_check.cpp -- exercises include/dhtgpu.hpp (C++11) against reference-shaped
// mock types (same member names as dht::Bucket / dht::Node / dht::InfoHash).
// Build-only on CPU (tests/test_abi.py); with --run on a GPU it compares the adapter
// against the oracle restatement (test infrastructure) and exits non-zero on mismatch.
#include <array>
#include <chrono>
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
    const bool host_only = argc >= 2 && std::strcmp(argv[1], "--host") == 0;
    if (argc < 2 || (std::strcmp(argv[1], "--run") != 0 && !host_only)) { std::puts("built"); return 0; }
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
    int bad = 0;
    std::vector<mock::InfoHash> targets(300);
    std::vector<uint8_t> tb(20 * 300);
    orc_gen_ids(101, 0, 300, tb.data());
    for (int i = 0; i < 300; ++i) std::memcpy(targets[i].d.data(), &tb[20 * i], 20);
    if (host_only) {
        // no device: the adapter's host walks (what single calls run) against the oracle
        std::map<mock::InfoHash, std::weak_ptr<mock::Node>> cache;
        std::vector<std::shared_ptr<mock::Node>> keep;
        for (int i = 0; i < 5000; ++i) {
            auto n = std::make_shared<mock::Node>();
            std::memcpy(n->id.d.data(), &ids[20 * i], 20);
            n->expired = (rnd() % 4) == 0;
            n->client = (rnd() % 10) == 0;
            n->good = true;
            cache[n->id] = n;
            if (rnd() % 8) keep.push_back(n);
        }
        std::vector<uint8_t> sorted, acc;
        for (const auto& kv : cache) {
            sorted.insert(sorted.end(), kv.first.d.begin(), kv.first.d.end());
            auto n = kv.second.lock();
            acc.push_back(n && !n->isExpired() && !n->isClient());
        }
        for (int i = 0; i < 300; ++i) {
            for (size_t count : {1, 8, 14, 40}) {
                uint32_t want[64];
                std::vector<std::shared_ptr<mock::Node>> got;
                dhtgpu::detail::find_closest_host(table, targets[i], 0L, count, got);
                uint32_t c = orc_find_closest(nb, firsts.data(), off.data(), nodes.data(), good.data(), &tb[20 * i],
                                              (uint32_t)count, want);
                if (got.size() != c) { ++bad; continue; }
                for (uint32_t r = 0; r < c; ++r)
                    if (std::memcmp(got[r]->id.data(), &nodes[20 * want[r]], 20)) ++bad;
                auto cg = dhtgpu::detail::cached_nodes_host(cache, targets[i], count);
                c = orc_cached_nodes(sorted.data(), cache.size(), acc.data(), &tb[20 * i], (uint32_t)count, want);
                if (cg.size() != c) { ++bad; continue; }
                for (uint32_t r = 0; r < c; ++r)
                    if (std::memcmp(cg[r]->id.data(), &sorted[20 * want[r]], 20)) ++bad;
            }
        }
        std::printf("adapter_check (host walks): %d mismatches\n", bad);
        return bad ? 1 : 0;
    }
    dhtgpu::Context ctx(0);
    // every batch to the device (threshold 1), and the default dispatch (host walk below it)
    ctx.min_device_batch = 1;
    auto batch = dhtgpu::findClosestNodesBatch(ctx, table, targets.data(), targets.size(), 0L, 8);
    auto one_dev = dhtgpu::findClosestNodes(ctx, table, targets[7], 0L, 8);
    ctx.min_device_batch = dhtgpu::kMinDeviceBatch;
    auto host = dhtgpu::findClosestNodesBatch(ctx, table, targets.data(), targets.size(), 0L, 8);
    if (one_dev != host[7]) ++bad;
    for (int i = 0; i < 300; ++i) {
        uint32_t want[32];
        uint32_t c = orc_find_closest(nb, firsts.data(), off.data(), nodes.data(), good.data(), &tb[20 * i], 8, want);
        auto one = dhtgpu::findClosestNodes(ctx, table, targets[i], 0L, 8);
        if (batch[i].size() != c || one.size() != c || host[i] != one) { ++bad; continue; }
        for (uint32_t r = 0; r < c; ++r)
            if (std::memcmp(batch[i][r]->id.data(), &nodes[20 * want[r]], 20) || batch[i][r] != one[r]) ++bad;
    }
    // single-call cost: the adapter (host walk over the reference-shaped std::list table) against
    // the oracle's restated reference body, and device batches around the dispatch threshold
    {
        using clk = std::chrono::steady_clock;
        const int reps = 200000;
        uint32_t sink = 0, want[32];
        auto t0 = clk::now();
        for (int i = 0; i < reps; ++i) sink += (uint32_t)dhtgpu::findClosestNodes(ctx, table, targets[i % 300], 0L, 8).size();
        auto t1 = clk::now();
        for (int i = 0; i < reps; ++i)
            sink += orc_find_closest(nb, firsts.data(), off.data(), nodes.data(), good.data(), &tb[20 * (i % 300)], 8, want);
        auto t2 = clk::now();
        const double a_us = std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
        const double c_us = std::chrono::duration<double, std::micro>(t2 - t1).count() / reps;
        std::printf("adapter_check: threshold min_device_batch=%zu; single findClosestNodes %.3f us (adapter) vs %.3f us "
                    "(reference body restated), ratio %.2f [sink %u]\n", dhtgpu::kMinDeviceBatch, a_us, c_us, a_us / c_us, sink);
        std::vector<mock::InfoHash> big(65536);
        std::vector<uint8_t> bb(20 * big.size());
        orc_gen_ids(202, 0, big.size(), bb.data());
        for (size_t i = 0; i < big.size(); ++i) std::memcpy(big[i].d.data(), &bb[20 * i], 20);
        for (size_t q : {64, 256, 1024, 4096, 65536}) {
            ctx.min_device_batch = 1;
            dhtgpu::findClosestNodesBatch(ctx, table, big.data(), q, 0L, 8);   // warm
            auto d0 = clk::now();
            auto dv = dhtgpu::findClosestNodesBatch(ctx, table, big.data(), q, 0L, 8);
            auto d1 = clk::now();
            ctx.min_device_batch = (size_t)-1;
            auto hv = dhtgpu::findClosestNodesBatch(ctx, table, big.data(), q, 0L, 8);
            auto d2 = clk::now();
            if (dv != hv) ++bad;
            std::printf("adapter_check: findClosestNodesBatch q=%zu device %.1f us, host walk %.1f us\n", q,
                        std::chrono::duration<double, std::micro>(d1 - d0).count(),
                        std::chrono::duration<double, std::micro>(d2 - d1).count());
        }
        ctx.min_device_batch = dhtgpu::kMinDeviceBatch;
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
    ctx.min_device_batch = 1;   // the device mirror for every batch
    auto cdev = dhtgpu::getCachedNodesBatch(ctx, cache, targets.data(), 300, 14);
    ctx.min_device_batch = dhtgpu::kMinDeviceBatch;
    for (int i = 0; i < 300; ++i) {
        auto got = dhtgpu::getCachedNodes(ctx, cache, targets[i], 14);   // host walk
        uint32_t want[32];
        uint32_t c = orc_cached_nodes(sorted.data(), cache.size(), acc.data(), &tb[20 * i], 14, want);
        if (got.size() != c || cdev[i] != got) { ++bad; continue; }
        for (uint32_t r = 0; r < c; ++r)
            if (std::memcmp(got[r]->id.data(), &sorted[20 * want[r]], 20)) ++bad;
    }
    {
        using clk = std::chrono::steady_clock;
        const int reps = 200000;
        uint32_t sink = 0, want[32];
        auto t0 = clk::now();
        for (int i = 0; i < reps; ++i) sink += (uint32_t)dhtgpu::getCachedNodes(ctx, cache, targets[i % 300], 14).size();
        auto t1 = clk::now();
        for (int i = 0; i < reps; ++i) sink += orc_cached_nodes(sorted.data(), cache.size(), acc.data(), &tb[20 * (i % 300)], 14, want);
        auto t2 = clk::now();
        const double a_us = std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
        const double c_us = std::chrono::duration<double, std::micro>(t2 - t1).count() / reps;
        std::printf("adapter_check: single getCachedNodes %.3f us (adapter, std::map walk + weak_ptr locks) vs %.3f us "
                    "(reference body restated over a sorted array), ratio %.2f [sink %u]\n", a_us, c_us, a_us / c_us, sink);
    }
    // the versioned form (upload skipped while the map is unchanged) gives the same nodes
    ctx.min_device_batch = 1;
    for (int i = 0; i < 50; ++i) {
        auto a = dhtgpu::getCachedNodes(ctx, cache, targets[i], 14, 7);
        auto b = dhtgpu::getCachedNodes(ctx, cache, targets[i], 14, 7);
        auto c0 = dhtgpu::getCachedNodes(ctx, cache, targets[i], 14);
        if (a != b || a != c0) ++bad;
    }
    ctx.min_device_batch = dhtgpu::kMinDeviceBatch;
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
        ctx.min_device_batch = 1;   // a device getCachedNodes between the two queries
        auto unused = dhtgpu::getCachedNodes(ctx, cache, targets[0], 14);
        (void)unused;
        ctx.min_device_batch = dhtgpu::kMinDeviceBatch;
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
