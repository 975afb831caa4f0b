/*
 * dhtgpu.hpp -- C++11 host adapter over the libdhtgpu C ABI (dhtgpu.h).
 *
 * Drop-in helpers with the reference's signatures and result shapes
 * (paths relative to the OpenDHT tree):
 *
 *   findClosestNodes(ctx, table, id, now, count)          <- RoutingTable::findClosestNodes
 *       (include/opendht/routing_table.h:56, src/routing_table.cpp:110-150)
 *   findClosestNodesBatch(ctx, table, targets, q, now, k)  new batched form (one launch)
 *   getCachedNodes(ctx, map, id, count)                    <- NodeCache::getCachedNodes
 *       (include/opendht/node_cache.h:31, src/node_cache.cpp:42-74)
 *   ClosestIndex                                           flat exact k-NN over a fixed id
 *       set: std::partial_sort(.., InfoHash::xorCmp) (include/opendht/infohash.h:179-194)
 *   bufferNodesBatch(ctx, af6, targets, nodes)             <- NetworkEngine::bufferNodes
 *       (src/network_engine.cpp:1003-1032), batched
 *
 * The templates are written against the reference's member names only -- a table is a
 * list of buckets with `.first` (InfoHash) and `.nodes` (list of Sp<Node>); a node has
 * `.id`, `isGood(now)`, `isExpired()`, `isClient()`; an InfoHash exposes `data()` (20
 * big-endian bytes) -- so they compile against dht::RoutingTable / NodeCache's map
 * without including OpenDHT headers here.
 *
 * Behaviour: results are identical to the reference (same nodes, same order).  On a
 * device error the helpers throw dhtgpu::Error; they never return different nodes.
 * The caller (single dht_thread, src/dhtrunner.cpp:115-150) owns the Context.
 *
 * Dispatch: a device call costs a fixed ~90 µs (snapshot + PCIe + launches) against
 * ~0.13 µs per findClosestNodes on one CPU core (bench.py find_closest / cpu_baseline), so
 * the helpers answer on the host -- the same walk as the reference body -- below
 * Context::min_device_batch targets (default kMinDeviceBatch = 1024, above the measured
 * crossover of ~740) and only larger batches go to the device.  A single call is therefore
 * as fast as the reference's own (tests/cpp/adapter_check.cpp reports both).
 */
#ifndef DHTGPU_HPP
#define DHTGPU_HPP

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <iterator>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "dhtgpu.h"

namespace dhtgpu {

class Error : public std::runtime_error {
public:
    Error(int code, const char* what)
        : std::runtime_error(std::string("libdhtgpu: ") + what + ": " + dhtgpu_strerror(code)), code_(code) {}
    int code() const { return code_; }
private:
    int code_;
};

inline void check(int code, const char* what) {
    if (code != DHTGPU_OK) throw Error(code, what);
}

/* Batches below this many targets are answered on the host (see Dispatch above). */
static const size_t kMinDeviceBatch = 1024;

/* RAII owner of one device context. */
class Context {
public:
    explicit Context(int device = 0) : ctx_(nullptr) { check(dhtgpu_ctx_create(device, &ctx_), "ctx_create"); }
    ~Context() { dhtgpu_ctx_destroy(ctx_); }
    Context(const Context&) = delete;
    Context& operator=(const Context&) = delete;
    dhtgpu_ctx* get() const { return ctx_; }
    size_t min_device_batch = kMinDeviceBatch;   // smallest batch sent to the device
    uint64_t cache_version_ = 0;   // NodeCache mirror: version and size of the last upload
    size_t cache_size_ = 0;
private:
    dhtgpu_ctx* ctx_;
};

namespace detail {
template <class H>
inline void put_id(std::vector<uint8_t>& out, const H& h) {
    const uint8_t* p = h.data();
    out.insert(out.end(), p, p + DHTGPU_HASH_LEN);
}

/* InfoHash::xorCmp(a, b) < 0 for target t (include/opendht/infohash.h:179-194): at the first
 * byte where a and b differ, the one whose byte XOR t's is smaller is closer. */
inline bool xor_closer(const uint8_t* t, const uint8_t* a, const uint8_t* b) {
    for (unsigned i = 0; i < DHTGPU_HASH_LEN; ++i)
        if (a[i] != b[i]) return (uint8_t)(a[i] ^ t[i]) < (uint8_t)(b[i] ^ t[i]);
    return false;
}

/* The reference's findClosestNodes walk on the host (src/routing_table.cpp:110-150): the
 * target's bucket (findBucket, :153-166: the last whose first <= id), then one bucket on each
 * side per round until `count` good nodes are held, each inserted in xorCmp order. */
template <class Table, class HashT, class TimePoint, class NodePtr>
void find_closest_host(const Table& table, const HashT& id, TimePoint now, size_t count, std::vector<NodePtr>& nodes) {
    nodes.clear();
    const auto begin = table.begin(), end = table.end();
    if (begin == end) return;
    const uint8_t* t = id.data();
    auto b = begin;
    for (;;) {
        auto nx = std::next(b);
        if (nx == end || std::memcmp(t, nx->first.data(), DHTGPU_HASH_LEN) < 0) break;
        b = nx;
    }
    auto insert_bucket = [&](const decltype(*begin)& bk) {
        for (const auto& n : bk.nodes) {
            if (!n->isGood(now)) continue;
            auto here = std::find_if(nodes.begin(), nodes.end(), [&](const NodePtr& o) {
                return xor_closer(t, n->id.data(), o->id.data());
            });
            nodes.insert(here, n);
        }
    };
    auto itn = b;
    auto itp = b == begin ? end : std::prev(b);
    while (nodes.size() < count && (itn != end || itp != end)) {
        if (itn != end) { insert_bucket(*itn); ++itn; }
        if (itp != end) { insert_bucket(*itp); itp = itp == begin ? end : std::prev(itp); }
    }
    if (nodes.size() > count) nodes.resize(count);
}

/* The reference's getCachedNodes walk on the host (src/node_cache.cpp:42-74): out of
 * lower_bound(id), each step takes the XOR-closer of the two neighbours; accepted = lock()
 * succeeds && !isExpired() && !isClient().  O(log N + visited) -- no pass over the map. */
template <class NodeMap, class HashT>
std::vector<std::shared_ptr<typename NodeMap::mapped_type::element_type>>
cached_nodes_host(const NodeMap& c, const HashT& id, size_t count) {
    std::vector<std::shared_ptr<typename NodeMap::mapped_type::element_type>> res;
    const uint8_t* t = id.data();
    auto it_n = c.lower_bound(id);
    auto it_p = it_n;
    const auto end = c.cend();
    auto dec = [&](decltype(it_p)& it) {   // cbegin() -> cend(), else prev()
        auto ret = it;
        it = it == c.cbegin() ? end : std::prev(it);
        return ret;
    };
    if (!c.empty()) dec(it_p);
    while (res.size() < count && (it_n != end || it_p != end)) {
        decltype(it_n) it;
        if (it_p == end) it = it_n++;
        else if (it_n == end) it = dec(it_p);
        else it = xor_closer(t, it_p->first.data(), it_n->first.data()) ? dec(it_p) : it_n++;
        if (auto n = it->second.lock())
            if (!n->isExpired() && !n->isClient()) res.push_back(n);
    }
    return res;
}
}  // namespace detail

/* Snapshot of a RoutingTable at time `now`: bucket firsts, per-bucket node ranges,
 * node ids, the isGood(now) mask, and the node handles to map indices back. */
template <class Table, class TimePoint>
struct TableSnapshot {
    typedef typename std::decay<decltype(*std::declval<const Table&>().begin()->nodes.begin())>::type NodePtr;
    std::vector<uint8_t> firsts, ids, good;
    std::vector<uint32_t> off;
    std::vector<NodePtr> nodes;

    TableSnapshot(const Table& table, TimePoint now) {
        for (const auto& b : table) {
            detail::put_id(firsts, b.first);
            off.push_back((uint32_t)nodes.size());
            for (const auto& n : b.nodes) {
                detail::put_id(ids, n->id);
                good.push_back(n->isGood(now) ? 1 : 0);
                nodes.push_back(n);
            }
        }
        off.push_back((uint32_t)nodes.size());
    }
    uint32_t nbuckets() const { return (uint32_t)(firsts.size() / DHTGPU_HASH_LEN); }
};

/* RoutingTable::findClosestNodes for a batch of targets (one device launch). */
template <class Table, class HashT, class TimePoint>
std::vector<std::vector<typename TableSnapshot<Table, TimePoint>::NodePtr>>
findClosestNodesBatch(Context& ctx, const Table& table, const HashT* targets, size_t q, TimePoint now,
                      size_t count) {
    typedef typename TableSnapshot<Table, TimePoint>::NodePtr NodePtr;
    std::vector<std::vector<NodePtr>> res(q);
    if (q == 0 || count == 0) return res;
    if (q < ctx.min_device_batch || count > DHTGPU_MAX_K) {   // the host walk (Dispatch)
        for (size_t i = 0; i < q; ++i) detail::find_closest_host(table, targets[i], now, count, res[i]);
        return res;
    }
    TableSnapshot<Table, TimePoint> snap(table, now);
    std::vector<uint8_t> t;
    t.reserve(q * DHTGPU_HASH_LEN);
    for (size_t i = 0; i < q; ++i) detail::put_id(t, targets[i]);
    std::vector<uint32_t> idx(q * count), cnt(q);
    check(dhtgpu_find_closest(ctx.get(), snap.nbuckets(), snap.firsts.data(), snap.off.data(),
                              snap.ids.empty() ? nullptr : snap.ids.data(),
                              snap.good.empty() ? nullptr : snap.good.data(), t.data(), (uint32_t)q,
                              (uint32_t)count, idx.data(), cnt.data()),
          "find_closest");
    for (size_t i = 0; i < q; ++i) {
        res[i].reserve(cnt[i]);
        for (uint32_t r = 0; r < cnt[i]; ++r) res[i].push_back(snap.nodes[idx[i * count + r]]);
    }
    return res;
}

/* Drop-in for RoutingTable::findClosestNodes(id, now, count): one target is always below
 * the device threshold, so this is the host walk (the reference's cost, no snapshot). */
template <class Table, class HashT, class TimePoint>
std::vector<typename TableSnapshot<Table, TimePoint>::NodePtr>
findClosestNodes(Context& ctx, const Table& table, const HashT& id, TimePoint now, size_t count = 8) {
    if (ctx.min_device_batch > 1) {
        std::vector<typename TableSnapshot<Table, TimePoint>::NodePtr> res;
        detail::find_closest_host(table, id, now, count, res);
        return res;
    }
    return std::move(findClosestNodesBatch(ctx, table, &id, 1, now, count)[0]);
}

/* NodeCache::getCachedNodes over one address family's map (std::map<InfoHash, weak_ptr<Node>>,
 * include/opendht/node_cache.h:43, src/node_cache.cpp:42-74), batched.  The map's keys go to
 * the context's NodeCache mirror (dhtgpu_cache_set: a set of its own, sorted on the device --
 * the context's k-NN id set is not touched); `version` != 0 equal to the previous call's skips
 * that upload (the caller bumps it whenever the map changes).  Accepted = lock() succeeds &&
 * !isExpired() && !isClient(), evaluated at call time; walk order preserved. */
template <class NodeMap, class HashT>
void getCachedNodesRaw(Context& ctx, const NodeMap& map, const HashT* targets, size_t q, size_t count,
                       std::vector<std::shared_ptr<typename NodeMap::mapped_type::element_type>>& locked,
                       std::vector<std::vector<uint32_t>>& out, uint64_t version = 0) {
    std::vector<uint8_t> ids, accept;
    const bool upload = version == 0 || version != ctx.cache_version_ || map.size() != ctx.cache_size_;
    if (upload) ids.reserve(map.size() * DHTGPU_HASH_LEN);
    locked.clear();
    accept.reserve(map.size());
    for (const auto& kv : map) {
        if (upload) detail::put_id(ids, kv.first);
        auto n = kv.second.lock();
        accept.push_back(n && !n->isExpired() && !n->isClient() ? 1 : 0);
        locked.push_back(n);
    }
    if (upload) {
        check(dhtgpu_cache_set(ctx.get(), ids.empty() ? nullptr : ids.data(), map.size(), version), "cache_set");
        ctx.cache_version_ = version;
        ctx.cache_size_ = map.size();
    }
    std::vector<uint8_t> t;
    for (size_t i = 0; i < q; ++i) detail::put_id(t, targets[i]);
    std::vector<uint32_t> idx(q * count), cnt(q);
    out.assign(q, std::vector<uint32_t>());
    if (q == 0) return;
    check(dhtgpu_cache_nodes(ctx.get(), accept.empty() ? nullptr : accept.data(), t.data(), (uint32_t)q,
                             (uint32_t)count, idx.data(), cnt.data()),
          "cache_nodes");
    for (size_t i = 0; i < q; ++i) out[i].assign(idx.begin() + i * count, idx.begin() + i * count + cnt[i]);
}

/* NodeCache::getCachedNodes for a batch of targets.  The device path walks the map once per
 * batch (the accept mask is evaluated at call time, as the reference does per visited entry),
 * so it is taken only when the batch is large against the map (q >= min_device_batch and
 * q >= map.size() / 8: the walk then costs less than 8 entries per target); otherwise each
 * target takes the host walk, O(log N + count). */
template <class NodeMap, class HashT>
std::vector<std::vector<std::shared_ptr<typename NodeMap::mapped_type::element_type>>>
getCachedNodesBatch(Context& ctx, const NodeMap& map, const HashT* targets, size_t q, size_t count,
                    uint64_t version = 0) {
    std::vector<std::vector<std::shared_ptr<typename NodeMap::mapped_type::element_type>>> res(q);
    if (q == 0 || count == 0) return res;
    if (q < ctx.min_device_batch || q < map.size() / 8 || count > DHTGPU_MAX_K) {
        for (size_t i = 0; i < q; ++i) res[i] = detail::cached_nodes_host(map, targets[i], count);
        return res;
    }
    std::vector<std::shared_ptr<typename NodeMap::mapped_type::element_type>> locked;
    std::vector<std::vector<uint32_t>> out;
    getCachedNodesRaw(ctx, map, targets, q, count, locked, out, version);
    for (size_t i = 0; i < q; ++i)
        for (uint32_t j : out[i]) res[i].push_back(locked[j]);
    return res;
}

/* Drop-in for NodeCache::getCachedNodes(id, af, count): one target -- the host walk, as fast
 * as the reference body (no pass over the map, nothing uploaded). */
template <class NodeMap, class HashT>
std::vector<std::shared_ptr<typename NodeMap::mapped_type::element_type>>
getCachedNodes(Context& ctx, const NodeMap& map, const HashT& id, size_t count, uint64_t version = 0) {
    return std::move(getCachedNodesBatch(ctx, map, &id, 1, count, version)[0]);
}

/* Flat exact k-NN over a fixed id set kept resident in HBM (the batched
 * findClosestNodesBatch(targets[], k) of the north star): upload once, query many. */
class ClosestIndex {
public:
    explicit ClosestIndex(Context& ctx) : ctx_(ctx) {}
    template <class HashT>
    void assign(const HashT* ids, size_t n) {
        std::vector<uint8_t> b;
        b.reserve(n * DHTGPU_HASH_LEN);
        for (size_t i = 0; i < n; ++i) detail::put_id(b, ids[i]);
        check(dhtgpu_set_ids(ctx_.get(), b.empty() ? nullptr : b.data(), n), "set_ids");
    }
    /* out[i] = indices of the k ids closest to targets[i], ascending by XOR distance */
    template <class HashT>
    std::vector<std::vector<uint32_t>> query(const HashT* targets, size_t q, size_t k) const {
        std::vector<uint8_t> t;
        t.reserve(q * DHTGPU_HASH_LEN);
        for (size_t i = 0; i < q; ++i) detail::put_id(t, targets[i]);
        std::vector<uint32_t> idx(q * k), cnt(q);
        std::vector<std::vector<uint32_t>> res(q);
        if (q == 0) return res;
        // K6 per-batch prefix filter (large sets run over prefix sub-partitions inside the
        // library); the K1 streaming scan where K6's limits are exceeded (q > 2^22)
        int rc = dhtgpu_batch_topk(ctx_.get(), t.data(), (uint32_t)q, (uint32_t)k, idx.data(), cnt.data());
        if (rc == DHTGPU_ERANGE) rc = dhtgpu_topk(ctx_.get(), t.data(), (uint32_t)q, (uint32_t)k, idx.data(), cnt.data());
        check(rc, "topk");
        for (size_t i = 0; i < q; ++i) res[i].assign(idx.begin() + i * k, idx.begin() + i * k + cnt[i]);
        return res;
    }
private:
    Context& ctx_;
};

/* Drop-in for NetworkEngine::bufferNodes(af, id, nodes) (src/network_engine.cpp:1003-1032)
 * over a batch: nodes[i] (candidates for targets[i], e.g. findClosestNodes results) are
 * sorted by xorCmp to targets[i], the first SEND_NODES = 8 are packed as 26 (AF_INET) /
 * 38 (AF_INET6) byte records id || address || port.  Written against the reference's
 * member names: node->id, node->getAddr().getIPv4().sin_addr/.sin_port,
 * getIPv6().sin6_addr/.sin6_port. */
template <class HashT, class NodePtr>
std::vector<std::vector<uint8_t>> bufferNodesBatch(Context& ctx, int af_inet6, const HashT* targets,
                                                   const std::vector<std::vector<NodePtr>>& nodes) {
    const uint32_t alen = af_inet6 ? 16u : 4u, rec = 20 + alen + 2;
    const size_t q = nodes.size();
    std::vector<std::vector<uint8_t>> res(q);
    if (q == 0) return res;
    size_t c = 0;
    for (const auto& v : nodes) c = v.size() > c ? v.size() : c;
    if (c > 64) throw Error(DHTGPU_EINVAL, "bufferNodes: more than 64 candidates");
    std::vector<uint8_t> ids, tail, t;
    std::vector<uint32_t> cand(q * (c ? c : 1), DHTGPU_NONE);
    uint32_t n = 0;
    for (size_t i = 0; i < q; ++i) {
        detail::put_id(t, targets[i]);
        for (size_t j = 0; j < nodes[i].size(); ++j, ++n) {
            const auto& nd = nodes[i][j];
            detail::put_id(ids, nd->id);
            const uint8_t* a;
            const uint8_t* p;
            if (af_inet6) {
                const auto& sin6 = nd->getAddr().getIPv6();
                a = reinterpret_cast<const uint8_t*>(&sin6.sin6_addr);
                p = reinterpret_cast<const uint8_t*>(&sin6.sin6_port);
            } else {
                const auto& sin = nd->getAddr().getIPv4();
                a = reinterpret_cast<const uint8_t*>(&sin.sin_addr);
                p = reinterpret_cast<const uint8_t*>(&sin.sin_port);
            }
            tail.insert(tail.end(), a, a + alen);
            tail.insert(tail.end(), p, p + 2);
            cand[i * c + j] = n;
        }
    }
    std::vector<uint8_t> out(q * 8 * rec);
    std::vector<uint32_t> len(q);
    // the candidates' own ids (the context's k-NN id set is not touched)
    check(dhtgpu_buffer_nodes_ids(ctx.get(), ids.empty() ? nullptr : ids.data(), tail.empty() ? nullptr : tail.data(), n,
                                  af_inet6 ? 6u : 4u, t.data(), (uint32_t)q, cand.data(), (uint32_t)c, out.data(),
                                  len.data()),
          "buffer_nodes");
    for (size_t i = 0; i < q; ++i) res[i].assign(out.begin() + i * 8 * rec, out.begin() + i * 8 * rec + len[i]);
    return res;
}

}  // namespace dhtgpu

#endif /* DHTGPU_HPP */
