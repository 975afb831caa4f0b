// crawl.hip -- batched iterative searches over a synthetic network (SURVEY §8(f) f3,
// BASELINE.json configs[4]: dhtscanner-style crawl replay).
//
// The model (identical in the oracle, oracle/crawl_oracle.cpp, whose header states it in
// full): n node ids, some dead; node R's routing table is implicit -- bucket i holds up
// to 8 nodes of the subtree of nodes sharing exactly i leading bits with R, sampled
// deterministically from that subtree's range of the (w0, index)-sorted node order;
// find_node(R, t) answers the 8 XOR-closest nodes of the buckets it visits (R's
// RoutingTable::findClosestNodes, src/routing_table.cpp:110-150).  One iterative search
// per target (Dht::Search, src/search.h) with Search::insertNode's ordering and trimming
// (:636-722, SEARCH_NODES = 14), MAX_REQUESTED_SEARCH_NODES = 4 requests per round
// (include/opendht/dht.h:321, Dht::searchSendGetValues src/dht.cpp:313-378) and the isSynced stop
// rule (:734-747).
//
// Kernels:
//   k_net_sort   one wave per K4 bucket: sorts the bucket's {w0, index} entries by
//                (w0, index), giving the node order and the subtree ranges;
//   k_search     one lane per search, its SearchNode list resident in LDS (slot-major),
//                every round, request and insertion of the search in one launch.
#include "dhtgpu_dev.h"
#include "dhtgpu_internal.h"

namespace dhtgpu {
namespace {

// kAlphaMax bounds the run-time alpha (requests per round; the reference's MAX_REQUESTED_SEARCH_NODES
// = 4, include/opendht/dht.h:321, is the default; BASELINE cfg 5 states 3)
constexpr uint32_t kSearchNodes = 14, kTargetNodes = 8, kAlphaMax = 8, kBucket = 8, kLevels = 32;
constexpr uint32_t kListCap = 64, kDeadCap = 64;
constexpr uint32_t kQ = 1, kReplied = 2, kBad = 4;
constexpr int kSearchThreads = 64;

// one wave per bucket: entries [lo, hi) of `in` sorted by (w0, index) into `out`
__global__ __launch_bounds__(256) void k_net_sort(const uint2* __restrict__ in, const uint32_t* __restrict__ dir,
                                                 uint32_t nb, uint2* __restrict__ out) {
    const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= nb) return;
    const uint32_t lane = lane_id();
    const uint32_t lo = dir[b], hi = dir[b + 1], m = hi - lo;
    for (uint32_t c = 0; c < m; c += 64) {
        const bool act = c + lane < m;
        const uint2 e = act ? in[lo + c + lane] : make_uint2(0u, 0u);
        const unsigned long long key = ((unsigned long long)e.x << 32) | e.y;
        uint32_t rank = 0;
        for (uint32_t o = 0; o < m; o += 64) {
            const uint2 x = o + lane < m ? in[lo + o + lane] : make_uint2(DHT_NONE, DHT_NONE);
            const unsigned long long xk = ((unsigned long long)x.x << 32) | x.y;
            const uint32_t lim = m - o < 64 ? m - o : 64;
            for (uint32_t l = 0; l < lim; ++l) {
                const unsigned long long ok = ((unsigned long long)__builtin_amdgcn_readlane((int)(xk >> 32), (int)l) << 32) |
                                              (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)xk, (int)l);
                rank += ok < key;
            }
        }
        if (act) out[lo + rank] = e;
    }
}

struct Net {
    const uint32_t* planes;
    uint64_t stride;
    const uint2* sorted;   // {w0, index} in node order
    const uint32_t* dir;   // 2^B + 1 bucket starts (top B bits of w0)
    uint32_t B;
    uint64_t n;
    const uint8_t* dead;   // nullable
    uint64_t seed;

    __device__ uint32_t w0(uint32_t i) const { return planes[i]; }
    // first node-order position with w0 >= key (key <= 2^32)
    __device__ uint32_t lb(uint64_t key) const {
        if (key >= (1ull << 32)) return (uint32_t)n;
        const uint32_t k32 = (uint32_t)key;
        const uint32_t b = B ? k32 >> (32 - B) : 0u;
        uint32_t lo = dir[b], hi = dir[b + 1];
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (sorted[mid].x < k32) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    }
    // XOR order of ids a, b relative to t (da, db: their w0 distances); equal ids by index
    __device__ bool less(uint32_t da, uint32_t a, uint32_t db, uint32_t b, const uint32_t* t) const {
        if (da != db) return da < db;
        if (a == b) return false;
        for (int j = 1; j < DHT_W; ++j) {
            const uint32_t xa = planes[(uint64_t)j * stride + a] ^ t[j];
            const uint32_t xb = planes[(uint64_t)j * stride + b] ^ t[j];
            if (xa != xb) return xa < xb;
        }
        return a < b;
    }
    // append bucket i of node r (up to 8 node indices) to c[*cnt]
    __device__ void bucket(uint32_t r, uint32_t i, uint32_t* c, uint32_t* cnt) const {
        const uint32_t sh = 31 - i;
        const uint64_t pre = (uint64_t)(w0(r) >> sh) ^ 1ull;
        const uint32_t a = lb(pre << sh), b = lb((pre + 1) << sh);
        const uint32_t m = b - a;
        if (m <= kBucket) {
            for (uint32_t p = a; p < b; ++p) c[(*cnt)++] = sorted[p].y;
            return;
        }
        const uint64_t h = splitmix(seed, 32ull * r + i) % m;
        for (uint32_t j = 0; j < kBucket; ++j) c[(*cnt)++] = sorted[a + (h + (((uint64_t)j * m) >> 3)) % m].y;
    }
    // find_node(r, t): up to 8 nodes ascending by XOR distance (ans, returns count)
    __device__ uint32_t answer(uint32_t r, const uint32_t* t, uint32_t* ans) const {
        const uint32_t x = w0(r) ^ t[0];
        const uint32_t d = x ? (uint32_t)__clz((int)x) : 32u;
        uint32_t c[2 * kBucket], cnt = 0;
        for (uint32_t i = d; i < kLevels && cnt < kBucket; ++i) bucket(r, i, c, &cnt);
        for (int i = (int)(d < kLevels ? d : kLevels) - 1; i >= 0 && cnt < kBucket; --i) bucket(r, (uint32_t)i, c, &cnt);
        // top-8 by insertion into the sorted prefix of ans
        uint32_t na = 0, ad[kBucket];
        for (uint32_t k = 0; k < cnt; ++k) {
            const uint32_t v = c[k], dv = w0(v) ^ t[0];
            if (na == kBucket && !less(dv, v, ad[kBucket - 1], ans[kBucket - 1], t)) continue;
            uint32_t pos = na < kBucket ? na : kBucket - 1;
            while (pos > 0 && less(dv, v, ad[pos - 1], ans[pos - 1], t)) {
                ans[pos] = ans[pos - 1];
                ad[pos] = ad[pos - 1];
                --pos;
            }
            ans[pos] = v;
            ad[pos] = dv;
            if (na < kBucket) ++na;
        }
        return na;
    }
};

// the lane's SearchNode list, slot-major in LDS: element k of lane l at [k * 64 + l]
struct List {
    uint32_t* idx;
    uint32_t* d0;
    uint8_t* fl;
    uint32_t* exp;
    uint32_t len, nexp;
    uint32_t lane;
    __device__ uint32_t& I(uint32_t k) { return idx[k * kSearchThreads + lane]; }
    __device__ uint32_t& D(uint32_t k) { return d0[k * kSearchThreads + lane]; }
    __device__ uint8_t& F(uint32_t k) { return fl[k * kSearchThreads + lane]; }
    __device__ bool expired(uint32_t x) {
        for (uint32_t k = 0; k < nexp; ++k)
            if (exp[k * kSearchThreads + lane] == x) return true;
        return false;
    }
    __device__ void move(uint32_t to, uint32_t from) {
        I(to) = I(from);
        D(to) = D(from);
        F(to) = F(from);
    }
    // Search::insertNode, src/search.h:636-722 (the search is never "expired")
    __device__ void insert(const Net& net, const uint32_t* t, uint32_t x, bool token) {
        const uint32_t dx = net.w0(x) ^ t[0];
        uint32_t n = len;
        bool found = false;
        while (n > 0) {
            --n;
            if (I(n) == x) { found = true; break; }
            if (net.less(D(n), I(n), dx, x, t)) { ++n; break; }
        }
        if (!found) {
            uint32_t bad = 0;
            for (uint32_t k = 0; k < len; ++k) bad += (F(k) & kBad) != 0;
            const bool full = len - bad >= kSearchNodes;
            uint32_t tcut = len;
            while (tcut - bad > kSearchNodes) {
                --tcut;
                if (F(tcut) & kBad) bad--;
            }
            if (full) {
                if (tcut != len) len = tcut;
                if (n >= tcut) return;
            }
            for (uint32_t k = len; k > n; --k) move(k, k - 1);
            I(n) = x;
            D(n) = dx;
            F(n) = expired(x) ? (uint8_t)kBad : (uint8_t)0;
            if (F(n) & kBad) bad++;
            ++len;
            while (len - bad > kSearchNodes) {
                if (F(len - 1) & kBad) bad--;
                --len;
            }
            if (len > kListCap) len = kListCap;   // model limit
            if (n >= len) return;
        }
        if (token) F(n) |= kReplied;
    }
    __device__ bool synced() {   // Search::isSynced, src/search.h:734-747
        uint32_t i = 0;
        for (uint32_t k = 0; k < len; ++k) {
            if (F(k) & kBad) continue;
            if (!(F(k) & kReplied)) return false;
            if (++i == kTargetNodes) break;
        }
        return i > 0;
    }
};

__global__ __launch_bounds__(kSearchThreads) void k_search(Net net, const uint32_t* __restrict__ tp, uint64_t ts,
                                                         const uint32_t* __restrict__ searchers, uint32_t q,
                                                         uint32_t max_rounds, uint32_t alpha, uint32_t* __restrict__ out_idx,
                                                         uint8_t* __restrict__ out_flags,
                                                         uint32_t* __restrict__ out_len,
                                                         uint32_t* __restrict__ out_rounds,
                                                         uint32_t* __restrict__ out_queries) {
    __shared__ uint32_t s_idx[(kListCap + 1) * kSearchThreads];   // one spare slot: insert, trim, cap
    __shared__ uint32_t s_d0[(kListCap + 1) * kSearchThreads];
    __shared__ uint32_t s_exp[kDeadCap * kSearchThreads];
    __shared__ uint8_t s_fl[(kListCap + 1) * kSearchThreads];
    const uint32_t s = blockIdx.x * kSearchThreads + threadIdx.x;
    if (s >= q) return;
    List L{s_idx, s_d0, s_fl, s_exp, 0, 0, threadIdx.x};
    uint32_t t[DHT_W];
#pragma unroll
    for (int j = 0; j < DHT_W; ++j) t[j] = tp[(uint64_t)j * ts + s];
    const uint32_t me = searchers[s];
    uint32_t ans[kBucket];
    uint32_t na = net.answer(me, t, ans);
    for (uint32_t k = 0; k < na; ++k)
        if (ans[k] != me) L.insert(net, t, ans[k], false);
    uint32_t rounds = 0, queries = 0;
    for (; rounds < max_rounds; ++rounds) {
        if (L.synced()) break;
        uint32_t sel[kAlphaMax], ns = 0;
        for (uint32_t k = 0; k < L.len && ns < alpha; ++k)
            if (!(L.F(k) & (kBad | kQ | kReplied))) {   // canGet: not bad, not asked, no reply yet
                L.F(k) |= kQ;
                sel[ns++] = L.I(k);
            }
        if (!ns) break;
        queries += ns;
        for (uint32_t j = 0; j < ns; ++j) {
            const uint32_t r = sel[j];
            if (net.dead && net.dead[r]) {   // the request expires: the node is expired (bad)
                if (L.nexp < kDeadCap) L.exp[(L.nexp++) * kSearchThreads + L.lane] = r;
                for (uint32_t k = 0; k < L.len; ++k)
                    if (L.I(k) == r) L.F(k) |= kBad;
                continue;
            }
            na = net.answer(r, t, ans);
            for (uint32_t k = 0; k < na; ++k)
                if (ans[k] != me) L.insert(net, t, ans[k], false);
            L.insert(net, t, r, true);
        }
    }
    out_len[s] = L.len;
    for (uint32_t k = 0; k < kListCap; ++k) {
        out_idx[(uint64_t)s * kListCap + k] = k < L.len ? L.I(k) : DHT_NONE;
        out_flags[(uint64_t)s * kListCap + k] = k < L.len ? L.F(k) : (uint8_t)0;
    }
    out_rounds[s] = rounds;
    out_queries[s] = queries;
}

}  // namespace

uint32_t search_list_cap() { return kListCap; }

hipError_t launch_net_sort(const void* index_ws, uint64_t n, uint32_t B, uint2* out, hipStream_t s) {
    const uint2* pairs = static_cast<const uint2*>(index_ws);
    const uint32_t* dir = reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(index_ws) + (size_t)n * 8);
    const uint32_t nb = 1u << B;
    k_net_sort<<<(nb + 3) / 4, 256, 0, s>>>(pairs, dir, nb, out);
    return hipGetLastError();
}

hipError_t launch_search(const uint32_t* planes, uint64_t stride, const uint2* sorted, const void* index_ws,
                         uint64_t n, uint32_t B, const uint8_t* dead, uint64_t seed, const uint32_t* tp, uint64_t ts,
                         uint32_t q, const uint32_t* searchers, uint32_t max_rounds, uint32_t alpha, uint32_t* out_idx,
                         uint8_t* out_flags, uint32_t* out_len, uint32_t* out_rounds, uint32_t* out_queries,
                         hipStream_t s) {
    if (!q) return hipSuccess;
    if (alpha < 1 || alpha > kAlphaMax) return hipErrorInvalidValue;
    Net net{planes, stride, sorted,
            reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(index_ws) + (size_t)n * 8), B, n, dead, seed};
    k_search<<<(q + kSearchThreads - 1) / kSearchThreads, kSearchThreads, 0, s>>>(
        net, tp, ts, searchers, q, max_rounds, alpha, out_idx, out_flags, out_len, out_rounds, out_queries);
    return hipGetLastError();
}

}  // namespace dhtgpu
