// search.hip -- batched Dht::Search::insertNode (src/search.h:636-722) on gfx950.
//
// A search keeps its candidate nodes in XOR order to its target (closest first) and trims the
// list to SEARCH_NODES = 14 non-bad nodes (src/dht.h:308); SearchNode::isBad (:352-354) is
// node->isExpired() || candidate.  Every new node is inserted by a backward walk from the end
// (after the first node it is farther than), the list is trimmed before (full search) and
// after the insertion, a reply with a token clears the node's candidate flag, and a new
// search node triggers removeExpiredNode (:541-551: the last node whose node isRemovable(now)).
//
// One thread per search; insertions are applied in order from a CSR list.  The list rows live
// in the caller's device buffers (cap entries each); node ids are word planes of the caller's
// node table, node state one byte per node (bit0 isExpired(), bit1 isRemovable(now)).  The
// work is O(list length) per insertion, as in the reference: latency-bound, batched only to
// serve many searches (Dht::refill / searchStep over MAX_SEARCHES) per launch.
#include "dhtgpu_dev.h"
#include "dhtgpu_internal.h"

namespace dhtgpu {
namespace {

constexpr uint32_t kSearchNodes = 14;   // SEARCH_NODES, src/dht.h:308

struct Row {
    uint32_t* node;
    uint8_t* fl;     // bit0 candidate, bit1 replied
    uint32_t len;
    __device__ bool bad(uint32_t i, const uint8_t* st) const { return (st[node[i]] & 1u) || (fl[i] & 1u); }
};

// InfoHash::xorCmp(target; a, b) > 0: a farther than b (infohash.h:179-194)
__device__ __forceinline__ bool farther(const uint32_t* __restrict__ planes, uint64_t stride, uint32_t a, uint32_t b,
                                        const uint32_t* t) {
    for (int w = 0; w < DHT_W; ++w) {
        const uint32_t x = planes[(uint64_t)w * stride + a], y = planes[(uint64_t)w * stride + b];
        if (x != y) return (x ^ t[w]) > (y ^ t[w]);
    }
    return false;
}

__global__ __launch_bounds__(256) void k_search_insert(const uint32_t* __restrict__ planes, uint64_t stride,
                                                       const uint8_t* __restrict__ st, const uint32_t* __restrict__ tp,
                                                       uint64_t ts, uint32_t q, uint32_t cap, uint32_t* list_node,
                                                       uint8_t* list_flags, uint32_t* list_len, uint8_t* expired_io,
                                                       const uint64_t* __restrict__ ins_off,
                                                       const uint32_t* __restrict__ ins_node,
                                                       const uint8_t* __restrict__ ins_token, uint8_t* ins_added,
                                                       uint32_t* overflow) {
    const uint32_t s = blockIdx.x * 256 + threadIdx.x;
    if (s >= q) return;
    uint32_t t[DHT_W];
    load_id(tp, ts, s, t);
    Row r{list_node + (uint64_t)s * cap, list_flags + (uint64_t)s * cap, list_len[s]};
    bool expired = expired_io[s] != 0;
    for (uint64_t i = ins_off[s]; i < ins_off[s + 1]; ++i) {
        const uint32_t x = ins_node[i];
        bool found = false;
        uint32_t n = r.len;
        while (n != 0) {   // backward walk: the node itself, or the slot after a closer node
            --n;
            if (r.node[n] == x) { found = true; break; }
            if (farther(planes, stride, x, r.node[n], t)) { ++n; break; }
        }
        bool added = false, ok = true;
        if (!found) {
            uint32_t tcut = r.len, bad = 0;
            bool full = false;
            if (expired) {
                if (r.len >= kSearchNodes) { full = true; tcut = kSearchNodes; }
            } else {
                for (uint32_t j = 0; j < r.len; ++j) bad += r.bad(j, st);
                full = r.len - bad >= kSearchNodes;
                while (tcut - bad > kSearchNodes) {
                    --tcut;
                    if (r.bad(tcut, st)) bad--;
                }
            }
            if (full) {
                r.len = tcut;
                if (n >= tcut) ok = false;   // farther than every kept node: not inserted
            }
            if (ok) {
                if (r.len + 1 > cap) {       // the row cannot hold the list: reported, row left as is
                    atomicOr(overflow, 1u);
                    ok = false;
                } else {
                    for (uint32_t j = r.len; j > n; --j) {
                        r.node[j] = r.node[j - 1];
                        r.fl[j] = r.fl[j - 1];
                    }
                    r.node[n] = x;
                    r.fl[n] = 0;
                    ++r.len;
                    added = true;
                    if (st[x] & 1u) {
                        if (!expired) bad++;
                    } else if (expired) {
                        bad = r.len - 1;
                        expired = false;
                    }
                    while (r.len - bad > kSearchNodes) {
                        if (!expired && r.bad(r.len - 1, st)) bad--;
                        --r.len;
                    }
                }
            }
        }
        if (ok && ins_token[i] && n < r.len && r.node[n] == x) {   // a reply with a token
            r.fl[n] = (uint8_t)((r.fl[n] & ~1u) | 2u);
            expired = false;
        }
        if (added) {   // Search::removeExpiredNode: the last removable node
            for (uint32_t e = r.len; e != 0;) {
                --e;
                if (st[r.node[e]] & 2u) {
                    for (uint32_t j = e; j + 1 < r.len; ++j) {
                        r.node[j] = r.node[j + 1];
                        r.fl[j] = r.fl[j + 1];
                    }
                    --r.len;
                    break;
                }
            }
        }
        ins_added[i] = added ? 1 : 0;
    }
    for (uint32_t j = r.len; j < cap; ++j) {
        r.node[j] = DHT_NONE;
        r.fl[j] = 0;
    }
    list_len[s] = r.len;
    expired_io[s] = expired ? 1 : 0;
}

// RoutingTable::depth (src/routing_table.cpp:100-107) and InfoHash::lowbit (infohash.h:132-143)
// of every bucket of a table snapshot: lowbit = MSB-first index of the lowest set bit (-1 if 0),
// depth[b] = max(lowbit(first[b]), lowbit(first[b + 1])) + 1
__device__ __forceinline__ int lowbit_words(const uint32_t* w) {
    for (int j = DHT_W - 1; j >= 0; --j)
        if (w[j]) return 32 * j + 31 - (int)__builtin_ctz(w[j]);
    return -1;
}

__global__ __launch_bounds__(256) void k_table_stats(const uint32_t* __restrict__ fp, uint32_t nb,
                                                     int32_t* __restrict__ out_lowbit, uint32_t* __restrict__ out_depth) {
    const uint32_t b = blockIdx.x * 256 + threadIdx.x;
    if (b >= nb) return;
    uint32_t w[DHT_W];
    for (int j = 0; j < DHT_W; ++j) w[j] = fp[(uint64_t)j * nb + b];
    const int lb = lowbit_words(w);
    int lb2 = -1;
    if (b + 1 < nb) {
        for (int j = 0; j < DHT_W; ++j) w[j] = fp[(uint64_t)j * nb + b + 1];
        lb2 = lowbit_words(w);
    }
    out_lowbit[b] = lb;
    out_depth[b] = (uint32_t)((lb > lb2 ? lb : lb2) + 1);
}

}  // namespace

hipError_t launch_search_insert(const uint32_t* planes, uint64_t stride, const uint8_t* st, const uint32_t* tp,
                                uint64_t ts, uint32_t q, uint32_t cap, uint32_t* list_node, uint8_t* list_flags,
                                uint32_t* list_len, uint8_t* expired, const uint64_t* ins_off, const uint32_t* ins_node,
                                const uint8_t* ins_token, uint8_t* ins_added, uint32_t* overflow, hipStream_t s) {
    if (!q) return hipSuccess;
    k_search_insert<<<(q + 255) / 256, 256, 0, s>>>(planes, stride, st, tp, ts, q, cap, list_node, list_flags, list_len,
                                                    expired, ins_off, ins_node, ins_token, ins_added, overflow);
    return hipGetLastError();
}

hipError_t launch_table_stats(const uint32_t* fp, uint32_t nb, int32_t* out_lowbit, uint32_t* out_depth, hipStream_t s) {
    if (!nb) return hipSuccess;
    k_table_stats<<<(nb + 255) / 256, 256, 0, s>>>(fp, nb, out_lowbit, out_depth);
    return hipGetLastError();
}

}  // namespace dhtgpu
