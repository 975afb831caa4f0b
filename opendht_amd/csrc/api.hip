// api.hip -- the libdhtgpu C ABI (include/dhtgpu.h).  Owns device buffers and the
// stream; converts between the boundary's 20-byte big-endian ids and the device
// word-plane layout; never throws across the ABI.
#include <hip/hip_runtime.h>
#include <cstdio>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/dhtgpu.h"
#include "dhtgpu_internal.h"

using namespace dhtgpu;

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipMalloc(&p, bytes ? bytes : 16);
        if (e == hipSuccess) cap = bytes;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

int map_err(hipError_t e) {
    if (e == hipSuccess) return DHTGPU_OK;
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) return DHTGPU_ENOMEM;
    return DHTGPU_EDEVICE;
}

// DHTGPU_VERBOSE: name the failing HIP call on stderr (diagnostics; read once)
bool verbose() {
    static const bool v = getenv("DHTGPU_VERBOSE") != nullptr;
    return v;
}

#define DHT_TRY(expr)                                                                                  \
    do {                                                                                               \
        hipError_t _e = (expr);                                                                        \
        if (_e != hipSuccess) {                                                                        \
            if (verbose()) fprintf(stderr, "dhtgpu: %s at %s:%d: %s\n", hipGetErrorString(_e), __FILE__, __LINE__, #expr); \
            return map_err(_e);                                                                        \
        }                                                                                              \
    } while (0)

uint32_t pad_q(uint32_t q) { return (q + 63) & ~63u; }
inline size_t al256(size_t b) { return (b + 255) & ~size_t(255); }

}  // namespace

struct dhtgpu_ctx {
    int device = 0;
    int num_cus = 256;
    hipStream_t stream = nullptr;
    DevBuf planes;          // 5 * stride u32
    uint64_t n = 0, stride = 0;
    bool sorted = false;
    DevBuf staging;         // host<->device byte staging
    DevBuf targets;         // 5 * tstride u32
    DevBuf out_idx, out_cnt, rec, aux, aux2, aux3;
    bool has_ids = false;
    DevBuf gidx;            // shard -> global index map (dhtgpu_gen_ids_prefix), else unused
    bool has_gidx = false;
    bool map_global = true;  // prefix shard results: global stream indices (else shard-local)
    const uint32_t* out_map() const { return has_gidx && map_global ? gidx.as<uint32_t>() : nullptr; }
    uint32_t shard_pbits = 0;   // prefix shard: every id shares its top shard_pbits bits
    DevBuf w0s;                 // prefix shard: word 0 shifted left by shard_pbits (stride u32)
    DevBuf index;           // K4 workspace: entries | directory | partition scratch
    uint32_t index_B = 0;
    bool index_valid = false;
    DevBuf wire;            // wire-format staging (tails, candidates, blobs)
    DevBuf net_sorted;      // crawl model: {w0, index} in node order (index rebuilt by net_prepare)
    DevBuf net_dead;        // crawl model: dead mask (n bytes) or empty
    DevBuf net_io;          // crawl model: search-batch staging
    uint64_t net_seed = 0;
    bool net_valid = false, net_has_dead = false;
    // K6 workspaces: kBatchDepth slots used round-robin, so that up to kBatchDepth calls issued
    // on different streams run concurrently (one batch's latency-bound F3/F4 overlaps the next
    // batch's HBM-bound F2).  A call on a slot last used on another stream first waits for
    // that stream's work so far (an event recorded there at switch time, so calls that stay on
    // one stream pay nothing); calls on one stream keep plain stream order.
    struct BatchSlot {
        DevBuf ws;              // workspace; its zero-between-calls head (bitmap, counters) stays clean
        DevBuf out_idx, out_cnt;   // record mode: local results before the record conversion
        DevBuf sws;             // small-batch path workspace (zero between calls once cleaned)
        size_t zeroed = 0;      // leading workspace bytes known zero (the last call's clean head) ...
        size_t ctr_off = 0;     // ... but for the statistics words at this offset (batch_ctr_offset)
        uint64_t desc_sig = 0;  // sub-partition descriptors held by the workspace (launch_batch_topk)
        bool sclean = false;
        uint32_t spar = 0;      // small-batch path: the counter set its next call uses
        hipEvent_t done = nullptr;
        hipStream_t last = nullptr;
    };
    static constexpr int kBatchDepth = 4;
    BatchSlot bslot[kBatchDepth];
    // fallback-list length of the context's last completed K6 call, written by F4 into mapped
    // host memory (a hint read without any sync: it sizes the next call's fallback-scan grid)
    uint32_t* fb_hint = nullptr;
    uint32_t* fb_hint_dev = nullptr;
    int bnext = 0, blast = 0;
    bool last_small = false;   // the last K6-API call took the small-batch path
    uint64_t last_n = 0;       // ... else its plan: largest sub-partition, planned targets, sub-partitions
    uint32_t last_qp = 0, last_nsub = 1;
    uint32_t last_pf = 0;
    // Prefix sub-partitions of a large id set (built on the first K6 call K6 cannot plan in
    // one piece, e.g. the 2^27-id cfg-3 shard): the ids whose next sub_bits bits (after the
    // shard's own prefix) equal i, compacted in order, with their shifted word-0 plane; one K6
    // launch sequence then serves all of them.
    struct SubPart {
        DevBuf planes, map, gmap, w0s;   // planes: 5 * stride u32; map: sub -> ctx-local; gmap: sub -> global
        uint64_t n = 0, stride = 0;
        uint32_t span[32] = {};          // launch_cell_spans of w0s (host copy): F2's window bound
    };
    std::vector<SubPart> subs;
    std::vector<uint32_t> spans;   // [subs][32] the sub-partitions' span tables (BatchCall::spans)
    DevBuf cells;            // [subs][1 << cell_level()] u8 id counts per level-cell_level() prefix (F1's sibling rule)
    DevBuf hinv;             // [n] context-local index -> sub-partition handle
    uint32_t sub_bits = 0;
    bool subs_valid = false;
    bool subs_sorted = false;   // the sub-partitions are sorted by prefix (decided by the call that built them)
    // dhtgpu_set_sub_handles: sub-partitioned calls return handles (a sub-partition's offset +
    // its compacted index), no index-map read per result; sub_tab maps them back on request
    bool sub_handles = false;
    DevBuf sub_tab;   // HandleSub[subs.size()], built with the sub-partitions
    uint32_t shard_pval = 0;
    // lexicographically sorted views (sort.hip): of the main set when it was uploaded unsorted
    // (built on the first cached_nodes call), and the NodeCache mirror (dhtgpu_cache_set)
    struct SortedSet {
        DevBuf planes, perm;
        uint64_t n = 0, stride = 0;
        bool valid = false, unique = true;
    };
    SortedSet sview, cache;
    uint64_t cache_version = 0;
    DevBuf cache_in, sort_scratch, cache_acc;
    DevBuf srch;            // search_insert / table_stats staging
    // diagnostics: DHTGPU_DBG, the library's one diagnostics switch, read once at creation and
    // masked to kDbgAllowed -- bit 256: per-block phase stamps of F2 / F3 printed to stderr;
    // bit 2^23: K6 instead of KS for batches of <= 64 targets (both exact).  Neither changes a
    // result; every other bit is ignored (the result-altering measurement ablations of earlier
    // rounds are not in this library: DESIGN.md §5d)
    uint32_t dbg = 0;
    uint32_t search_alpha = 4;   // crawl model: requests per search round (MAX_REQUESTED_SEARCH_NODES)
    hipEvent_t next_ev[8] = {};   // dhtgpu_batch_events: the next K6 call records its kernels here
    bool has_next_ev = false;
    DevBuf stamps;

    hipError_t bind() { return hipSetDevice(device); }
    void invalidate_subs() {
        subs_valid = false;
        if (fb_hint) *fb_hint = 1u;   // a new set or split: the next call's list length is unknown
        for (auto& sp : subs)
            for (DevBuf* b : {&sp.planes, &sp.map, &sp.gmap, &sp.w0s}) b->release();
        subs.clear();
        sub_tab.release();
        cells.release();
        hinv.release();
        sub_bits = 0;
    }

    // upload q targets (20-byte big-endian, host) into target planes; returns stride
    hipError_t upload_targets(const uint8_t* t20, uint32_t q, uint64_t* ts) {
        const uint64_t s = pad_q(q);
        hipError_t e = staging.ensure((size_t)q * 20);
        if (e != hipSuccess) return e;
        if ((e = targets.ensure((size_t)s * 5 * 4)) != hipSuccess) return e;
        if ((e = hipMemcpyAsync(staging.p, t20, (size_t)q * 20, hipMemcpyHostToDevice, stream)) != hipSuccess) return e;
        if ((e = launch_pack(staging.as<uint8_t>(), q, targets.as<uint32_t>(), s, stream)) != hipSuccess) return e;
        *ts = s;
        return hipSuccess;
    }
};

extern "C" {

const char* dhtgpu_strerror(int code) {
    switch (code) {
        case DHTGPU_OK: return "ok";
        case DHTGPU_EINVAL: return "invalid argument";
        case DHTGPU_ENOMEM: return "device out of memory";
        case DHTGPU_EDEVICE: return "HIP device or kernel error";
        case DHTGPU_ENOIDS: return "no id set uploaded";
        case DHTGPU_EUNSORTED: return "id set holds duplicate ids (NodeCache keys are unique)";
        case DHTGPU_ERANGE: return "size out of range";
        default: return "unknown error";
    }
}

int dhtgpu_device_count(int* out) {
    if (!out) return DHTGPU_EINVAL;
    *out = 0;
    DHT_TRY(hipGetDeviceCount(out));
    return DHTGPU_OK;
}

int dhtgpu_ctx_create(int device, dhtgpu_ctx** out) {
    if (!out) return DHTGPU_EINVAL;
    *out = nullptr;
    int nd = 0;
    DHT_TRY(hipGetDeviceCount(&nd));
    if (device < 0 || device >= nd) return DHTGPU_EINVAL;
    auto* c = new (std::nothrow) dhtgpu_ctx;
    if (!c) return DHTGPU_ENOMEM;
    c->device = device;
    hipError_t e = c->bind();
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (const char* d = getenv("DHTGPU_DBG")) c->dbg = (uint32_t)strtoul(d, nullptr, 0) & kDbgAllowed;
    if (e == hipSuccess) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->num_cus = prop.multiProcessorCount;
    }
    if (e == hipSuccess) {   // F4's fallback-list hint: mapped, coherent host memory (F4 stores it system-scope)
        void* h = nullptr;
        e = hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent);
        if (e == hipSuccess) {
            c->fb_hint = static_cast<uint32_t*>(h);
            *c->fb_hint = 1u;   // unknown: assume a fallback list (full-size grid)
            void* d = nullptr;
            e = hipHostGetDevicePointer(&d, h, 0);
            c->fb_hint_dev = static_cast<uint32_t*>(d);
        }
    }
    if (e != hipSuccess) {
        dhtgpu_ctx_destroy(c);
        return map_err(e);
    }
    *out = c;
    return DHTGPU_OK;
}

void dhtgpu_ctx_destroy(dhtgpu_ctx* c) {
    if (!c) return;
    (void)c->bind();
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (auto& b : c->bslot) {   // slots last used on other streams: let that work finish
        if (b.last && b.last != c->stream) (void)hipStreamSynchronize(b.last);
        if (b.done) (void)hipEventDestroy(b.done);
    }
    for (DevBuf* b : {&c->planes, &c->staging, &c->targets, &c->out_idx, &c->out_cnt, &c->rec,
                      &c->aux, &c->aux2, &c->aux3, &c->index, &c->gidx, &c->wire,
                      &c->net_sorted, &c->net_dead, &c->net_io})
        b->release();
    for (auto& b : c->bslot)
        for (DevBuf* d : {&b.ws, &b.out_idx, &b.out_cnt, &b.sws}) d->release();
    c->invalidate_subs();
    if (c->fb_hint) (void)hipHostFree(c->fb_hint);
    for (DevBuf* b : {&c->stamps, &c->w0s, &c->sview.planes, &c->sview.perm,
                      &c->cache.planes, &c->cache.perm, &c->cache_in, &c->sort_scratch, &c->cache_acc, &c->srch})
        b->release();
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

void* dhtgpu_ctx_stream(dhtgpu_ctx* c) { return c ? (void*)c->stream : nullptr; }

uint64_t dhtgpu_num_ids(const dhtgpu_ctx* c) { return c && c->has_ids ? c->n : 0; }

static int finish_ids(dhtgpu_ctx* c, uint64_t n) {
    // zero the padding so tile streaming reads deterministic words
    const uint64_t s = c->stride;
    for (int w = 0; w < 5; ++w)
        DHT_TRY(launch_fill(c->planes.as<uint32_t>() + (uint64_t)w * s + n, s - n, 0u, c->stream));
    DHT_TRY(c->aux.ensure(16));
    DHT_TRY(hipMemsetAsync(c->aux.p, 0, 4, c->stream));
    DHT_TRY(launch_check_sorted(c->planes.as<uint32_t>(), s, n, c->aux.as<uint32_t>(), c->stream));
    uint32_t flag = 0;
    DHT_TRY(hipMemcpyAsync(&flag, c->aux.p, 4, hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipStreamSynchronize(c->stream));
    c->n = n;
    c->sorted = flag == 0;
    c->has_ids = true;
    return DHTGPU_OK;
}

static int alloc_ids(dhtgpu_ctx* c, uint64_t n) {
    if (n >= 0xFFFFFFFFull) return DHTGPU_ERANGE;
    c->has_ids = false;
    c->index_valid = false;
    c->net_valid = false;
    c->shard_pbits = 0;
    c->shard_pval = 0;
    c->has_gidx = false;
    c->invalidate_subs();
    c->sview.valid = false;
    c->stride = pad_ids(n ? n : 1);
    DHT_TRY(c->planes.ensure((size_t)c->stride * 5 * 4));
    return DHTGPU_OK;
}

int dhtgpu_set_ids(dhtgpu_ctx* c, const uint8_t* ids20, uint64_t n) {
    if (!c || (!ids20 && n)) return DHTGPU_EINVAL;
    DHT_TRY(c->bind());
    int r = alloc_ids(c, n);
    if (r) return r;
    const uint64_t chunk = 1ull << 22;   // 80 MB of staging at a time
    DHT_TRY(c->staging.ensure((size_t)std::min<uint64_t>(n ? n : 1, chunk) * 20));
    for (uint64_t i = 0; i < n; i += chunk) {
        const uint64_t m = std::min(chunk, n - i);
        DHT_TRY(hipMemcpyAsync(c->staging.p, ids20 + i * 20, (size_t)m * 20, hipMemcpyHostToDevice, c->stream));
        DHT_TRY(launch_pack(c->staging.as<uint8_t>(), m, c->planes.as<uint32_t>() + i, c->stride, c->stream));
        DHT_TRY(hipStreamSynchronize(c->stream));   // staging is reused
    }
    return finish_ids(c, n);
}

int dhtgpu_gen_ids(dhtgpu_ctx* c, uint64_t seed, uint64_t start, uint64_t n) {
    if (!c) return DHTGPU_EINVAL;
    DHT_TRY(c->bind());
    int r = alloc_ids(c, n);
    if (r) return r;
    DHT_TRY(launch_gen(seed, start, n, c->planes.as<uint32_t>(), c->stride, c->stream));
    return finish_ids(c, n);
}

int dhtgpu_gen_ids_prefix(dhtgpu_ctx* c, uint64_t seed, uint64_t start, uint64_t n, uint32_t pbits,
                          uint32_t pval) {
    if (!c || pbits > 16 || (pbits < 32 && pval >= (1u << pbits))) return DHTGPU_EINVAL;
    if (n >= 0xFFFFFFFFull || start + n > 0xFFFFFFFFull) return DHTGPU_ERANGE;
    DHT_TRY(c->bind());
    // the whole stream is generated into scratch, then the shard is compacted in order
    const uint64_t gs = pad_ids(n ? n : 1);
    DHT_TRY(c->staging.ensure((size_t)gs * 5 * 4));
    uint32_t* gen = c->staging.as<uint32_t>();
    DHT_TRY(launch_gen(seed, start, n, gen, gs, c->stream));
    DHT_TRY(c->aux.ensure((size_t)select_scratch_words(n) * 4 + 16));
    unsigned long long* d_total = reinterpret_cast<unsigned long long*>(c->aux.as<uint8_t>());
    uint32_t* scratch = reinterpret_cast<uint32_t*>(c->aux.as<uint8_t>() + 8);
    DHT_TRY(launch_select_prefix(gen, gs, n, pbits, pval, scratch, d_total, nullptr, 0, nullptr, 0, c->stream));
    unsigned long long m = 0;
    DHT_TRY(hipMemcpyAsync(&m, d_total, 8, hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipStreamSynchronize(c->stream));
    int r = alloc_ids(c, m);
    if (r) return r;
    DHT_TRY(c->gidx.ensure((size_t)(m ? m : 1) * 4));
    DHT_TRY(launch_select_prefix(gen, gs, n, pbits, pval, scratch, d_total, c->planes.as<uint32_t>(), c->stride,
                                 c->gidx.as<uint32_t>(), start, c->stream));
    r = finish_ids(c, m);
    if (r) return r;
    // the generation scratch (20 B per id of the whole stream) is not kept: a device may
    // hold several shard contexts of one large stream
    DHT_TRY(hipStreamSynchronize(c->stream));
    if (c->staging.cap > ((size_t)1 << 28)) c->staging.release();
    if (c->aux.cap > ((size_t)1 << 28)) c->aux.release();
    c->has_gidx = true;
    if (pbits) {
        DHT_TRY(c->w0s.ensure((size_t)c->stride * 4));
        DHT_TRY(launch_shift_w0(c->planes.as<uint32_t>(), c->stride, pbits, c->w0s.as<uint32_t>(), c->stream));
        c->shard_pbits = pbits;
        c->shard_pval = pval;
    }
    return DHTGPU_OK;
}

int dhtgpu_set_global_indices(dhtgpu_ctx* c, int on) {
    if (!c) return DHTGPU_EINVAL;
    c->map_global = on != 0;
    return DHTGPU_OK;
}

int dhtgpu_set_sub_handles(dhtgpu_ctx* c, int on) {
    if (!c) return DHTGPU_EINVAL;
    c->sub_handles = on != 0;
    return DHTGPU_OK;
}

static bool needs_subs(const dhtgpu_ctx* c, uint32_t q, uint32_t k);

// measurement only (not in include/): the phase-stamp buffer of DHTGPU_DBG=256 runs
int dhtgpu_debug_stamps(dhtgpu_ctx* c, void** dev_ptr, uint64_t* bytes) {
    if (!c || !dev_ptr || !bytes) return DHTGPU_EINVAL;
    *dev_ptr = c->stamps.p;
    *bytes = c->stamps.cap;
    return 0;
}

int dhtgpu_sub_handles_active(dhtgpu_ctx* c, uint32_t q, uint32_t k) {
    if (!c || !c->has_ids) return 0;
    return c->sub_handles && !(small_supported(c->n, q, k) && !(c->dbg & (1u << 23))) && needs_subs(c, q, k) ? 1 : 0;
}

int dhtgpu_handles_to_indices_dev(dhtgpu_ctx* c, const uint32_t* handles, uint64_t m, uint32_t* out_idx,
                                  uint32_t idx_base, void* stream) {
    if (!c || (m && (!handles || !out_idx))) return DHTGPU_EINVAL;
    if (!c->subs_valid) return DHTGPU_EINVAL;   // no sub-partitioned call has built the handle space
    if (!m) return DHTGPU_OK;
    DHT_TRY(c->bind());
    const bool global = c->has_gidx && c->map_global;
    DHT_TRY(launch_handles_to_idx(c->sub_tab.as<HandleSub>(), (uint32_t)c->subs.size(), handles, m, out_idx, global,
                                  global ? 0u : idx_base, stream ? (hipStream_t)stream : c->stream));
    return DHTGPU_OK;
}

int dhtgpu_select_prefix_dev(dhtgpu_ctx* c, const uint32_t* planes, uint64_t stride, uint64_t n, uint32_t pbits,
                             uint32_t pval, uint32_t* out_planes, uint64_t out_stride, uint32_t* out_gidx,
                             uint64_t* out_count, void* stream) {
    if (!c || !out_count || pbits > 16 || (pbits < 32 && pval >= (1u << pbits))) return DHTGPU_EINVAL;
    if (n && (!planes || !out_planes)) return DHTGPU_EINVAL;
    DHT_TRY(c->bind());
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    DHT_TRY(c->aux.ensure((size_t)select_scratch_words(n) * 4 + 16));
    unsigned long long* d_total = reinterpret_cast<unsigned long long*>(c->aux.as<uint8_t>());
    uint32_t* scratch = reinterpret_cast<uint32_t*>(c->aux.as<uint8_t>() + 8);
    DHT_TRY(launch_select_prefix(planes, stride, n, pbits, pval, scratch, d_total, nullptr, 0, nullptr, 0, s));
    unsigned long long m = 0;
    DHT_TRY(hipMemcpyAsync(&m, d_total, 8, hipMemcpyDeviceToHost, s));
    DHT_TRY(hipStreamSynchronize(s));
    if (m > out_stride) return DHTGPU_ERANGE;
    DHT_TRY(launch_select_prefix(planes, stride, n, pbits, pval, scratch, d_total, out_planes, out_stride, out_gidx,
                                 0, s));
    DHT_TRY(hipStreamSynchronize(s));
    *out_count = m;
    return DHTGPU_OK;
}

int dhtgpu_get_ids(dhtgpu_ctx* c, uint64_t first, uint64_t n, uint8_t* out20) {
    if (!c || (!out20 && n)) return DHTGPU_EINVAL;
    if (!c->has_ids) return DHTGPU_ENOIDS;
    if (first > c->n || n > c->n - first) return DHTGPU_ERANGE;
    if (!n) return DHTGPU_OK;
    DHT_TRY(c->bind());
    DHT_TRY(c->staging.ensure((size_t)n * 20));
    DHT_TRY(launch_unpack(c->planes.as<uint32_t>(), c->stride, first, n, c->staging.as<uint8_t>(), c->stream));
    DHT_TRY(hipMemcpyAsync(out20, c->staging.p, (size_t)n * 20, hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipStreamSynchronize(c->stream));
    return DHTGPU_OK;
}

int dhtgpu_ids_dev(dhtgpu_ctx* c, const uint32_t** planes, uint64_t* stride) {
    if (!c || !planes || !stride) return DHTGPU_EINVAL;
    if (!c->has_ids) return DHTGPU_ENOIDS;
    *planes = c->planes.as<uint32_t>();
    *stride = c->stride;
    return DHTGPU_OK;
}

int dhtgpu_topk_dev(dhtgpu_ctx* c, const uint32_t* tp, uint64_t ts, uint32_t q, uint32_t k,
                    uint32_t* out_idx, uint32_t* out_cnt, uint32_t* out_rec, uint32_t idx_base,
                    void* stream) {
    if (!c || k == 0 || k > DHTGPU_MAX_K || (q && !tp)) return DHTGPU_EINVAL;
    if (!out_rec && (!out_idx || !out_cnt)) return DHTGPU_EINVAL;
    if (!c->has_ids) return DHTGPU_ENOIDS;
    if (!q) return DHTGPU_OK;
    DHT_TRY(c->bind());
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    const ScanPlan p = plan_scan(c->n, q, k, c->num_cus);
    const uint32_t* gidx = c->out_map();
    const bool one = p.splits == 1 || c->n == 0;
    if (one && !out_rec) {   // one pass writes the final form directly
        DHT_TRY(launch_scan(c->planes.as<uint32_t>(), c->stride, c->n, p, tp, ts, q, k, out_idx, out_cnt, out_rec,
                            gidx, idx_base, s));
        return DHTGPU_OK;
    }
    // local indices (merged over id-range splits when the batch is too small to fill the
    // chip), then turned into candidate records or mapped to the final form
    uint32_t* li = out_idx;
    uint32_t* lc = out_cnt;
    if (out_rec) {
        DHT_TRY(c->out_idx.ensure((size_t)q * k * 4));
        DHT_TRY(c->out_cnt.ensure((size_t)q * 4));
        li = c->out_idx.as<uint32_t>();
        lc = c->out_cnt.as<uint32_t>();
    }
    if (one) {
        DHT_TRY(launch_scan(c->planes.as<uint32_t>(), c->stride, c->n, p, tp, ts, q, k, li, lc, nullptr, nullptr, 0,
                            s));
    } else {
        DHT_TRY(c->rec.ensure((size_t)p.splits * q * k * 6 * 4));
        DHT_TRY(launch_scan(c->planes.as<uint32_t>(), c->stride, c->n, p, tp, ts, q, k, nullptr, nullptr,
                            c->rec.as<uint32_t>(), nullptr, 0, s));
        DHT_TRY(launch_merge(c->rec.as<uint32_t>(), p.splits, q, k, tp, ts, k, li, lc, s));
    }
    if (out_rec)
        DHT_TRY(launch_rec3(li, (uint64_t)q * k, c->planes.as<uint32_t>(), c->stride, idx_base, gidx, out_rec, s));
    else
        DHT_TRY(launch_map_idx(li, (uint64_t)q * k, gidx, idx_base, s));
    return DHTGPU_OK;
}

int dhtgpu_merge_dev(const uint32_t* rec, uint32_t lists, uint32_t q, uint32_t k_in,
                     const uint32_t* tp, uint64_t ts, uint32_t k, uint32_t* out_idx,
                     uint32_t* out_cnt, uint32_t* ties, uint32_t tie_cap, void* stream) {
    if (!rec || !tp || !out_idx || !out_cnt || k == 0 || k > DHTGPU_MAX_K || lists == 0 || k_in == 0 ||
        k_in > DHTGPU_MAX_K)
        return DHTGPU_EINVAL;
    if (lists > DHTGPU_MAX_LISTS) return DHTGPU_ERANGE;
    if (lists > 1 && !ties) return DHTGPU_EINVAL;   // cross-list ties must be listed
    if (!q) return DHTGPU_OK;
    DHT_TRY(launch_merge3(rec, lists, q, k_in, tp, ts, k, out_idx, out_cnt, ties, tie_cap, (hipStream_t)stream));
    return DHTGPU_OK;
}

int dhtgpu_tie_words_dev(dhtgpu_ctx* c, const uint32_t* rec, uint32_t q, uint32_t k, uint32_t idx_base,
                         const uint32_t* ties, uint32_t tie_cap, uint32_t row_base, uint32_t* out_words,
                         void* stream) {
    if (!c || !rec || !out_words || k == 0 || k > DHTGPU_MAX_K) return DHTGPU_EINVAL;
    if (!c->has_ids) return DHTGPU_ENOIDS;
    if (!q) return DHTGPU_OK;
    DHT_TRY(c->bind());
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    // records name ids by global index: the prefix shard's ascending map, else idx_base + local
    const uint32_t* gmap = c->out_map();
    DHT_TRY(launch_tie_words(rec, q, k, ties, tie_cap, row_base, c->planes.as<uint32_t>(), c->stride, c->n, gmap,
                             gmap ? 0u : idx_base, out_words, s));
    return DHTGPU_OK;
}

int dhtgpu_merge_ties_dev(const uint32_t* rec, const uint32_t* words, uint32_t lists, uint32_t q, uint32_t k_in,
                          const uint32_t* tp, uint64_t ts, uint32_t k, const uint32_t* ties, uint32_t tie_cap,
                          uint32_t* out_idx, uint32_t* out_cnt, void* stream) {
    if (!rec || !words || !tp || !out_idx || !out_cnt || k == 0 || k > DHTGPU_MAX_K || lists == 0 || k_in == 0 ||
        k_in > DHTGPU_MAX_K)
        return DHTGPU_EINVAL;
    if (lists > DHTGPU_MAX_LISTS) return DHTGPU_ERANGE;
    if (!q || (ties && !tie_cap)) return DHTGPU_OK;
    DHT_TRY(launch_merge_full(rec, words, lists, q, k_in, tp, ts, k, ties, tie_cap, out_idx, out_cnt,
                              (hipStream_t)stream));
    return DHTGPU_OK;
}

int dhtgpu_pack_dev(const uint8_t* ids20, uint64_t n, uint32_t* planes, uint64_t stride, void* stream) {
    if ((!ids20 || !planes) && n) return DHTGPU_EINVAL;
    if (stride < n) return DHTGPU_EINVAL;
    DHT_TRY(launch_pack(ids20, n, planes, stride, (hipStream_t)stream));
    return DHTGPU_OK;
}

int dhtgpu_gen_dev(uint64_t seed, uint64_t start, uint64_t n, uint32_t* planes, uint64_t stride,
                   void* stream) {
    if (!planes && n) return DHTGPU_EINVAL;
    if (stride < n) return DHTGPU_EINVAL;
    DHT_TRY(launch_gen(seed, start, n, planes, stride, (hipStream_t)stream));
    return DHTGPU_OK;
}

int dhtgpu_topk(dhtgpu_ctx* c, const uint8_t* t20, uint32_t q, uint32_t k, uint32_t* out_idx,
                uint32_t* out_cnt) {
    if (!c || k == 0 || k > DHTGPU_MAX_K || (q && (!t20 || !out_idx || !out_cnt))) return DHTGPU_EINVAL;
    if (!c->has_ids) return DHTGPU_ENOIDS;
    if (!q) return DHTGPU_OK;
    DHT_TRY(c->bind());
    uint64_t ts = 0;
    DHT_TRY(c->upload_targets(t20, q, &ts));
    DHT_TRY(c->aux2.ensure((size_t)q * k * 4));
    DHT_TRY(c->aux3.ensure((size_t)q * 4));
    int r = dhtgpu_topk_dev(c, c->targets.as<uint32_t>(), ts, q, k, c->aux2.as<uint32_t>(),
                            c->aux3.as<uint32_t>(), nullptr, 0, c->stream);
    if (r) return r;
    DHT_TRY(hipMemcpyAsync(out_idx, c->aux2.p, (size_t)q * k * 4, hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipMemcpyAsync(out_cnt, c->aux3.p, (size_t)q * 4, hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipStreamSynchronize(c->stream));
    return DHTGPU_OK;
}

int dhtgpu_index_build(dhtgpu_ctx* c, void* stream) {
    if (!c) return DHTGPU_EINVAL;
    if (!c->has_ids) return DHTGPU_ENOIDS;
    DHT_TRY(c->bind());
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    const uint32_t B = index_bits(c->n);
    DHT_TRY(c->index.ensure(index_bytes(c->n, B)));
    DHT_TRY(launch_index_build(c->planes.as<uint32_t>(), c->stride, c->n, B, c->index.p, s));
    c->index_B = B;
    c->index_valid = true;
    return DHTGPU_OK;
}

int dhtgpu_index_build_timed(dhtgpu_ctx* c, void* stream, float* ms4) {
    if (!c || !ms4) return DHTGPU_EINVAL;
    if (!c->has_ids) return DHTGPU_ENOIDS;
    DHT_TRY(c->bind());
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    const uint32_t B = index_bits(c->n);
    DHT_TRY(c->index.ensure(index_bytes(c->n, B)));
    hipEvent_t ev[5];
    for (int i = 0; i < 5; ++i) DHT_TRY(hipEventCreate(&ev[i]));
    hipError_t e = launch_index_build(c->planes.as<uint32_t>(), c->stride, c->n, B, c->index.p, s, ev);
    if (e == hipSuccess) e = hipEventSynchronize(ev[4]);
    for (int i = 0; e == hipSuccess && i < 4; ++i) e = hipEventElapsedTime(&ms4[i], ev[i], ev[i + 1]);
    for (int i = 0; i < 5; ++i) (void)hipEventDestroy(ev[i]);
    DHT_TRY(e);
    c->index_B = B;
    c->index_valid = true;
    return DHTGPU_OK;
}

int dhtgpu_index_topk_dev(dhtgpu_ctx* c, const uint32_t* tp, uint64_t ts, uint32_t q, uint32_t k,
                          uint32_t* out_idx, uint32_t* out_cnt, uint32_t* out_rec, uint32_t idx_base,
                          void* stream) {
    if (!c || k == 0 || k > DHTGPU_MAX_K || (q && !tp)) return DHTGPU_EINVAL;
    if (!out_rec && (!out_idx || !out_cnt)) return DHTGPU_EINVAL;
    if (!c->has_ids || !c->index_valid) return DHTGPU_ENOIDS;
    if (!q) return DHTGPU_OK;
    DHT_TRY(c->bind());
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    const uint32_t* gidx = c->out_map();
    uint32_t* li = out_idx;
    uint32_t* lc = out_cnt;
    if (out_rec) {   // candidate records for a cross-shard merge
        DHT_TRY(c->out_idx.ensure((size_t)q * k * 4));
        DHT_TRY(c->out_cnt.ensure((size_t)q * 4));
        li = c->out_idx.as<uint32_t>();
        lc = c->out_cnt.as<uint32_t>();
    }
    DHT_TRY(launch_index_query(c->index.p, c->n, c->index_B, c->planes.as<uint32_t>(), c->stride, tp, ts, q, k,
                               li, lc, s));
    if (out_rec)
        DHT_TRY(launch_rec3(li, (uint64_t)q * k, c->planes.as<uint32_t>(), c->stride, idx_base, gidx, out_rec, s));
    else
        DHT_TRY(launch_map_idx(li, (uint64_t)q * k, gidx, idx_base, s));
    return DHTGPU_OK;
}

int dhtgpu_index_topk(dhtgpu_ctx* c, const uint8_t* t20, uint32_t q, uint32_t k, uint32_t* out_idx,
                      uint32_t* out_cnt) {
    if (!c || k == 0 || k > DHTGPU_MAX_K || (q && (!t20 || !out_idx || !out_cnt))) return DHTGPU_EINVAL;
    if (!c->has_ids) return DHTGPU_ENOIDS;
    if (!q) return DHTGPU_OK;
    DHT_TRY(c->bind());
    if (!c->index_valid) {
        int r = dhtgpu_index_build(c, c->stream);
        if (r) return r;
    }
    uint64_t ts = 0;
    DHT_TRY(c->upload_targets(t20, q, &ts));
    DHT_TRY(c->aux2.ensure((size_t)q * k * 4));
    DHT_TRY(c->aux3.ensure((size_t)q * 4));
    int r = dhtgpu_index_topk_dev(c, c->targets.as<uint32_t>(), ts, q, k, c->aux2.as<uint32_t>(),
                                  c->aux3.as<uint32_t>(), nullptr, 0, c->stream);
    if (r) return r;
    DHT_TRY(hipMemcpyAsync(out_idx, c->aux2.p, (size_t)q * k * 4, hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipMemcpyAsync(out_cnt, c->aux3.p, (size_t)q * 4, hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipStreamSynchronize(c->stream));
    return DHTGPU_OK;
}

// ---- K6 -------------------------------------------------------------------------------------
// The workspace slot for a call on stream s: the next slot (round-robin) whose last user was s
// (stream order suffices, no wait), else the next unused one, else the next in turn (which
// then waits for its last stream).  Stream-affine, so that up to kBatchDepth streams in flight
// never wait on each other (plain round-robin over 3 streams made every call wait).
static int pick_slot(dhtgpu_ctx* c, hipStream_t s) {
    constexpr int D = dhtgpu_ctx::kBatchDepth;
    int si = -1;
    for (int i = 0; i < D && si < 0; ++i)
        if (c->bslot[(c->bnext + i) % D].last == s) si = (c->bnext + i) % D;
    for (int i = 0; i < D && si < 0; ++i)
        if (!c->bslot[(c->bnext + i) % D].last) si = (c->bnext + i) % D;
    if (si < 0) si = c->bnext;
    c->bnext = (si + 1) % D;
    return si;
}

// One K6 launch sequence on workspace slot `si` (stream s): waits for the slot's previous user
// when that was another stream, cleans the workspace head when needed.
static int batch_slot_run(dhtgpu_ctx* c, int si, BatchCall bc, hipStream_t s, hipEvent_t* ev) {
    dhtgpu_ctx::BatchSlot& b = c->bslot[si];
    // a slot last used on another stream: wait for that stream's work so far (it includes the
    // slot's previous call); same stream: stream order suffices
    if (b.last && b.last != s) {
        if (!b.done) DHT_TRY(hipEventCreateWithFlags(&b.done, hipEventDisableTiming));
        DHT_TRY(hipEventRecord(b.done, b.last));
        DHT_TRY(hipStreamWaitEvent(s, b.done, 0));
    }
    uint64_t n_plan = bc.nsub ? 0 : bc.n;   // the plan is the largest sub-partition's
    for (uint32_t i = 0; i < bc.nsub; ++i) n_plan = std::max<uint64_t>(n_plan, bc.subs[i].n);
    const uint32_t nsub = bc.nsub ? bc.nsub : 1u;
    const uint32_t pf = (bc.cells ? kPlanCells : 0u) | (bc.sorted ? kPlanSorted : 0u);
    const size_t need = batch_bytes(n_plan, bc.q, bc.q_plan, bc.k, c->num_cus, nsub, pf);
    const size_t head = batch_clean_bytes(n_plan, bc.q_plan, bc.k, c->num_cus, nsub, pf);
    const size_t ctr_off = batch_ctr_offset(n_plan, bc.q_plan, bc.k, c->num_cus, nsub, pf);
    if (need > b.ws.cap) {   // reallocated: nothing of it is known
        b.zeroed = 0;
        b.desc_sig = 0;
    }
    DHT_TRY(b.ws.ensure(need));
    bc.fb_hint = c->fb_hint;
    bc.fb_hint_dev = c->fb_hint_dev;
    // the head is zero after a call but for the statistics words ctr[0..3] (F1 resets them at the
    // start of the next call): a head laid out with its counters elsewhere (another bitmap size --
    // a sub-partitioned call, then a one-set call) would meet them inside another array (a partition
    // count: stale survivors gathered by F3), so it is zeroed again
    if (b.zeroed < head || (b.zeroed && b.ctr_off != ctr_off)) DHT_TRY(hipMemsetAsync(b.ws.p, 0, head, s));
    b.zeroed = 0;   // re-established below once every launch went through
    if (bc.dbg & 256u) {   // phase stamps (zeroed when allocated)
        const bool fresh = !c->stamps.p;
        DHT_TRY(c->stamps.ensure((size_t)3 * 8192 * 16 * 8));
        if (fresh) DHT_TRY(hipMemsetAsync(c->stamps.p, 0, (size_t)3 * 8192 * 16 * 8, s));
        bc.stamps = c->stamps.as<unsigned long long>();
    }
    bc.ws = b.ws.p;
    bc.desc_sig = &b.desc_sig;
    DHT_TRY(launch_batch_topk(bc, s));
    b.last = s;
    b.zeroed = head;   // the call leaves its clean head zero (but for ctr[0..3])
    b.ctr_off = ctr_off;
    c->blast = si;
    c->last_n = n_plan;
    c->last_qp = bc.q_plan;
    c->last_nsub = nsub;
    c->last_pf = pf;
    return DHTGPU_OK;
}

// Build the prefix sub-partitions: the smallest split into 2^s parts of <= 2^24 expected ids
// (s <= 8), each compacted from the context's planes and then sorted by its ids (stable: equal
// ids keep their index order, so index ties break the same way), with its shifted word-0 plane,
// its index maps, its level-19 cell counts and the context's inverse handle map.  Prefix order
// is the layout K6 wants: an F2 workgroup's contiguous range of a sub-partition covers a narrow
// prefix range, so its survivors fall into a few partitions (long, coalesced bucket runs instead
// of a few entries in every partition) and a partition's survivors, results and result-map
// entries sit in a narrow index window (F3's gathers and record words hit lines they share).
static int build_subs(dhtgpu_ctx* c, bool sort) {
    if (c->subs_valid) return DHTGPU_OK;
    c->invalidate_subs();
    uint32_t sb = 1;
    while (sb < 8 && (c->n >> sb) > (1ull << 24)) ++sb;
    const uint32_t P = c->shard_pbits + sb;   // prefix bits every id of a sub-partition shares
    if (P > 24) return DHTGPU_ERANGE;
    hipStream_t s = c->stream;
    DHT_TRY(c->aux.ensure((size_t)select_scratch_words(c->n) * 4 + 16));
    unsigned long long* d_total = reinterpret_cast<unsigned long long*>(c->aux.as<uint8_t>());
    uint32_t* scratch = reinterpret_cast<uint32_t*>(c->aux.as<uint8_t>() + 8);
    const uint32_t* planes = c->planes.as<uint32_t>();
    c->subs.resize((size_t)1 << sb);
    for (uint32_t i = 0; i < (1u << sb); ++i) {
        const uint32_t pv = (c->shard_pval << sb) | i;
        DHT_TRY(launch_select_prefix(planes, c->stride, c->n, P, pv, scratch, d_total, nullptr, 0, nullptr, 0, s));
        unsigned long long m = 0;
        DHT_TRY(hipMemcpyAsync(&m, d_total, 8, hipMemcpyDeviceToHost, s));
        DHT_TRY(hipStreamSynchronize(s));
        dhtgpu_ctx::SubPart& sp = c->subs[i];
        sp.n = m;
        sp.stride = pad_ids(m ? m : 1);
        DHT_TRY(sp.planes.ensure((size_t)sp.stride * 5 * 4));
        DHT_TRY(sp.map.ensure((size_t)sp.stride * 4));
        DHT_TRY(sp.w0s.ensure((size_t)sp.stride * 4));
        for (int w = 0; w < 5; ++w)   // deterministic padding words (F2 may read them, masked)
            DHT_TRY(launch_fill(sp.planes.as<uint32_t>() + (uint64_t)w * sp.stride + m, sp.stride - m, 0u, s));
        DHT_TRY(launch_select_prefix(planes, c->stride, c->n, P, pv, scratch, d_total, sp.planes.as<uint32_t>(),
                                     sp.stride, sp.map.as<uint32_t>(), 0, s));
        if (sort && m > 1) {   // prefix order (stable sort of the compacted ids; perm -> context-local map)
            DevBuf sorted, perm, sscr;
            int unique = 1;
            hipError_t e = sorted.ensure((size_t)sp.stride * 5 * 4);
            if (e == hipSuccess) e = perm.ensure((size_t)m * 4);
            if (e == hipSuccess) e = sscr.ensure(sort_scratch_bytes(m));
            for (int w = 0; e == hipSuccess && w < 5; ++w)
                e = launch_fill(sorted.as<uint32_t>() + (uint64_t)w * sp.stride + m, sp.stride - m, 0u, s);
            if (e == hipSuccess)
                e = launch_sort_ids(sp.planes.as<uint32_t>(), sp.stride, m, sorted.as<uint32_t>(), sp.stride,
                                    perm.as<uint32_t>(), sscr.p, &unique, s);
            if (e == hipSuccess) e = launch_map_idx(perm.as<uint32_t>(), m, sp.map.as<uint32_t>(), 0, s);
            if (e == hipSuccess) e = hipMemcpyAsync(sp.map.p, perm.p, (size_t)m * 4, hipMemcpyDeviceToDevice, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e == hipSuccess) std::swap(sp.planes, sorted);
            sorted.release();
            perm.release();
            sscr.release();
            DHT_TRY(e);
        }
        DHT_TRY(launch_shift_w0(sp.planes.as<uint32_t>(), sp.stride, P, sp.w0s.as<uint32_t>(), s));
        if (c->has_gidx) {   // sub -> global stream index, composed once
            DHT_TRY(sp.gmap.ensure((size_t)sp.stride * 4));
            DHT_TRY(hipMemcpyAsync(sp.gmap.p, sp.map.p, (size_t)m * 4, hipMemcpyDeviceToDevice, s));
            DHT_TRY(launch_map_idx(sp.gmap.as<uint32_t>(), m, c->gidx.as<uint32_t>(), 0, s));
        }
    }
    // level-cell_level() id counts of every sub-partition (sibling marking, BatchCall::cells)
    const size_t ncell = (size_t)1 << cell_level();
    DHT_TRY(c->cells.ensure(c->subs.size() * ncell));
    {
        DevBuf cnt;   // (DevBuf frees nothing by itself: released on every path)
        hipError_t e = cnt.ensure(ncell * 4);
        for (size_t i = 0; e == hipSuccess && i < c->subs.size(); ++i)
            e = launch_cell_counts(c->subs[i].w0s.as<uint32_t>(), c->subs[i].n, cnt.as<uint32_t>(),
                                   c->cells.as<uint8_t>() + i * ncell, s);
        for (size_t i = 0; sort && e == hipSuccess && i < c->subs.size(); ++i) {   // window bounds (sorted subs)
            e = launch_cell_spans(c->subs[i].w0s.as<uint32_t>(), c->subs[i].n, cnt.as<uint32_t>(), s);
            if (e == hipSuccess) e = hipMemcpyAsync(c->subs[i].span, cnt.p, 32 * 4, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
        }
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        cnt.release();
        DHT_TRY(e);
        c->spans.assign(sort ? c->subs.size() * 32 : 0, 0u);
        for (size_t i = 0; sort && i < c->subs.size(); ++i)
            std::copy(c->subs[i].span, c->subs[i].span + 32, c->spans.begin() + i * 32);
    }
    DHT_TRY(c->hinv.ensure((size_t)(c->n ? c->n : 1) * 4));
    {
        uint64_t o = 0;
        for (const auto& sp : c->subs) {
            DHT_TRY(launch_handle_inverse(sp.map.as<uint32_t>(), sp.n, (uint32_t)o, c->hinv.as<uint32_t>(), s));
            o += sp.n;
        }
    }
    std::vector<HandleSub> tab(c->subs.size());
    uint64_t off = 0;
    for (size_t i = 0; i < tab.size(); ++i) {
        const dhtgpu_ctx::SubPart& sp = c->subs[i];
        tab[i] = HandleSub{sp.n, sp.map.as<uint32_t>(), c->has_gidx ? sp.gmap.as<uint32_t>() : nullptr, (uint32_t)off, 0u};
        off += sp.n;
    }
    DHT_TRY(c->sub_tab.ensure(tab.size() * sizeof(HandleSub)));
    DHT_TRY(hipMemcpyAsync(c->sub_tab.p, tab.data(), tab.size() * sizeof(HandleSub), hipMemcpyHostToDevice, s));
    DHT_TRY(hipStreamSynchronize(s));
    c->sub_bits = sb;
    c->subs_valid = true;
    c->subs_sorted = sort;
    return DHTGPU_OK;
}

// A K6 call over prefix sub-partitions, all of them in ONE launch sequence.  A target is
// answered from its own sub-partition (F1 routes it by the sub_bits bits after the shard
// prefix): when that holds >= k ids, every id of it is XOR-closer to the target than every id
// outside it, so its top-k is the set's.  Targets whose sub-partition is short of k ids (or
// whose partition overflowed) take F4's scan over the whole set.  A split K6 cannot plan
// (strongly clustered ids: one sub-partition far above 2^24) takes the K1 scan.
static int batch_run_subs(dhtgpu_ctx* c, const uint32_t* tp, uint64_t ts, uint32_t q, uint32_t k, uint32_t* out_idx,
                          uint32_t* out_cnt, uint32_t* out_rec, uint32_t idx_base, hipStream_t s, hipEvent_t* ev) {
    // Prefix-sorted sub-partitions: an F2 range's survivors fall into a few partitions that the
    // range owns, so F2 writes them straight to their buckets with no stage (k_f2_direct: a few KB
    // of LDS, F3 workgroups of the other call in flight beside it) and F3's reads stay inside
    // narrow index windows.  The cfg-3 broadcast rank (2^20 targets on 1.25e8 ids, ~22 % of the
    // ids survive): 1.16 -> 0.43 ms per call; the prefix rank (~3 %): 0.149 -> 0.135 ms, the
    // 2^27-id shard 0.157 -> 0.148-0.152 (profiles/r06/experiments).  Below ~2 % survivors a
    // wave's runs would be one or two entries: index order.  Decided once, by the call that
    // builds them.
    bool sort = false;
    {
        uint32_t sbe = 1;
        while (sbe < 8 && (c->n >> sbe) > (1ull << 24)) ++sbe;
        const uint64_t nsub_e = c->n >> sbe;
        const double qsub = (double)q / (double)(1u << sbe);
        uint32_t lm = 0;
        while (lm < 19 && (nsub_e >> (lm + 1)) >= 4ull * k) ++lm;
        lm = lm + 1 < 19 ? lm + 1 : 19;
        sort = 1.0 - std::exp(-qsub / (double)(1ull << lm)) > 0.02;
    }
    int r = build_subs(c, sort);
    if (r) return r;
    const uint32_t sb = c->sub_bits, S = 1u << sb;
    const uint32_t pf = kPlanCells | (c->subs_sorted ? kPlanSorted : 0u);
    const uint32_t P = c->shard_pbits + sb;
    const uint32_t q_plan = std::max<uint32_t>(1u, (uint32_t)(((uint64_t)q + S - 1) >> sb));
    uint64_t n_max = 0;
    for (const auto& sp : c->subs) n_max = std::max<uint64_t>(n_max, sp.n);
    const bool handles = c->sub_handles && !out_rec;
    if (!batch_supported(n_max, q_plan, k, c->num_cus, S, pf)) {
        if (!handles) return dhtgpu_topk_dev(c, tp, ts, q, k, out_idx, out_cnt, out_rec, idx_base, s);
        // handles on the K1 route: context-local indices, then their handles
        const bool mg = c->map_global;
        c->map_global = false;
        r = dhtgpu_topk_dev(c, tp, ts, q, k, out_idx, out_cnt, nullptr, 0, s);
        c->map_global = mg;
        if (r) return r;
        DHT_TRY(launch_idx_to_handles(c->hinv.as<uint32_t>(), out_idx, (uint64_t)q * k, s));
        return DHTGPU_OK;
    }
    const bool global = !handles && c->has_gidx && c->map_global && !out_rec;
    const int si = pick_slot(c, s);
    dhtgpu_ctx::BatchSlot& b = c->bslot[si];
    // record form: the index rows are scratch (K6 stores the records themselves)
    uint32_t* li = out_idx;
    uint32_t* lc = out_cnt;
    if (out_rec) {
        DHT_TRY(b.out_idx.ensure((size_t)q * k * 4));
        DHT_TRY(b.out_cnt.ensure((size_t)q * 4));
        li = b.out_idx.as<uint32_t>();
        lc = b.out_cnt.as<uint32_t>();
    }
    std::vector<SubSpec> specs(S);
    uint64_t off = 0;
    for (uint32_t i = 0; i < S; ++i) {
        const dhtgpu_ctx::SubPart& sp = c->subs[i];
        specs[i] = SubSpec{sp.planes.as<uint32_t>(), sp.w0s.as<uint32_t>(), sp.stride, sp.n,
                           handles ? nullptr : global ? sp.gmap.as<uint32_t>() : sp.map.as<uint32_t>(),
                           handles ? (uint32_t)off : 0u};
        off += sp.n;
    }
    BatchCall bc{};
    bc.planes = c->planes.as<uint32_t>();   // F4's scan: the whole set
    bc.stride = c->stride;
    bc.n = c->n;
    bc.tp = tp;
    bc.ts = ts;
    bc.q = q;
    bc.q_plan = q_plan;
    bc.k = k;
    bc.skip = P;
    bc.pval = c->shard_pval;
    bc.cells = c->cells.as<uint8_t>();
    bc.spans = c->spans.empty() ? nullptr : c->spans.data();
    bc.sorted = c->subs_sorted ? 1u : 0u;
    bc.gidx = global ? c->gidx.as<uint32_t>() : nullptr;
    bc.base = 0;
    bc.out_idx = li;
    bc.out_cnt = lc;
    bc.num_cus = c->num_cus;
    bc.dbg = c->dbg;
    bc.ev = ev;
    bc.subs = specs.data();
    bc.nsub = S;
    bc.sub_shift = c->shard_pbits;
    bc.sub_bits = sb;
    bc.out_rec = out_rec;   // every K6 writer of a row stores its records
    bc.rec_gidx = c->out_map();
    bc.rec_base = idx_base;
    bc.handles = handles ? 1u : 0u;
    bc.htab = c->sub_tab.as<HandleSub>();
    bc.hinv = c->hinv.as<uint32_t>();
    if (handles) bc.base = kHandleMark;   // whole-set fallback rows, marked for the pass after F4
    r = batch_slot_run(c, si, bc, s, ev);
    if (r) return r;
    if (!out_rec && !handles && !global && idx_base) {   // (record form: K6 wrote the records)
        DHT_TRY(launch_map_idx(out_idx, (uint64_t)q * k, nullptr, idx_base, s));
    }
    return DHTGPU_OK;
}

// Batches of at most 64 targets: one pass over word 0 + one workgroup per target prefix (KS).
static int small_run(dhtgpu_ctx* c, const uint32_t* tp, uint64_t ts, uint32_t q, uint32_t k, uint32_t* out_idx,
                     uint32_t* out_cnt, uint32_t* out_rec, uint32_t idx_base, hipStream_t s, hipEvent_t* ev) {
    const int si = pick_slot(c, s);
    dhtgpu_ctx::BatchSlot& b = c->bslot[si];
    if (b.last && b.last != s) {   // the slot's previous user on another stream
        if (!b.done) DHT_TRY(hipEventCreateWithFlags(&b.done, hipEventDisableTiming));
        DHT_TRY(hipEventRecord(b.done, b.last));
        DHT_TRY(hipStreamWaitEvent(s, b.done, 0));
    }
    if (b.sws.cap < small_bytes()) b.sclean = false;
    DHT_TRY(b.sws.ensure(small_bytes()));
    if (!b.sclean) {
        DHT_TRY(hipMemsetAsync(b.sws.p, 0, small_bytes(), s));
        b.spar = 0;
    }
    b.sclean = true;   // the kernels leave it zero
    const uint32_t* gidx = c->out_map();
    uint32_t* li = out_idx;
    uint32_t* lc = out_cnt;
    if (out_rec) {
        DHT_TRY(b.out_idx.ensure((size_t)q * k * 4));
        DHT_TRY(b.out_cnt.ensure((size_t)q * 4));
        li = b.out_idx.as<uint32_t>();
        lc = b.out_cnt.as<uint32_t>();
    }
    BatchCall bc{};
    bc.planes = c->planes.as<uint32_t>();
    bc.stride = c->stride;
    bc.n = c->n;
    bc.tp = tp;
    bc.ts = ts;
    bc.q = q;
    bc.q_plan = q;
    bc.k = k;
    bc.skip = c->shard_pbits;
    bc.w0s = c->shard_pbits ? c->w0s.as<uint32_t>() : nullptr;
    bc.gidx = out_rec ? nullptr : gidx;
    bc.base = out_rec ? 0u : idx_base;
    bc.out_idx = li;
    bc.out_cnt = lc;
    bc.num_cus = c->num_cus;
    bc.ev = ev;
    if (hipError_t e = launch_small_topk(bc, b.sws.p, b.spar, s)) {
        b.sclean = false;   // S1 may have counted into this call's set: the next call re-zeroes it all
        return map_err(e);
    }
    b.spar ^= 1u;
    b.last = s;
    c->last_small = true;
    if (out_rec)
        DHT_TRY(launch_rec3(li, (uint64_t)q * k, c->planes.as<uint32_t>(), c->stride, idx_base, gidx, out_rec, s));
    return DHTGPU_OK;
}

static bool needs_subs(const dhtgpu_ctx* c, uint32_t q, uint32_t k) {
    return c->n > (1ull << 24) && !batch_supported(c->n, q, k, c->num_cus) && q <= (1u << 22);
}

static int batch_run(dhtgpu_ctx* c, const uint32_t* tp, uint64_t ts, uint32_t q, uint32_t k, uint32_t* out_idx,
                     uint32_t* out_cnt, uint32_t* out_rec, uint32_t idx_base, hipStream_t s, hipEvent_t* ev) {
    hipEvent_t evs[8];
    if (!ev && c->has_next_ev) {   // armed by dhtgpu_batch_events: this call only
        for (int i = 0; i < 8; ++i) evs[i] = c->next_ev[i];
        c->has_next_ev = false;
        ev = evs;
    }
    // DHTGPU_DBG bit 2^23: K6 for small batches too (comparison runs; the same exact results)
    if (small_supported(c->n, q, k) && !(c->dbg & (1u << 23)))
        return small_run(c, tp, ts, q, k, out_idx, out_cnt, out_rec, idx_base, s, ev);
    c->last_small = false;
    if (needs_subs(c, q, k)) return batch_run_subs(c, tp, ts, q, k, out_idx, out_cnt, out_rec, idx_base, s, ev);
    if (!batch_supported(c->n, q, k, c->num_cus)) return DHTGPU_ERANGE;
    const int si = pick_slot(c, s);
    dhtgpu_ctx::BatchSlot& b = c->bslot[si];
    const uint32_t* gidx = c->out_map();
    uint32_t* li = out_idx;
    uint32_t* lc = out_cnt;
    if (out_rec) {   // record form: the index rows are scratch (K6 stores the records themselves)
        DHT_TRY(b.out_idx.ensure((size_t)q * k * 4));
        DHT_TRY(b.out_cnt.ensure((size_t)q * 4));
        li = b.out_idx.as<uint32_t>();
        lc = b.out_cnt.as<uint32_t>();
    }
    BatchCall bc{};
    bc.planes = c->planes.as<uint32_t>();
    bc.stride = c->stride;
    bc.n = c->n;
    bc.tp = tp;
    bc.ts = ts;
    bc.q = q;
    bc.q_plan = q;
    bc.k = k;
    bc.skip = c->shard_pbits;
    bc.pval = c->shard_pval;
    bc.w0s = c->shard_pbits ? c->w0s.as<uint32_t>() : nullptr;
    bc.gidx = out_rec ? nullptr : gidx;
    bc.base = out_rec ? 0u : idx_base;
    bc.out_idx = li;
    bc.out_cnt = lc;
    bc.num_cus = c->num_cus;
    bc.dbg = c->dbg;
    bc.ev = ev;
    bc.out_rec = out_rec;   // every K6 writer of a row stores its records
    bc.rec_gidx = gidx;
    bc.rec_base = idx_base;
    return batch_slot_run(c, si, bc, s, ev);   // (record form: K6 writes the records itself)
}

int dhtgpu_batch_topk_dev(dhtgpu_ctx* c, const uint32_t* tp, uint64_t ts, uint32_t q, uint32_t k,
                          uint32_t* out_idx, uint32_t* out_cnt, uint32_t* out_rec, uint32_t idx_base,
                          void* stream) {
    if (!c || k == 0 || k > DHTGPU_MAX_K || (q && !tp)) return DHTGPU_EINVAL;
    if (!out_rec && (!out_idx || !out_cnt)) return DHTGPU_EINVAL;
    if (!c->has_ids) return DHTGPU_ENOIDS;
    if (!q) return DHTGPU_OK;
    DHT_TRY(c->bind());
    return batch_run(c, tp, ts, q, k, out_idx, out_cnt, out_rec, idx_base,
                     stream ? (hipStream_t)stream : c->stream, nullptr);
}

int dhtgpu_batch_events(dhtgpu_ctx* c, void** ev8) {
    if (!c || !ev8) return DHTGPU_EINVAL;
    for (int i = 0; i < 8; ++i) {
        if (!ev8[i]) return DHTGPU_EINVAL;
        c->next_ev[i] = (hipEvent_t)ev8[i];
    }
    c->has_next_ev = true;
    return DHTGPU_OK;
}

int dhtgpu_batch_topk_timed(dhtgpu_ctx* c, const uint32_t* tp, uint64_t ts, uint32_t q, uint32_t k,
                            uint32_t* out_idx, uint32_t* out_cnt, void* stream, float* ms4, uint32_t* stats4) {
    if (!c || !ms4 || k == 0 || k > DHTGPU_MAX_K || !q || !tp || !out_idx || !out_cnt) return DHTGPU_EINVAL;
    if (!c->has_ids) return DHTGPU_ENOIDS;
    DHT_TRY(c->bind());
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    hipEvent_t ev[8];   // start/stop per kernel, recorded by the kernels' own dispatches
    for (int i = 0; i < 8; ++i) DHT_TRY(hipEventCreate(&ev[i]));
    int r = batch_run(c, tp, ts, q, k, out_idx, out_cnt, nullptr, 0, s, ev);
    hipError_t e = r ? hipSuccess : hipStreamSynchronize(s);
    if (!r && e == hipSuccess) e = hipEventSynchronize(ev[7]);
    for (int i = 0; !r && e == hipSuccess && i < 4; ++i) e = hipEventElapsedTime(&ms4[i], ev[2 * i], ev[2 * i + 1]);
    for (int i = 0; i < 8; ++i) (void)hipEventDestroy(ev[i]);
    if (r) return r;
    DHT_TRY(e);
    if (stats4 && c->last_small) {   // the small-batch path keeps no statistics
        for (int i = 0; i < 4; ++i) stats4[i] = 0;
    } else if (stats4) {
        DHT_TRY(batch_read_stats(c->bslot[c->blast].ws.p, c->last_n, q, c->last_qp, k, c->num_cus, stats4, s,
                                 c->last_nsub, c->last_pf));
    }
    return DHTGPU_OK;
}

int dhtgpu_batch_topk(dhtgpu_ctx* c, const uint8_t* t20, uint32_t q, uint32_t k, uint32_t* out_idx,
                      uint32_t* out_cnt) {
    if (!c || k == 0 || k > DHTGPU_MAX_K || (q && (!t20 || !out_idx || !out_cnt))) return DHTGPU_EINVAL;
    if (!c->has_ids) return DHTGPU_ENOIDS;
    if (!q) return DHTGPU_OK;
    DHT_TRY(c->bind());
    uint64_t ts = 0;
    DHT_TRY(c->upload_targets(t20, q, &ts));
    DHT_TRY(c->aux2.ensure((size_t)q * k * 4));
    DHT_TRY(c->aux3.ensure((size_t)q * 4));
    int r = batch_run(c, c->targets.as<uint32_t>(), ts, q, k, c->aux2.as<uint32_t>(), c->aux3.as<uint32_t>(),
                      nullptr, 0, c->stream, nullptr);
    if (r) return r;
    DHT_TRY(hipMemcpyAsync(out_idx, c->aux2.p, (size_t)q * k * 4, hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipMemcpyAsync(out_cnt, c->aux3.p, (size_t)q * 4, hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipStreamSynchronize(c->stream));
    return DHTGPU_OK;
}

int dhtgpu_find_closest(dhtgpu_ctx* c, uint32_t nb, const uint8_t* firsts20, const uint32_t* off,
                        const uint8_t* node_ids20, const uint8_t* good, const uint8_t* t20,
                        uint32_t q, uint32_t count, uint32_t* out_idx, uint32_t* out_cnt) {
    if (!c || count == 0 || count > DHTGPU_MAX_K) return DHTGPU_EINVAL;
    if (q && (!t20 || !out_idx || !out_cnt)) return DHTGPU_EINVAL;
    if (nb > 256 || (nb && (!firsts20 || !off))) return DHTGPU_EINVAL;
    if (!q) return DHTGPU_OK;
    if (nb == 0) {   // empty table: empty result (src/routing_table.cpp:116)
        for (uint32_t i = 0; i < q; ++i) {
            out_cnt[i] = 0;
            for (uint32_t r = 0; r < count; ++r) out_idx[(size_t)i * count + r] = DHTGPU_NONE;
        }
        return DHTGPU_OK;
    }
    const uint32_t nn = off[nb];
    if (nn && (!node_ids20 || !good)) return DHTGPU_EINVAL;
    for (uint32_t b = 0; b < nb; ++b)
        if (off[b] > off[b + 1]) return DHTGPU_EINVAL;
    DHT_TRY(c->bind());
    // host snapshot -> one device blob: firsts planes | off | gcnt | node planes | good
    const uint64_t ns = pad_q(nn ? nn : 1);
    std::vector<uint32_t> fp((size_t)5 * nb), gcnt(nb);
    for (uint32_t b = 0; b < nb; ++b) {
        for (int w = 0; w < 5; ++w) {
            const uint8_t* p = firsts20 + 20 * b + 4 * w;
            fp[(size_t)w * nb + b] = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
        }
        uint32_t g = 0;
        for (uint32_t i = off[b]; i < off[b + 1]; ++i) g += good[i] != 0;
        gcnt[b] = g;
    }
    const size_t o_fp = 0, o_off = o_fp + fp.size() * 4, o_g = o_off + (size_t)(nb + 1) * 4,
                 o_np = (o_g + (size_t)nb * 4 + 15) & ~size_t(15), o_good = o_np + (size_t)ns * 5 * 4,
                 total = o_good + nn + 16;
    DHT_TRY(c->aux.ensure(total));
    uint8_t* base = c->aux.as<uint8_t>();
    DHT_TRY(hipMemcpyAsync(base + o_fp, fp.data(), fp.size() * 4, hipMemcpyHostToDevice, c->stream));
    DHT_TRY(hipMemcpyAsync(base + o_off, off, (size_t)(nb + 1) * 4, hipMemcpyHostToDevice, c->stream));
    DHT_TRY(hipMemcpyAsync(base + o_g, gcnt.data(), (size_t)nb * 4, hipMemcpyHostToDevice, c->stream));
    if (nn) {
        DHT_TRY(hipMemcpyAsync(base + o_good, good, nn, hipMemcpyHostToDevice, c->stream));
        DHT_TRY(c->staging.ensure((size_t)std::max<uint64_t>(nn, q) * 20));
        DHT_TRY(hipMemcpyAsync(c->staging.p, node_ids20, (size_t)nn * 20, hipMemcpyHostToDevice, c->stream));
        DHT_TRY(launch_pack(c->staging.as<uint8_t>(), nn, (uint32_t*)(base + o_np), ns, c->stream));
        DHT_TRY(hipStreamSynchronize(c->stream));   // staging reused for targets
    }
    uint64_t ts = 0;
    DHT_TRY(c->upload_targets(t20, q, &ts));
    DHT_TRY(c->aux2.ensure((size_t)q * count * 4));
    DHT_TRY(c->aux3.ensure((size_t)q * 4));
    DHT_TRY(launch_find_closest(nb, (const uint32_t*)(base + o_fp), (const uint32_t*)(base + o_off),
                                (const uint32_t*)(base + o_g), (const uint32_t*)(base + o_np), ns,
                                base + o_good, c->targets.as<uint32_t>(), ts, q, count,
                                c->aux2.as<uint32_t>(), c->aux3.as<uint32_t>(), c->stream));
    DHT_TRY(hipMemcpyAsync(out_idx, c->aux2.p, (size_t)q * count * 4, hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipMemcpyAsync(out_cnt, c->aux3.p, (size_t)q * 4, hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipStreamSynchronize(c->stream));
    return DHTGPU_OK;
}

int dhtgpu_classify_dev(const uint32_t* planes, uint64_t stride, uint64_t n, uint32_t nb,
                        const uint32_t* d_fp, const uint32_t* myid_words, uint8_t* out_bucket,
                        unsigned long long* d_hist, void* stream) {
    if (!d_fp || !myid_words || !d_hist || nb == 0 || nb > 256 || (n && !planes)) return DHTGPU_EINVAL;
    DHT_TRY(launch_classify(planes, stride, n, nb, d_fp, myid_words, out_bucket, d_hist, (hipStream_t)stream));
    return DHTGPU_OK;
}

int dhtgpu_classify(dhtgpu_ctx* c, uint32_t nb, const uint8_t* firsts20, const uint8_t* myid20,
                    uint8_t* out_bucket, uint64_t* hist161) {
    if (!c || !firsts20 || !myid20 || !hist161 || nb == 0 || nb > 256) return DHTGPU_EINVAL;
    if (!c->has_ids) return DHTGPU_ENOIDS;
    DHT_TRY(c->bind());
    std::vector<uint32_t> fp((size_t)5 * nb);
    uint32_t my[5];
    auto be = [](const uint8_t* p) {
        return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
    };
    for (uint32_t b = 0; b < nb; ++b)
        for (int w = 0; w < 5; ++w) fp[(size_t)w * nb + b] = be(firsts20 + 20 * b + 4 * w);
    for (int w = 0; w < 5; ++w) my[w] = be(myid20 + 4 * w);
    DHT_TRY(c->aux.ensure(fp.size() * 4 + 161 * 8 + 64));
    uint8_t* base = c->aux.as<uint8_t>();
    unsigned long long* d_hist = (unsigned long long*)(base + ((fp.size() * 4 + 15) & ~size_t(15)));
    DHT_TRY(hipMemcpyAsync(base, fp.data(), fp.size() * 4, hipMemcpyHostToDevice, c->stream));
    DHT_TRY(hipMemsetAsync(d_hist, 0, 161 * 8, c->stream));
    uint8_t* d_bucket = nullptr;
    if (out_bucket && c->n) {
        DHT_TRY(c->aux2.ensure((size_t)c->n + 16));
        d_bucket = c->aux2.as<uint8_t>();
    }
    DHT_TRY(launch_classify(c->planes.as<uint32_t>(), c->stride, c->n, nb, (const uint32_t*)base, my,
                            d_bucket, d_hist, c->stream));
    if (d_bucket) DHT_TRY(hipMemcpyAsync(out_bucket, d_bucket, (size_t)c->n, hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipMemcpyAsync(hist161, d_hist, 161 * 8, hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipStreamSynchronize(c->stream));
    return DHTGPU_OK;
}

// Sort n ids (planes, stride) into `out` (sorted planes + permutation); synchronises.
static int sort_into(dhtgpu_ctx* c, const uint32_t* planes, uint64_t stride, uint64_t n, dhtgpu_ctx::SortedSet& out) {
    out.valid = false;
    out.n = n;
    out.stride = pad_ids(n ? n : 1);
    DHT_TRY(out.planes.ensure((size_t)out.stride * 5 * 4));
    DHT_TRY(out.perm.ensure((size_t)out.stride * 4));
    DHT_TRY(c->sort_scratch.ensure(sort_scratch_bytes(n)));
    int unique = 1;
    DHT_TRY(launch_sort_ids(planes, stride, n, out.planes.as<uint32_t>(), out.stride, out.perm.as<uint32_t>(),
                            c->sort_scratch.p, &unique, c->stream));
    DHT_TRY(hipStreamSynchronize(c->stream));
    if (c->sort_scratch.cap > ((size_t)1 << 30)) c->sort_scratch.release();   // large sorts: do not keep GBs
    out.unique = unique != 0;
    out.valid = true;
    return DHTGPU_OK;
}

// The getCachedNodes walk of q targets over a sorted set (perm nullable), accept[] in caller order.
static int cached_walk(dhtgpu_ctx* c, const uint32_t* planes, uint64_t stride, uint64_t n, const uint32_t* perm,
                       const uint8_t* accept, const uint8_t* t20, uint32_t q, uint32_t count, const uint32_t* gidx,
                       uint32_t* out_idx, uint32_t* out_cnt) {
    uint8_t* d_acc = nullptr;
    if (accept && n) {
        DHT_TRY(c->cache_acc.ensure((size_t)n + 16));
        d_acc = c->cache_acc.as<uint8_t>();
        DHT_TRY(hipMemcpyAsync(d_acc, accept, (size_t)n, hipMemcpyHostToDevice, c->stream));
    }
    uint64_t ts = 0;
    DHT_TRY(c->upload_targets(t20, q, &ts));
    DHT_TRY(c->aux2.ensure((size_t)q * count * 4));
    DHT_TRY(c->aux3.ensure((size_t)q * 4));
    DHT_TRY(launch_cached(planes, stride, n, perm, d_acc, c->targets.as<uint32_t>(), ts, q, count,
                          c->aux2.as<uint32_t>(), c->aux3.as<uint32_t>(), c->stream));
    if (gidx) DHT_TRY(launch_map_idx(c->aux2.as<uint32_t>(), (uint64_t)q * count, gidx, 0, c->stream));
    DHT_TRY(hipMemcpyAsync(out_idx, c->aux2.p, (size_t)q * count * 4, hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipMemcpyAsync(out_cnt, c->aux3.p, (size_t)q * 4, hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipStreamSynchronize(c->stream));
    return DHTGPU_OK;
}

int dhtgpu_cached_nodes(dhtgpu_ctx* c, const uint8_t* accept, const uint8_t* t20, uint32_t q,
                        uint32_t count, uint32_t* out_idx, uint32_t* out_cnt) {
    if (!c || count == 0 || count > DHTGPU_MAX_K || (q && (!t20 || !out_idx || !out_cnt))) return DHTGPU_EINVAL;
    if (!c->has_ids) return DHTGPU_ENOIDS;
    DHT_TRY(c->bind());
    if (c->sorted) {
        if (!q) return DHTGPU_OK;
        return cached_walk(c, c->planes.as<uint32_t>(), c->stride, c->n, nullptr, accept, t20, q, count, c->out_map(),
                           out_idx, out_cnt);
    }
    // an unsorted upload: walk its lexicographically sorted view (built once per id set)
    if (!c->sview.valid) {
        int r = sort_into(c, c->planes.as<uint32_t>(), c->stride, c->n, c->sview);
        if (r) return r;
    }
    if (!c->sview.unique) return DHTGPU_EUNSORTED;
    if (!q) return DHTGPU_OK;
    return cached_walk(c, c->sview.planes.as<uint32_t>(), c->sview.stride, c->n, c->sview.perm.as<uint32_t>(), accept,
                       t20, q, count, c->out_map(), out_idx, out_cnt);
}

int dhtgpu_cache_set(dhtgpu_ctx* c, const uint8_t* ids20, uint64_t n, uint64_t version) {
    if (!c || (!ids20 && n)) return DHTGPU_EINVAL;
    if (n >= 0xFFFFFFFFull) return DHTGPU_ERANGE;
    if (version && c->cache.valid && version == c->cache_version && n == c->cache.n) return DHTGPU_OK;
    DHT_TRY(c->bind());
    c->cache.valid = false;
    c->cache_version = 0;
    const uint64_t st = pad_ids(n ? n : 1);
    DHT_TRY(c->cache_in.ensure((size_t)st * 5 * 4));
    const uint64_t chunk = 1ull << 22;
    DHT_TRY(c->staging.ensure((size_t)std::min<uint64_t>(n ? n : 1, chunk) * 20));
    for (uint64_t i = 0; i < n; i += chunk) {
        const uint64_t m = std::min(chunk, n - i);
        DHT_TRY(hipMemcpyAsync(c->staging.p, ids20 + i * 20, (size_t)m * 20, hipMemcpyHostToDevice, c->stream));
        DHT_TRY(launch_pack(c->staging.as<uint8_t>(), m, c->cache_in.as<uint32_t>() + i, st, c->stream));
        DHT_TRY(hipStreamSynchronize(c->stream));   // staging is reused
    }
    int r = sort_into(c, c->cache_in.as<uint32_t>(), st, n, c->cache);
    if (r) return r;
    if (!c->cache.unique) {
        c->cache.valid = false;
        return DHTGPU_EUNSORTED;
    }
    c->cache_version = version;
    return DHTGPU_OK;
}

int dhtgpu_cache_nodes(dhtgpu_ctx* c, const uint8_t* accept, const uint8_t* t20, uint32_t q, uint32_t count,
                       uint32_t* out_idx, uint32_t* out_cnt) {
    if (!c || count == 0 || count > DHTGPU_MAX_K || (q && (!t20 || !out_idx || !out_cnt))) return DHTGPU_EINVAL;
    if (!c->cache.valid) return DHTGPU_ENOIDS;
    if (!q) return DHTGPU_OK;
    DHT_TRY(c->bind());
    return cached_walk(c, c->cache.planes.as<uint32_t>(), c->cache.stride, c->cache.n, c->cache.perm.as<uint32_t>(),
                       accept, t20, q, count, nullptr, out_idx, out_cnt);
}

int dhtgpu_cache_sorted(dhtgpu_ctx* c, uint32_t* perm) {
    if (!c || (!perm && c->cache.n)) return DHTGPU_EINVAL;
    if (!c->cache.valid) return DHTGPU_ENOIDS;
    if (!c->cache.n) return DHTGPU_OK;
    DHT_TRY(c->bind());
    DHT_TRY(hipMemcpyAsync(perm, c->cache.perm.p, (size_t)c->cache.n * 4, hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipStreamSynchronize(c->stream));
    return DHTGPU_OK;
}

// ---- a11 / f4: compact node wire format ------------------------------------------------

int dhtgpu_buffer_nodes_dev(dhtgpu_ctx* c, const uint8_t* node_tail, uint32_t af, const uint32_t* tp, uint64_t ts,
                            uint32_t q, const uint32_t* cand, uint32_t nc, uint8_t* out, uint32_t* out_len,
                            void* stream) {
    if (!c || (af != 4 && af != 6) || nc > 64) return DHTGPU_EINVAL;
    if (q && (!tp || !out || !out_len || (nc && (!cand || !node_tail)))) return DHTGPU_EINVAL;
    if (!c->has_ids) return DHTGPU_ENOIDS;
    if (!q) return DHTGPU_OK;
    DHT_TRY(c->bind());
    DHT_TRY(launch_wire_encode(c->planes.as<uint32_t>(), c->stride, node_tail, af == 4 ? 4u : 16u, tp, ts, q, cand,
                               nc, out, out_len, stream ? (hipStream_t)stream : c->stream));
    return DHTGPU_OK;
}

static int buffer_nodes_impl(dhtgpu_ctx* c, const uint32_t* planes, uint64_t stride, uint64_t n,
                             const uint8_t* node_tail, uint32_t af, const uint8_t* t20, uint32_t q,
                             const uint32_t* cand, uint32_t nc, uint8_t* out, uint32_t* out_len, size_t lead) {
    // every candidate must name a node (the kernel reads its planes and tail)
    for (size_t i = 0; i < (size_t)q * nc; ++i)
        if (cand[i] != DHTGPU_NONE && cand[i] >= n) return DHTGPU_EINVAL;
    const uint32_t alen = af == 4 ? 4u : 16u, rec = 20 + alen + 2;
    const size_t tl = (size_t)n * (alen + 2), cl = (size_t)q * nc * 4, ol = (size_t)q * 8 * rec, ll = (size_t)q * 4;
    DHT_TRY(c->wire.ensure(lead + al256(tl) + al256(cl) + al256(ol) + al256(ll) + 256));
    uint8_t* base = c->wire.as<uint8_t>() + lead;
    uint8_t* d_tail = base;
    uint32_t* d_cand = reinterpret_cast<uint32_t*>(base + al256(tl));
    uint8_t* d_out = base + al256(tl) + al256(cl);
    uint32_t* d_len = reinterpret_cast<uint32_t*>(d_out + al256(ol));
    if (tl) DHT_TRY(hipMemcpyAsync(d_tail, node_tail, tl, hipMemcpyHostToDevice, c->stream));
    if (cl) DHT_TRY(hipMemcpyAsync(d_cand, cand, cl, hipMemcpyHostToDevice, c->stream));
    uint64_t ts = 0;
    DHT_TRY(c->upload_targets(t20, q, &ts));
    DHT_TRY(launch_wire_encode(planes, stride, d_tail, alen, c->targets.as<uint32_t>(), ts, q, d_cand, nc, d_out,
                               d_len, c->stream));
    DHT_TRY(hipMemcpyAsync(out, d_out, ol, hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipMemcpyAsync(out_len, d_len, ll, hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipStreamSynchronize(c->stream));
    return DHTGPU_OK;
}

int dhtgpu_buffer_nodes(dhtgpu_ctx* c, const uint8_t* node_tail, uint32_t af, const uint8_t* t20, uint32_t q,
                        const uint32_t* cand, uint32_t nc, uint8_t* out, uint32_t* out_len) {
    if (!c || (af != 4 && af != 6) || nc > 64) return DHTGPU_EINVAL;
    if (q && (!t20 || !out || !out_len || (nc && (!cand || !node_tail)))) return DHTGPU_EINVAL;
    if (!c->has_ids) return DHTGPU_ENOIDS;
    if (!q) return DHTGPU_OK;
    DHT_TRY(c->bind());
    return buffer_nodes_impl(c, c->planes.as<uint32_t>(), c->stride, c->n, node_tail, af, t20, q, cand, nc, out,
                             out_len, 0);
}

int dhtgpu_buffer_nodes_ids(dhtgpu_ctx* c, const uint8_t* node_ids20, const uint8_t* node_tail, uint32_t nn,
                            uint32_t af, const uint8_t* t20, uint32_t q, const uint32_t* cand, uint32_t nc,
                            uint8_t* out, uint32_t* out_len) {
    if (!c || (af != 4 && af != 6) || nc > 64) return DHTGPU_EINVAL;
    if (q && (!t20 || !out || !out_len || (nc && (!cand || !node_tail)))) return DHTGPU_EINVAL;
    if (nn && (!node_ids20 || !node_tail)) return DHTGPU_EINVAL;
    if (!q) return DHTGPU_OK;
    DHT_TRY(c->bind());
    // the nodes' planes lead the wire scratch (sized for the whole call first: ensure() may
    // reallocate); the context's id set is left alone
    const uint64_t ns = pad_q(nn ? nn : 1);
    const size_t lead = al256((size_t)ns * 5 * 4);
    const uint32_t alen = af == 4 ? 4u : 16u, rec = 20 + alen + 2;
    DHT_TRY(c->wire.ensure(lead + al256((size_t)nn * (alen + 2)) + al256((size_t)q * nc * 4) +
                           al256((size_t)q * 8 * rec) + al256((size_t)q * 4) + 256));
    if (nn) {
        DHT_TRY(c->staging.ensure((size_t)nn * 20));
        DHT_TRY(hipMemcpyAsync(c->staging.p, node_ids20, (size_t)nn * 20, hipMemcpyHostToDevice, c->stream));
        DHT_TRY(launch_pack(c->staging.as<uint8_t>(), nn, c->wire.as<uint32_t>(), ns, c->stream));
        DHT_TRY(hipStreamSynchronize(c->stream));   // staging is reused for the targets
    }
    return buffer_nodes_impl(c, c->wire.as<uint32_t>(), ns, nn, node_tail, af, t20, q, cand, nc, out, out_len, lead);
}

int dhtgpu_deserialize_nodes(dhtgpu_ctx* c, uint32_t af, const uint8_t* myid20, const uint8_t* blob,
                             const uint64_t* msg_off, uint32_t m, const uint8_t* from_af, const uint8_t* from_addr,
                             uint8_t* out_ids20, uint8_t* out_tail, uint8_t* out_status, uint8_t* msg_status,
                             uint32_t* out_nrec) {
    if (!c || (af != 4 && af != 6) || !myid20 || !out_nrec) return DHTGPU_EINVAL;
    if (m && (!msg_off || !from_af || !from_addr || !msg_status)) return DHTGPU_EINVAL;
    *out_nrec = 0;
    if (!m) return DHTGPU_OK;
    const uint32_t alen = af == 4 ? 4u : 16u, rl = 20 + alen + 2;
    // per-message record ranges; a length that is not a whole number of records is the
    // reference's WRONG_NODE_INFO_BUF_LEN (the message's nodes are not used)
    std::vector<uint32_t> rs((size_t)m + 1, 0);
    for (uint32_t i = 0; i < m; ++i) {
        if (msg_off[i + 1] < msg_off[i]) return DHTGPU_EINVAL;
        const uint64_t len = msg_off[i + 1] - msg_off[i];
        msg_status[i] = len % rl ? 1 : 0;
        const uint64_t nr = len % rl ? 0 : len / rl;
        if ((uint64_t)rs[i] + nr > 0xFFFFFFF0ull) return DHTGPU_ERANGE;
        rs[i + 1] = rs[i] + (uint32_t)nr;
    }
    const uint32_t nrec = rs[m];
    *out_nrec = nrec;
    if (!nrec) return DHTGPU_OK;
    if (!blob || !out_ids20 || !out_tail || !out_status) return DHTGPU_EINVAL;
    DHT_TRY(c->bind());
    const uint64_t blen = msg_off[m];
    const size_t sz[] = {(size_t)blen, ((size_t)m + 1) * 8, ((size_t)m + 1) * 4, 32, m, (size_t)m * 16,
                         (size_t)nrec * 20, (size_t)nrec * (alen + 2), nrec};
    size_t tot = 0;
    for (size_t x : sz) tot += al256(x);
    DHT_TRY(c->wire.ensure(tot));
    uint8_t* p[9];
    uint8_t* w = c->wire.as<uint8_t>();
    for (int i = 0; i < 9; ++i) {
        p[i] = w;
        w += al256(sz[i]);
    }
    DHT_TRY(hipMemcpyAsync(p[0], blob, sz[0], hipMemcpyHostToDevice, c->stream));
    DHT_TRY(hipMemcpyAsync(p[1], msg_off, sz[1], hipMemcpyHostToDevice, c->stream));
    DHT_TRY(hipMemcpyAsync(p[2], rs.data(), sz[2], hipMemcpyHostToDevice, c->stream));
    DHT_TRY(hipMemcpyAsync(p[3], myid20, 20, hipMemcpyHostToDevice, c->stream));
    DHT_TRY(hipMemcpyAsync(p[4], from_af, sz[4], hipMemcpyHostToDevice, c->stream));
    DHT_TRY(hipMemcpyAsync(p[5], from_addr, sz[5], hipMemcpyHostToDevice, c->stream));
    DHT_TRY(launch_wire_decode(p[0], reinterpret_cast<const uint64_t*>(p[1]), reinterpret_cast<const uint32_t*>(p[2]),
                               m, nrec, af, p[3], p[4], p[5], p[6], p[7], p[8], c->stream));
    DHT_TRY(hipMemcpyAsync(out_ids20, p[6], sz[6], hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipMemcpyAsync(out_tail, p[7], sz[7], hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipMemcpyAsync(out_status, p[8], sz[8], hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipStreamSynchronize(c->stream));
    return DHTGPU_OK;
}

// RoutingTable::depth (src/routing_table.cpp:100-107) over a table snapshot: one more than
// the larger lowbit (infohash.h:132-143) of the bucket's first and of the next bucket's.
int dhtgpu_table_depth(uint32_t nb, const uint8_t* firsts20, uint32_t b, uint32_t* out_depth) {
    if (!out_depth || (nb && !firsts20) || (nb && b >= nb)) return DHTGPU_EINVAL;
    *out_depth = 0;
    if (!nb) return DHTGPU_OK;
    auto lowbit = [](const uint8_t* h) -> int {
        int i = 19;
        while (i >= 0 && h[i] == 0) --i;
        if (i < 0) return -1;
        int j = 7;
        while (((h[i] >> (7 - j)) & 1) == 0) --j;
        return 8 * i + j;
    };
    const int bit1 = lowbit(firsts20 + 20 * (size_t)b);
    const int bit2 = b + 1 < nb ? lowbit(firsts20 + 20 * (size_t)(b + 1)) : -1;
    *out_depth = (uint32_t)(std::max(bit1, bit2) + 1);
    return DHTGPU_OK;
}

// ---- a10: Search::insertNode, batched ---------------------------------------------------------
int dhtgpu_search_insert(dhtgpu_ctx* c, const uint8_t* node_ids20, const uint8_t* node_state, uint32_t nn,
                         const uint8_t* t20, uint32_t q, uint32_t cap, uint32_t* list_node, uint8_t* list_flags,
                         uint32_t* list_len, uint8_t* search_expired, const uint64_t* ins_off, const uint32_t* ins_node,
                         const uint8_t* ins_token, uint8_t* ins_added) {
    if (!c || cap == 0 || cap > 4096) return DHTGPU_EINVAL;
    if (q && (!t20 || !list_node || !list_flags || !list_len || !search_expired || !ins_off)) return DHTGPU_EINVAL;
    if (!q) return DHTGPU_OK;
    const uint64_t m = ins_off[q];
    if (m && (!ins_node || !ins_token || !ins_added)) return DHTGPU_EINVAL;
    if (nn && (!node_ids20 || !node_state)) return DHTGPU_EINVAL;
    for (uint32_t i = 0; i < q; ++i) {   // every index the kernel follows must name a node
        if (ins_off[i + 1] < ins_off[i] || list_len[i] > cap) return DHTGPU_EINVAL;
        for (uint32_t j = 0; j < list_len[i]; ++j)
            if (list_node[(size_t)i * cap + j] >= nn) return DHTGPU_EINVAL;
    }
    for (uint64_t i = 0; i < m; ++i)
        if (ins_node[i] >= nn) return DHTGPU_EINVAL;
    DHT_TRY(c->bind());
    const uint64_t ns = pad_q(nn ? nn : 1);
    const size_t sz[] = {(size_t)ns * 20, (size_t)nn, (size_t)q * cap * 4, (size_t)q * cap, (size_t)q * 4, (size_t)q,
                         ((size_t)q + 1) * 8, (size_t)m * 4, (size_t)m, (size_t)m, 16};
    size_t tot = 0;
    for (size_t x : sz) tot += al256(x);
    DHT_TRY(c->srch.ensure(tot));
    uint8_t* p[11];
    uint8_t* w = c->srch.as<uint8_t>();
    for (int i = 0; i < 11; ++i) {
        p[i] = w;
        w += al256(sz[i]);
    }
    if (nn) {
        DHT_TRY(c->staging.ensure((size_t)nn * 20));
        DHT_TRY(hipMemcpyAsync(c->staging.p, node_ids20, (size_t)nn * 20, hipMemcpyHostToDevice, c->stream));
        DHT_TRY(launch_pack(c->staging.as<uint8_t>(), nn, reinterpret_cast<uint32_t*>(p[0]), ns, c->stream));
        DHT_TRY(hipMemcpyAsync(p[1], node_state, nn, hipMemcpyHostToDevice, c->stream));
        DHT_TRY(hipStreamSynchronize(c->stream));   // staging is reused for the targets
    }
    DHT_TRY(hipMemcpyAsync(p[2], list_node, sz[2], hipMemcpyHostToDevice, c->stream));
    DHT_TRY(hipMemcpyAsync(p[3], list_flags, sz[3], hipMemcpyHostToDevice, c->stream));
    DHT_TRY(hipMemcpyAsync(p[4], list_len, sz[4], hipMemcpyHostToDevice, c->stream));
    DHT_TRY(hipMemcpyAsync(p[5], search_expired, sz[5], hipMemcpyHostToDevice, c->stream));
    DHT_TRY(hipMemcpyAsync(p[6], ins_off, sz[6], hipMemcpyHostToDevice, c->stream));
    if (m) {
        DHT_TRY(hipMemcpyAsync(p[7], ins_node, sz[7], hipMemcpyHostToDevice, c->stream));
        DHT_TRY(hipMemcpyAsync(p[8], ins_token, sz[8], hipMemcpyHostToDevice, c->stream));
    }
    DHT_TRY(hipMemsetAsync(p[10], 0, 4, c->stream));
    uint64_t ts = 0;
    DHT_TRY(c->upload_targets(t20, q, &ts));
    DHT_TRY(launch_search_insert(reinterpret_cast<uint32_t*>(p[0]), ns, p[1], c->targets.as<uint32_t>(), ts, q, cap,
                                 reinterpret_cast<uint32_t*>(p[2]), p[3], reinterpret_cast<uint32_t*>(p[4]), p[5],
                                 reinterpret_cast<const uint64_t*>(p[6]), reinterpret_cast<const uint32_t*>(p[7]), p[8],
                                 p[9], reinterpret_cast<uint32_t*>(p[10]), c->stream));
    uint32_t overflow = 0;
    DHT_TRY(hipMemcpyAsync(&overflow, p[10], 4, hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipMemcpyAsync(list_node, p[2], sz[2], hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipMemcpyAsync(list_flags, p[3], sz[3], hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipMemcpyAsync(list_len, p[4], sz[4], hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipMemcpyAsync(search_expired, p[5], sz[5], hipMemcpyDeviceToHost, c->stream));
    if (m) DHT_TRY(hipMemcpyAsync(ins_added, p[9], sz[9], hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipStreamSynchronize(c->stream));
    return overflow ? DHTGPU_ERANGE : DHTGPU_OK;
}

// ---- a4 / a6: InfoHash::lowbit and RoutingTable::depth of every bucket ---------------------------
int dhtgpu_table_stats(dhtgpu_ctx* c, uint32_t nb, const uint8_t* firsts20, int32_t* out_lowbit, uint32_t* out_depth) {
    if (!c || (nb && (!firsts20 || !out_lowbit || !out_depth))) return DHTGPU_EINVAL;
    if (!nb) return DHTGPU_OK;
    DHT_TRY(c->bind());
    std::vector<uint32_t> fp((size_t)5 * nb);
    for (uint32_t b = 0; b < nb; ++b)
        for (int w = 0; w < 5; ++w) {
            const uint8_t* q4 = firsts20 + 20 * (size_t)b + 4 * w;
            fp[(size_t)w * nb + b] = ((uint32_t)q4[0] << 24) | ((uint32_t)q4[1] << 16) | ((uint32_t)q4[2] << 8) | q4[3];
        }
    const size_t a = al256(fp.size() * 4), bsz = al256((size_t)nb * 4);
    DHT_TRY(c->srch.ensure(a + 2 * bsz));
    uint8_t* base = c->srch.as<uint8_t>();
    DHT_TRY(hipMemcpyAsync(base, fp.data(), fp.size() * 4, hipMemcpyHostToDevice, c->stream));
    DHT_TRY(launch_table_stats(reinterpret_cast<uint32_t*>(base), nb, reinterpret_cast<int32_t*>(base + a),
                               reinterpret_cast<uint32_t*>(base + a + bsz), c->stream));
    DHT_TRY(hipMemcpyAsync(out_lowbit, base + a, (size_t)nb * 4, hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipMemcpyAsync(out_depth, base + a + bsz, (size_t)nb * 4, hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipStreamSynchronize(c->stream));
    return DHTGPU_OK;
}

// ---- f3: crawl replay (iterative searches over a synthetic network) ----------------------
int dhtgpu_net_prepare(dhtgpu_ctx* c, const uint8_t* dead, uint64_t table_seed) {
    if (!c) return DHTGPU_EINVAL;
    if (!c->has_ids || !c->n) return DHTGPU_ENOIDS;
    if (c->has_gidx) return DHTGPU_EINVAL;   // the network is the whole uploaded id set
    int r = dhtgpu_index_build(c, c->stream);
    if (r) return r;
    DHT_TRY(c->net_sorted.ensure((size_t)c->n * 8));
    DHT_TRY(launch_net_sort(c->index.p, c->n, c->index_B, c->net_sorted.as<uint2>(), c->stream));
    c->net_has_dead = dead != nullptr;
    if (dead) {
        DHT_TRY(c->net_dead.ensure((size_t)c->n));
        DHT_TRY(hipMemcpyAsync(c->net_dead.p, dead, (size_t)c->n, hipMemcpyHostToDevice, c->stream));
    }
    DHT_TRY(hipStreamSynchronize(c->stream));
    c->net_seed = table_seed;
    c->net_valid = true;
    return DHTGPU_OK;
}

int dhtgpu_set_search_alpha(dhtgpu_ctx* c, uint32_t alpha) {
    if (!c || alpha < 1 || alpha > 8) return DHTGPU_EINVAL;
    c->search_alpha = alpha;
    return DHTGPU_OK;
}

int dhtgpu_search_batch_dev(dhtgpu_ctx* c, const uint32_t* tp, uint64_t ts, uint32_t q, const uint32_t* searchers,
                            uint32_t max_rounds, uint32_t* out_idx, uint8_t* out_flags, uint32_t* out_len,
                            uint32_t* out_rounds, uint32_t* out_queries, void* stream) {
    if (!c || (q && (!tp || !searchers || !out_idx || !out_flags || !out_len || !out_rounds || !out_queries)))
        return DHTGPU_EINVAL;
    if (!c->net_valid || !c->index_valid) return DHTGPU_ENOIDS;
    if (!q) return DHTGPU_OK;
    DHT_TRY(c->bind());
    DHT_TRY(launch_search(c->planes.as<uint32_t>(), c->stride, c->net_sorted.as<uint2>(), c->index.p, c->n,
                          c->index_B, c->net_has_dead ? c->net_dead.as<uint8_t>() : nullptr, c->net_seed, tp, ts, q,
                          searchers, max_rounds, c->search_alpha, out_idx, out_flags, out_len, out_rounds, out_queries,
                          stream ? (hipStream_t)stream : c->stream));
    return DHTGPU_OK;
}

int dhtgpu_search_batch(dhtgpu_ctx* c, const uint8_t* t20, uint32_t q, const uint32_t* searchers, uint32_t max_rounds,
                        uint32_t* out_idx, uint8_t* out_flags, uint32_t* out_len, uint32_t* out_rounds,
                        uint32_t* out_queries) {
    if (!c || (q && (!t20 || !searchers || !out_idx || !out_flags || !out_len || !out_rounds || !out_queries)))
        return DHTGPU_EINVAL;
    if (!c->net_valid) return DHTGPU_ENOIDS;
    if (!q) return DHTGPU_OK;
    for (uint32_t i = 0; i < q; ++i)
        if (searchers[i] >= c->n) return DHTGPU_EINVAL;
    DHT_TRY(c->bind());
    const size_t L = search_list_cap();
    const size_t sz[] = {(size_t)q * 4, (size_t)q * L * 4, (size_t)q * L, (size_t)q * 4, (size_t)q * 4, (size_t)q * 4};
    size_t tot = 0;
    for (size_t x : sz) tot += al256(x);
    DHT_TRY(c->net_io.ensure(tot));
    uint8_t* p[6];
    uint8_t* w = c->net_io.as<uint8_t>();
    for (int i = 0; i < 6; ++i) {
        p[i] = w;
        w += al256(sz[i]);
    }
    uint64_t ts = 0;
    DHT_TRY(c->upload_targets(t20, q, &ts));
    DHT_TRY(hipMemcpyAsync(p[0], searchers, sz[0], hipMemcpyHostToDevice, c->stream));
    int r = dhtgpu_search_batch_dev(c, c->targets.as<uint32_t>(), ts, q, (const uint32_t*)p[0], max_rounds,
                                    (uint32_t*)p[1], p[2], (uint32_t*)p[3], (uint32_t*)p[4], (uint32_t*)p[5], c->stream);
    if (r) return r;
    DHT_TRY(hipMemcpyAsync(out_idx, p[1], sz[1], hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipMemcpyAsync(out_flags, p[2], sz[2], hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipMemcpyAsync(out_len, p[3], sz[3], hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipMemcpyAsync(out_rounds, p[4], sz[4], hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipMemcpyAsync(out_queries, p[5], sz[5], hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipStreamSynchronize(c->stream));
    return DHTGPU_OK;
}

}  // extern "C"
