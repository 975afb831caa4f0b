// api.hip -- the libdhtgpu C ABI (include/dhtgpu.h).  Owns device buffers and the
// stream; converts between the boundary's 20-byte big-endian ids and the device
// word-plane layout; never throws across the ABI.
#include <hip/hip_runtime.h>

#include <algorithm>
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

#define DHT_TRY(expr)                                 \
    do {                                              \
        hipError_t _e = (expr);                       \
        if (_e != hipSuccess) return map_err(_e);     \
    } while (0)

uint32_t pad_q(uint32_t q) { return (q + 63) & ~63u; }

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
        bool clean = false;
        hipEvent_t done = nullptr;
        hipStream_t last = nullptr;
    };
    static constexpr int kBatchDepth = 4;
    BatchSlot bslot[kBatchDepth];
    int bnext = 0, blast = 0;

    hipError_t bind() { return hipSetDevice(device); }

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
        case DHTGPU_EUNSORTED: return "id set is not lexicographically sorted and unique";
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
    if (e == hipSuccess) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->num_cus = prop.multiProcessorCount;
    }
    if (e != hipSuccess) {
        delete c;
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
        for (DevBuf* d : {&b.ws, &b.out_idx, &b.out_cnt}) d->release();
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
    c->has_gidx = false;
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
    }
    return DHTGPU_OK;
}

int dhtgpu_set_global_indices(dhtgpu_ctx* c, int on) {
    if (!c) return DHTGPU_EINVAL;
    c->map_global = on != 0;
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
    const ScanPlan p = plan_scan(c->n, q, c->num_cus);
    const uint32_t* gidx = c->out_map();
    if ((p.splits == 1 || c->n == 0) && !gidx) {   // one pass writes the final form directly
        DHT_TRY(launch_scan(c->planes.as<uint32_t>(), c->stride, c->n, p, tp, ts, q, k, out_idx,
                            out_cnt, out_rec, idx_base, s));
        return DHTGPU_OK;
    }
    // local indices (merged over id-range splits when the batch is too small to fill
    // the chip), then mapped to global indices or turned into candidate records
    uint32_t* li = out_idx;
    uint32_t* lc = out_cnt;
    if (out_rec) {
        DHT_TRY(c->out_idx.ensure((size_t)q * k * 4));
        DHT_TRY(c->out_cnt.ensure((size_t)q * 4));
        li = c->out_idx.as<uint32_t>();
        lc = c->out_cnt.as<uint32_t>();
    }
    if (p.splits == 1 || c->n == 0) {
        DHT_TRY(launch_scan(c->planes.as<uint32_t>(), c->stride, c->n, p, tp, ts, q, k, li, lc, nullptr, 0, s));
    } else {
        DHT_TRY(c->rec.ensure((size_t)p.splits * q * k * 6 * 4));
        DHT_TRY(launch_scan(c->planes.as<uint32_t>(), c->stride, c->n, p, tp, ts, q, k, nullptr, nullptr,
                            c->rec.as<uint32_t>(), 0, s));
        DHT_TRY(launch_merge(c->rec.as<uint32_t>(), p.splits, q, k, tp, ts, k, li, lc, s));
    }
    if (out_rec)
        DHT_TRY(launch_rec_from_idx(li, (uint64_t)q * k, c->planes.as<uint32_t>(), c->stride, idx_base, gidx,
                                    out_rec, s));
    else
        DHT_TRY(launch_map_idx(li, (uint64_t)q * k, gidx, idx_base, s));
    return DHTGPU_OK;
}

int dhtgpu_merge_dev(const uint32_t* rec, uint32_t lists, uint32_t q, uint32_t k_in,
                     const uint32_t* tp, uint64_t ts, uint32_t k, uint32_t* out_idx,
                     uint32_t* out_cnt, void* stream) {
    if (!rec || !tp || !out_idx || !out_cnt || k == 0 || k > DHTGPU_MAX_K || lists == 0 || k_in == 0)
        return DHTGPU_EINVAL;
    if ((size_t)lists * k_in * 24 > 160 * 1024) return DHTGPU_ERANGE;
    if (!q) return DHTGPU_OK;
    DHT_TRY(launch_merge(rec, lists, q, k_in, tp, ts, k, out_idx, out_cnt, (hipStream_t)stream));
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
        DHT_TRY(launch_rec_from_idx(li, (uint64_t)q * k, c->planes.as<uint32_t>(), c->stride, idx_base, gidx,
                                    out_rec, s));
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

static int batch_run(dhtgpu_ctx* c, const uint32_t* tp, uint64_t ts, uint32_t q, uint32_t k, uint32_t* out_idx,
                     uint32_t* out_cnt, uint32_t* out_rec, uint32_t idx_base, hipStream_t s, hipEvent_t* ev) {
    if (!batch_supported(c->n, q, k, c->num_cus)) return DHTGPU_ERANGE;
    dhtgpu_ctx::BatchSlot& b = c->bslot[c->bnext];
    // a slot last used on another stream: wait for that stream's work so far (it includes the
    // slot's previous call); same stream: stream order suffices
    if (b.last && b.last != s) {
        if (!b.done) DHT_TRY(hipEventCreateWithFlags(&b.done, hipEventDisableTiming));
        DHT_TRY(hipEventRecord(b.done, b.last));
        DHT_TRY(hipStreamWaitEvent(s, b.done, 0));
    }
    const size_t need = batch_bytes(c->n, q, k, c->num_cus);
    if (need > b.ws.cap) b.clean = false;
    DHT_TRY(b.ws.ensure(need));
    if (!b.clean) DHT_TRY(hipMemsetAsync(b.ws.p, 0, batch_clean_bytes(), s));
    b.clean = false;   // re-established below once every launch went through
    c->blast = c->bnext;
    c->bnext = (c->bnext + 1) % dhtgpu_ctx::kBatchDepth;
    const uint32_t* gidx = c->out_map();
    uint32_t* li = out_idx;
    uint32_t* lc = out_cnt;
    if (out_rec) {   // local indices first, then candidate records for a cross-shard merge
        DHT_TRY(b.out_idx.ensure((size_t)q * k * 4));
        DHT_TRY(b.out_cnt.ensure((size_t)q * 4));
        li = b.out_idx.as<uint32_t>();
        lc = b.out_cnt.as<uint32_t>();
    }
    DHT_TRY(launch_batch_topk(b.ws.p, c->planes.as<uint32_t>(), c->stride, c->n, tp, ts, q, k,
                              out_rec ? nullptr : gidx, out_rec ? 0u : idx_base, li, lc, c->num_cus, c->shard_pbits,
                              c->shard_pbits ? c->w0s.as<uint32_t>() : nullptr, s, ev));
    if (out_rec)
        DHT_TRY(launch_rec_from_idx(li, (uint64_t)q * k, c->planes.as<uint32_t>(), c->stride, idx_base, gidx,
                                    out_rec, s));
    b.last = s;
    b.clean = true;
    return DHTGPU_OK;
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

int dhtgpu_batch_topk_timed(dhtgpu_ctx* c, const uint32_t* tp, uint64_t ts, uint32_t q, uint32_t k,
                            uint32_t* out_idx, uint32_t* out_cnt, void* stream, float* ms4, uint32_t* stats4) {
    if (!c || !ms4 || k == 0 || k > DHTGPU_MAX_K || !q || !tp || !out_idx || !out_cnt) return DHTGPU_EINVAL;
    if (!c->has_ids) return DHTGPU_ENOIDS;
    DHT_TRY(c->bind());
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    hipEvent_t ev[8];   // start/stop per kernel, recorded by the kernels' dispatches
    for (int i = 0; i < 8; ++i) DHT_TRY(hipEventCreate(&ev[i]));
    int r = batch_run(c, tp, ts, q, k, out_idx, out_cnt, nullptr, 0, s, ev);
    hipError_t e = r ? hipSuccess : hipEventSynchronize(ev[7]);
    for (int i = 0; !r && e == hipSuccess && i < 4; ++i) e = hipEventElapsedTime(&ms4[i], ev[2 * i], ev[2 * i + 1]);
    for (int i = 0; i < 8; ++i) (void)hipEventDestroy(ev[i]);
    if (r) return r;
    DHT_TRY(e);
    if (stats4) {
        DHT_TRY(batch_read_stats(c->bslot[c->blast].ws.p, c->n, q, k, c->num_cus, stats4, s));
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

int dhtgpu_cached_nodes(dhtgpu_ctx* c, const uint8_t* accept, const uint8_t* t20, uint32_t q,
                        uint32_t count, uint32_t* out_idx, uint32_t* out_cnt) {
    if (!c || count == 0 || count > DHTGPU_MAX_K || (q && (!t20 || !out_idx || !out_cnt))) return DHTGPU_EINVAL;
    if (!c->has_ids) return DHTGPU_ENOIDS;
    if (!c->sorted) return DHTGPU_EUNSORTED;
    if (!q) return DHTGPU_OK;
    DHT_TRY(c->bind());
    uint8_t* d_acc = nullptr;
    if (accept && c->n) {
        DHT_TRY(c->aux.ensure((size_t)c->n + 16));
        d_acc = c->aux.as<uint8_t>();
        DHT_TRY(hipMemcpyAsync(d_acc, accept, (size_t)c->n, hipMemcpyHostToDevice, c->stream));
    }
    uint64_t ts = 0;
    DHT_TRY(c->upload_targets(t20, q, &ts));
    DHT_TRY(c->aux2.ensure((size_t)q * count * 4));
    DHT_TRY(c->aux3.ensure((size_t)q * 4));
    DHT_TRY(launch_cached(c->planes.as<uint32_t>(), c->stride, c->n, d_acc, c->targets.as<uint32_t>(),
                          ts, q, count, c->aux2.as<uint32_t>(), c->aux3.as<uint32_t>(), c->stream));
    if (c->out_map())
        DHT_TRY(launch_map_idx(c->aux2.as<uint32_t>(), (uint64_t)q * count, c->gidx.as<uint32_t>(), 0, c->stream));
    DHT_TRY(hipMemcpyAsync(out_idx, c->aux2.p, (size_t)q * count * 4, hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipMemcpyAsync(out_cnt, c->aux3.p, (size_t)q * 4, hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipStreamSynchronize(c->stream));
    return DHTGPU_OK;
}

// ---- a11 / f4: compact node wire format ------------------------------------------------
static inline size_t al256(size_t b) { return (b + 255) & ~size_t(255); }

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

int dhtgpu_buffer_nodes(dhtgpu_ctx* c, const uint8_t* node_tail, uint32_t af, const uint8_t* t20, uint32_t q,
                        const uint32_t* cand, uint32_t nc, uint8_t* out, uint32_t* out_len) {
    if (!c || (af != 4 && af != 6) || nc > 64) return DHTGPU_EINVAL;
    if (q && (!t20 || !out || !out_len || (nc && (!cand || !node_tail)))) return DHTGPU_EINVAL;
    if (!c->has_ids) return DHTGPU_ENOIDS;
    if (!q) return DHTGPU_OK;
    DHT_TRY(c->bind());
    const uint32_t alen = af == 4 ? 4u : 16u, rec = 20 + alen + 2;
    const size_t tl = (size_t)c->n * (alen + 2), cl = (size_t)q * nc * 4, ol = (size_t)q * 8 * rec, ll = (size_t)q * 4;
    DHT_TRY(c->wire.ensure(al256(tl) + al256(cl) + al256(ol) + al256(ll) + 256));
    uint8_t* base = c->wire.as<uint8_t>();
    uint8_t* d_tail = base;
    uint32_t* d_cand = reinterpret_cast<uint32_t*>(base + al256(tl));
    uint8_t* d_out = base + al256(tl) + al256(cl);
    uint32_t* d_len = reinterpret_cast<uint32_t*>(d_out + al256(ol));
    if (tl) DHT_TRY(hipMemcpyAsync(d_tail, node_tail, tl, hipMemcpyHostToDevice, c->stream));
    if (cl) DHT_TRY(hipMemcpyAsync(d_cand, cand, cl, hipMemcpyHostToDevice, c->stream));
    uint64_t ts = 0;
    DHT_TRY(c->upload_targets(t20, q, &ts));
    DHT_TRY(launch_wire_encode(c->planes.as<uint32_t>(), c->stride, d_tail, alen, c->targets.as<uint32_t>(), ts, q,
                               d_cand, nc, d_out, d_len, c->stream));
    DHT_TRY(hipMemcpyAsync(out, d_out, ol, hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipMemcpyAsync(out_len, d_len, ll, hipMemcpyDeviceToHost, c->stream));
    DHT_TRY(hipStreamSynchronize(c->stream));
    return DHTGPU_OK;
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
                          searchers, max_rounds, out_idx, out_flags, out_len, out_rounds, out_queries,
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
