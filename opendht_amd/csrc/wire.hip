// wire.hip -- compact node wire format on the device.
//
// Encode = NetworkEngine::bufferNodes (src/network_engine.cpp:1003-1032): the candidate
// nodes of each target (typically its findClosestNodes / k-NN result) are sorted by
// InfoHash::xorCmp to the target, the first SEND_NODES = 8 (:62) are kept and written as
// id (20 B) || address (4 B IPv4 / 16 B IPv6) || port (2 B), the address and port bytes
// exactly as the node's sockaddr holds them (network order): 26 / 38-byte records.
//
// Decode = NetworkEngine::deserializeNodes (:849-887) per record: deserializeIPv4/6
// (:831-846), skip the own id (:858-859), loopback -> the sender's address with the
// record's port (:861-865; SockAddr::isLoopback, src/utils.cpp:115-128), then
// NetworkEngine::isMartian (:362-386).  isNodeBlacklisted is host policy state and stays
// with the caller.  Status per record: 0 accepted, 1 own id, 2 martian.
#include "dhtgpu_dev.h"
#include "dhtgpu_internal.h"

namespace dhtgpu {
namespace {

constexpr uint32_t kSendNodes = 8;   // SEND_NODES, src/network_engine.cpp:62

// one wave per target; lane j holds candidate j (c <= 64)
__global__ __launch_bounds__(256) void k_wire_encode(const uint32_t* __restrict__ planes, uint64_t stride,
                                                    const uint8_t* __restrict__ tail, uint32_t alen,
                                                    const uint32_t* __restrict__ tp, uint64_t ts, uint32_t q,
                                                    const uint32_t* __restrict__ cand, uint32_t c,
                                                    uint8_t* __restrict__ out, uint32_t* __restrict__ out_len) {
    const uint32_t lane = lane_id();
    const uint32_t qi = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (qi >= q) return;
    const uint32_t x = lane < c ? cand[(uint64_t)qi * c + lane] : DHT_NONE;
    const bool act = x != DHT_NONE;
    uint32_t d[DHT_W];
#pragma unroll
    for (int j = 0; j < DHT_W; ++j) {
        const uint32_t tj = tp[(uint64_t)j * ts + qi];
        d[j] = act ? planes[(uint64_t)j * stride + x] ^ tj : 0u;
    }
    // rank = candidates strictly closer, then equal ids in candidate order
    const uint64_t am = __ballot(act);
    uint32_t rank = 0;
    for (uint64_t it = am; it; it &= it - 1) {
        const uint32_t o = (uint32_t)__ffsll((long long)it) - 1;
        bool less = false, decided = false;
#pragma unroll
        for (int j = 0; j < DHT_W; ++j) {
            const uint32_t od = __builtin_amdgcn_readlane((int)d[j], (int)o);
            if (!decided && od != d[j]) {
                less = od < d[j];
                decided = true;
            }
        }
        if (!decided) less = o < lane;
        rank += less;
    }
    const uint32_t valid = (uint32_t)__popcll(am);
    const uint32_t nnode = valid < kSendNodes ? valid : kSendNodes;
    const uint32_t rec = 20 + alen + 2;
    if (act && rank < kSendNodes) {
        uint8_t* dst = out + ((uint64_t)qi * kSendNodes + rank) * rec;
#pragma unroll
        for (int j = 0; j < DHT_W; ++j) {
            const uint32_t w = planes[(uint64_t)j * stride + x];
            dst[4 * j] = (uint8_t)(w >> 24);
            dst[4 * j + 1] = (uint8_t)(w >> 16);
            dst[4 * j + 2] = (uint8_t)(w >> 8);
            dst[4 * j + 3] = (uint8_t)w;
        }
        const uint8_t* src = tail + (uint64_t)x * (alen + 2);
        for (uint32_t b = 0; b < alen + 2; ++b) dst[20 + b] = src[b];
    }
    if (lane == 0) out_len[qi] = nnode * rec;
}

// one thread per record
__global__ __launch_bounds__(256) void k_wire_decode(const uint8_t* __restrict__ blob,
                                                    const uint64_t* __restrict__ msg_off,
                                                    const uint32_t* __restrict__ rec_start, uint32_t m,
                                                    uint32_t af, const uint8_t* __restrict__ myid,
                                                    const uint8_t* __restrict__ from_af,
                                                    const uint8_t* __restrict__ from_addr,
                                                    uint8_t* __restrict__ out_ids, uint8_t* __restrict__ out_tail,
                                                    uint8_t* __restrict__ out_status) {
    const uint32_t r = blockIdx.x * 256 + threadIdx.x;
    if (r >= rec_start[m]) return;
    uint32_t lo = 0, hi = m;   // message: largest i with rec_start[i] <= r
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (rec_start[mid] <= r) lo = mid;
        else hi = mid;
    }
    const uint32_t alen = af == 4 ? 4u : 16u, rl = 20 + alen + 2;
    const uint8_t* rec = blob + msg_off[lo] + (uint64_t)(r - rec_start[lo]) * rl;
    bool self = true;
    for (int b = 0; b < 20; ++b) {
        out_ids[(uint64_t)r * 20 + b] = rec[b];
        self = self && rec[b] == myid[b];
    }
    uint8_t a[16];
    for (uint32_t b = 0; b < alen; ++b) a[b] = rec[20 + b];
    const uint8_t p0 = rec[20 + alen], p1 = rec[21 + alen];
    bool loop;
    if (af == 4) {
        loop = a[0] == 127;
    } else {
        loop = a[15] == 1;
        for (int b = 0; b < 15; ++b) loop = loop && a[b] == 0;
    }
    if (loop && from_af[lo] == af)
        for (uint32_t b = 0; b < alen; ++b) a[b] = from_addr[(uint64_t)lo * 16 + b];
    uint8_t* ot = out_tail + (uint64_t)r * (alen + 2);
    for (uint32_t b = 0; b < alen; ++b) ot[b] = a[b];
    ot[alen] = p0;
    ot[alen + 1] = p1;
    bool martian = p0 == 0 && p1 == 0;
    if (af == 4) {
        martian = martian || a[0] == 0 || (a[0] & 0xE0) == 0xE0;
    } else {
        bool zero = true, v4map = a[10] == 0xFF && a[11] == 0xFF;
        for (int b = 0; b < 16; ++b) zero = zero && a[b] == 0;
        for (int b = 0; b < 10; ++b) v4map = v4map && a[b] == 0;
        martian = martian || a[0] == 0xFF || (a[0] == 0xFE && (a[1] & 0xC0) == 0x80) || zero || v4map;
    }
    out_status[r] = self ? 1 : (martian ? 2 : 0);
}

}  // namespace

hipError_t launch_wire_encode(const uint32_t* planes, uint64_t stride, const uint8_t* tail, uint32_t alen,
                              const uint32_t* tp, uint64_t ts, uint32_t q, const uint32_t* cand, uint32_t c,
                              uint8_t* out, uint32_t* out_len, hipStream_t s) {
    if (!q) return hipSuccess;
    k_wire_encode<<<(q + 3) / 4, 256, 0, s>>>(planes, stride, tail, alen, tp, ts, q, cand, c, out, out_len);
    return hipGetLastError();
}

hipError_t launch_wire_decode(const uint8_t* blob, const uint64_t* msg_off, const uint32_t* rec_start, uint32_t m,
                              uint32_t nrec, uint32_t af, const uint8_t* myid, const uint8_t* from_af,
                              const uint8_t* from_addr, uint8_t* out_ids, uint8_t* out_tail, uint8_t* out_status,
                              hipStream_t s) {
    if (!nrec) return hipSuccess;
    k_wire_decode<<<(nrec + 255) / 256, 256, 0, s>>>(blob, msg_off, rec_start, m, af, myid, from_af, from_addr,
                                                     out_ids, out_tail, out_status);
    return hipGetLastError();
}

}  // namespace dhtgpu
