// comm.cpp -- device buffers and the RCCL communicator of the multi-view pipeline.
//
// The reference runs every ProcessProblem on device 0 and hands depth maps between passes through
// depths*.dmb files (ACMMP.cpp:653-678).  Here one process drives one GPU; between passes the
// depth maps a geom pass reads are broadcast from the rank that owns each view, HBM to HBM over
// xGMI (grouped ncclBroadcast, one per view), and uploaded into the engine device-to-device
// (acmmp_upload_depths_device).  RCCL is /opt/rocm's, on the same HIP runtime as the engine; the
// 128-byte unique id is the only thing the host side has to carry between processes.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "acmmp.h"
#include "engine.h"

static_assert(sizeof(ncclUniqueId) == ACMMP_COMM_ID_BYTES, "ncclUniqueId size");

struct acmmp_comm {
    int device = 0, nranks = 1, rank = 0;
    ncclComm_t nccl = nullptr;
    hipStream_t stream = nullptr;
    double* d_scratch = nullptr;
    int scratch_n = 0;
    hipEvent_t after = nullptr;         // acmmp_comm_after: engine-stream work the next collectives wait for
};

namespace {

acmmp_status from_hip(hipError_t e) {
    return e == hipSuccess ? ACMMP_OK : (e == hipErrorOutOfMemory ? ACMMP_ERR_OUT_OF_MEMORY : ACMMP_ERR_HIP);
}
acmmp_status from_nccl(ncclResult_t r) { return r == ncclSuccess ? ACMMP_OK : ACMMP_ERR_COMM; }

#define TRY_HIP(expr) do { const acmmp_status s_ = from_hip(expr); if (s_ != ACMMP_OK) return s_; } while (0)
#define TRY_NCCL(expr) do { const acmmp_status s_ = from_nccl(expr); if (s_ != ACMMP_OK) return s_; } while (0)

}  // namespace

extern "C" {

acmmp_status acmmp_device_alloc(int device, size_t bytes, void** ptr) {
    if (!ptr) return ACMMP_ERR_INVALID_ARGUMENT;
    *ptr = nullptr;
    TRY_HIP(hipSetDevice(device));
    TRY_HIP(hipMalloc(ptr, bytes ? bytes : 1));
    return ACMMP_OK;
}

acmmp_status acmmp_device_free(int device, void* ptr) {
    if (!ptr) return ACMMP_OK;
    TRY_HIP(hipSetDevice(device));
    TRY_HIP(hipFree(ptr));
    return ACMMP_OK;
}

acmmp_status acmmp_memcpy(int device, void* dst, const void* src, size_t bytes, int kind) {
    if ((!dst || !src) && bytes) return ACMMP_ERR_INVALID_ARGUMENT;
    static const hipMemcpyKind kinds[3] = {hipMemcpyHostToDevice, hipMemcpyDeviceToHost, hipMemcpyDeviceToDevice};
    if (kind < 0 || kind > 2) return ACMMP_ERR_INVALID_ARGUMENT;
    TRY_HIP(hipSetDevice(device));
    TRY_HIP(kind == 1 ? acmmp::d2h(dst, src, bytes) : hipMemcpy(dst, src, bytes, kinds[kind]));
    return ACMMP_OK;
}

acmmp_status acmmp_device_checksum(int device, const void* ptr, size_t bytes, uint64_t* out) {
    if (!out || (!ptr && bytes) || bytes % 4) return ACMMP_ERR_INVALID_ARGUMENT;
    *out = 0;
    if (!bytes) return ACMMP_OK;
    TRY_HIP(hipSetDevice(device));
    unsigned long long* d = nullptr;
    TRY_HIP(hipMalloc(&d, sizeof(*d)));
    unsigned long long h = 0;
    hipError_t e = hipMemsetAsync(d, 0, sizeof(*d), nullptr);
    if (e == hipSuccess) e = acmmp::launch_checksum(ptr, bytes, d, nullptr);
    if (e == hipSuccess) e = hipMemcpy(&h, d, sizeof(h), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    TRY_HIP(e);
    *out = h;
    return ACMMP_OK;
}

acmmp_status acmmp_device_identity(int device, char* pci_bus_id, int len, uint8_t uuid[16]) {
    if (!pci_bus_id || len < 16 || !uuid) return ACMMP_ERR_INVALID_ARGUMENT;
    TRY_HIP(hipDeviceGetPCIBusId(pci_bus_id, len, device));
    hipDevice_t dv;
    TRY_HIP(hipDeviceGet(&dv, device));
    hipUUID u;
    TRY_HIP(hipDeviceGetUuid(&u, dv));
    std::memcpy(uuid, u.bytes, 16);
    return ACMMP_OK;
}

acmmp_status acmmp_clock_probe(int device, float warm_ms, double out[4]) {
    if (!out) return ACMMP_ERR_INVALID_ARGUMENT;
    TRY_HIP(hipSetDevice(device));
    int cus = 0;
    TRY_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    const int blocks = std::max(1, cus) * 16;            // 4 waves of 256 lanes per block: 16 per SIMD
    std::vector<float> rnd(65536);
    uint32_t x = 0x9e3779b9u;
    for (float& r : rnd) {                               // uniform in [-1, 1): random operands, not zeros
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        r = static_cast<float>(x >> 8) * (2.0f / 16777216.0f) - 1.0f;
    }
    float *d_rnd = nullptr, *d_sink = nullptr;
    acmmp::ClockStamp* d_st = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    hipError_t e = hipMalloc(&d_rnd, rnd.size() * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&d_sink, static_cast<size_t>(blocks) * 256 * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&d_st, static_cast<size_t>(blocks) * sizeof(acmmp::ClockStamp));
    if (e == hipSuccess) e = hipMemcpy(d_rnd, rnd.data(), rnd.size() * sizeof(float), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    std::vector<acmmp::ClockStamp> st(blocks);
    float ms = 0.f;
    int iters = 4096;
    // size one launch to ~5 ms, keep the chip under that load for warm_ms, then one stamped launch
    for (int k = 0; e == hipSuccess && k < 3; ++k) {
        e = hipEventRecord(e0, nullptr);
        if (e == hipSuccess) e = acmmp::launch_clock_probe(d_rnd, iters, blocks, nullptr, d_sink, nullptr);
        if (e == hipSuccess) e = hipEventRecord(e1, nullptr);
        if (e == hipSuccess) e = hipEventSynchronize(e1);
        if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
        if (e == hipSuccess && ms > 0.f) iters = std::max(256, std::min(1 << 22, static_cast<int>(iters * 5.0f / ms)));
    }
    const int warm = std::max(0, static_cast<int>(warm_ms / 5.0f));
    for (int k = 0; e == hipSuccess && k < warm; ++k)
        e = acmmp::launch_clock_probe(d_rnd, iters, blocks, nullptr, d_sink, nullptr);
    if (e == hipSuccess) e = hipEventRecord(e0, nullptr);
    if (e == hipSuccess) e = acmmp::launch_clock_probe(d_rnd, iters, blocks, d_st, d_sink, nullptr);
    if (e == hipSuccess) e = hipEventRecord(e1, nullptr);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    if (e == hipSuccess) e = hipMemcpy(st.data(), d_st, st.size() * sizeof(st[0]), hipMemcpyDeviceToHost);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipFree(d_rnd);
    (void)hipFree(d_sink);
    (void)hipFree(d_st);
    TRY_HIP(e);
    std::vector<double> ghz;
    for (const acmmp::ClockStamp& c : st)
        if (c.ticks > 0) ghz.push_back(static_cast<double>(c.cycles) / static_cast<double>(c.ticks) * 0.1);
    if (ghz.empty()) return ACMMP_ERR_HIP;
    std::sort(ghz.begin(), ghz.end());
    out[0] = ghz[ghz.size() / 2];
    out[1] = ghz.front();
    out[2] = ghz.back();
    out[3] = ms;
    return ACMMP_OK;
}

acmmp_status acmmp_comm_unique_id(uint8_t id[ACMMP_COMM_ID_BYTES]) {
    if (!id) return ACMMP_ERR_INVALID_ARGUMENT;
    ncclUniqueId u;
    TRY_NCCL(ncclGetUniqueId(&u));
    std::memcpy(id, &u, sizeof u);
    return ACMMP_OK;
}

acmmp_status acmmp_comm_create(int device, const uint8_t id[ACMMP_COMM_ID_BYTES], int nranks, int rank,
                               acmmp_comm** out) {
    if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks) return ACMMP_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    TRY_HIP(hipSetDevice(device));
    acmmp_comm* c = new acmmp_comm();
    c->device = device; c->nranks = nranks; c->rank = rank;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    acmmp_status s = from_hip(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    if (s == ACMMP_OK) s = from_nccl(ncclCommInitRank(&c->nccl, nranks, u, rank));
    if (s != ACMMP_OK) { acmmp_comm_destroy(c); return s; }
    *out = c;
    return ACMMP_OK;
}

void acmmp_comm_destroy(acmmp_comm* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->nccl) (void)ncclCommDestroy(c->nccl);
    if (c->d_scratch) (void)hipFree(c->d_scratch);
    if (c->after) (void)hipEventDestroy(c->after);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

acmmp_status acmmp_comm_after(acmmp_comm* c, acmmp_ctx* ctx) {
    if (!c || !ctx) return ACMMP_ERR_INVALID_ARGUMENT;
    int dev = 0;
    hipStream_t s = nullptr;
    acmmp_status st = acmmp::engine_stream(ctx, &dev, &s);
    if (st != ACMMP_OK) return st;
    if (dev != c->device) return ACMMP_ERR_INVALID_ARGUMENT;
    TRY_HIP(hipSetDevice(c->device));
    if (!c->after) TRY_HIP(hipEventCreateWithFlags(&c->after, hipEventDisableTiming));
    // the engine stream's work so far -> an event the communicator's stream waits on: device-side order,
    // no host wait (a later record re-arms the same event; a wait already queued keeps its snapshot)
    TRY_HIP(hipEventRecord(c->after, s));
    TRY_HIP(hipStreamWaitEvent(c->stream, c->after, 0));
    return ACMMP_OK;
}

acmmp_status acmmp_comm_broadcast(acmmp_comm* c, int n, void* const* bufs, const size_t* bytes, const int* roots) {
    if (!c || n < 0 || (n > 0 && (!bufs || !bytes || !roots))) return ACMMP_ERR_INVALID_ARGUMENT;
    for (int i = 0; i < n; ++i)
        if (!bufs[i] || roots[i] < 0 || roots[i] >= c->nranks) return ACMMP_ERR_INVALID_ARGUMENT;
    TRY_HIP(hipSetDevice(c->device));
    TRY_NCCL(ncclGroupStart());
    for (int i = 0; i < n; ++i) {
        const ncclResult_t r = ncclBroadcast(bufs[i], bufs[i], bytes[i], ncclUint8, roots[i], c->nccl, c->stream);
        if (r != ncclSuccess) { (void)ncclGroupEnd(); return ACMMP_ERR_COMM; }
    }
    TRY_NCCL(ncclGroupEnd());
    TRY_HIP(hipStreamSynchronize(c->stream));
    return ACMMP_OK;
}

acmmp_status acmmp_comm_allreduce_max(acmmp_comm* c, double* vals, int n) {
    if (!c || n < 0 || (n > 0 && !vals)) return ACMMP_ERR_INVALID_ARGUMENT;
    if (n == 0) return ACMMP_OK;
    TRY_HIP(hipSetDevice(c->device));
    if (c->scratch_n < n) {
        if (c->d_scratch) TRY_HIP(hipFree(c->d_scratch));
        c->d_scratch = nullptr;
        TRY_HIP(hipMalloc(reinterpret_cast<void**>(&c->d_scratch), sizeof(double) * n));
        c->scratch_n = n;
    }
    TRY_HIP(hipMemcpyAsync(c->d_scratch, vals, sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
    TRY_NCCL(ncclAllReduce(c->d_scratch, c->d_scratch, n, ncclFloat64, ncclMax, c->nccl, c->stream));
    TRY_HIP(hipMemcpyAsync(vals, c->d_scratch, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream));
    TRY_HIP(hipStreamSynchronize(c->stream));
    return ACMMP_OK;
}

acmmp_status acmmp_comm_band_exchange(acmmp_comm* c, acmmp_ctx* ctx, int colour, int rank_up, int rank_down) {
    if (!c || !ctx || colour < 0 || colour > 1 || rank_up >= c->nranks || rank_down >= c->nranks ||
        rank_up == c->rank || rank_down == c->rank)
        return ACMMP_ERR_INVALID_ARGUMENT;
    acmmp::BandBuffers b{};
    acmmp_status st = acmmp::band_buffers(ctx, colour, &b);
    if (st != ACMMP_OK) return st;
    int r[8];
    if ((st = acmmp_band_halo_ranges(ctx, r)) != ACMMP_OK) return st;
    // (rows, peer, send?) for the four transfers; a band with no neighbour on one side has empty ranges
    const int ops[4][4] = {{r[0], r[1], rank_up, 1}, {r[2], r[3], rank_up, 0}, {r[4], r[5], rank_down, 1},
                           {r[6], r[7], rank_down, 0}};
    TRY_HIP(hipSetDevice(b.device));
    TRY_NCCL(ncclGroupStart());
    for (const auto& op : ops) {
        if (op[1] <= op[0]) continue;
        if (op[2] < 0) { (void)ncclGroupEnd(); return ACMMP_ERR_INVALID_ARGUMENT; }
        const size_t off = static_cast<size_t>(op[0]) * b.Wh, n = static_cast<size_t>(op[1] - op[0]) * b.Wh;
        void* bufs[3] = {b.plane + off, b.cost + off, b.sel + off};
        const size_t bytes[3] = {sizeof(float4) * n, sizeof(float) * n, sizeof(uint32_t) * n};
        for (int k = 0; k < 3; ++k) {
            const ncclResult_t res = op[3] ? ncclSend(bufs[k], bytes[k], ncclUint8, op[2], c->nccl, b.stream)
                                           : ncclRecv(bufs[k], bytes[k], ncclUint8, op[2], c->nccl, b.stream);
            if (res != ncclSuccess) { (void)ncclGroupEnd(); return ACMMP_ERR_COMM; }
        }
    }
    TRY_NCCL(ncclGroupEnd());
    return ACMMP_OK;
}

acmmp_status acmmp_run_patchmatch_band(acmmp_ctx* ctx, acmmp_comm* c, uint64_t seed, int row0, int row1,
                                       int rank_up, int rank_down) {
    if (!ctx || (!c && (rank_up >= 0 || rank_down >= 0))) return ACMMP_ERR_INVALID_ARGUMENT;
    acmmp_status st = acmmp_band_begin(ctx, seed, row0, row1);
    while (st == ACMMP_OK && acmmp_band_sweeps_left(ctx) > 0) {
        int colour = 0;
        st = acmmp_band_sweep(ctx, &colour);
        if (st == ACMMP_OK && c) st = acmmp_comm_band_exchange(c, ctx, colour, rank_up, rank_down);
    }
    if (st != ACMMP_OK) return st;
    return acmmp_band_end(ctx, 1);
}

}  // extern "C"
