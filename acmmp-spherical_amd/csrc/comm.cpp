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

#include <cstring>
#include <string>
#include <vector>

#include "acmmp.h"

static_assert(sizeof(ncclUniqueId) == ACMMP_COMM_ID_BYTES, "ncclUniqueId size");

struct acmmp_comm {
    int device = 0, nranks = 1, rank = 0;
    ncclComm_t nccl = nullptr;
    hipStream_t stream = nullptr;
    double* d_scratch = nullptr;
    int scratch_n = 0;
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
    TRY_HIP(hipMemcpy(dst, src, bytes, kinds[kind]));
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
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
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

}  // extern "C"
