// multi.hip — the multi-GPU entry points of the C-ABI.
//
// Rows partition naturally: A is split into contiguous row blocks of equal
// estimated device cost (ias_partition_rows), every GPU holds all of B and
// computes its block of C with the single-GPU engine; the only exchange is
// concatenating C.  Two forms:
//
//  * ias_csr_mul_csr_multi — one process driving N devices (one host thread
//    per device, each with its own plan and stream); C is assembled in host
//    memory (or on the first device), block after block in row order.  This
//    is what `spgemm-gpu --gpus N` runs.
//  * ias_dist_* — one process per GPU over RCCL (xGMI): each rank computes
//    its block and the row-sharded C is concatenated on every rank by an
//    allgatherv (per-rank counts by ncclAllGather, then one ncclBroadcast per
//    root into that root's slice of the output, in one group; row pointers
//    shifted by the rank's global nnz offset).  RCCL has no v-variant.
//    librccl is opened at first use (dlopen, RTLD_LOCAL), so libias.so has no
//    link-time RCCL dependency that could clash with a host framework's own.
//
// The reference is single-device; its multi-threaded CPU kernels split rows
// the same way (CPU/detail/csr/common_csr.h:95-189, OpenMP over rows).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "ias.h"
#include "ias_internal.hpp"

using namespace ias;

#define HIPC(x)                                                                   \
    do {                                                                          \
        hipError_t _e = (x);                                                      \
        if (_e != hipSuccess) {                                                   \
            set_last_error("%s failed: %s", #x, hipGetErrorString(_e));           \
            return _e == hipErrorOutOfMemory ? IAS_ERROR_OUT_OF_MEMORY : IAS_ERROR_DEVICE; \
        }                                                                         \
    } while (0)

namespace {

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

extern "C" ias_status ias_csr_mul_csr_multi(const ias_csr *A, const ias_csr *B, ias_csr *C, int32_t ndev,
                                            const int32_t *devices, const ias_opts *opts, ias_report *rep) {
    if (!A || !B || !C || ndev < 1) return IAS_ERROR_INVALID_ARGUMENT;
    if (A->cols != B->rows) return IAS_ERROR_DIMENSION_MISMATCH;
    ias_opts base;
    if (opts) base = *opts;
    else ias_opts_default(&base);
    const int out_mem = base.output_memory >= 0 ? base.output_memory : IAS_MEMORY_HOST;
    std::vector<int32_t> devs(ndev);
    for (int d = 0; d < ndev; ++d) devs[d] = devices ? devices[d] : d;
    if (rep) memset(rep, 0, sizeof *rep);
    std::vector<int64_t> bounds(ndev + 1);
    IAS_TRY(ias_partition_rows(A, B, ndev, bounds.data()));

    // every device computes its block into host memory
    std::vector<ias_csr> part(ndev);
    std::vector<ias_report> prep(ndev);
    std::vector<ias_status> st(ndev, IAS_SUCCESS);
    const double t0 = now_ms();
    std::vector<std::thread> th;
    for (int d = 0; d < ndev; ++d)
        th.emplace_back([&, d] {
            ias_csr view{};
            st[d] = ias_csr_row_view(A, bounds[d], bounds[d + 1], &view);
            if (st[d] != IAS_SUCCESS) return;
            ias_opts o = base;
            o.device = devs[d];
            o.plan = nullptr;    // a plan per device
            o.stream = nullptr;
            o.output_memory = IAS_MEMORY_HOST;
            memset(&part[d], 0, sizeof part[d]);
            st[d] = ias_csr_mul_csr(&view, B, &part[d], &o, &prep[d]);
        });
    for (auto &t : th) t.join();
    for (int d = 0; d < ndev; ++d)
        if (st[d] != IAS_SUCCESS) {
            for (auto &p : part) ias_csr_free(&p);
            return st[d];
        }
    const double t1 = now_ms();

    // concatenate the blocks (row pointers shifted by the blocks before)
    int64_t nnz = 0;
    for (auto &p : part) nnz += p.nnz;
    ias_csr H{};
    ias_status s = ias_csr_alloc(&H, A->rows, B->cols, nnz, IAS_MEMORY_HOST, 0);
    if (s == IAS_SUCCESS) {
        int64_t off = 0;
        H.row_ptr[0] = 0;
        for (int d = 0; d < ndev; ++d) {
            const ias_csr &p = part[d];
            const int64_t r0 = bounds[d];
            for (int64_t i = 0; i < p.rows; ++i) H.row_ptr[r0 + i + 1] = p.row_ptr[i + 1] + off;
            if (p.nnz) {
                memcpy(H.col + off, p.col, sizeof(int32_t) * (size_t)p.nnz);
                memcpy(H.val + off, p.val, sizeof(double) * (size_t)p.nnz);
            }
            off += p.nnz;
        }
    }
    for (auto &p : part) ias_csr_free(&p);
    if (s != IAS_SUCCESS) return s;
    if (out_mem == IAS_MEMORY_DEVICE) {
        ias_csr D{};
        s = ias_csr_copy(&H, &D, IAS_MEMORY_DEVICE, devs[0]);
        ias_csr_free(&H);
        if (s != IAS_SUCCESS) return s;
        *C = D;
    } else {
        *C = H;
    }
    if (rep) {
        for (int d = 0; d < ndev; ++d) {
            rep->flops += prep[d].flops;
            rep->ms_total = std::max(rep->ms_total, prep[d].ms_total);
            rep->ms_upload = std::max(rep->ms_upload, prep[d].ms_upload);
            rep->ms_download = std::max(rep->ms_download, prep[d].ms_download);
            rep->max_row_products = std::max(rep->max_row_products, prep[d].max_row_products);
            rep->max_row_nnz = std::max(rep->max_row_nnz, prep[d].max_row_nnz);
        }
        rep->nnz_c = nnz;
        (void)t0;
        (void)t1;
    }
    return IAS_SUCCESS;
}

// ------------------------------------------------------------------ RCCL
namespace {

struct Rccl {
    ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*AllGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Broadcast)(const void *, void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char *(*GetErrorString)(ncclResult_t) = nullptr;
    bool ok = false;
};

const Rccl *rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            set_last_error("librccl not found: %s", dlerror());
            return;
        }
        auto sym = [&](const char *n) { return dlsym(h, n); };
        r.GetUniqueId = (decltype(r.GetUniqueId))sym("ncclGetUniqueId");
        r.CommInitRank = (decltype(r.CommInitRank))sym("ncclCommInitRank");
        r.CommDestroy = (decltype(r.CommDestroy))sym("ncclCommDestroy");
        r.AllGather = (decltype(r.AllGather))sym("ncclAllGather");
        r.Broadcast = (decltype(r.Broadcast))sym("ncclBroadcast");
        r.GroupStart = (decltype(r.GroupStart))sym("ncclGroupStart");
        r.GroupEnd = (decltype(r.GroupEnd))sym("ncclGroupEnd");
        r.GetErrorString = (decltype(r.GetErrorString))sym("ncclGetErrorString");
        r.ok = r.GetUniqueId && r.CommInitRank && r.CommDestroy && r.AllGather && r.Broadcast && r.GroupStart &&
               r.GroupEnd;
        if (!r.ok) set_last_error("librccl lacks a needed symbol");
    });
    return r.ok ? &r : nullptr;
}

#define RCCL_TRY(call)                                                                   \
    do {                                                                                 \
        const ncclResult_t rc_ = (call);                                                 \
        if (rc_ != ncclSuccess) {                                                        \
            set_last_error("%s: %s", #call, R->GetErrorString ? R->GetErrorString(rc_) : "rccl error"); \
            return IAS_ERROR_DEVICE;                                                     \
        }                                                                                \
    } while (0)

__global__ void k_shift_ends(const int64_t *rp, int64_t rows, int64_t off, int64_t *out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < rows) out[i] = rp[i + 1] - rp[0] + off;
}

}  // namespace

struct ias_dist {
    ncclComm_t comm = nullptr;
    int rank = 0, nranks = 1, device = 0;
    ias_plan *plan = nullptr;
};

extern "C" ias_status ias_dist_unique_id(char *id, int32_t id_len) {
    if (!id || id_len < (int32_t)sizeof(ncclUniqueId)) return IAS_ERROR_INVALID_ARGUMENT;
    const Rccl *R = rccl();
    if (!R) return IAS_ERROR_DEVICE;
    ncclUniqueId u;
    RCCL_TRY(R->GetUniqueId(&u));
    memcpy(id, &u, sizeof u);
    return IAS_SUCCESS;
}

extern "C" ias_status ias_dist_create(ias_dist **out, const char *id, int32_t nranks, int32_t rank, int32_t device) {
    if (!out || !id || nranks < 1 || rank < 0 || rank >= nranks) return IAS_ERROR_INVALID_ARGUMENT;
    const Rccl *R = rccl();
    if (!R) return IAS_ERROR_DEVICE;
    HIPC(hipSetDevice(device));
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    ias_dist *d = new ias_dist;
    d->rank = rank;
    d->nranks = nranks;
    d->device = device;
    const ncclResult_t rc = R->CommInitRank(&d->comm, nranks, u, rank);
    if (rc != ncclSuccess) {
        set_last_error("ncclCommInitRank: %s", R->GetErrorString ? R->GetErrorString(rc) : "rccl error");
        delete d;
        return IAS_ERROR_DEVICE;
    }
    const ias_status s = ias_plan_create(&d->plan, device, nullptr);
    if (s != IAS_SUCCESS) {
        R->CommDestroy(d->comm);
        delete d;
        return s;
    }
    *out = d;
    return IAS_SUCCESS;
}

extern "C" ias_status ias_dist_destroy(ias_dist *d) {
    if (!d) return IAS_SUCCESS;
    const Rccl *R = rccl();
    if (d->plan) ias_plan_destroy(d->plan);
    if (R && d->comm) R->CommDestroy(d->comm);
    delete d;
    return IAS_SUCCESS;
}

extern "C" ias_status ias_dist_allgatherv_csr(ias_dist *d, const ias_csr *Cl, ias_csr *Cf, void *stream) {
    if (!d || !Cl || !Cf) return IAS_ERROR_INVALID_ARGUMENT;
    if (Cl->memory != IAS_MEMORY_DEVICE || Cl->device != d->device) return IAS_ERROR_INVALID_ARGUMENT;
    const Rccl *R = rccl();
    if (!R) return IAS_ERROR_DEVICE;
    HIPC(hipSetDevice(d->device));
    hipStream_t s = (hipStream_t)stream;
    const int P = d->nranks;
    // per-rank (rows, nnz)
    int64_t *cnt = nullptr;
    HIPC(hipMalloc(&cnt, sizeof(int64_t) * 2 * (P + 1)));
    std::vector<int64_t> h(2 * (P + 1));
    h[0] = Cl->rows;
    h[1] = Cl->nnz;
    HIPC(hipMemcpyAsync(cnt + 2 * P, h.data(), 2 * sizeof(int64_t), hipMemcpyHostToDevice, s));
    RCCL_TRY(R->AllGather(cnt + 2 * P, cnt, 2, ncclInt64, d->comm, s));
    HIPC(hipMemcpyAsync(h.data(), cnt, sizeof(int64_t) * 2 * P, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    hipFree(cnt);
    std::vector<int64_t> roff(P + 1, 0), noff(P + 1, 0);
    for (int r = 0; r < P; ++r) {
        roff[r + 1] = roff[r] + h[2 * r];
        noff[r + 1] = noff[r] + h[2 * r + 1];
    }
    ias_csr F{};
    IAS_TRY(ias_csr_alloc(&F, roff[P], Cl->cols, noff[P], IAS_MEMORY_DEVICE, d->device));
    HIPC(hipMemsetAsync(F.row_ptr, 0, sizeof(int64_t), s));
    // this rank's row ends, shifted into the global numbering, land in place
    if (Cl->rows > 0)
        k_shift_ends<<<(unsigned)((Cl->rows + 255) / 256), 256, 0, s>>>(Cl->row_ptr, Cl->rows, noff[d->rank],
                                                                        F.row_ptr + 1 + roff[d->rank]);
    HIPC(hipGetLastError());
    RCCL_TRY(R->GroupStart());
    for (int r = 0; r < P; ++r) {
        const bool me = r == d->rank;
        const int64_t rows = h[2 * r], nnz = h[2 * r + 1];
        if (rows > 0)
            RCCL_TRY(R->Broadcast(F.row_ptr + 1 + roff[r], F.row_ptr + 1 + roff[r], (size_t)rows, ncclInt64, r,
                                  d->comm, s));
        if (nnz > 0) {
            RCCL_TRY(R->Broadcast(me ? (const void *)Cl->col : nullptr, F.col + noff[r], (size_t)nnz, ncclInt32, r,
                                  d->comm, s));
            RCCL_TRY(R->Broadcast(me ? (const void *)Cl->val : nullptr, F.val + noff[r], (size_t)nnz, ncclFloat64, r,
                                  d->comm, s));
        }
    }
    RCCL_TRY(R->GroupEnd());
    HIPC(hipStreamSynchronize(s));
    *Cf = F;
    return IAS_SUCCESS;
}

extern "C" ias_status ias_dist_csr_mul_csr(ias_dist *d, const ias_csr *A, const ias_csr *B, ias_csr *C,
                                           int32_t gather, int32_t order, ias_report *rep) {
    if (!d || !A || !B || !C) return IAS_ERROR_INVALID_ARGUMENT;
    if (A->cols != B->rows) return IAS_ERROR_DIMENSION_MISMATCH;
    std::vector<int64_t> bounds(d->nranks + 1);
    IAS_TRY(ias_partition_rows(A, B, d->nranks, bounds.data()));
    ias_csr view{};
    IAS_TRY(ias_csr_row_view(A, bounds[d->rank], bounds[d->rank + 1], &view));
    ias_opts o;
    ias_opts_default(&o);
    o.order = order;
    o.device = d->device;
    o.plan = d->plan;
    o.output_memory = IAS_MEMORY_DEVICE;
    ias_csr L{};
    IAS_TRY(ias_csr_mul_csr(&view, B, &L, &o, rep));
    if (!gather) {
        *C = L;
        return IAS_SUCCESS;
    }
    const ias_status s = ias_dist_allgatherv_csr(d, &L, C, nullptr);
    ias_csr_free(&L);
    return s;
}
