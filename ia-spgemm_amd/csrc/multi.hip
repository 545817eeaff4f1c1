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
#include <condition_variable>
#include <map>
#include <memory>
#include <string>
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

// The exchange step's two collectives, behind one interface:
// RCCL for one process per GPU, and a loopback (in-process, memcpy) form for
// P ranks driven by P host threads of one process — on one GPU or several —
// so the sharding, the per-root offsets and the row-pointer fix-up run at
// P > 1 where RCCL cannot (it allows one rank per device in a communicator).
struct Bcast {
    const void *send;   // the root's source (others: ignored)
    void *recv;
    size_t bytes;
    int root;
};
struct Transport {
    virtual ~Transport() {}
    // recv[r * n .. r * n + n) = rank r's send[0 .. n), device buffers
    virtual ias_status allgather_i64(const int64_t *send, int64_t *recv, size_t n, hipStream_t s) = 0;
    // every op of the list as one group (the same list on every rank)
    virtual ias_status bcast_group(const std::vector<Bcast> &ops, hipStream_t s) = 0;
};

struct RcclTransport : Transport {
    const Rccl *R;
    ncclComm_t comm;
    RcclTransport(const Rccl *r, ncclComm_t c) : R(r), comm(c) {}
    ~RcclTransport() override {
        if (comm) R->CommDestroy(comm);
    }
    ias_status allgather_i64(const int64_t *send, int64_t *recv, size_t n, hipStream_t s) override {
        RCCL_TRY(R->AllGather(send, recv, n, ncclInt64, comm, s));
        return IAS_SUCCESS;
    }
    ias_status bcast_group(const std::vector<Bcast> &ops, hipStream_t s) override {
        RCCL_TRY(R->GroupStart());
        for (const Bcast &b : ops) {
            // 8-byte elements where the size allows (the C arrays), bytes otherwise
            const bool w8 = b.bytes % 8 == 0;
            const ncclResult_t rc = R->Broadcast(b.send, b.recv, w8 ? b.bytes / 8 : b.bytes, w8 ? ncclInt64 : ncclInt8,
                                                 b.root, comm, s);
            if (rc != ncclSuccess) {
                R->GroupEnd();
                set_last_error("ncclBroadcast: %s", R->GetErrorString ? R->GetErrorString(rc) : "rccl error");
                return IAS_ERROR_DEVICE;
            }
        }
        RCCL_TRY(R->GroupEnd());
        return IAS_SUCCESS;
    }
};

// Loopback group: P ranks of one process meet at a host barrier; every rank
// posts its (already complete: its stream is synchronised first) send
// buffers, copies what it receives from the peers' buffers with
// hipMemcpyAsync on its own stream, drains it, and meets the others again
// before returning (no peer buffer is released while still being read).
struct LoopGroup {
    int P;
    std::mutex mu;
    std::condition_variable cv;
    int waiting = 0;
    uint64_t gen = 0;
    std::vector<const void *> posted;                 // allgather: per rank
    std::vector<std::vector<Bcast>> posted_ops;       // bcast: per rank
    explicit LoopGroup(int p) : P(p), posted(p), posted_ops(p) {}
    bool broken = false;   // a rank gave up waiting: the group is unusable
    // false when the peers did not all arrive within `secs` (a rank failed
    // before reaching the collective): every rank then returns an error
    // instead of waiting forever
    bool barrier(double secs = 300.0) {
        std::unique_lock<std::mutex> g(mu);
        if (broken) return false;
        const uint64_t my = gen;
        if (++waiting == P) {
            waiting = 0;
            ++gen;
            cv.notify_all();
            return true;
        }
        const bool ok = cv.wait_for(g, std::chrono::duration<double>(secs), [&] { return gen != my || broken; });
        if (!ok || broken) {
            broken = true;
            cv.notify_all();
            return false;
        }
        return true;
    }
};
std::mutex &loop_registry_mu() {
    static std::mutex *m = new std::mutex;
    return *m;
}
std::map<std::string, std::weak_ptr<LoopGroup>> &loop_registry() {
    static auto *m = new std::map<std::string, std::weak_ptr<LoopGroup>>;
    return *m;
}

struct LoopTransport : Transport {
    std::shared_ptr<LoopGroup> g;
    int rank;
    LoopTransport(std::shared_ptr<LoopGroup> grp, int r) : g(std::move(grp)), rank(r) {}
    static ias_status lost() {
        set_last_error("loopback group: a peer rank did not reach the collective");
        return IAS_ERROR_DEVICE;
    }
    ias_status allgather_i64(const int64_t *send, int64_t *recv, size_t n, hipStream_t s) override {
        HIPC(hipStreamSynchronize(s));
        g->posted[rank] = send;
        if (!g->barrier()) return lost();
        hipError_t e = hipSuccess;
        for (int r = 0; r < g->P && e == hipSuccess; ++r)
            e = hipMemcpyAsync(recv + (size_t)r * n, g->posted[r], n * sizeof(int64_t), hipMemcpyDefault, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        const bool met = g->barrier();   // every peer done reading this rank's buffer (also on error)
        HIPC(e);
        return met ? IAS_SUCCESS : lost();
    }
    ias_status bcast_group(const std::vector<Bcast> &ops, hipStream_t s) override {
        HIPC(hipStreamSynchronize(s));
        g->posted_ops[rank] = ops;
        if (!g->barrier()) return lost();
        hipError_t e = hipSuccess;
        for (size_t k = 0; k < ops.size() && e == hipSuccess; ++k) {
            const auto &root_ops = g->posted_ops[ops[k].root];
            const void *src = k < root_ops.size() ? root_ops[k].send : nullptr;
            if (!src) {
                e = hipErrorInvalidValue;
                break;
            }
            if (src != ops[k].recv && ops[k].bytes)
                e = hipMemcpyAsync(ops[k].recv, src, ops[k].bytes, hipMemcpyDefault, s);
        }
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        const bool met = g->barrier();
        if (!met) return lost();
        if (e != hipSuccess) {
            set_last_error("loopback broadcast: %s", hipGetErrorString(e));
            return IAS_ERROR_DEVICE;
        }
        return IAS_SUCCESS;
    }
};

}  // namespace

struct ias_dist {
    std::unique_ptr<Transport> tr;
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

static ias_status dist_finish(ias_dist *d, int32_t device, ias_dist **out) {
    const ias_status s = ias_plan_create(&d->plan, device, nullptr);
    if (s != IAS_SUCCESS) {
        delete d;
        return s;
    }
    *out = d;
    return IAS_SUCCESS;
}

extern "C" ias_status ias_dist_create(ias_dist **out, const char *id, int32_t nranks, int32_t rank, int32_t device) {
    if (!out || !id || nranks < 1 || rank < 0 || rank >= nranks) return IAS_ERROR_INVALID_ARGUMENT;
    const Rccl *R = rccl();
    if (!R) return IAS_ERROR_DEVICE;
    HIPC(hipSetDevice(device));
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    ncclComm_t comm = nullptr;
    const ncclResult_t rc = R->CommInitRank(&comm, nranks, u, rank);
    if (rc != ncclSuccess) {
        set_last_error("ncclCommInitRank: %s", R->GetErrorString ? R->GetErrorString(rc) : "rccl error");
        return IAS_ERROR_DEVICE;
    }
    ias_dist *d = new ias_dist;
    d->tr.reset(new RcclTransport(R, comm));
    d->rank = rank;
    d->nranks = nranks;
    d->device = device;
    return dist_finish(d, device, out);
}

extern "C" ias_status ias_dist_create_loopback(ias_dist **out, const char *group, int32_t nranks, int32_t rank,
                                               int32_t device) {
    if (!out || !group || nranks < 1 || rank < 0 || rank >= nranks) return IAS_ERROR_INVALID_ARGUMENT;
    HIPC(hipSetDevice(device));
    std::shared_ptr<LoopGroup> g;
    {
        std::lock_guard<std::mutex> lk(loop_registry_mu());
        auto &reg = loop_registry();
        auto it = reg.find(group);
        if (it != reg.end()) g = it->second.lock();
        if (g && g->P != nranks) {
            set_last_error("loopback group '%s' has %d ranks, not %d", group, g->P, nranks);
            return IAS_ERROR_INVALID_ARGUMENT;
        }
        if (!g) {
            g = std::make_shared<LoopGroup>(nranks);
            reg[group] = g;
        }
    }
    ias_dist *d = new ias_dist;
    d->tr.reset(new LoopTransport(g, rank));
    d->rank = rank;
    d->nranks = nranks;
    d->device = device;
    return dist_finish(d, device, out);
}

extern "C" ias_status ias_dist_destroy(ias_dist *d) {
    if (!d) return IAS_SUCCESS;
    if (d->plan) ias_plan_destroy(d->plan);
    delete d;
    return IAS_SUCCESS;
}

extern "C" ias_status ias_dist_allgatherv_csr(ias_dist *d, const ias_csr *Cl, ias_csr *Cf, void *stream) {
    if (!d || !Cl || !Cf) return IAS_ERROR_INVALID_ARGUMENT;
    if (Cl->memory != IAS_MEMORY_DEVICE || Cl->device != d->device) return IAS_ERROR_INVALID_ARGUMENT;
    HIPC(hipSetDevice(d->device));
    hipStream_t s = (hipStream_t)stream;
    const int P = d->nranks;
    // C_local may be a row view: its entries start at row_ptr[0].  Read on the
    // caller's stream after the work it queued (a non-blocking stream may
    // still be producing C_local).
    int64_t rp0 = 0;
    if (Cl->rows > 0) {
        HIPC(hipMemcpyAsync(&rp0, Cl->row_ptr, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        HIPC(hipStreamSynchronize(s));
    }
    // per-rank (rows, nnz)
    std::vector<int64_t> h(2 * (P + 1));
    {
        void *cntv = nullptr;
        IAS_TRY(dev_alloc(&cntv, sizeof(int64_t) * 2 * (P + 1), d->device));
        int64_t *cnt = (int64_t *)cntv;
        h[0] = Cl->rows;
        h[1] = Cl->nnz;
        hipError_t e = hipMemcpyAsync(cnt + 2 * P, h.data(), 2 * sizeof(int64_t), hipMemcpyHostToDevice, s);
        ias_status st = e == hipSuccess ? d->tr->allgather_i64(cnt + 2 * P, cnt, 2, s) : IAS_ERROR_DEVICE;
        if (st == IAS_SUCCESS) {
            e = hipMemcpyAsync(h.data(), cnt, sizeof(int64_t) * 2 * P, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e != hipSuccess) st = IAS_ERROR_DEVICE;
        }
        if (e != hipSuccess) set_last_error("allgatherv counts: %s", hipGetErrorString(e));
        hipStreamSynchronize(s);
        dev_free(cnt, d->device);
        IAS_TRY(st);
    }
    std::vector<int64_t> roff(P + 1, 0), noff(P + 1, 0);
    for (int r = 0; r < P; ++r) {
        roff[r + 1] = roff[r] + h[2 * r];
        noff[r + 1] = noff[r] + h[2 * r + 1];
    }
    ias_csr F{};
    IAS_TRY(ias_csr_alloc(&F, roff[P], Cl->cols, noff[P], IAS_MEMORY_DEVICE, d->device));
    struct Guard {
        ias_csr *F;
        hipStream_t s;
        ~Guard() {
            if (F) {
                hipStreamSynchronize(s);
                ias_csr_free(F);
            }
        }
    } guard{&F, s};
    auto hipc = [](hipError_t e) -> ias_status {
        if (e == hipSuccess) return IAS_SUCCESS;
        set_last_error("allgatherv: %s", hipGetErrorString(e));
        return e == hipErrorOutOfMemory ? IAS_ERROR_OUT_OF_MEMORY : IAS_ERROR_DEVICE;
    };
    IAS_TRY(hipc(hipMemsetAsync(F.row_ptr, 0, sizeof(int64_t), s)));
    // this rank's row ends, shifted into the global numbering, land in place
    if (Cl->rows > 0)
        k_shift_ends<<<(unsigned)((Cl->rows + 255) / 256), 256, 0, s>>>(Cl->row_ptr, Cl->rows, noff[d->rank],
                                                                        F.row_ptr + 1 + roff[d->rank]);
    IAS_TRY(hipc(hipGetLastError()));
    std::vector<Bcast> ops;
    for (int r = 0; r < P; ++r) {
        const bool me = r == d->rank;
        const int64_t rows = h[2 * r], nnz = h[2 * r + 1];
        if (rows > 0) {
            int64_t *slot = F.row_ptr + 1 + roff[r];
            ops.push_back(Bcast{slot, slot, sizeof(int64_t) * (size_t)rows, r});
        }
        if (nnz > 0) {
            ops.push_back(Bcast{me ? (const void *)(Cl->col + rp0) : nullptr, F.col + noff[r],
                                sizeof(int32_t) * (size_t)nnz, r});
            ops.push_back(Bcast{me ? (const void *)(Cl->val + rp0) : nullptr, F.val + noff[r],
                                sizeof(double) * (size_t)nnz, r});
        }
    }
    IAS_TRY(d->tr->bcast_group(ops, s));
    IAS_TRY(hipc(hipStreamSynchronize(s)));
    *Cf = F;
    guard.F = nullptr;
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
