// ias_api.hip — C-ABI glue of libias.so: memory, plans, the SpGEMM entry
// points (CSR / COO / ELL over the shared engine), two-phase form, sums,
// flops, row views and multi-GPU helpers.  Reference counterparts are cited
// per function in include/ias.h.
#include "ias.h"
#include "ias_internal.hpp"
#include "spgemm_engine.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

namespace ias {

static thread_local char g_last_error[512] = "";
static thread_local uint32_t g_last_diag = 0u;
void set_last_diag(uint32_t flags) { g_last_diag = flags; }

void set_last_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_last_error, sizeof g_last_error, fmt, ap);
    va_end(ap);
}

void *host_alloc(size_t bytes, bool zero) {
    void *p = zero ? calloc(bytes ? bytes : 1, 1) : malloc(bytes ? bytes : 1);
    return p;
}
void host_free(void *p) { free(p); }

#define HIPC(x)                                                                   \
    do {                                                                          \
        hipError_t _e = (x);                                                      \
        if (_e != hipSuccess) {                                                   \
            set_last_error("%s failed: %s", #x, hipGetErrorString(_e));           \
            return _e == hipErrorOutOfMemory ? IAS_ERROR_OUT_OF_MEMORY : IAS_ERROR_DEVICE; \
        }                                                                         \
    } while (0)

// Device blocks of the library-allocated outputs and staging copies go
// through a small per-device cache: blocks up to 256 MiB are rounded to a
// power of two and kept on free (up to 1 GiB per device) instead of
// hipFree'd — hipFree costs hundreds of µs (it synchronises the device and
// unmaps), which dominated calls on small operands (K1 through the DIA kernel:
// 0.43 ms per call around a 32 µs kernel).  Returning a block to the cache
// keeps hipFree's ordering guarantee: the device is synchronised first (a few
// µs when idle), so no kernel of any stream — an error path's side streams, a
// caller's own work on a library-allocated output — still reads or writes a
// block a later call may be handed.  When hipMalloc runs out of memory the
// device's cached free blocks are released and the allocation retried once.
namespace {
struct BlockCache {
    static constexpr size_t MAX_BLOCK = 256ull << 20, MAX_TOTAL = 1ull << 30;
    std::mutex mu;
    std::map<std::pair<int, size_t>, std::vector<void *>> free;   // (device, size) -> blocks
    std::map<void *, size_t> size_of;                           // cached-class blocks in use or free
    // freed blocks whose last users may still run: they join `free` after one
    // device-wide synchronisation, taken when an allocation would reuse them
    // (one sync per call that allocates, not one per freed array).  Each
    // pending block is numbered from a per-device counter that only grows;
    // a sync settles exactly the blocks numbered below the counter's value
    // read before it (another thread may settle or queue blocks meanwhile, so
    // positions in the vector mean nothing).
    struct Pending {
        void *p;
        size_t size;
        uint64_t seq;
    };
    std::vector<Pending> pending[64];
    uint64_t next_seq[64] = {};
    size_t held[64] = {};
    // pending blocks queued before a device sync that then completed -> free
    // (caller holds the lock; `upto` = next_seq[device] read under the lock
    // BEFORE that sync)
    void settle(int device, uint64_t upto) {
        auto &v = pending[device];
        size_t k = 0;
        for (size_t i = 0; i < v.size(); ++i) {
            if (v[i].seq < upto) free[{device, v[i].size}].push_back(v[i].p);
            else v[k++] = v[i];
        }
        v.resize(k);
    }
    static size_t round(size_t b) {
        size_t r = 256;
        while (r < b) r <<= 1;
        return r;
    }
    // hipFree every cached free block of `device` (caller holds no lock)
    size_t trim(int device) {
        std::vector<void *> drop;
        size_t bytes = 0;
        uint64_t snap;
        {
            std::lock_guard<std::mutex> g(mu);
            snap = next_seq[device];
        }
        (void)hipDeviceSynchronize();
        {
            std::lock_guard<std::mutex> g(mu);
            settle(device, snap);
            for (auto it = free.begin(); it != free.end();) {
                if (it->first.first == device) {
                    for (void *q : it->second) {
                        drop.push_back(q);
                        size_of.erase(q);
                        bytes += it->first.second;
                    }
                    held[device] -= it->first.second * it->second.size();
                    it = free.erase(it);
                } else {
                    ++it;
                }
            }
        }
        for (void *q : drop) hipFree(q);
        return bytes;
    }
    size_t held_bytes(int device) {
        std::lock_guard<std::mutex> g(mu);
        return device >= 0 && device < 64 ? held[device] : 0;
    }
};
BlockCache &cache() {
    static BlockCache *c = new BlockCache;   // never destroyed: blocks may be freed at exit
    return *c;
}
}  // namespace

ias_status dev_alloc(void **p, size_t bytes, int device) {
    *p = nullptr;
    HIPC(hipSetDevice(device));
    if (bytes == 0) bytes = 8;
    BlockCache &c = cache();
    const bool cached = bytes <= BlockCache::MAX_BLOCK && device >= 0 && device < 64;
    const size_t want = cached ? BlockCache::round(bytes) : bytes;
    if (cached) {
        bool sync = false;
        uint64_t snap = 0;
        {
            std::lock_guard<std::mutex> g(c.mu);
            auto it = c.free.find({device, want});
            if (it != c.free.end() && !it->second.empty()) {
                *p = it->second.back();
                it->second.pop_back();
                c.held[device] -= want;
                return IAS_SUCCESS;
            }
            for (auto &b : c.pending[device]) sync = sync || b.size == want;
            snap = c.next_seq[device];
        }
        if (sync) {
            // a freed block of this size exists: wait for its last users (only
            // the blocks pending before this sync are settled by it)
            HIPC(hipDeviceSynchronize());
            std::lock_guard<std::mutex> g(c.mu);
            c.settle(device, snap);
            auto it = c.free.find({device, want});
            if (it != c.free.end() && !it->second.empty()) {
                *p = it->second.back();
                it->second.pop_back();
                c.held[device] -= want;
                return IAS_SUCCESS;
            }
        }
    }
    hipError_t e = hipMalloc(p, want);
    if (e == hipErrorOutOfMemory && device >= 0 && device < 64) {
        (void)hipGetLastError();
        release_device_memory(device, nullptr);
        e = hipMalloc(p, want);
    }
    HIPC(e);
    if (cached) {
        std::lock_guard<std::mutex> g(c.mu);
        c.size_of[*p] = want;
    }
    return IAS_SUCCESS;
}
ias_status dev_free(void *p, int device) {
    if (!p) return IAS_SUCCESS;
    BlockCache &c = cache();
    bool keep = false;
    {
        std::lock_guard<std::mutex> g(c.mu);
        auto it = c.size_of.find(p);
        if (it != c.size_of.end() && device >= 0 && device < 64) {
            if (c.held[device] + it->second <= BlockCache::MAX_TOTAL) keep = true;
            else c.size_of.erase(it);
        }
    }
    HIPC(hipSetDevice(device));
    if (keep) {
        // hipFree's ordering: nothing still running may touch the block once
        // a later call is handed it — the block waits in `pending` until an
        // allocation synchronises the device (dev_alloc)
        std::lock_guard<std::mutex> g(c.mu);
        const size_t r = c.size_of[p];
        c.pending[device].push_back({p, r, c.next_seq[device]++});
        c.held[device] += r;
        return IAS_SUCCESS;
    }
    HIPC(hipFree(p));
    return IAS_SUCCESS;
}
ias_status dev_copy_h2d(void *dst, const void *src, size_t bytes, int device) {
    if (!bytes) return IAS_SUCCESS;
    HIPC(hipSetDevice(device));
    HIPC(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    return IAS_SUCCESS;
}
ias_status dev_copy_d2h(void *dst, const void *src, size_t bytes, int device) {
    if (!bytes) return IAS_SUCCESS;
    HIPC(hipSetDevice(device));
    HIPC(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return IAS_SUCCESS;
}
ias_status dev_memset(void *p, int value, size_t bytes, int device) {
    if (!bytes) return IAS_SUCCESS;
    HIPC(hipSetDevice(device));
    HIPC(hipMemset(p, value, bytes));
    return IAS_SUCCESS;
}

ias_status check_csr_host(const ias_csr *A) {
    if (A->rows < 0 || A->cols < 0 || A->nnz < 0) return IAS_ERROR_INVALID_ARGUMENT;
    if (A->rows > INT32_MAX || A->cols > INT32_MAX) return IAS_ERROR_OVERFLOW;
    if (!A->row_ptr) return IAS_ERROR_INVALID_ARGUMENT;
    if (A->nnz > 0 && (!A->col || !A->val)) return IAS_ERROR_INVALID_ARGUMENT;
    return IAS_SUCCESS;
}

// Generic copy of one array between host/device memories.
static ias_status move_bytes(void **dst, const void *src, size_t bytes, int src_mem, int src_dev,
                             int dst_mem, int dst_dev) {
    *dst = nullptr;
    if (dst_mem == IAS_MEMORY_DEVICE) {
        IAS_TRY(dev_alloc(dst, bytes, dst_dev));
        if (!bytes || !src) return IAS_SUCCESS;
        HIPC(hipSetDevice(dst_dev));
        if (src_mem == IAS_MEMORY_DEVICE) HIPC(hipMemcpy(*dst, src, bytes, hipMemcpyDeviceToDevice));
        else HIPC(hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice));
    } else {
        *dst = host_alloc(bytes, false);
        if (!*dst) return IAS_ERROR_OUT_OF_MEMORY;
        if (!bytes || !src) return IAS_SUCCESS;
        if (src_mem == IAS_MEMORY_DEVICE) {
            HIPC(hipSetDevice(src_dev));
            HIPC(hipMemcpy(*dst, src, bytes, hipMemcpyDeviceToHost));
        } else {
            memcpy(*dst, src, bytes);
        }
    }
    return IAS_SUCCESS;
}

static void release(void *p, int mem, int dev) {
    if (!p) return;
    if (mem == IAS_MEMORY_DEVICE) dev_free(p, dev);
    else free(p);
}

}  // namespace ias

using namespace ias;

// =================================================================== misc
extern "C" int ias_abi_version(void) { return IAS_ABI_VERSION; }

extern "C" const char *ias_status_string(ias_status s) {
    switch (s) {
        case IAS_SUCCESS: return "success";
        case IAS_ERROR_INVALID_ARGUMENT: return "invalid argument";
        case IAS_ERROR_DIMENSION_MISMATCH: return "dimension mismatch";
        case IAS_ERROR_OUT_OF_MEMORY: return "out of memory";
        case IAS_ERROR_DEVICE: return "device error";
        case IAS_ERROR_IO: return "I/O error";
        case IAS_ERROR_FORMAT: return "bad Matrix-Market format";
        case IAS_ERROR_UNSUPPORTED: return "unsupported";
        case IAS_ERROR_INFEASIBLE: return "format infeasible under the size gate";
        case IAS_ERROR_OVERFLOW: return "index overflow";
        case IAS_ERROR_UNAVAILABLE: return "runtime unavailable";
        case IAS_ERROR_INSUFFICIENT_CAPACITY: return "insufficient capacity";
    }
    return "unknown status";
}

extern "C" const char *ias_last_error(void) { return g_last_error; }
extern "C" uint32_t ias_last_diag(void) { return g_last_diag; }

extern "C" ias_status ias_device_count(int32_t *count) {
    if (!count) return IAS_ERROR_INVALID_ARGUMENT;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *count = 0;
        set_last_error("hipGetDeviceCount: %s", hipGetErrorString(e));
        return IAS_ERROR_DEVICE;
    }
    *count = n;
    return IAS_SUCCESS;
}

extern "C" void ias_opts_default(ias_opts *o) {
    if (!o) return;
    memset(o, 0, sizeof *o);
    o->order = IAS_ORDER_REFERENCE;
    o->output_memory = -1;
    o->device = -1;
}

extern "C" ias_status ias_plan_create(ias_plan **plan, int32_t device, void *stream) {
    if (!plan) return IAS_ERROR_INVALID_ARGUMENT;
    *plan = nullptr;
    int32_t n = 0;
    IAS_TRY(ias_device_count(&n));
    if (device < 0 || device >= n) {
        set_last_error("device %d not present (%d devices)", device, n);
        return IAS_ERROR_DEVICE;
    }
    std::unique_ptr<ias_plan> p(new ias_plan());
    IAS_TRY(p->init(device, stream));
    *plan = p.release();
    return IAS_SUCCESS;
}

extern "C" ias_status ias_plan_destroy(ias_plan *plan) {
    delete plan;
    return IAS_SUCCESS;
}

// =================================================================== memory
extern "C" ias_status ias_csr_alloc(ias_csr *m, int64_t rows, int64_t cols, int64_t nnz,
                                    int32_t memory, int32_t device) {
    if (!m || rows < 0 || cols < 0 || nnz < 0) return IAS_ERROR_INVALID_ARGUMENT;
    memset(m, 0, sizeof *m);
    m->rows = rows; m->cols = cols; m->nnz = nnz; m->memory = memory; m->device = device;
    void *a = nullptr, *b = nullptr, *c = nullptr;
    ias_status s;
    if ((s = move_bytes(&a, nullptr, sizeof(int64_t) * (rows + 1), memory, device, memory, device)) ||
        (s = move_bytes(&b, nullptr, sizeof(int32_t) * nnz, memory, device, memory, device)) ||
        (s = move_bytes(&c, nullptr, sizeof(double) * nnz, memory, device, memory, device))) {
        release(a, memory, device); release(b, memory, device); release(c, memory, device);
        memset(m, 0, sizeof *m);
        return s;
    }
    m->row_ptr = (int64_t *)a; m->col = (int32_t *)b; m->val = (double *)c;
    return IAS_SUCCESS;
}

// Copies rebase: a row view (row_ptr[0] != 0, col/val addressed absolutely,
// see ias_csr_row_view) becomes a standalone matrix with row_ptr[0] == 0.
extern "C" ias_status ias_csr_copy(const ias_csr *src, ias_csr *dst, int32_t memory,
                                   int32_t device) {
    if (!src || !dst || !src->row_ptr || src->rows < 0) return IAS_ERROR_INVALID_ARGUMENT;
    int64_t ends[2] = {0, 0};
    if (src->memory == IAS_MEMORY_DEVICE) {
        IAS_TRY(dev_copy_d2h(&ends[0], src->row_ptr, sizeof(int64_t), src->device));
        IAS_TRY(dev_copy_d2h(&ends[1], src->row_ptr + src->rows, sizeof(int64_t), src->device));
    } else {
        ends[0] = src->row_ptr[0];
        ends[1] = src->row_ptr[src->rows];
    }
    const int64_t base = ends[0], nnz = ends[1] - ends[0];
    if (nnz < 0) return IAS_ERROR_INVALID_ARGUMENT;
    ias_csr t{};
    t.rows = src->rows; t.cols = src->cols; t.nnz = nnz; t.memory = memory; t.device = device;
    void *a = nullptr, *b = nullptr, *c = nullptr;
    ias_status s;
    if ((s = move_bytes(&a, src->row_ptr, sizeof(int64_t) * (src->rows + 1), src->memory, src->device, memory, device)) ||
        (s = move_bytes(&b, src->col ? src->col + base : nullptr, sizeof(int32_t) * nnz, src->memory, src->device, memory, device)) ||
        (s = move_bytes(&c, src->val ? src->val + base : nullptr, sizeof(double) * nnz, src->memory, src->device, memory, device))) {
        release(a, memory, device); release(b, memory, device); release(c, memory, device);
        return s;
    }
    t.row_ptr = (int64_t *)a; t.col = (int32_t *)b; t.val = (double *)c;
    if (base != 0) {
        if (memory == IAS_MEMORY_DEVICE) {
            s = ias_shift_device(t.row_ptr, src->rows + 1, -base, nullptr);
            if (s == IAS_SUCCESS && hipDeviceSynchronize() != hipSuccess) s = IAS_ERROR_DEVICE;
        } else {
            for (int64_t i = 0; i <= src->rows; ++i) t.row_ptr[i] -= base;
        }
        if (s != IAS_SUCCESS) {
            release(a, memory, device); release(b, memory, device); release(c, memory, device);
            return s;
        }
    }
    *dst = t;
    return IAS_SUCCESS;
}

extern "C" ias_status ias_csr_free(ias_csr *m) {
    if (!m) return IAS_ERROR_INVALID_ARGUMENT;
    release(m->row_ptr, m->memory, m->device);
    release(m->col, m->memory, m->device);
    release(m->val, m->memory, m->device);
    memset(m, 0, sizeof *m);
    return IAS_SUCCESS;
}
extern "C" ias_status ias_coo_free(ias_coo *m) {
    if (!m) return IAS_ERROR_INVALID_ARGUMENT;
    release(m->row_offset, m->memory, m->device);
    release(m->row, m->memory, m->device);
    release(m->col, m->memory, m->device);
    release(m->val, m->memory, m->device);
    memset(m, 0, sizeof *m);
    return IAS_SUCCESS;
}
extern "C" ias_status ias_ell_free(ias_ell *m) {
    if (!m) return IAS_ERROR_INVALID_ARGUMENT;
    release(m->nnz_row, m->memory, m->device);
    release(m->col, m->memory, m->device);
    release(m->val, m->memory, m->device);
    memset(m, 0, sizeof *m);
    return IAS_SUCCESS;
}
extern "C" ias_status ias_dia_free(ias_dia *m) {
    if (!m) return IAS_ERROR_INVALID_ARGUMENT;
    release(m->diagonal_offsets, m->memory, m->device);
    release(m->diagonal_ind, m->memory, m->device);
    release(m->val, m->memory, m->device);
    memset(m, 0, sizeof *m);
    return IAS_SUCCESS;
}

extern "C" ias_status ias_coo_copy(const ias_coo *src, ias_coo *dst, int32_t memory, int32_t device) {
    if (!src || !dst) return IAS_ERROR_INVALID_ARGUMENT;
    ias_coo t = *src;
    t.memory = memory; t.device = device;
    void *a = nullptr, *b = nullptr, *c = nullptr, *d = nullptr;
    ias_status s;
    if ((s = move_bytes(&a, src->row_offset, sizeof(int64_t) * (src->rows + 1), src->memory, src->device, memory, device)) ||
        (s = move_bytes(&b, src->row, sizeof(int32_t) * src->nnz, src->memory, src->device, memory, device)) ||
        (s = move_bytes(&c, src->col, sizeof(int32_t) * src->nnz, src->memory, src->device, memory, device)) ||
        (s = move_bytes(&d, src->val, sizeof(double) * src->nnz, src->memory, src->device, memory, device))) {
        release(a, memory, device); release(b, memory, device); release(c, memory, device); release(d, memory, device);
        return s;
    }
    t.row_offset = (int64_t *)a; t.row = (int32_t *)b; t.col = (int32_t *)c; t.val = (double *)d;
    *dst = t;
    return IAS_SUCCESS;
}

extern "C" ias_status ias_ell_copy(const ias_ell *src, ias_ell *dst, int32_t memory, int32_t device) {
    if (!src || !dst) return IAS_ERROR_INVALID_ARGUMENT;
    ias_ell t = *src;
    t.memory = memory; t.device = device;
    const size_t rk = (size_t)src->rows * (size_t)src->max_nnz_per_row;
    void *a = nullptr, *b = nullptr, *c = nullptr;
    ias_status s;
    if ((s = move_bytes(&a, src->nnz_row, sizeof(int32_t) * src->rows, src->memory, src->device, memory, device)) ||
        (s = move_bytes(&b, src->col, sizeof(int32_t) * rk, src->memory, src->device, memory, device)) ||
        (s = move_bytes(&c, src->val, sizeof(double) * rk, src->memory, src->device, memory, device))) {
        release(a, memory, device); release(b, memory, device); release(c, memory, device);
        return s;
    }
    t.nnz_row = (int32_t *)a; t.col = (int32_t *)b; t.val = (double *)c;
    *dst = t;
    return IAS_SUCCESS;
}

extern "C" ias_status ias_dia_copy(const ias_dia *src, ias_dia *dst, int32_t memory, int32_t device) {
    if (!src || !dst) return IAS_ERROR_INVALID_ARGUMENT;
    ias_dia t = *src;
    t.memory = memory; t.device = device;
    const size_t rn = (size_t)src->rows * (size_t)src->num_diagonals;
    const size_t span = (size_t)std::max<int64_t>(src->rows + src->cols - 1, 0);
    void *a = nullptr, *b = nullptr, *c = nullptr;
    ias_status s;
    if ((s = move_bytes(&a, src->diagonal_offsets, sizeof(int32_t) * src->num_diagonals, src->memory, src->device, memory, device)) ||
        (s = move_bytes(&b, src->diagonal_ind, sizeof(int32_t) * span, src->memory, src->device, memory, device)) ||
        (s = move_bytes(&c, src->val, sizeof(double) * rn, src->memory, src->device, memory, device))) {
        release(a, memory, device); release(b, memory, device); release(c, memory, device);
        return s;
    }
    t.diagonal_offsets = (int32_t *)a; t.diagonal_ind = (int32_t *)b; t.val = (double *)c;
    *dst = t;
    return IAS_SUCCESS;
}

// =================================================================== SpGEMM
namespace {

// When the caller passes no plan (and no stream), a per-device default plan
// kept for the life of the process serves the call — as a cuSPARSE handle
// would — so repeated one-shot calls do not re-create streams, events and the
// workspace (the first K3' call spent ~120 ms of its 133 ms there).  A call
// that finds the default plan busy (another host thread) or brings its own
// stream gets a temporary plan.  IAS_DEFAULT_PLAN=0 always uses temporaries.
struct DefaultPlans {
    std::mutex mu;
    std::map<int, ias_plan *> plan;
    std::map<int, bool> busy;
};
DefaultPlans &default_plans() {
    static DefaultPlans *d = new DefaultPlans;   // never destroyed (plans may be in use at exit)
    return *d;
}
}  // namespace

size_t ias::release_device_memory(int device, const ias_plan *keep) {
    size_t bytes = cache().trim(device);
    DefaultPlans &d = default_plans();
    std::lock_guard<std::mutex> g(d.mu);
    auto it = d.plan.find(device);
    if (it != d.plan.end() && it->second && it->second != keep && !d.busy[device])
        bytes += it->second->release_workspace();
    return bytes;
}

namespace {
bool default_plan_on() {
    static const bool on = [] {
        const char *e = getenv("IAS_DEFAULT_PLAN");
        return !(e && *e == '0');
    }();
    return on;
}
struct PlanGuard {
    ias_plan *p = nullptr;
    bool owned = false, pooled = false;
    int dev = 0;
    ~PlanGuard() {
        if (owned) ias_plan_destroy(p);
        if (pooled) {
            DefaultPlans &d = default_plans();
            std::lock_guard<std::mutex> g(d.mu);
            d.busy[dev] = false;
        }
    }
    ias_status acquire(const ias_opts &o, int device) {
        if (o.plan) {
            p = o.plan;
            return IAS_SUCCESS;
        }
        if (!o.stream && default_plan_on()) {
            DefaultPlans &d = default_plans();
            std::unique_lock<std::mutex> g(d.mu);
            if (!d.busy[device]) {
                ias_plan *&dp = d.plan[device];
                if (!dp) {
                    g.unlock();
                    ias_plan *np = nullptr;
                    IAS_TRY(ias_plan_create(&np, device, nullptr));
                    g.lock();
                    if (!dp) dp = np;
                    else ias_plan_destroy(np);
                }
                if (!d.busy[device]) {
                    d.busy[device] = true;
                    pooled = true;
                    dev = device;
                    p = dp;
                    return IAS_SUCCESS;
                }
            }
        }
        owned = true;
        return ias_plan_create(&p, device, o.stream);
    }
};

// Device-resident copies of host operands, released at scope exit.
struct Staged {
    std::vector<std::pair<void *, int>> owned;
    ~Staged() {
        for (auto &x : owned) dev_free(x.first, x.second);
    }
    template <typename T>
    ias_status stage(const T *src, size_t count, int mem, int srcdev, int device, const T **out) {
        if (mem == IAS_MEMORY_DEVICE && srcdev == device) {
            *out = src;
            return IAS_SUCCESS;
        }
        void *d = nullptr;
        IAS_TRY(move_bytes(&d, src, sizeof(T) * count, mem, srcdev, IAS_MEMORY_DEVICE, device));
        owned.push_back({d, device});
        *out = (const T *)d;
        return IAS_SUCCESS;
    }
};

// A CSR operand on the compute device: the caller's when already there, else
// a rebased copy owned (and freed) by this holder.
struct StagedCsr {
    ias_csr own{};
    const ias_csr *use = nullptr;
    bool owned = false;
    ~StagedCsr() {
        if (owned) ias_csr_free(&own);
    }
    ias_status stage(const ias_csr *m, int device) {
        if (m->memory == IAS_MEMORY_DEVICE && m->device == device) {
            use = m;
            return IAS_SUCCESS;
        }
        IAS_TRY(ias_csr_copy(m, &own, IAS_MEMORY_DEVICE, device));
        owned = true;
        use = &own;
        return IAS_SUCCESS;
    }
    const ias_csr *get() const { return use; }
};

ias_opts resolve(const ias_opts *opts) {
    ias_opts o;
    ias_opts_default(&o);
    if (opts) o = *opts;
    return o;
}

int pick_device(const ias_opts &o, int a_mem, int a_dev) {
    if (o.device >= 0) return o.device;
    if (a_mem == IAS_MEMORY_DEVICE) return a_dev;
    return 0;
}

// host wall clock (ms) for the synchronous PCIe staging of host operands
double host_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

double ms_since(hipEvent_t a, hipEvent_t b) {
    float t = 0;
    hipEventElapsedTime(&t, a, b);
    return t;
}

}  // namespace

extern "C" ias_status ias_csr_mul_csr(const ias_csr *A, const ias_csr *B, ias_csr *C,
                                      const ias_opts *opts, ias_report *rep) {
    if (!A || !B || !C) return IAS_ERROR_INVALID_ARGUMENT;
    IAS_TRY(check_csr_host(A));
    IAS_TRY(check_csr_host(B));
    if (A->cols != B->rows) return IAS_ERROR_DIMENSION_MISMATCH;
    const ias_opts o = resolve(opts);
    if (o.order != IAS_ORDER_REFERENCE && o.order != IAS_ORDER_SORTED) return IAS_ERROR_INVALID_ARGUMENT;
    const int device = pick_device(o, A->memory, A->device);
    const int out_mem = o.output_memory >= 0 ? o.output_memory : A->memory;
    if (rep) memset(rep, 0, sizeof *rep);
    PlanGuard pg;
    IAS_TRY(pg.acquire(o, device));
    ias_plan *plan = pg.p;
    HIPC(hipSetDevice(plan->device));
    hipStream_t s = (hipStream_t)plan->stream;

    // Operands not resident on the compute device are copied there (rebased,
    // so host row views work); resident ones, views included, are used as-is.
    StagedCsr sa, sb;
    const double t_up = host_ms();
    IAS_TRY(sa.stage(A, plan->device));
    const ias_csr *dA = sa.get(), *dB = dA;
    if (B != A) {
        IAS_TRY(sb.stage(B, plan->device));
        dB = sb.get();
    }
    if (rep && (sa.owned || sb.owned)) rep->ms_upload = host_ms() - t_up;
    dev::Rows ra{dA->row_ptr, nullptr, 0, dA->col, dA->val};
    dev::Rows rb{dB->row_ptr, nullptr, 0, dB->col, dB->val};
    ias_csr D{};
    plan->last_a = plan->last_b = nullptr;
    IAS_TRY(plan->symbolic(ra, rb, A->rows, B->cols, dA->nnz, rep));
    const int64_t nnz = plan->nnz_total;
    IAS_TRY(ias_csr_alloc(&D, A->rows, B->cols, nnz, IAS_MEMORY_DEVICE, plan->device));
    HIPC(hipMemcpyAsync(D.row_ptr, plan->bufs[ias_plan::B_PTR].p, sizeof(int64_t) * (A->rows + 1),
                        hipMemcpyDeviceToDevice, s));
    dev::Out out{D.row_ptr, 0, D.col, D.val, nullptr, 0, 0, nullptr};
    ias_status stn = plan->numeric(ra, rb, out, rep);
    if (stn == IAS_SUCCESS && o.order == IAS_ORDER_SORTED)
        stn = ias_sort_rows_device(plan, D.row_ptr, A->rows, D.col, D.val, plan->max_nnz);
    if (stn != IAS_SUCCESS) {
        ias_csr_free(&D);
        return stn;
    }
    HIPC(hipStreamSynchronize(s));
    if (out_mem == IAS_MEMORY_HOST) {
        ias_csr H{};
        const double t_dn = host_ms();
        ias_status cs = ias_csr_copy(&D, &H, IAS_MEMORY_HOST, 0);
        if (rep) rep->ms_download = host_ms() - t_dn;
        ias_csr_free(&D);
        if (cs != IAS_SUCCESS) return cs;
        *C = H;
    } else {
        *C = D;
    }
    return IAS_SUCCESS;
}

extern "C" ias_status ias_coo_mul_coo(const ias_coo *A, const ias_coo *B, ias_coo *C,
                                      const ias_opts *opts, ias_report *rep) {
    if (!A || !B || !C) return IAS_ERROR_INVALID_ARGUMENT;
    if (!A->choice || !B->choice) return IAS_ERROR_INFEASIBLE;
    if (A->cols != B->rows) return IAS_ERROR_DIMENSION_MISMATCH;
    const ias_opts o = resolve(opts);
    const int device = pick_device(o, A->memory, A->device);
    const int out_mem = o.output_memory >= 0 ? o.output_memory : A->memory;
    if (rep) memset(rep, 0, sizeof *rep);
    PlanGuard pg;
    IAS_TRY(pg.acquire(o, device));
    ias_plan *plan = pg.p;
    HIPC(hipSetDevice(plan->device));
    hipStream_t s = (hipStream_t)plan->stream;
    Staged st;
    const int64_t *ap, *bp;
    const int32_t *ac, *bc;
    const double *av, *bv;
    const double t_up = host_ms();
    IAS_TRY(st.stage(A->row_offset, A->rows + 1, A->memory, A->device, plan->device, &ap));
    IAS_TRY(st.stage(A->col, A->nnz, A->memory, A->device, plan->device, &ac));
    IAS_TRY(st.stage(A->val, A->nnz, A->memory, A->device, plan->device, &av));
    if (B == A) {
        bp = ap; bc = ac; bv = av;
    } else {
        IAS_TRY(st.stage(B->row_offset, B->rows + 1, B->memory, B->device, plan->device, &bp));
        IAS_TRY(st.stage(B->col, B->nnz, B->memory, B->device, plan->device, &bc));
        IAS_TRY(st.stage(B->val, B->nnz, B->memory, B->device, plan->device, &bv));
    }
    if (rep && !st.owned.empty()) rep->ms_upload = host_ms() - t_up;
    dev::Rows ra{ap, nullptr, 0, ac, av};
    dev::Rows rb{bp, nullptr, 0, bc, bv};
    IAS_TRY(plan->symbolic(ra, rb, A->rows, B->cols, A->nnz, rep));
    const int64_t nnz = plan->nnz_total;
    ias_coo D{};
    D.rows = A->rows; D.cols = B->cols; D.nnz = nnz; D.memory = IAS_MEMORY_DEVICE;
    D.device = plan->device; D.choice = 1;
    void *p0 = nullptr, *p1 = nullptr, *p2 = nullptr, *p3 = nullptr;
    IAS_TRY(dev_alloc(&p0, sizeof(int64_t) * (A->rows + 1), plan->device));
    D.row_offset = (int64_t *)p0;
    ias_status sa;
    if ((sa = dev_alloc(&p1, sizeof(int32_t) * nnz, plan->device)) ||
        (sa = dev_alloc(&p2, sizeof(int32_t) * nnz, plan->device)) ||
        (sa = dev_alloc(&p3, sizeof(double) * nnz, plan->device))) {
        D.row = (int32_t *)p1; D.col = (int32_t *)p2; D.val = (double *)p3;
        ias_coo_free(&D);
        return sa;
    }
    D.row = (int32_t *)p1; D.col = (int32_t *)p2; D.val = (double *)p3;
    HIPC(hipMemcpyAsync(D.row_offset, plan->bufs[ias_plan::B_PTR].p,
                        sizeof(int64_t) * (A->rows + 1), hipMemcpyDeviceToDevice, s));
    dev::Out out{D.row_offset, 0, D.col, D.val, D.row, o.order == IAS_ORDER_SORTED ? 0 : 1, 1, nullptr};
    ias_status stn = plan->numeric(ra, rb, out, rep);
    if (stn == IAS_SUCCESS && o.order == IAS_ORDER_SORTED)
        stn = ias_sort_rows_device(plan, D.row_offset, A->rows, D.col, D.val, plan->max_nnz);
    if (stn != IAS_SUCCESS) {
        ias_coo_free(&D);
        return stn;
    }
    HIPC(hipStreamSynchronize(s));
    if (out_mem == IAS_MEMORY_HOST) {
        ias_coo H{};
        const double t_dn = host_ms();
        ias_status cs = ias_coo_copy(&D, &H, IAS_MEMORY_HOST, 0);
        if (rep) rep->ms_download = host_ms() - t_dn;
        ias_coo_free(&D);
        if (cs != IAS_SUCCESS) return cs;
        *C = H;
    } else {
        *C = D;
    }
    return IAS_SUCCESS;
}

extern "C" ias_status ias_ell_mul_ell(const ias_ell *A, const ias_ell *B, ias_ell *C,
                                      const ias_opts *opts, ias_report *rep) {
    if (!A || !B || !C) return IAS_ERROR_INVALID_ARGUMENT;
    if (!A->choice || !B->choice) return IAS_ERROR_INFEASIBLE;
    if (A->cols != B->rows) return IAS_ERROR_DIMENSION_MISMATCH;
    const ias_opts o = resolve(opts);
    const int device = pick_device(o, A->memory, A->device);
    const int out_mem = o.output_memory >= 0 ? o.output_memory : A->memory;
    if (rep) memset(rep, 0, sizeof *rep);
    PlanGuard pg;
    IAS_TRY(pg.acquire(o, device));
    ias_plan *plan = pg.p;
    HIPC(hipSetDevice(plan->device));
    hipStream_t s = (hipStream_t)plan->stream;
    Staged st;
    const int32_t *an, *bn, *ac, *bc;
    const double *av, *bv;
    const size_t ak = (size_t)A->rows * A->max_nnz_per_row, bk = (size_t)B->rows * B->max_nnz_per_row;
    const double t_up = host_ms();
    IAS_TRY(st.stage(A->nnz_row, A->rows, A->memory, A->device, plan->device, &an));
    IAS_TRY(st.stage(A->col, ak, A->memory, A->device, plan->device, &ac));
    IAS_TRY(st.stage(A->val, ak, A->memory, A->device, plan->device, &av));
    if (B == A) {
        bn = an; bc = ac; bv = av;
    } else {
        IAS_TRY(st.stage(B->nnz_row, B->rows, B->memory, B->device, plan->device, &bn));
        IAS_TRY(st.stage(B->col, bk, B->memory, B->device, plan->device, &bc));
        IAS_TRY(st.stage(B->val, bk, B->memory, B->device, plan->device, &bv));
    }
    if (rep && !st.owned.empty()) rep->ms_upload = host_ms() - t_up;
    dev::Rows ra{nullptr, an, A->max_nnz_per_row, ac, av};
    dev::Rows rb{nullptr, bn, B->max_nnz_per_row, bc, bv};
    IAS_TRY(plan->symbolic(ra, rb, A->rows, B->cols, (int64_t)ak, rep));
    const int32_t K = plan->max_nnz;
    ias_ell D{};
    D.rows = A->rows; D.cols = B->cols; D.nnz = plan->nnz_total; D.max_nnz_per_row = K;
    D.choice = 1; D.memory = IAS_MEMORY_DEVICE; D.device = plan->device;
    const size_t ck = (size_t)A->rows * (size_t)K;
    void *p0 = nullptr, *p1 = nullptr, *p2 = nullptr;
    ias_status sa;
    if ((sa = dev_alloc(&p0, sizeof(int32_t) * A->rows, plan->device)) ||
        (sa = dev_alloc(&p1, sizeof(int32_t) * ck, plan->device)) ||
        (sa = dev_alloc(&p2, sizeof(double) * ck, plan->device))) {
        D.nnz_row = (int32_t *)p0; D.col = (int32_t *)p1; D.val = (double *)p2;
        ias_ell_free(&D);
        return sa;
    }
    D.nnz_row = (int32_t *)p0; D.col = (int32_t *)p1; D.val = (double *)p2;
    HIPC(hipMemcpyAsync(D.nnz_row, plan->bufs[ias_plan::B_NNZ].p, sizeof(int32_t) * A->rows,
                        hipMemcpyDeviceToDevice, s));
    HIPC(hipMemsetAsync(D.col, 0, sizeof(int32_t) * ck, s));
    HIPC(hipMemsetAsync(D.val, 0, sizeof(double) * ck, s));
    dev::Out out{nullptr, K, D.col, D.val, nullptr, 0, 0, nullptr};
    ias_status stn = plan->numeric(ra, rb, out, rep);
    if (stn == IAS_SUCCESS && o.order == IAS_ORDER_SORTED)
        stn = ias_sort_rows_ell_device(plan, D.nnz_row, A->rows, K, D.col, D.val);
    if (stn != IAS_SUCCESS) {
        ias_ell_free(&D);
        return stn;
    }
    HIPC(hipStreamSynchronize(s));
    if (out_mem == IAS_MEMORY_HOST) {
        ias_ell H{};
        const double t_dn = host_ms();
        ias_status cs = ias_ell_copy(&D, &H, IAS_MEMORY_HOST, 0);
        if (rep) rep->ms_download = host_ms() - t_dn;
        ias_ell_free(&D);
        if (cs != IAS_SUCCESS) return cs;
        *C = H;
    } else {
        *C = D;
    }
    return IAS_SUCCESS;
}

extern "C" ias_status ias_device_release(int32_t device, int64_t *released) {
    int32_t n = 0;
    IAS_TRY(ias_device_count(&n));
    if (device < 0 || device >= n) return IAS_ERROR_INVALID_ARGUMENT;
    HIPC(hipSetDevice(device));
    const size_t b = release_device_memory(device, nullptr);
    if (released) *released = (int64_t)b;
    return IAS_SUCCESS;
}

extern "C" ias_status ias_device_cached_bytes(int32_t device, int64_t *bytes) {
    if (!bytes) return IAS_ERROR_INVALID_ARGUMENT;
    size_t b = cache().held_bytes(device);
    DefaultPlans &d = default_plans();
    {
        std::lock_guard<std::mutex> g(d.mu);
        auto it = d.plan.find(device);
        if (it != d.plan.end() && it->second) b += it->second->workspace_bytes();
    }
    *bytes = (int64_t)b;
    return IAS_SUCCESS;
}

// ------------------------------------------------------------------- two-phase
static ias_status check_dev_csr(const ias_csr *A, const ias_plan *plan) {
    if (!A) return IAS_ERROR_INVALID_ARGUMENT;
    IAS_TRY(check_csr_host(A));
    if (A->memory != IAS_MEMORY_DEVICE || A->device != plan->device) return IAS_ERROR_INVALID_ARGUMENT;
    return IAS_SUCCESS;
}

extern "C" ias_status ias_csr_mul_csr_nnz(ias_plan *plan, const ias_csr *A, const ias_csr *B,
                                          int64_t *nnz_c, int64_t *row_ptr_c, ias_report *rep) {
    if (!plan || !nnz_c) return IAS_ERROR_INVALID_ARGUMENT;
    IAS_TRY(check_dev_csr(A, plan));
    IAS_TRY(check_dev_csr(B, plan));
    if (A->cols != B->rows) return IAS_ERROR_DIMENSION_MISMATCH;
    if (rep) memset(rep, 0, sizeof *rep);
    dev::Rows ra{A->row_ptr, nullptr, 0, A->col, A->val};
    dev::Rows rb{B->row_ptr, nullptr, 0, B->col, B->val};
    IAS_TRY(plan->symbolic(ra, rb, A->rows, B->cols, A->nnz, rep));
    plan->last_a = A->col;
    plan->last_b = B->col;
    *nnz_c = plan->nnz_total;
    if (row_ptr_c) {
        HIPC(hipMemcpyAsync(row_ptr_c, plan->bufs[ias_plan::B_PTR].p, sizeof(int64_t) * (A->rows + 1),
                            hipMemcpyDeviceToDevice, (hipStream_t)plan->stream));
        HIPC((hipError_t)host_wait(plan->stream));
    }
    return IAS_SUCCESS;
}

extern "C" ias_status ias_csr_mul_csr_compute(ias_plan *plan, const ias_csr *A, const ias_csr *B,
                                              ias_csr *C, int32_t order, ias_report *rep) {
    if (!plan || !C) return IAS_ERROR_INVALID_ARGUMENT;
    IAS_TRY(check_dev_csr(A, plan));
    IAS_TRY(check_dev_csr(B, plan));
    if (plan->last_a != A->col || plan->last_b != B->col || plan->n_rows != A->rows)
        return IAS_ERROR_INVALID_ARGUMENT;
    if (C->memory != IAS_MEMORY_DEVICE || C->device != plan->device || !C->row_ptr ||
        (plan->nnz_total > 0 && (!C->col || !C->val)))
        return IAS_ERROR_INVALID_ARGUMENT;
    if (C->nnz < plan->nnz_total) return IAS_ERROR_INSUFFICIENT_CAPACITY;
    hipStream_t s = (hipStream_t)plan->stream;
    HIPC(hipSetDevice(plan->device));
    HIPC(hipMemcpyAsync(C->row_ptr, plan->bufs[ias_plan::B_PTR].p, sizeof(int64_t) * (A->rows + 1),
                        hipMemcpyDeviceToDevice, s));
    C->rows = A->rows;
    C->cols = B->cols;
    C->nnz = plan->nnz_total;
    dev::Rows ra{A->row_ptr, nullptr, 0, A->col, A->val};
    dev::Rows rb{B->row_ptr, nullptr, 0, B->col, B->val};
    dev::Out out{C->row_ptr, 0, C->col, C->val, nullptr, 0, 0, nullptr};
    IAS_TRY(plan->numeric(ra, rb, out, rep));
    if (order == IAS_ORDER_SORTED)
        IAS_TRY(ias_sort_rows_device(plan, C->row_ptr, A->rows, C->col, C->val, plan->max_nnz));
    // C is complete when this returns (callers may read or free it at once,
    // from any stream), as the reference's timer sync does (GPU/detail/utime.h).
    HIPC((hipError_t)host_wait(s));
    return IAS_SUCCESS;
}

extern "C" ias_status ias_csr_mul_csr_into(ias_plan *plan, const ias_csr *A, const ias_csr *B, ias_csr *C,
                                           int32_t order, ias_report *rep) {
    if (!plan || !C) return IAS_ERROR_INVALID_ARGUMENT;
    IAS_TRY(check_dev_csr(A, plan));
    IAS_TRY(check_dev_csr(B, plan));
    if (A->cols != B->rows) return IAS_ERROR_DIMENSION_MISMATCH;
    if (order != IAS_ORDER_REFERENCE && order != IAS_ORDER_SORTED) return IAS_ERROR_INVALID_ARGUMENT;
    if (C->memory != IAS_MEMORY_DEVICE || C->device != plan->device || !C->row_ptr || C->nnz < 0 ||
        (C->nnz > 0 && (!C->col || !C->val)))
        return IAS_ERROR_INVALID_ARGUMENT;
    if (rep) memset(rep, 0, sizeof *rep);
    hipStream_t s = (hipStream_t)plan->stream;
    HIPC(hipSetDevice(plan->device));
    plan->last_a = plan->last_b = nullptr;   // the two-phase state is overwritten
    dev::Rows ra{A->row_ptr, nullptr, 0, A->col, A->val};
    dev::Rows rb{B->row_ptr, nullptr, 0, B->col, B->val};
    C->rows = A->rows;
    C->cols = B->cols;
    int64_t nnz = 0;
    // the two-phase engine behind one call: nnz, then values when they fit
    IAS_TRY(plan->symbolic(ra, rb, A->rows, B->cols, A->nnz, rep));
    nnz = plan->nnz_total;
    HIPC(hipMemcpyAsync(C->row_ptr, plan->bufs[ias_plan::B_PTR].p, sizeof(int64_t) * (A->rows + 1),
                        hipMemcpyDeviceToDevice, s));
    if (nnz > C->nnz) {
        HIPC(hipStreamSynchronize(s));
        set_last_error("C needs %lld entries, capacity %lld", (long long)nnz, (long long)C->nnz);
        C->nnz = nnz;
        return IAS_ERROR_INSUFFICIENT_CAPACITY;
    }
    dev::Out out{C->row_ptr, 0, C->col, C->val, nullptr, 0, 0, nullptr};
    IAS_TRY(plan->numeric(ra, rb, out, rep));
    C->nnz = nnz;
    if (order == IAS_ORDER_SORTED)
        IAS_TRY(ias_sort_rows_device(plan, C->row_ptr, A->rows, C->col, C->val, 0));
    HIPC((hipError_t)host_wait(s));
    return IAS_SUCCESS;
}

int ias::host_wait(void *stream) {
    static const long spin_us = [] {
        const char *e = getenv("IAS_SPIN_US");
        return e && *e ? atol(e) : 200L;
    }();
    hipStream_t s = (hipStream_t)stream;
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t e = hipStreamQuery(s);
        if (e != hipErrorNotReady) return (int)e;
        if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us))
            return (int)hipStreamSynchronize(s);
    }
}

// =================================================================== helpers
extern "C" ias_status ias_csr_row_view(const ias_csr *A, int64_t r0, int64_t r1, ias_csr *view) {
    if (!A || !view || r0 < 0 || r1 < r0 || r1 > A->rows) return IAS_ERROR_INVALID_ARGUMENT;
    ias_csr v = *A;
    v.rows = r1 - r0;
    v.row_ptr = A->row_ptr + r0;
    if (A->memory == IAS_MEMORY_HOST) {
        v.nnz = A->row_ptr[r1] - A->row_ptr[r0];
    } else {
        int64_t e[2];
        IAS_TRY(dev_copy_d2h(&e[0], A->row_ptr + r0, sizeof(int64_t), A->device));
        IAS_TRY(dev_copy_d2h(&e[1], A->row_ptr + r1, sizeof(int64_t), A->device));
        v.nnz = e[1] - e[0];
    }
    *view = v;
    return IAS_SUCCESS;
}

extern "C" ias_status ias_row_ptr_shift(int64_t *row_ptr, int64_t count, int64_t offset,
                                        int32_t device, void *stream) {
    if (!row_ptr || count < 0) return IAS_ERROR_INVALID_ARGUMENT;
    HIPC(hipSetDevice(device));
    return ias_shift_device(row_ptr, count, offset, stream);
}
