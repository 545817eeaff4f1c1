// mkl_baseline.cpp — the reference's Algorithm 1 (MKL_MUL_MKL,
// IA-SPGEMM-CPU_release/detail/csr/common_csr.h:18-47, timed as main.cpp:746-748)
// on the host cores, MKL loaded at run time.  MKL is a third-party runtime of
// the image (/opt/conda/lib/libmkl_rt.so); its published sparse BLAS ABI is
// declared here by hand (no mkl.h in the image).  The GNU threading layer is
// selected because the rest of the process uses libgomp: MKL's default Intel
// layer next to libgomp returns a wrong C.
#include "ias.h"
#include "ias_internal.hpp"

#include <dlfcn.h>
#include <sys/time.h>

#include <mutex>
#include <vector>

using namespace ias;

namespace {

typedef void *sparse_matrix_t;
struct matrix_descr {
    int type, mode, diag;
};
enum {
    SPARSE_STATUS_SUCCESS = 0,
    SPARSE_INDEX_BASE_ZERO = 0,
    SPARSE_OPERATION_NON_TRANSPOSE = 10,
    SPARSE_MATRIX_TYPE_GENERAL = 20,
    SPARSE_FILL_MODE_FULL = 42,
    SPARSE_DIAG_NON_UNIT = 50,
    SPARSE_STAGE_FULL_MULT = 90,
    MKL_THREADING_GNU = 3,
    MKL_INTERFACE_LP64 = 0,
    MKL_INTERFACE_ILP64 = 1,
};

template <typename I>
struct Api {
    int (*create_csr)(sparse_matrix_t *, int, I, I, I *, I *, I *, double *);
    int (*sp2m)(int, matrix_descr, sparse_matrix_t, int, matrix_descr, sparse_matrix_t, int,
                sparse_matrix_t *);
    int (*export_csr)(sparse_matrix_t, int *, I *, I *, I **, I **, I **, double **);
    int (*destroy)(sparse_matrix_t);
};

struct Mkl {
    void *h = nullptr;
    int iface = -1;   // interface layer chosen at first use
    int (*set_threading_layer)(int) = nullptr;
    int (*set_interface_layer)(int) = nullptr;
    void (*set_num_threads)(int) = nullptr;
    void (*get_version_string)(char *, int) = nullptr;
    void *create = nullptr, *sp2m = nullptr, *exp = nullptr, *destroy = nullptr;
    bool load() {
        if (h) return true;
        const char *env = getenv("IAS_MKL_PATH");
        const char *cands[] = {env, "libmkl_rt.so", "libmkl_rt.so.1", "libmkl_rt.so.2",
                               "/opt/conda/lib/libmkl_rt.so.1", "/opt/conda/lib/libmkl_rt.so",
                               "/opt/intel/oneapi/mkl/latest/lib/intel64/libmkl_rt.so"};
        for (const char *c : cands) {
            if (!c) continue;
            h = dlopen(c, RTLD_NOW | RTLD_LOCAL);
            if (h) break;
        }
        if (!h) return false;
        set_threading_layer = (int (*)(int))dlsym(h, "MKL_Set_Threading_Layer");
        set_interface_layer = (int (*)(int))dlsym(h, "MKL_Set_Interface_Layer");
        set_num_threads = (void (*)(int))dlsym(h, "MKL_Set_Num_Threads");
        get_version_string = (void (*)(char *, int))dlsym(h, "MKL_Get_Version_String");
        create = dlsym(h, "mkl_sparse_d_create_csr");
        sp2m = dlsym(h, "mkl_sparse_sp2m");
        exp = dlsym(h, "mkl_sparse_d_export_csr");
        destroy = dlsym(h, "mkl_sparse_destroy");
        if (!create || !sp2m || !exp || !destroy || !set_threading_layer) {
            dlclose(h);
            h = nullptr;
            return false;
        }
        // Layers must be fixed before ANY other MKL call (even the version
        // query), or MKL initialises with its Intel OpenMP layer, which next to
        // libgomp returns a wrong C.
        const char *e = getenv("IAS_MKL_ILP64");
        iface = (e && atoi(e)) ? MKL_INTERFACE_ILP64 : MKL_INTERFACE_LP64;
        if (set_interface_layer) set_interface_layer(iface);
        set_threading_layer(MKL_THREADING_GNU);
        return true;
    }
};

Mkl g_mkl;
std::mutex g_mu;

double now_ms() {
    timeval t;
    gettimeofday(&t, nullptr);
    return t.tv_sec * 1000.0 + t.tv_usec / 1000.0;
}

template <typename I>
ias_status run(const ias_csr *A, const ias_csr *B, ias_csr *C, double *ms) {
    Api<I> api;
    api.create_csr = (decltype(api.create_csr))g_mkl.create;
    api.sp2m = (decltype(api.sp2m))g_mkl.sp2m;
    api.export_csr = (decltype(api.export_csr))g_mkl.exp;
    api.destroy = (decltype(api.destroy))g_mkl.destroy;
    // MKL arrays (copied before the timer like main.cpp:709-743)
    std::vector<I> ap(A->rows + 1), ac(A->nnz), bp(B->rows + 1), bc(B->nnz);
    std::vector<double> av(A->val, A->val + A->nnz), bv(B->val, B->val + B->nnz);
    for (int64_t i = 0; i <= A->rows; ++i) ap[i] = (I)(A->row_ptr[i] - A->row_ptr[0]);
    for (int64_t i = 0; i < A->nnz; ++i) ac[i] = (I)A->col[A->row_ptr[0] + i];
    for (int64_t i = 0; i <= B->rows; ++i) bp[i] = (I)(B->row_ptr[i] - B->row_ptr[0]);
    for (int64_t i = 0; i < B->nnz; ++i) bc[i] = (I)B->col[B->row_ptr[0] + i];
    if (A->row_ptr[0] != 0) av.assign(A->val + A->row_ptr[0], A->val + A->row_ptr[0] + A->nnz);
    if (B->row_ptr[0] != 0) bv.assign(B->val + B->row_ptr[0], B->val + B->row_ptr[0] + B->nnz);

    sparse_matrix_t ma = nullptr, mb = nullptr, mc = nullptr;
    matrix_descr d{SPARSE_MATRIX_TYPE_GENERAL, SPARSE_FILL_MODE_FULL, SPARSE_DIAG_NON_UNIT};
    int idx = 0;
    I rows = 0, cols = 0, *rs = nullptr, *re = nullptr, *ci = nullptr;
    double *vals = nullptr;
    const double t0 = now_ms();
    int st = api.create_csr(&ma, SPARSE_INDEX_BASE_ZERO, (I)A->rows, (I)A->cols, ap.data(),
                            ap.data() + 1, ac.data(), av.data());
    if (st == 0)
        st = api.create_csr(&mb, SPARSE_INDEX_BASE_ZERO, (I)B->rows, (I)B->cols, bp.data(),
                            bp.data() + 1, bc.data(), bv.data());
    if (st == 0)
        st = api.sp2m(SPARSE_OPERATION_NON_TRANSPOSE, d, ma, SPARSE_OPERATION_NON_TRANSPOSE, d, mb,
                      SPARSE_STAGE_FULL_MULT, &mc);
    if (st == 0) st = api.export_csr(mc, &idx, &rows, &cols, &rs, &re, &ci, &vals);
    const double t1 = now_ms();
    ias_status out = IAS_SUCCESS;
    if (st != 0) {
        set_last_error("MKL sparse status %d", st);
        out = IAS_ERROR_DEVICE;
    } else {
        const int64_t nnz = rows > 0 ? (int64_t)re[rows - 1] : 0;
        ias_csr M{};
        out = ias_csr_alloc(&M, rows, cols, nnz, IAS_MEMORY_HOST, 0);
        if (out == IAS_SUCCESS) {
            // rows_start/rows_end may leave gaps in general; compact.
            int64_t at = 0;
            M.row_ptr[0] = 0;
            for (I i = 0; i < rows; ++i) {
                for (I p = rs[i]; p < re[i]; ++p, ++at) {
                    M.col[at] = (int32_t)ci[p];
                    M.val[at] = vals[p];
                }
                M.row_ptr[i + 1] = at;
            }
            M.nnz = at;
            *C = M;
        }
    }
    if (ma) api.destroy(ma);
    if (mb) api.destroy(mb);
    if (mc) api.destroy(mc);
    if (ms) *ms = t1 - t0;
    return out;
}

}  // namespace

extern "C" ias_status ias_mkl_available(int32_t *available, char *version, int32_t version_len) {
    std::lock_guard<std::mutex> lk(g_mu);
    const bool ok = g_mkl.load();
    if (available) *available = ok ? 1 : 0;
    if (version && version_len > 0) {
        version[0] = 0;
        if (ok && g_mkl.get_version_string) g_mkl.get_version_string(version, version_len);
    }
    return ok ? IAS_SUCCESS : IAS_ERROR_UNAVAILABLE;
}

extern "C" ias_status ias_mkl_sp2m(const ias_csr *A, const ias_csr *B, ias_csr *C, int32_t threads,
                                   double *ms) {
    if (!A || !B || !C) return IAS_ERROR_INVALID_ARGUMENT;
    if (A->memory != IAS_MEMORY_HOST || B->memory != IAS_MEMORY_HOST) return IAS_ERROR_INVALID_ARGUMENT;
    if (A->cols != B->rows) return IAS_ERROR_DIMENSION_MISMATCH;
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_mkl.load()) {
        set_last_error("libmkl_rt not found (set IAS_MKL_PATH)");
        return IAS_ERROR_UNAVAILABLE;
    }
    if (threads > 0 && g_mkl.set_num_threads) g_mkl.set_num_threads(threads);
    if (g_mkl.iface == MKL_INTERFACE_ILP64) return run<long long>(A, B, C, ms);
    if (A->nnz > INT32_MAX || B->nnz > INT32_MAX) {
        set_last_error("LP64 MKL cannot index nnz > 2^31; run with IAS_MKL_ILP64=1");
        return IAS_ERROR_OVERFLOW;
    }
    return run<int>(A, B, C, ms);
}
