// convert_dev.hip — the format layer on the device: CSRtoCOO,
// CSRtoELL and CSRtoDIA (coo/common_coo.h:29-66, ell/common_ell.h:30-77,
// dia/common_dia.h:29-96) for a CSR already resident in HBM, so the CLI's
// trans_time is spent on the GPU and the converted operand never crosses
// PCIe.  Outputs are byte-identical to the host conversions in convert.cpp
// (tests/test_gpu_parity.py::test_device_conversions), including the padding
// (ELL column 0 / value 0.0), absent diagonals (diagonal_ind 0) and the
// "later duplicate overwrites" rule of CSRtoDIA.
//
// All three are HBM-streaming passes over the CSR (12 B/entry read, 16-20 B
// per stored slot written); rows are walked by 16-lane groups so short and
// long rows both keep the wave's loads coalesced.
#include "ias.h"
#include "ias_internal.hpp"

#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>

namespace ias {
namespace {

#define DHIPC(x)                                                                  \
    do {                                                                          \
        hipError_t _e = (x);                                                      \
        if (_e != hipSuccess) {                                                   \
            set_last_error("%s failed: %s", #x, hipGetErrorString(_e));           \
            return _e == hipErrorOutOfMemory ? IAS_ERROR_OUT_OF_MEMORY : IAS_ERROR_DEVICE; \
        }                                                                         \
    } while (0)

constexpr int CV_BLOCK = 256;
constexpr int CV_GROUP = 16;   // lanes per row

inline unsigned grid_for(int64_t items, int per_block) {
    const int64_t g = (items + per_block - 1) / per_block;
    return (unsigned)std::max<int64_t>(std::min<int64_t>(g, 1 << 20), 1);
}

// Row r's entries for the group (grid-strided over rows).
#define CV_ROWS(rows)                                                              \
    const int64_t lane_ = threadIdx.x % CV_GROUP;                                  \
    const int64_t groups_ = (int64_t)gridDim.x * (CV_BLOCK / CV_GROUP);            \
    for (int64_t r = (int64_t)blockIdx.x * (CV_BLOCK / CV_GROUP) + threadIdx.x / CV_GROUP; \
         r < (rows); r += groups_)

__global__ __launch_bounds__(CV_BLOCK) void k_cv_rebase(const int64_t *__restrict__ rp, int64_t n,
                                                        int64_t base, int64_t *__restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * CV_BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * CV_BLOCK)
        out[i] = rp[i] - base;
}

__global__ __launch_bounds__(CV_BLOCK) void k_cv_coo_rows(const int64_t *__restrict__ rp, int64_t rows,
                                                          int32_t *__restrict__ row) {
    CV_ROWS(rows) {
        const int64_t b = rp[r] - rp[0], e = rp[r + 1] - rp[0];
        for (int64_t p = b + lane_; p < e; p += CV_GROUP) row[p] = (int32_t)r;
    }
}

__global__ __launch_bounds__(CV_BLOCK) void k_cv_max_len(const int64_t *__restrict__ rp, int64_t rows,
                                                         unsigned long long *__restrict__ mx) {
    unsigned long long m = 0;
    for (int64_t i = (int64_t)blockIdx.x * CV_BLOCK + threadIdx.x; i < rows; i += (int64_t)gridDim.x * CV_BLOCK)
        m = std::max<unsigned long long>(m, (unsigned long long)(rp[i + 1] - rp[i]));
    for (int o = 32; o > 0; o >>= 1) m = std::max<unsigned long long>(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0 && m) atomicMax(mx, m);
}

__global__ __launch_bounds__(CV_BLOCK) void k_cv_ell_fill(const int64_t *__restrict__ rp, int64_t rows,
                                                          const int32_t *__restrict__ col,
                                                          const double *__restrict__ val, int64_t K,
                                                          int32_t *__restrict__ nnz_row,
                                                          int32_t *__restrict__ ecol,
                                                          double *__restrict__ eval) {
    CV_ROWS(rows) {
        const int64_t b = rp[r], len = rp[r + 1] - b;
        for (int64_t t = lane_; t < len; t += CV_GROUP) {
            ecol[r * K + t] = col[b + t];
            eval[r * K + t] = val[b + t];
        }
        if (lane_ == 0) nnz_row[r] = (int32_t)len;
    }
}

// flag[(rows - i) + j] = 1 for every stored (i, j); idempotent plain stores.
__global__ __launch_bounds__(CV_BLOCK) void k_cv_dia_mark(const int64_t *__restrict__ rp, int64_t rows,
                                                          const int32_t *__restrict__ col,
                                                          int32_t *__restrict__ flag) {
    CV_ROWS(rows) {
        for (int64_t p = rp[r] + lane_; p < rp[r + 1]; p += CV_GROUP) flag[(rows - r) + col[p]] = 1;
    }
}

// slot = exclusive scan of flag: offsets[slot] = idx - rows for present
// diagonals; diagonal_ind[idx - 1] = slot or 0 when absent.
__global__ __launch_bounds__(CV_BLOCK) void k_cv_dia_index(const int32_t *__restrict__ flag,
                                                           const int32_t *__restrict__ slot, int64_t span,
                                                           int64_t rows, int32_t *__restrict__ offsets,
                                                           int32_t *__restrict__ dind) {
    for (int64_t idx = (int64_t)blockIdx.x * CV_BLOCK + threadIdx.x; idx < span;
         idx += (int64_t)gridDim.x * CV_BLOCK) {
        const bool on = flag[idx] != 0;
        if (on) offsets[slot[idx]] = (int32_t)(idx - rows);
        if (idx >= 1) dind[idx - 1] = on ? slot[idx] : 0;
    }
}

// One thread per row, entries in stored order: a later duplicate (i, j)
// overwrites an earlier one exactly as the reference's sequential loop.
__global__ __launch_bounds__(CV_BLOCK) void k_cv_dia_vals(const int64_t *__restrict__ rp, int64_t rows,
                                                          const int32_t *__restrict__ col,
                                                          const double *__restrict__ val,
                                                          const int32_t *__restrict__ slot, int64_t nd,
                                                          double *__restrict__ dval) {
    for (int64_t r = (int64_t)blockIdx.x * CV_BLOCK + threadIdx.x; r < rows; r += (int64_t)gridDim.x * CV_BLOCK)
        for (int64_t p = rp[r]; p < rp[r + 1]; ++p) dval[r * nd + slot[(rows - r) + col[p]]] = val[p];
}

__global__ __launch_bounds__(CV_BLOCK) void k_cv_col_count(const int32_t *__restrict__ col, int64_t nnz,
                                                           unsigned long long *__restrict__ cnt) {
    for (int64_t p = (int64_t)blockIdx.x * CV_BLOCK + threadIdx.x; p < nnz; p += (int64_t)gridDim.x * CV_BLOCK)
        atomicAdd(&cnt[col[p]], 1ull);
}

__global__ __launch_bounds__(CV_BLOCK) void k_cv_iota(int32_t *__restrict__ idx, int64_t n) {
    for (int64_t p = (int64_t)blockIdx.x * CV_BLOCK + threadIdx.x; p < n; p += (int64_t)gridDim.x * CV_BLOCK)
        idx[p] = (int32_t)p;
}

// Aᵀ entry k = A entry idx[k] (idx sorted stably by column): column = its row.
__global__ __launch_bounds__(CV_BLOCK) void k_cv_t_gather(const int32_t *__restrict__ idx,
                                                          const int32_t *__restrict__ row,
                                                          const double *__restrict__ val, int64_t nnz,
                                                          int32_t *__restrict__ tcol,
                                                          double *__restrict__ tval) {
    for (int64_t k = (int64_t)blockIdx.x * CV_BLOCK + threadIdx.x; k < nnz; k += (int64_t)gridDim.x * CV_BLOCK) {
        const int32_t e = idx[k];
        tcol[k] = row[e];
        tval[k] = val[e];
    }
}

double csr_bytes_dev(const ias_csr *A) {
    return 4.0 * (double)(A->rows + 1 + A->nnz + 3) + 8.0 * (double)A->nnz;
}

template <typename T>
ias_status alloc_n(T **p, int64_t n, int device) {
    return dev_alloc((void **)p, sizeof(T) * (size_t)std::max<int64_t>(n, 0), device);
}

struct DevBuf {
    void *p = nullptr;
    int device = 0;
    ~DevBuf() {
        if (p) dev_free(p, device);
    }
};

}  // namespace

ias_status csr_to_coo_device(const ias_csr *A, ias_coo *out, double gate) {
    ias_coo C{};
    C.rows = A->rows; C.cols = A->cols; C.nnz = A->nnz; C.choice = 1;
    C.memory = IAS_MEMORY_DEVICE; C.device = A->device;
    if (gate > 0 && !(ias_sizeof_coo(&C) < gate * csr_bytes_dev(A))) {
        C.choice = 0;
        *out = C;
        return IAS_ERROR_INFEASIBLE;
    }
    DHIPC(hipSetDevice(A->device));
    int64_t base = 0;
    IAS_TRY(dev_copy_d2h(&base, A->row_ptr, sizeof(int64_t), A->device));
    ias_status s = IAS_SUCCESS;
    if ((s = alloc_n(&C.row_offset, A->rows + 1, A->device)) != IAS_SUCCESS ||
        (s = alloc_n(&C.row, A->nnz, A->device)) != IAS_SUCCESS ||
        (s = alloc_n(&C.col, A->nnz, A->device)) != IAS_SUCCESS ||
        (s = alloc_n(&C.val, A->nnz, A->device)) != IAS_SUCCESS) {
        ias_coo_free(&C);
        return s;
    }
    hipLaunchKernelGGL(k_cv_rebase, dim3(grid_for(A->rows + 1, CV_BLOCK)), dim3(CV_BLOCK), 0, 0,
                       A->row_ptr, A->rows + 1, base, C.row_offset);
    if (A->rows > 0)
        hipLaunchKernelGGL(k_cv_coo_rows, dim3(grid_for(A->rows, CV_BLOCK / CV_GROUP)), dim3(CV_BLOCK), 0, 0,
                           A->row_ptr, A->rows, C.row);
    if (A->nnz > 0) {
        hipMemcpyAsync(C.col, A->col + base, sizeof(int32_t) * A->nnz, hipMemcpyDeviceToDevice, 0);
        hipMemcpyAsync(C.val, A->val + base, sizeof(double) * A->nnz, hipMemcpyDeviceToDevice, 0);
    }
    const hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess || hipGetLastError() != hipSuccess) {
        set_last_error("csr_to_coo_device: %s", hipGetErrorString(e));
        ias_coo_free(&C);
        return IAS_ERROR_DEVICE;
    }
    *out = C;
    return IAS_SUCCESS;
}

ias_status csr_to_ell_device(const ias_csr *A, ias_ell *out, double gate) {
    DHIPC(hipSetDevice(A->device));
    DevBuf mx;
    mx.device = A->device;
    IAS_TRY(dev_alloc(&mx.p, sizeof(unsigned long long), A->device));
    IAS_TRY(dev_memset(mx.p, 0, sizeof(unsigned long long), A->device));
    if (A->rows > 0)
        hipLaunchKernelGGL(k_cv_max_len, dim3(grid_for(A->rows, CV_BLOCK)), dim3(CV_BLOCK), 0, 0, A->row_ptr,
                           A->rows, (unsigned long long *)mx.p);
    unsigned long long K = 0;
    IAS_TRY(dev_copy_d2h(&K, mx.p, sizeof(K), A->device));
    if (K > (unsigned long long)INT32_MAX) return IAS_ERROR_OVERFLOW;
    ias_ell E{};
    E.rows = A->rows; E.cols = A->cols; E.nnz = A->nnz; E.max_nnz_per_row = (int32_t)K; E.choice = 1;
    E.memory = IAS_MEMORY_DEVICE; E.device = A->device;
    if (gate > 0 && !(ias_sizeof_ell(&E) < gate * csr_bytes_dev(A))) {
        E.choice = 0;
        *out = E;
        return IAS_ERROR_INFEASIBLE;
    }
    const int64_t rk = A->rows * (int64_t)K;
    ias_status s = IAS_SUCCESS;
    if ((s = alloc_n(&E.nnz_row, A->rows, A->device)) != IAS_SUCCESS ||
        (s = alloc_n(&E.col, rk, A->device)) != IAS_SUCCESS ||
        (s = alloc_n(&E.val, rk, A->device)) != IAS_SUCCESS ||
        (s = dev_memset(E.col, 0, sizeof(int32_t) * rk, A->device)) != IAS_SUCCESS ||
        (s = dev_memset(E.val, 0, sizeof(double) * rk, A->device)) != IAS_SUCCESS) {
        ias_ell_free(&E);
        return s;
    }
    if (A->rows > 0)
        hipLaunchKernelGGL(k_cv_ell_fill, dim3(grid_for(A->rows, CV_BLOCK / CV_GROUP)), dim3(CV_BLOCK), 0, 0,
                           A->row_ptr, A->rows, A->col, A->val, (int64_t)K, E.nnz_row, E.col, E.val);
    const hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess || hipGetLastError() != hipSuccess) {
        set_last_error("csr_to_ell_device: %s", hipGetErrorString(e));
        ias_ell_free(&E);
        return IAS_ERROR_DEVICE;
    }
    *out = E;
    return IAS_SUCCESS;
}

ias_status csr_to_dia_device(const ias_csr *A, ias_dia *out, double gate) {
    DHIPC(hipSetDevice(A->device));
    const int64_t span = A->rows + A->cols;   // index (rows - i) + j in [1, span)
    if (span + 1 > (int64_t)INT32_MAX) return IAS_ERROR_OVERFLOW;   // hipcub scan length is int
    DevBuf flag, slot, tmp;
    flag.device = slot.device = tmp.device = A->device;
    IAS_TRY(dev_alloc(&flag.p, sizeof(int32_t) * (size_t)(span + 1), A->device));
    IAS_TRY(dev_alloc(&slot.p, sizeof(int32_t) * (size_t)(span + 1), A->device));
    IAS_TRY(dev_memset(flag.p, 0, sizeof(int32_t) * (size_t)(span + 1), A->device));
    int32_t *fl = (int32_t *)flag.p, *sl = (int32_t *)slot.p;
    if (A->rows > 0)
        hipLaunchKernelGGL(k_cv_dia_mark, dim3(grid_for(A->rows, CV_BLOCK / CV_GROUP)), dim3(CV_BLOCK), 0, 0,
                           A->row_ptr, A->rows, A->col, fl);
    // slot[0..span] = exclusive scan of flag[0..span] (flag[span] == 0): slot[span] = nd.
    size_t tmp_bytes = 0;
    DHIPC(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, fl, sl, (int)(span + 1), 0));
    IAS_TRY(dev_alloc(&tmp.p, tmp_bytes, A->device));
    DHIPC(hipcub::DeviceScan::ExclusiveSum(tmp.p, tmp_bytes, fl, sl, (int)(span + 1), 0));
    int32_t nd = 0;
    IAS_TRY(dev_copy_d2h(&nd, sl + span, sizeof(int32_t), A->device));
    ias_dia D{};
    D.rows = A->rows; D.cols = A->cols; D.num_diagonals = nd; D.choice = 1;
    D.memory = IAS_MEMORY_DEVICE; D.device = A->device;
    if (gate > 0 && !(ias_sizeof_dia(&D) < gate * csr_bytes_dev(A))) {
        D.choice = 0;
        *out = D;
        return IAS_ERROR_INFEASIBLE;
    }
    const int64_t rn = A->rows * (int64_t)nd;
    ias_status s = IAS_SUCCESS;
    if ((s = alloc_n(&D.diagonal_offsets, nd, A->device)) != IAS_SUCCESS ||
        (s = alloc_n(&D.diagonal_ind, std::max<int64_t>(span - 1, 0), A->device)) != IAS_SUCCESS ||
        (s = alloc_n(&D.val, rn, A->device)) != IAS_SUCCESS ||
        (s = dev_memset(D.val, 0, sizeof(double) * rn, A->device)) != IAS_SUCCESS) {
        ias_dia_free(&D);
        return s;
    }
    if (span > 0)
        hipLaunchKernelGGL(k_cv_dia_index, dim3(grid_for(span, CV_BLOCK)), dim3(CV_BLOCK), 0, 0, fl, sl, span,
                           A->rows, D.diagonal_offsets, D.diagonal_ind);
    if (A->rows > 0 && nd > 0)
        hipLaunchKernelGGL(k_cv_dia_vals, dim3(grid_for(A->rows, CV_BLOCK)), dim3(CV_BLOCK), 0, 0, A->row_ptr,
                           A->rows, A->col, A->val, sl, (int64_t)nd, D.val);
    const hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess || hipGetLastError() != hipSuccess) {
        set_last_error("csr_to_dia_device: %s", hipGetErrorString(e));
        ias_dia_free(&D);
        return IAS_ERROR_DEVICE;
    }
    *out = D;
    return IAS_SUCCESS;
}

// Aᵀ (mkl_dcsrcsc in GPU/main.cu:260-269; host counting sort in convert.cpp):
// column counts -> row pointers, and a stable LSD radix sort of the entry
// indices by column, so each row of Aᵀ lists source rows in ascending order
// (duplicates in stored order), exactly as the host counting sort.
ias_status csr_transpose_device(const ias_csr *A, ias_csr *AT) {
    DHIPC(hipSetDevice(A->device));
    if (A->nnz > (int64_t)INT32_MAX || A->cols + 1 > (int64_t)INT32_MAX) return IAS_ERROR_OVERFLOW;
    int64_t base = 0;
    IAS_TRY(dev_copy_d2h(&base, A->row_ptr, sizeof(int64_t), A->device));
    const int64_t nnz = A->nnz, cols = A->cols;
    ias_csr T{};
    IAS_TRY(ias_csr_alloc(&T, A->cols, A->rows, nnz, IAS_MEMORY_DEVICE, A->device));
    DevBuf cnt, row, kin, kout, iin, iout, tmp;
    cnt.device = row.device = kin.device = kout.device = iin.device = iout.device = tmp.device = A->device;
    ias_status s = IAS_SUCCESS;
    auto fail = [&](ias_status st) {
        ias_csr_free(&T);
        return st;
    };
    if ((s = dev_alloc(&cnt.p, sizeof(unsigned long long) * (size_t)(cols + 1), A->device)) != IAS_SUCCESS ||
        (s = dev_memset(cnt.p, 0, sizeof(unsigned long long) * (size_t)(cols + 1), A->device)) != IAS_SUCCESS ||
        (s = dev_alloc(&row.p, sizeof(int32_t) * (size_t)nnz, A->device)) != IAS_SUCCESS ||
        (s = dev_alloc(&iin.p, sizeof(int32_t) * (size_t)nnz, A->device)) != IAS_SUCCESS ||
        (s = dev_alloc(&iout.p, sizeof(int32_t) * (size_t)nnz, A->device)) != IAS_SUCCESS ||
        (s = dev_alloc(&kout.p, sizeof(int32_t) * (size_t)nnz, A->device)) != IAS_SUCCESS)
        return fail(s);
    const int32_t *col = A->col + base;
    const double *val = A->val + base;
    if (nnz > 0) {
        hipLaunchKernelGGL(k_cv_col_count, dim3(grid_for(nnz, CV_BLOCK)), dim3(CV_BLOCK), 0, 0, col, nnz,
                           (unsigned long long *)cnt.p);
        hipLaunchKernelGGL(k_cv_coo_rows, dim3(grid_for(A->rows, CV_BLOCK / CV_GROUP)), dim3(CV_BLOCK), 0, 0,
                           A->row_ptr, A->rows, (int32_t *)row.p);
        hipLaunchKernelGGL(k_cv_iota, dim3(grid_for(nnz, CV_BLOCK)), dim3(CV_BLOCK), 0, 0, (int32_t *)iin.p, nnz);
    }
    // row_ptr of Aᵀ = exclusive scan of the column counts (cols + 1 entries)
    size_t tb = 0, tb2 = 0;
    unsigned long long *cp = (unsigned long long *)cnt.p;
    DHIPC(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cp, (unsigned long long *)T.row_ptr, (int)(cols + 1), 0));
    int end_bit = 1;
    while (end_bit < 31 && ((int64_t)1 << end_bit) < cols) ++end_bit;
    DHIPC(hipcub::DeviceRadixSort::SortPairs(nullptr, tb2, col, (int32_t *)kout.p, (const int32_t *)iin.p,
                                             (int32_t *)iout.p, (int)nnz, 0, end_bit, 0));
    if ((s = dev_alloc(&tmp.p, std::max(tb, tb2), A->device)) != IAS_SUCCESS) return fail(s);
    tb = tb2 = std::max(tb, tb2);
    DHIPC(hipcub::DeviceScan::ExclusiveSum(tmp.p, tb, cp, (unsigned long long *)T.row_ptr, (int)(cols + 1), 0));
    if (nnz > 0) {
        DHIPC(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb2, col, (int32_t *)kout.p, (const int32_t *)iin.p,
                                                 (int32_t *)iout.p, (int)nnz, 0, end_bit, 0));
        hipLaunchKernelGGL(k_cv_t_gather, dim3(grid_for(nnz, CV_BLOCK)), dim3(CV_BLOCK), 0, 0,
                           (const int32_t *)iout.p, (const int32_t *)row.p, val, nnz, T.col, T.val);
    }
    const hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess || hipGetLastError() != hipSuccess) {
        set_last_error("csr_transpose_device: %s", hipGetErrorString(e));
        return fail(IAS_ERROR_DEVICE);
    }
    *AT = T;
    return IAS_SUCCESS;
}

}  // namespace ias
