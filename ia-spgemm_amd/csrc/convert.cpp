// convert.cpp — format layer (CSRtoCOO/ELL/DIA and back), transpose, size
// models, verified sums, GetFlop and flops-balanced row partitioning.
// CSR -> COO/ELL/DIA and the transpose of a device-resident CSR run on the
// device (convert_dev.hip); everything else here is host code that stages device
// operands through the host (not on the timed path).
#include "ias.h"
#include "ias_internal.hpp"

#include <algorithm>
#include <vector>

using namespace ias;

namespace {

// Host copy of a CSR if it lives on a device; `h` owns it then.
struct HostCsr {
    ias_csr h{};
    const ias_csr *m = nullptr;
    bool owned = false;
    ~HostCsr() {
        if (owned) ias_csr_free(&h);
    }
    ias_status get(const ias_csr *A) {
        if (A->memory == IAS_MEMORY_DEVICE) {
            IAS_TRY(ias_csr_copy(A, &h, IAS_MEMORY_HOST, 0));
            owned = true;
            m = &h;
        } else {
            m = A;
        }
        return IAS_SUCCESS;
    }
};

double csr_bytes(const ias_csr *A) { return 4.0 * (double)(A->rows + 1 + A->nnz + 3) + 8.0 * (double)A->nnz; }

template <typename T>
ias_status to_memory(T *host, int32_t memory, int32_t device,
                     ias_status (*copy)(const T *, T *, int32_t, int32_t),
                     ias_status (*freef)(T *)) {
    if (memory != IAS_MEMORY_DEVICE) return IAS_SUCCESS;
    T d{};
    ias_status s = copy(host, &d, IAS_MEMORY_DEVICE, device);
    freef(host);
    if (s != IAS_SUCCESS) return s;
    *host = d;
    return IAS_SUCCESS;
}

}  // namespace

// ------------------------------------------------------------------ sizes
extern "C" double ias_sizeof_csr(const ias_csr *A) { return A ? csr_bytes(A) : 0.0; }
extern "C" double ias_sizeof_coo(const ias_coo *A) {
    return A ? 4.0 * (double)(A->rows + 1 + 2 * A->nnz + 3) + 8.0 * (double)A->nnz : 0.0;
}
extern "C" double ias_sizeof_ell(const ias_ell *A) {
    if (!A) return 0.0;
    const double rk = (double)A->rows * (double)A->max_nnz_per_row;
    return 4.0 * ((double)A->rows + rk + 4.0) + 8.0 * rk;
}
extern "C" double ias_sizeof_dia(const ias_dia *A) {
    if (!A) return 0.0;
    return 4.0 * (double)(A->rows + A->cols - 1 + A->num_diagonals + 3) +
           8.0 * (double)A->rows * (double)A->num_diagonals;
}

// ------------------------------------------------------------------ CSR -> X
extern "C" ias_status ias_csr_to_coo(const ias_csr *A, ias_coo *out, double gate) {
    if (!A || !out) return IAS_ERROR_INVALID_ARGUMENT;
    if (A->memory == IAS_MEMORY_DEVICE) return csr_to_coo_device(A, out, gate);
    HostCsr H;
    IAS_TRY(H.get(A));
    const ias_csr *M = H.m;
    ias_coo C{};
    C.rows = M->rows; C.cols = M->cols; C.nnz = M->nnz; C.choice = 1;
    if (gate > 0 && !(ias_sizeof_coo(&C) < gate * csr_bytes(M))) {
        C.choice = 0;
        C.memory = A->memory; C.device = A->device;
        *out = C;
        return IAS_ERROR_INFEASIBLE;
    }
    C.row_offset = (int64_t *)host_alloc(sizeof(int64_t) * (M->rows + 1));
    C.row = (int32_t *)host_alloc(sizeof(int32_t) * M->nnz);
    C.col = (int32_t *)host_alloc(sizeof(int32_t) * M->nnz);
    C.val = (double *)host_alloc(sizeof(double) * M->nnz);
    if (!C.row_offset || !C.row || !C.col || !C.val) {
        ias_coo_free(&C);
        return IAS_ERROR_OUT_OF_MEMORY;
    }
    for (int64_t i = 0; i < M->rows; ++i) {
        C.row_offset[i] = M->row_ptr[i] - M->row_ptr[0];
        for (int64_t p = M->row_ptr[i]; p < M->row_ptr[i + 1]; ++p) {
            const int64_t at = p - M->row_ptr[0];
            C.row[at] = (int32_t)i;
            C.col[at] = M->col[p];
            C.val[at] = M->val[p];
        }
    }
    C.row_offset[M->rows] = M->nnz;
    IAS_TRY(to_memory<ias_coo>(&C, A->memory, A->device, ias_coo_copy, ias_coo_free));
    *out = C;
    return IAS_SUCCESS;
}

extern "C" ias_status ias_csr_to_ell(const ias_csr *A, ias_ell *out, double gate) {
    if (!A || !out) return IAS_ERROR_INVALID_ARGUMENT;
    if (A->memory == IAS_MEMORY_DEVICE) return csr_to_ell_device(A, out, gate);
    HostCsr H;
    IAS_TRY(H.get(A));
    const ias_csr *M = H.m;
    int64_t K = 0;
    for (int64_t i = 0; i < M->rows; ++i) K = std::max<int64_t>(K, M->row_ptr[i + 1] - M->row_ptr[i]);
    if (K > INT32_MAX) return IAS_ERROR_OVERFLOW;
    ias_ell E{};
    E.rows = M->rows; E.cols = M->cols; E.nnz = M->nnz; E.max_nnz_per_row = (int32_t)K; E.choice = 1;
    if (gate > 0 && !(ias_sizeof_ell(&E) < gate * csr_bytes(M))) {
        E.choice = 0;
        E.memory = A->memory; E.device = A->device;
        *out = E;
        return IAS_ERROR_INFEASIBLE;
    }
    const size_t rk = (size_t)M->rows * (size_t)K;
    E.nnz_row = (int32_t *)host_alloc(sizeof(int32_t) * M->rows);
    E.col = (int32_t *)host_alloc(sizeof(int32_t) * rk);
    E.val = (double *)host_alloc(sizeof(double) * rk);
    if (!E.nnz_row || !E.col || !E.val) {
        ias_ell_free(&E);
        return IAS_ERROR_OUT_OF_MEMORY;
    }
    for (int64_t i = 0; i < M->rows; ++i) {
        int64_t t = 0;
        for (int64_t p = M->row_ptr[i]; p < M->row_ptr[i + 1]; ++p, ++t) {
            E.col[i * K + t] = M->col[p];
            E.val[i * K + t] = M->val[p];
        }
        E.nnz_row[i] = (int32_t)t;
    }
    IAS_TRY(to_memory<ias_ell>(&E, A->memory, A->device, ias_ell_copy, ias_ell_free));
    *out = E;
    return IAS_SUCCESS;
}

// CSRtoDIA semantics (dia/common_dia.h:29-96): diagonal present when any
// stored entry lies on it; a later duplicate (i,j) overwrites an earlier one.
extern "C" ias_status ias_csr_to_dia(const ias_csr *A, ias_dia *out, double gate) {
    if (!A || !out) return IAS_ERROR_INVALID_ARGUMENT;
    if (A->memory == IAS_MEMORY_DEVICE) return csr_to_dia_device(A, out, gate);
    HostCsr H;
    IAS_TRY(H.get(A));
    const ias_csr *M = H.m;
    const int64_t span = M->rows + M->cols;   // index (rows - i) + j in [1, span)
    std::vector<int32_t> map((size_t)std::max<int64_t>(span, 1), -1);
    int64_t nd = 0;
    for (int64_t i = 0; i < M->rows; ++i)
        for (int64_t p = M->row_ptr[i]; p < M->row_ptr[i + 1]; ++p) {
            const int64_t idx = (M->rows - i) + M->col[p];
            if (map[(size_t)idx] < 0) {
                map[(size_t)idx] = 0;
                ++nd;
            }
        }
    ias_dia D{};
    D.rows = M->rows; D.cols = M->cols; D.num_diagonals = (int32_t)nd; D.choice = 1;
    if (gate > 0 && !(ias_sizeof_dia(&D) < gate * csr_bytes(M))) {
        D.choice = 0;
        D.memory = A->memory; D.device = A->device;
        *out = D;
        return IAS_ERROR_INFEASIBLE;
    }
    const size_t rn = (size_t)M->rows * (size_t)nd;
    D.diagonal_offsets = (int32_t *)host_alloc(sizeof(int32_t) * nd);
    D.diagonal_ind = (int32_t *)host_alloc(sizeof(int32_t) * std::max<int64_t>(span - 1, 0));
    D.val = (double *)host_alloc(sizeof(double) * rn);
    if (!D.diagonal_offsets || !D.diagonal_ind || !D.val) {
        ias_dia_free(&D);
        return IAS_ERROR_OUT_OF_MEMORY;
    }
    int32_t d = 0;
    for (int64_t idx = 0; idx < span; ++idx)
        if (map[(size_t)idx] >= 0) {
            map[(size_t)idx] = d;
            D.diagonal_offsets[d] = (int32_t)(idx - M->rows);
            ++d;
        }
    for (int64_t i = 0; i < M->rows; ++i)
        for (int64_t p = M->row_ptr[i]; p < M->row_ptr[i + 1]; ++p) {
            const int32_t slot = map[(size_t)((M->rows - i) + M->col[p])];
            D.val[(size_t)i * nd + slot] = M->val[p];
        }
    for (int64_t idx = 1; idx < span; ++idx) D.diagonal_ind[idx - 1] = std::max(map[(size_t)idx], 0);
    IAS_TRY(to_memory<ias_dia>(&D, A->memory, A->device, ias_dia_copy, ias_dia_free));
    *out = D;
    return IAS_SUCCESS;
}

// ------------------------------------------------------------------ X -> CSR
extern "C" ias_status ias_coo_to_csr(const ias_coo *A, ias_csr *out) {
    if (!A || !out || !A->choice) return IAS_ERROR_INVALID_ARGUMENT;
    ias_csr view{A->rows, A->cols, A->nnz, A->row_offset, A->col, A->val, A->memory, A->device};
    return ias_csr_copy(&view, out, A->memory, A->device);
}

extern "C" ias_status ias_ell_to_csr(const ias_ell *A, ias_csr *out) {
    if (!A || !out || !A->choice) return IAS_ERROR_INVALID_ARGUMENT;
    ias_ell h{};
    const ias_ell *M = A;
    if (A->memory == IAS_MEMORY_DEVICE) {
        IAS_TRY(ias_ell_copy(A, &h, IAS_MEMORY_HOST, 0));
        M = &h;
    }
    int64_t nnz = 0;
    for (int64_t i = 0; i < M->rows; ++i) nnz += M->nnz_row[i];
    ias_csr C{};
    ias_status s = ias_csr_alloc(&C, M->rows, M->cols, nnz, IAS_MEMORY_HOST, 0);
    if (s == IAS_SUCCESS) {
        const int64_t K = M->max_nnz_per_row;
        C.row_ptr[0] = 0;
        for (int64_t i = 0; i < M->rows; ++i) {
            C.row_ptr[i + 1] = C.row_ptr[i] + M->nnz_row[i];
            for (int64_t t = 0; t < M->nnz_row[i]; ++t) {
                C.col[C.row_ptr[i] + t] = M->col[i * K + t];
                C.val[C.row_ptr[i] + t] = M->val[i * K + t];
            }
        }
        s = to_memory<ias_csr>(&C, A->memory, A->device, ias_csr_copy, ias_csr_free);
    }
    if (M == &h) ias_ell_free(&h);
    if (s == IAS_SUCCESS) *out = C;
    return s;
}

extern "C" ias_status ias_dia_to_csr(const ias_dia *A, ias_csr *out) {
    if (!A || !out || !A->choice) return IAS_ERROR_INVALID_ARGUMENT;
    ias_dia h{};
    const ias_dia *M = A;
    if (A->memory == IAS_MEMORY_DEVICE) {
        IAS_TRY(ias_dia_copy(A, &h, IAS_MEMORY_HOST, 0));
        M = &h;
    }
    const int32_t nd = M->num_diagonals;
    int64_t nnz = 0;
    for (int32_t d = 0; d < nd; ++d) {
        const int64_t o = M->diagonal_offsets[d];
        const int64_t lo = std::max<int64_t>(0, -o), hi = std::min<int64_t>(M->rows, M->cols - o);
        if (hi > lo) nnz += hi - lo;
    }
    ias_csr C{};
    ias_status s = ias_csr_alloc(&C, M->rows, M->cols, nnz, IAS_MEMORY_HOST, 0);
    if (s == IAS_SUCCESS) {
        int64_t at = 0;
        C.row_ptr[0] = 0;
        for (int64_t i = 0; i < M->rows; ++i) {
            for (int32_t d = 0; d < nd; ++d) {
                const int64_t j = i + M->diagonal_offsets[d];
                if (j < 0 || j >= M->cols) continue;
                C.col[at] = (int32_t)j;
                C.val[at] = M->val[(size_t)i * nd + d];
                ++at;
            }
            C.row_ptr[i + 1] = at;
        }
        s = to_memory<ias_csr>(&C, A->memory, A->device, ias_csr_copy, ias_csr_free);
    }
    if (M == &h) ias_dia_free(&h);
    if (s == IAS_SUCCESS) *out = C;
    return s;
}

// Aᵀ by a stable counting sort on column (rows of Aᵀ ascend by source row).
extern "C" ias_status ias_csr_transpose(const ias_csr *A, ias_csr *AT) {
    if (!A || !AT) return IAS_ERROR_INVALID_ARGUMENT;
    if (A->memory == IAS_MEMORY_DEVICE) return csr_transpose_device(A, AT);
    HostCsr H;
    IAS_TRY(H.get(A));
    const ias_csr *M = H.m;
    ias_csr T{};
    IAS_TRY(ias_csr_alloc(&T, M->cols, M->rows, M->nnz, IAS_MEMORY_HOST, 0));
    std::vector<int64_t> cnt((size_t)M->cols + 1, 0);
    for (int64_t p = M->row_ptr[0]; p < M->row_ptr[M->rows]; ++p) cnt[(size_t)M->col[p] + 1]++;
    for (int64_t j = 0; j < M->cols; ++j) cnt[(size_t)j + 1] += cnt[(size_t)j];
    for (int64_t j = 0; j <= M->cols; ++j) T.row_ptr[j] = cnt[(size_t)j];
    for (int64_t i = 0; i < M->rows; ++i)
        for (int64_t p = M->row_ptr[i]; p < M->row_ptr[i + 1]; ++p) {
            const int64_t at = cnt[(size_t)M->col[p]]++;
            T.col[at] = (int32_t)i;
            T.val[at] = M->val[p];
        }
    IAS_TRY(to_memory<ias_csr>(&T, A->memory, A->device, ias_csr_copy, ias_csr_free));
    *AT = T;
    return IAS_SUCCESS;
}

// ------------------------------------------------------------------ sums / flops
extern "C" ias_status ias_flops(const ias_csr *A, const ias_csr *B, int64_t *flops) {
    if (!A || !B || !flops) return IAS_ERROR_INVALID_ARGUMENT;
    HostCsr HA, HB;
    IAS_TRY(HA.get(A));
    IAS_TRY(HB.get(B));
    const ias_csr *a = HA.m, *b = HB.m;
    int64_t total = 0;
#pragma omp parallel for reduction(+ : total) schedule(static)
    for (int64_t i = 0; i < a->rows; ++i)
        for (int64_t p = a->row_ptr[i]; p < a->row_ptr[i + 1]; ++p) {
            const int32_t j = a->col[p];
            total += b->row_ptr[j + 1] - b->row_ptr[j];
        }
    *flops = total;
    return IAS_SUCCESS;
}

template <typename T, typename GET>
static ias_status sum_array(const T *p, size_t n, int memory, int device, GET, double *sum) {
    std::vector<T> tmp;
    const T *h = p;
    if (memory == IAS_MEMORY_DEVICE && n) {
        tmp.resize(n);
        IAS_TRY(dev_copy_d2h(tmp.data(), p, sizeof(T) * n, device));
        h = tmp.data();
    }
    double s = 0.0;
    for (size_t i = 0; i < n; ++i) s += (double)h[i];
    *sum = s;
    return IAS_SUCCESS;
}

extern "C" ias_status ias_sum_csr(const ias_csr *A, double *sum) {
    if (!A || !sum) return IAS_ERROR_INVALID_ARGUMENT;
    return sum_array(A->val, (size_t)A->nnz, A->memory, A->device, 0, sum);
}
extern "C" ias_status ias_sum_coo(const ias_coo *A, double *sum) {
    if (!A || !sum) return IAS_ERROR_INVALID_ARGUMENT;
    return sum_array(A->val, (size_t)A->nnz, A->memory, A->device, 0, sum);
}
extern "C" ias_status ias_sum_ell(const ias_ell *A, double *sum) {
    if (!A || !sum) return IAS_ERROR_INVALID_ARGUMENT;
    return sum_array(A->val, (size_t)A->rows * (size_t)A->max_nnz_per_row, A->memory, A->device, 0, sum);
}
extern "C" ias_status ias_sum_dia(const ias_dia *A, double *sum) {
    if (!A || !sum) return IAS_ERROR_INVALID_ARGUMENT;
    return sum_array(A->val, (size_t)A->rows * (size_t)A->num_diagonals, A->memory, A->device, 0, sum);
}

// ------------------------------------------------------------------ partition
extern "C" ias_status ias_partition_rows(const ias_csr *A, const ias_csr *B, int32_t nparts,
                                         int64_t *bounds) {
    if (!A || !B || !bounds || nparts < 1) return IAS_ERROR_INVALID_ARGUMENT;
    HostCsr HA, HB;
    IAS_TRY(HA.get(A));
    IAS_TRY(HB.get(B));
    const ias_csr *a = HA.m, *b = HB.m;
    // Estimated device cost per row, in tenths of a product: a fixed cost per
    // row (binning, per-row passes, launch share) plus its products, weighted
    // by the symbolic path they take: LDS bins (<= 16,384 products), the
    // 8-wave sym5 bins (<= 32,768: 2.4x), hash partitions (beyond: 4.4x).
    // Calibrated on MI355X (non-negative least squares over K3' and the eight
    // rank shards of K4 run one at a time, bench.py --as-rank all; round 5:
    // 1.39 ns per row, 7.6 / 18.2 / 33.6 ps per product of the three classes;
    // DESIGN.md §6), so the rank holding R-MAT's hub rows gets fewer.
    // When C's columns fit the column bitmap (CBM_MAX_COLS), every row beyond
    // 16,384 products takes k_sym_cbm instead (serial K3': 0.55 ms for 27.5 M
    // products, ~20 ps per product: CBM).
    constexpr int64_t ROW_COST = 1830, SMALL = 10, MID = 24, BIG = 44, CBM = 26, MID_MIN = 16384, BIG_MIN = 32768;
    const bool cbm = b->cols <= CBM_MAX_COLS;
    std::vector<int64_t> pref((size_t)a->rows + 1, 0);
    for (int64_t i = 0; i < a->rows; ++i) {
        int64_t prod = 0;
        for (int64_t p = a->row_ptr[i]; p < a->row_ptr[i + 1]; ++p) {
            const int32_t j = a->col[p];
            prod += b->row_ptr[j + 1] - b->row_ptr[j];
        }
        const int64_t w = ROW_COST + prod * (prod <= MID_MIN ? SMALL : cbm ? CBM : prod > BIG_MIN ? BIG : MID);
        pref[(size_t)i + 1] = pref[(size_t)i] + w;
    }
    const int64_t total = pref[(size_t)a->rows];
    bounds[0] = 0;
    for (int32_t k = 1; k < nparts; ++k) {
        const int64_t target = (int64_t)((__int128)total * k / nparts);
        const int64_t r = std::lower_bound(pref.begin(), pref.end(), target) - pref.begin();
        bounds[k] = std::max(bounds[k - 1], std::min<int64_t>(r, a->rows));
    }
    bounds[nparts] = a->rows;
    return IAS_SUCCESS;
}
