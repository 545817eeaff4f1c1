// dia.hip — DIA x DIA for banded inputs (replaces DIA_mul_DIA,
// IA-SPGEMM-CPU_release/detail/dia/common_dia.h:101-195, and the unused
// DIA_MUL_DIA_DEV, GPU/detail/dia_dev/common_dia_dev.h:138-182).
//
// C's diagonal set is computed on the host from the offsets alone, exactly as
// the reference's triple loop decides it (dia:107-140: offset a+b exists when
// some row i has i+a in [0, A.cols) and i+a+b in [0, B.cols)).  For every C
// slot the contributing (A diagonal, B diagonal) pairs are listed in the
// reference's loop order (ja ascending), so one lane per C element
//     C[i][slot] = ((0.0 + A[i][ja0]*B[i+a0][kb0]) + A[i][ja1]*B[i+a1][kb1]) ...
// reproduces the reference's sums bit for bit (-ffp-contract=off).  One lane
// per element makes the C store fully coalesced (row-major rows x nd_C); A
// and B rows are re-read from L2 by the nd_C lanes of a row.  The kernel is
// HBM-bound (~0.4 flop/byte at 7 diagonals), so no MFMA: DESIGN.md §DIA.
#include "ias.h"
#include "ias_internal.hpp"
#include "spgemm_engine.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

namespace ias {
namespace dev {

struct DiaPairs {
    const int32_t *start;  // nd_C + 1
    const int32_t *ja;     // A diagonal slot of each pair
    const int32_t *kb;     // B diagonal slot of each pair
};

__global__ __launch_bounds__(256) void k_dia_mul(int64_t rows, int64_t a_cols, int64_t b_cols,
                                                 int32_t nda, const int32_t *__restrict__ offa,
                                                 const double *__restrict__ va, int32_t ndb,
                                                 const int32_t *__restrict__ offb,
                                                 const double *__restrict__ vb, int32_t ndc,
                                                 DiaPairs pairs, double *__restrict__ vc) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= rows * ndc) return;
    const int64_t i = e / ndc;
    const int32_t slot = (int32_t)(e - i * ndc);
    double acc = 0.0;
    for (int32_t p = pairs.start[slot]; p < pairs.start[slot + 1]; ++p) {
        const int32_t ja = pairs.ja[p], kb = pairs.kb[p];
        const int64_t acol = i + offa[ja];
        if (acol < 0 || acol >= a_cols) continue;
        const int64_t bcol = acol + offb[kb];
        if (bcol < 0 || bcol >= b_cols) continue;
        const double prod = va[i * nda + ja] * vb[acol * ndb + kb];
        acc = acc + prod;
    }
    vc[e] = acc;
}

__global__ void k_dia_index(int32_t ndc, const int32_t *offc, int64_t rows, int32_t *ind) {
    const int32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d < ndc) ind[offc[d] + rows - 1] = d;
}

}  // namespace dev
}  // namespace ias

using namespace ias;

// Host: C diagonal set and per-slot pair lists (reference loop order).
static void dia_plan(const int32_t *offa, int32_t nda, const int32_t *offb, int32_t ndb,
                     int64_t rows, int64_t a_cols, int64_t b_cols, std::vector<int32_t> &offc,
                     std::vector<int32_t> &start, std::vector<int32_t> &ja,
                     std::vector<int32_t> &kb) {
    std::vector<int64_t> reach;
    for (int32_t x = 0; x < nda; ++x)
        for (int32_t y = 0; y < ndb; ++y) {
            const int64_t oa = offa[x], ob = offb[y];
            int64_t lo = 0, hi = rows;
            lo = std::max(lo, -oa);
            hi = std::min(hi, a_cols - oa);
            lo = std::max(lo, -oa - ob);
            hi = std::min(hi, b_cols - oa - ob);
            if (lo < hi) reach.push_back(oa + ob);
        }
    std::sort(reach.begin(), reach.end());
    reach.erase(std::unique(reach.begin(), reach.end()), reach.end());
    offc.assign(reach.begin(), reach.end());
    const int32_t ndc = (int32_t)offc.size();
    start.assign(ndc + 1, 0);
    std::vector<std::vector<std::pair<int32_t, int32_t>>> lists(ndc);
    for (int32_t x = 0; x < nda; ++x)
        for (int32_t y = 0; y < ndb; ++y) {
            const int64_t o = (int64_t)offa[x] + offb[y];
            auto it = std::lower_bound(reach.begin(), reach.end(), o);
            if (it != reach.end() && *it == o) lists[it - reach.begin()].push_back({x, y});
        }
    ja.clear();
    kb.clear();
    for (int32_t d = 0; d < ndc; ++d) {
        for (auto &pr : lists[d]) {
            ja.push_back(pr.first);
            kb.push_back(pr.second);
        }
        start[d + 1] = (int32_t)ja.size();
    }
}

#define HIPC(x)                                                                   \
    do {                                                                          \
        hipError_t _e = (x);                                                      \
        if (_e != hipSuccess) {                                                   \
            set_last_error("%s failed: %s", #x, hipGetErrorString(_e));           \
            return _e == hipErrorOutOfMemory ? IAS_ERROR_OUT_OF_MEMORY : IAS_ERROR_DEVICE; \
        }                                                                         \
    } while (0)

extern "C" ias_status ias_dia_mul_dia(const ias_dia *A, const ias_dia *B, ias_dia *C,
                                      const ias_opts *opts, ias_report *rep) {
    if (!A || !B || !C) return IAS_ERROR_INVALID_ARGUMENT;
    if (!A->choice || !B->choice) return IAS_ERROR_INFEASIBLE;
    if (A->cols != B->rows) return IAS_ERROR_DIMENSION_MISMATCH;
    ias_opts o;
    ias_opts_default(&o);
    if (opts) o = *opts;
    if (rep) memset(rep, 0, sizeof *rep);
    const int device = o.device >= 0 ? o.device : (A->memory == IAS_MEMORY_DEVICE ? A->device : 0);
    const int out_mem = o.output_memory >= 0 ? o.output_memory : A->memory;
    HIPC(hipSetDevice(device));

    // offsets on the host (tiny)
    std::vector<int32_t> offa(A->num_diagonals), offb(B->num_diagonals);
    if (A->num_diagonals) {
        if (A->memory == IAS_MEMORY_DEVICE)
            IAS_TRY(dev_copy_d2h(offa.data(), A->diagonal_offsets, 4 * offa.size(), A->device));
        else memcpy(offa.data(), A->diagonal_offsets, 4 * offa.size());
    }
    if (B->num_diagonals) {
        if (B->memory == IAS_MEMORY_DEVICE)
            IAS_TRY(dev_copy_d2h(offb.data(), B->diagonal_offsets, 4 * offb.size(), B->device));
        else memcpy(offb.data(), B->diagonal_offsets, 4 * offb.size());
    }
    std::vector<int32_t> offc, pst, pja, pkb;
    dia_plan(offa.data(), A->num_diagonals, offb.data(), B->num_diagonals, A->rows, A->cols,
             B->cols, offc, pst, pja, pkb);
    const int32_t ndc = (int32_t)offc.size();

    hipStream_t s = (hipStream_t)o.stream;
    bool own = false;
    if (!s && o.plan) s = (hipStream_t)((ias_plan *)o.plan)->stream;
    if (!s) {
        HIPC(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        own = true;
    }
    struct Cleanup {
        std::vector<void *> p;
        int dev;
        hipStream_t s;
        bool own;
        ~Cleanup() {
            for (void *x : p) dev_free(x, dev);
            if (own) hipStreamDestroy(s);
        }
    } cl{{}, device, s, own};
    auto stage = [&](const void *src, size_t bytes, int mem, int sdev, const void **out) -> ias_status {
        if (mem == IAS_MEMORY_DEVICE && sdev == device) {
            *out = src;
            return IAS_SUCCESS;
        }
        void *d = nullptr;
        IAS_TRY(dev_alloc(&d, bytes, device));
        cl.p.push_back(d);
        if (bytes) {
            if (mem == IAS_MEMORY_DEVICE) HIPC(hipMemcpy(d, src, bytes, hipMemcpyDeviceToDevice));
            else HIPC(hipMemcpy(d, src, bytes, hipMemcpyHostToDevice));
        }
        *out = d;
        return IAS_SUCCESS;
    };
    const void *da_off, *da_val, *db_off, *db_val;
    const size_t na = (size_t)A->rows * A->num_diagonals, nb = (size_t)B->rows * B->num_diagonals;
    IAS_TRY(stage(A->diagonal_offsets, 4 * offa.size(), A->memory, A->device, &da_off));
    IAS_TRY(stage(A->val, 8 * na, A->memory, A->device, &da_val));
    if (B == A) {
        db_off = da_off;
        db_val = da_val;
    } else {
        IAS_TRY(stage(B->diagonal_offsets, 4 * offb.size(), B->memory, B->device, &db_off));
        IAS_TRY(stage(B->val, 8 * nb, B->memory, B->device, &db_val));
    }
    // pair tables (host -> device, a few hundred bytes)
    std::vector<int32_t> tab;
    tab.insert(tab.end(), pst.begin(), pst.end());
    tab.insert(tab.end(), pja.begin(), pja.end());
    tab.insert(tab.end(), pkb.begin(), pkb.end());
    const void *dtab;
    IAS_TRY(stage(tab.data(), 4 * tab.size(), IAS_MEMORY_HOST, 0, &dtab));

    ias_dia D{};
    D.rows = A->rows;
    D.cols = B->cols;
    D.num_diagonals = ndc;
    D.choice = 1;
    D.memory = IAS_MEMORY_DEVICE;
    D.device = device;
    const int64_t span = std::max<int64_t>(A->rows + B->cols - 1, 0);
    void *p0 = nullptr, *p1 = nullptr, *p2 = nullptr;
    ias_status sa;
    if ((sa = dev_alloc(&p0, 4 * (size_t)ndc, device)) || (sa = dev_alloc(&p1, 4 * (size_t)span, device)) ||
        (sa = dev_alloc(&p2, 8 * (size_t)A->rows * ndc, device))) {
        D.diagonal_offsets = (int32_t *)p0; D.diagonal_ind = (int32_t *)p1; D.val = (double *)p2;
        ias_dia_free(&D);
        return sa;
    }
    D.diagonal_offsets = (int32_t *)p0; D.diagonal_ind = (int32_t *)p1; D.val = (double *)p2;
    HIPC(hipMemcpyAsync(D.diagonal_offsets, offc.data(), 4 * (size_t)ndc, hipMemcpyHostToDevice, s));
    HIPC(hipMemsetAsync(D.diagonal_ind, 0, 4 * (size_t)span, s));

    hipEvent_t e0, e1;
    HIPC(hipEventCreate(&e0));
    HIPC(hipEventCreate(&e1));
    HIPC(hipEventRecord(e0, s));
    const int64_t n = A->rows * (int64_t)ndc;
    if (ndc > 0) {
        dev::k_dia_index<<<(ndc + 255) / 256, 256, 0, s>>>(ndc, D.diagonal_offsets, A->rows, D.diagonal_ind);
        if (n > 0) {
            const int32_t *t = (const int32_t *)dtab;
            dev::DiaPairs pr{t, t + pst.size(), t + pst.size() + pja.size()};
            dev::k_dia_mul<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(
                A->rows, A->cols, B->cols, A->num_diagonals, (const int32_t *)da_off,
                (const double *)da_val, B->num_diagonals, (const int32_t *)db_off,
                (const double *)db_val, ndc, pr, D.val);
        }
    }
    HIPC(hipGetLastError());
    HIPC(hipEventRecord(e1, s));
    HIPC(hipStreamSynchronize(s));
    if (rep) {
        float t = 0;
        hipEventElapsedTime(&t, e0, e1);
        rep->ms_total = t;
        rep->ms_numeric = t;
        int64_t fl = 0;   // multiply pairs actually formed (in-range)
        for (int32_t d = 0; d < ndc; ++d)
            for (int32_t p = pst[d]; p < pst[d + 1]; ++p) {
                const int64_t oa = offa[pja[p]], ob = offb[pkb[p]];
                int64_t lo = std::max<int64_t>(0, std::max<int64_t>(-oa, -oa - ob));
                int64_t hi = std::min<int64_t>(A->rows, std::min<int64_t>(A->cols - oa, B->cols - oa - ob));
                if (hi > lo) fl += hi - lo;
            }
        rep->flops = fl;
        rep->nnz_c = n;
    }
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    if (out_mem == IAS_MEMORY_HOST) {
        ias_dia H{};
        ias_status cs = ias_dia_copy(&D, &H, IAS_MEMORY_HOST, 0);
        ias_dia_free(&D);
        if (cs != IAS_SUCCESS) return cs;
        *C = H;
    } else {
        *C = D;
    }
    return IAS_SUCCESS;
}
