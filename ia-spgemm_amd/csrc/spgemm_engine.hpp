// spgemm_engine.hpp — host-side engine state (the ias_plan behind the ABI).
#pragma once

#include "ias.h"
#include "spgemm_kernels.hpp"

#include <cstdint>

namespace ias {

constexpr int MAX_BINS = 8;      // 0 = empty rows, 1..6 = LDS bins, 7 = global table
constexpr int MAX_BIN_LDS = 6;

struct BinSpec {
    int32_t nbins;
    int32_t upper[MAX_BINS];
};

// Device-side counters, copied to the host after binning and after the scan.
struct Counters {
    unsigned long long flops;
    unsigned long long sym_ws;      // global-table slots needed by symbolic rows
    unsigned long long num_ws;      // global-table slots needed by numeric rows
    int32_t max_prod;
    int32_t max_nnz;
    int32_t sym_count[MAX_BINS];
    int32_t num_count[MAX_BINS];
};

}  // namespace ias

struct ias_plan {
    enum { B_PROD, B_NNZ, B_SLIST, B_NLIST, B_SOFF, B_NOFF, B_CNT, B_PTR, B_PART, B_WS, B_TMP0, B_TMP1, B_TMP2, B_TMP3, B_TMP4, B_TMP5, B_COUNT };
    struct Buf {
        void *p = nullptr;
        size_t cap = 0;
    };
    int device = 0;
    void *stream = nullptr;
    bool own_stream = false;
    Buf bufs[B_COUNT];
    hipEvent_t ev[8] = {};
    void *host_counters = nullptr;

    // state carried from symbolic() to numeric()
    int64_t n_rows = 0;
    int64_t nnz_total = 0;
    int64_t flops = 0;
    int32_t max_prod = 0;
    int32_t max_nnz = 0;
    int32_t num_count[ias::MAX_BINS] = {};
    unsigned long long num_ws = 0;
    // identity of the operands of the last symbolic() (checked by compute)
    const void *last_a = nullptr, *last_b = nullptr;

    ~ias_plan();
    ias_status init(int device, void *stream);
    ias_status reserve(void **buf, size_t *cap, size_t bytes);
    ias_status symbolic(const ias::dev::Rows &A, const ias::dev::Rows &B, int64_t rows,
                        int64_t cols, ias_report *rep);
    ias_status numeric(const ias::dev::Rows &A, const ias::dev::Rows &B, const ias::dev::Out &out,
                       ias_report *rep);
    ias_status shift(int64_t *p, int64_t n, int64_t off);
};

namespace ias {
using Plan = ias_plan;
}
