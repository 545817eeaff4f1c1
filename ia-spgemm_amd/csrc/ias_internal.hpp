// ias_internal.hpp — shared host-side helpers of libias.so (not part of the ABI).
#pragma once

#include "ias.h"

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

namespace ias {

// Host allocation that never returns NULL for a zero-sized request.
void *host_alloc(size_t bytes, bool zero = true);
void host_free(void *p);

// Device helpers (defined in ias_device.hip; all return an ias_status).
ias_status dev_alloc(void **p, size_t bytes, int device);
ias_status dev_free(void *p, int device);
ias_status dev_copy_h2d(void *dst, const void *src, size_t bytes, int device);
ias_status dev_copy_d2h(void *dst, const void *src, size_t bytes, int device);
ias_status dev_memset(void *p, int value, size_t bytes, int device);
// Out-of-memory relief: hipFree the device's cached free blocks and the
// workspace of its idle default plan (never `keep`, the plan of the caller);
// returns the bytes released.
size_t release_device_memory(int device, const ias_plan *keep);

// Host wait for a stream's work (returns a hipError_t): polls for up to
// IAS_SPIN_US microseconds (default 200), then blocks.  A blocking wait wakes
// the host tens of µs after the GPU finishes, which small products (K1: a
// few tens of µs per kernel, two host reads per call) would pay per wait.
int host_wait(void *stream);

// Record the last HIP/internal error message for ias_status_string's detail.
void set_last_error(const char *fmt, ...);
void set_last_diag(uint32_t flags);   // ias_last_diag() of the calling thread

inline bool is_device(int32_t memory) { return memory == IAS_MEMORY_DEVICE; }

// C columns up to which the symbolic pass's longest rows take the LDS column
// bitmap (k_sym_cbm; spgemm.hip's CBM_MAXW words of 32 columns)
constexpr int64_t CBM_MAX_COLS = 36096ll * 32;

// Shape/pointer sanity of a CSR operand (no element scan).
ias_status check_csr_host(const ias_csr *A);

// Device-side row utilities used by the entry points (sort_rows.hip).
// Sort every row of a device CSR (ptr) by column, values following.
ias_status ias_sort_rows_device(ias_plan *plan, const int64_t *ptr, int64_t rows, int32_t *col,
                                double *val, int32_t max_nnz);
// Same for a device ELL (row i at i*K, nnz_row[i] entries).
ias_status ias_sort_rows_ell_device(ias_plan *plan, const int32_t *nnz_row, int64_t rows,
                                    int32_t K, int32_t *col, double *val);
ias_status ias_shift_device(int64_t *p, int64_t n, int64_t off, void *stream);

// CSR -> COO / ELL / DIA for a device-resident CSR (convert_dev.hip); outputs
// on the same device, byte-identical to the host conversions in convert.cpp.
ias_status csr_to_coo_device(const ias_csr *A, ias_coo *out, double gate);
ias_status csr_to_ell_device(const ias_csr *A, ias_ell *out, double gate);
ias_status csr_to_dia_device(const ias_csr *A, ias_dia *out, double gate);
ias_status csr_transpose_device(const ias_csr *A, ias_csr *AT);

}  // namespace ias

#define IAS_TRY(expr)                                   \
    do {                                                \
        ias_status _s = (expr);                         \
        if (_s != IAS_SUCCESS) return _s;               \
    } while (0)
