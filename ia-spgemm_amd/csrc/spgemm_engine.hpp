// spgemm_engine.hpp — host-side engine state (the ias_plan behind the ABI).
#pragma once

#include "ias.h"
#include "spgemm_kernels.hpp"

#include <cstdint>

namespace ias {

constexpr int MAX_BINS = 48;   // 0 = nothing to do, 1..nval = LDS (value) bins, nval+1 =
                               // hash partitions, nval+2 = global-memory table,
                               // nval+3.. = direct-write LDS bins, then streaming bins

// How a pass bins its rows by `key` (products or nnz).
struct BinSpec {
    int32_t nval;              // value bins 1..nval cover key <= upper[nval]
    int32_t ndw;               // direct-write bins nval+3 .. nval+2+ndw
    int32_t nst;               // streaming bins (by products) after the direct-write bins
    int32_t upper[MAX_BINS];   // per LDS bin, indexed by bin number
    int32_t ratio_num;         // value class iff prod * ratio_den > key * ratio_num
    int32_t ratio_den;         //   (ratio_den == 0: every row is value class)
    int32_t part_cap;          // keys per hash partition in bin nval+1
    int32_t wide_min;          // key >= wide_min -> bin nval+2 (0: never)
    int32_t dcap[MAX_BINS];    // duplicate-list capacity per LDS bin (symbolic; 0: none)
    int32_t part_dcap_div;     // partitioned rows: duplicate list of min(key / div, max) (0: none)
    int32_t part_dcap_max;
    int32_t ft;                // give every listed row a first-touch bitmap
    int32_t zero_nnz;          // write nnz_row = 0 for empty and partitioned rows
    int32_t ent_key;           // > 0: LDS bin i also needs ent_key * (A entries of the row) <= upper[i]
                               // (sym2 stages the row's entry bases in LDS, upper/ent_key of them)
    int32_t short_base;        // > 0: rows marked short (stv -5) -> bins short_base + 0/1/2 by
                               // products <= 64 / 128 / 256 (numeric pass of the short rows)
};

// Device-side counters, copied to the host after each binning.
struct Counters {
    unsigned long long flops;
    unsigned long long items;     // (row, partition) work items
    unsigned long long bm_words;  // first-touch bitmap words
    unsigned long long ws_slots;  // global-table slots
    unsigned long long dup_slots; // duplicate-list slots
    unsigned long long st_prod, st_nnz;   // products / C entries of the streaming rows
    unsigned long long items_cur, bm_cur, ws_cur, dup_cur;   // scatter-pass cursors
    unsigned long long part_prod, pb_cur;   // products of partitioned rows (bucket space) + cursor
    unsigned long long nnz_total;           // nnz(C) (k_bin_count of the numeric binning)
    long long a_base;                       // A's first entry (row_ptr[0]; k_an_rows)
    unsigned long long n2_units, n2_bunits, n2_dunits;   // k_num2_fill: all units, class ends
    int32_t max_prod;
    int32_t max_nnz;
    int32_t overflow;
    int32_t cbm_hits;             // k_sym_cbm branches taken (IAS_CBM_FORCE set: ias_last_diag)
    int32_t s3_retry[16];         // sym3 / sym4: rows handed to sym2, per bin (bin & 15; retry lists)
    int32_t wide_b;               // a selected B row ends beyond 2^30 entries: no sym3 (32-bit offsets)
    int32_t wide_v;               // one ends beyond 2^29: k_num2 with 64-bit gather addresses
    int32_t count[MAX_BINS];      // rows per bin (counting pass)
    int32_t cursor[MAX_BINS];     // scatter-pass cursors
};

}  // namespace ias

struct ias_plan {
    enum {
        B_AXS, B_AXL, B_AXV, B_AXP, B_POFF, B_TCOL, B_DUPV, B_PART2, B_PROD, B_NNZ, B_SLIST, B_NLIST, B_SITEM, B_NITEM, B_BMOFF, B_BITS, B_BPREF, B_WSOFF,
        B_CNT, B_CNT2, B_PTR, B_PART, B_WS, B_DUPOFF, B_DUPN, B_DUPT, B_DUPP,
        B_TMP0, B_TMP1, B_TMP2, B_TMP3, B_TMP4, B_TMP5,
        // partition buckets of the symbolic pass
        B_PFIRST, B_PBOFF, B_PBKT, B_PSPAN,
        // work units of the row-unit numeric pass (num2)
        B_N2CNT, B_N2OFF, B_N2UNIT,
        // the column-slice symbolic's per-row work-space cursors
        B_CBSCUR,
        // sym3's retry lists (rows whose possible-duplicate list overflowed)
        B_S3RETRY,
        // k_sym_gtab's global tables (keys, own) for the two bins beyond SYM2_MAX
        B_GTKEY, B_GTOWN, B_COUNT
    };
    struct Buf {
        void *p = nullptr;
        size_t cap = 0;
    };
    int device = 0;
    void *stream = nullptr;
    bool own_stream = false;
    Buf bufs[B_COUNT];
    hipEvent_t ev[8] = {};
    // bin kernels run concurrently on side streams forked from / joined to
    // `stream` (a CU then holds work of several bins at once, and the tail of
    // one bin overlaps the next)
    static constexpr int NSIDE = 4;
    void *side[NSIDE] = {};
    hipEvent_t fork_ev = nullptr;
    hipEvent_t join_ev[NSIDE] = {};
    ias_status fork();
    ias_status join();
    bool serial = false;   // IAS_SERIAL=1: everything on `stream` (per-kernel profiling)
    // small products (flops < SMALL_FLOPS): the bins run on `stream` too — a
    // fork / join across queues costs ~30 us of event latency each, more than
    // the bins of a small product overlap
    bool small = false;
    static constexpr int64_t SMALL_FLOPS = 64ll << 20;
    void *side_stream(int i) const { return (serial || small) ? stream : side[i % NSIDE]; }
    void *host_counters = nullptr;

    // state carried from symbolic() to numeric() (and the row sort)
    int64_t n_rows = 0;
    int64_t n_cols = 0;      // C's columns
    bool cbm_path = false;   // partitioned rows: one LDS column bitmap per row (k_sym_cbm)
    bool wide_v = false;     // B entries beyond 2^29 among the selected rows (k_num2<true, …>)
    bool wide_redo = false;  // this call's analysis redone with the bins of B beyond 2^30 entries
    int64_t n_entries = 0;   // stored entries of A (expanded-A length)
    int64_t nnz_total = 0;
    int64_t flops = 0;
    int32_t max_prod = 0;
    int32_t max_nnz = 0;
    int32_t num_count[ias::MAX_BINS] = {};
    unsigned long long num_items = 0;
    int64_t st_prod = 0, st_nnz = 0;
    int64_t n2_units = 0;   // work units of the row-unit numeric pass
    int64_t n2_bunits = 0;  //   of which the first belong to rows with > 1024 duplicates,
    int64_t n2_dunits = 0;  //   and up to here to rows with duplicates
    hipEvent_t fix_ev[2] = {}; // units of class 0 / class 1 done: their fix-ups may start
    hipEvent_t n2_ev[6] = {};  // around each streaming-pass launch: ms_stream = their sum
    // symbolic stream balancing fed back from the previous call: each bin's
    // measured duration beside the others per estimated product (ns; 0: not
    // measured yet) and the events around its launches
    double sym_w[ias::MAX_BINS] = {};
    double sym_est_prev[ias::MAX_BINS] = {};   // the last call's estimated products per bin
    // rows each sym3 / sym4 / sym5 bin handed to sym2 on the last call (-1:
    // unknown): this call's retry grids are sized from them
    int32_t retry_prev[16] = {-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};
    int32_t retry_upper[16] = {};       // the product bound of the bin each count belongs to
    int32_t retry_upper_cur[16] = {};   //   (this call's, until its counts are read)
    hipEvent_t bin_ev[2 * ias::MAX_BINS] = {};
    bool bin_rec[ias::MAX_BINS] = {};
    unsigned long long num_ws = 0;
    // identity of the operands of the last symbolic() (checked by compute)
    const void *last_a = nullptr, *last_b = nullptr;

    ~ias_plan();
    ias_status init(int device, void *stream);
    ias_status reserve(void **buf, size_t *cap, size_t bytes);
    ias_status reserve(int which, size_t bytes) { return reserve(&bufs[which].p, &bufs[which].cap, bytes); }
    // hipFree every workspace buffer once the plan's streams are idle (they
    // grow again on the next call); returns the bytes freed
    size_t release_workspace();
    size_t workspace_bytes() const;
    // a_entries: stored entries of A (CSR: nnz of the view; ELL: rows * width)
    ias_status analysis_launch(const ias::dev::Rows &A, const ias::dev::Rows &B, int64_t rows,
                               int64_t a_entries);
    const double *ax_aval = nullptr;   // A.val + the view's base (set after the analysis read-back)
    ias_status symbolic(const ias::dev::Rows &A, const ias::dev::Rows &B, int64_t rows,
                        int64_t cols, int64_t a_entries, ias_report *rep);
    ias::dev::AxView ax_view();
    ias_status numeric(const ias::dev::Rows &A, const ias::dev::Rows &B, const ias::dev::Out &out,
                       ias_report *rep);
};

namespace ias {
using Plan = ias_plan;
}
