/*
 * ias.h — C-ABI of the MI355X-native IA-SpGEMM engine (libias.so).
 *
 * This is the drop-in boundary for the reference's row-wise SpGEMM path.
 * The reference (hipdac-lab/IA-SpGEMM) has no library: its "operator API" is a
 * set of header-only free functions over POD structs called from main().  Every
 * entry point below names the reference function it replaces (file:line, paths
 * relative to IA-SPGEMM-CPU_release/ unless prefixed GPU/).
 *
 * Conventions:
 *   - plain pointers and sizes, no torch / HIP types in any signature
 *     (streams are passed as `void*` holding a hipStream_t);
 *   - int64 row pointers and counts everywhere (the reference's `int` overflows
 *     at nnz(C) > 2^31, format.h:36-38); int32 column indices; fp64 values;
 *   - outputs are library-allocated, caller frees with ias_*_free()
 *     (reference: callee mallocs C, caller calls FreeXMatrix);
 *   - every entry point returns an ias_status instead of exit()/ignored MKL
 *     statuses (reference: GPU/detail/common.h:62-77 exits);
 *   - no hidden global state: everything per-call lives in an ias_plan, so the
 *     library is reentrant per stream.
 *   - a matrix lives either on the host or on one HIP device (`memory`,
 *     `device`); compute entry points accept both and return C where
 *     opts->output_memory says.
 */
#ifndef IAS_H
#define IAS_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IAS_ABI_VERSION 6   /* 2: ias_report gained ms_stream, stream_products, stream_nnz;
                               3: ias_csr_mul_csr_into (single pass);
                               4: input-aware selector (features, images, MatNet);
                               5: ias_report.stream_launches;
                               6: ias_last_diag */

typedef enum ias_status {
    IAS_SUCCESS = 0,
    IAS_ERROR_INVALID_ARGUMENT = 1,
    IAS_ERROR_DIMENSION_MISMATCH = 2,
    IAS_ERROR_OUT_OF_MEMORY = 3,
    IAS_ERROR_DEVICE = 4,          /* HIP runtime error or no device */
    IAS_ERROR_IO = 5,              /* fopen / short read */
    IAS_ERROR_FORMAT = 6,          /* bad Matrix-Market banner / size line */
    IAS_ERROR_UNSUPPORTED = 7,     /* complex or dense-array .mtx, ... */
    IAS_ERROR_INFEASIBLE = 8,      /* format gate said `choice = false` */
    IAS_ERROR_OVERFLOW = 9,        /* an index does not fit its type */
    IAS_ERROR_UNAVAILABLE = 10,    /* optional runtime (MKL) not present */
    IAS_ERROR_INSUFFICIENT_CAPACITY = 11 /* caller-provided C too small */
} ias_status;

typedef enum ias_memory { IAS_MEMORY_HOST = 0, IAS_MEMORY_DEVICE = 1 } ias_memory;

/* Output column order inside each row of C. */
typedef enum ias_order {
    /* The order the reference kernel of that format emits, value-for-value:
     * CSR and ELL: reverse first-touch (CSR_MUL_CSR linked-list head insertion,
     * csr/common_csr.h:164-187; ELL_MUL_ELL ell/common_ell.h:163-185);
     * COO: forward first-touch (COO_MUL_COO linear probe, coo/common_coo.h:136-156).
     * Values are summed in the reference's product order without FMA
     * contraction, so integer and fp64 results are bit-identical to it. */
    IAS_ORDER_REFERENCE = 0,
    /* Ascending column index inside each row (MKL/cuSPARSE-like canonical). */
    IAS_ORDER_SORTED = 1
} ias_order;

/* CsrMatrix (detail/format.h:31-41). */
typedef struct ias_csr {
    int64_t rows, cols, nnz;
    int64_t *row_ptr;   /* rows+1 entries; row i is [row_ptr[i], row_ptr[i+1]) */
    int32_t *col;       /* nnz */
    double  *val;       /* nnz */
    int32_t memory;     /* ias_memory */
    int32_t device;     /* HIP ordinal when memory == IAS_MEMORY_DEVICE */
} ias_csr;

/* CooMatrix (detail/format.h:17-29): row-sorted COO carrying row_offset. */
typedef struct ias_coo {
    int64_t rows, cols, nnz;
    int64_t *row_offset; /* rows+1 */
    int32_t *row;        /* nnz */
    int32_t *col;        /* nnz */
    double  *val;        /* nnz */
    int32_t memory, device;
    int32_t choice;      /* reference `choice`: 0 = infeasible under the size gate */
    int32_t reserved;
} ias_coo;

/* EllMatrix (detail/format.h:66-76); col/val are rows x max_nnz_per_row,
 * row-major, padding = column 0 / value 0.0 (malloc2d zero-fill). */
typedef struct ias_ell {
    int64_t rows, cols, nnz;
    int32_t max_nnz_per_row;
    int32_t choice;
    int32_t *nnz_row;    /* rows */
    int32_t *col;
    double  *val;
    int32_t memory, device;
} ias_ell;

/* DiaMatrix (detail/format.h:56-64); val is rows x num_diagonals row-major:
 * val[i*nd + d] = A(i, i + diagonal_offsets[d]) (0.0 where out of range).
 * diagonal_ind has rows+cols-1 entries: diagonal_ind[off + rows - 1] = slot
 * of offset `off` (0 where the diagonal is absent, as the reference). */
typedef struct ias_dia {
    int64_t rows, cols;
    int32_t num_diagonals;
    int32_t choice;
    int32_t *diagonal_offsets; /* num_diagonals, ascending */
    int32_t *diagonal_ind;     /* rows + cols - 1 */
    double  *val;
    int32_t memory, device;
} ias_dia;

/* Per-call options. Zero-initialise and set what you need (ias_opts_default). */
typedef struct ias_opts {
    int32_t order;          /* ias_order */
    int32_t output_memory;  /* ias_memory for C; -1 = same as A */
    int32_t device;         /* HIP device used for compute; -1 = A's device, else 0 */
    int32_t reserved0;
    void   *stream;         /* hipStream_t; NULL = the plan's own stream */
    struct ias_plan *plan;  /* optional workspace cache reused across calls */
} ias_opts;

/* Per-call measurements (device time by hipEvents on the compute stream). */
typedef struct ias_report {
    double  ms_total;       /* first kernel -> last byte of C written */
    double  ms_analysis;    /* row products + binning */
    double  ms_symbolic;    /* per-row nnz + scan */
    double  ms_numeric;     /* accumulate + write C */
    double  ms_upload;      /* host->device of A,B when given on the host */
    double  ms_download;    /* device->host of C when returned on the host */
    int64_t flops;          /* GetFlop (csr/common_csr.h:290-304): multiply pairs */
    int64_t nnz_c;
    int64_t max_row_products;
    int64_t max_row_nnz;
    /* the step's largest pass, the streaming numeric pass (k_num2: rows
       resolved by the symbolic bitmap, C written without a hash table), timed
       with events on its own stream (the sum of its launches' durations) */
    double  ms_stream;
    int64_t stream_products; /* products it processed */
    int64_t stream_nnz;      /* entries of C it wrote */
    int32_t stream_launches; /* its launches: up to 3 (rows by duplicate class,
                                each class's fix-ups overlapping the rest) */
    int32_t kernel;          /* ias_dia_mul_dia: the kernel that ran (IAS_DIA_KERNEL_*) */
} ias_report;
/* ias_report.kernel of ias_dia_mul_dia */
#define IAS_DIA_KERNEL_TILE 1   /* k_dia_tile: LDS row tiles, VALU, bitwise */
#define IAS_DIA_KERNEL_MFMA 2   /* k_dia_mfma: v_mfma_f64_16x16x4f64 dense blocks */
#define IAS_DIA_KERNEL_PAIRS 3  /* k_dia_mul: one thread per C element (wide bands) */

typedef struct ias_mtx_info {
    int32_t is_pattern, is_real, is_integer, is_symmetric; /* main.cpp:171-189 */
    int64_t rows, cols;
    int64_t nnz_file;       /* entries listed in the file (nnzA_mtx_report) */
} ias_mtx_info;

typedef struct ias_plan ias_plan;

/* ---------------------------------------------------------------- misc */
int         ias_abi_version(void);
const char *ias_status_string(ias_status s);
/* Detail of the last failure on the calling thread ("" if none). */
const char *ias_last_error(void);
/* Diagnostics of the calling thread's last symbolic pass (the nnz phase of a
 * CSR product): with the environment variable IAS_CBM_FORCE set (a test knob:
 * bits 1 = the column-bitmap symbolic's minima table in global memory,
 * 2 = its duplicates found by a sweep instead of the list, 4 = its first-touch
 * words in global memory; 0 = no forcing), the OR of the IAS_DIAG_CBM_*
 * branches its rows took; 0 otherwise, and 0 after a call that stopped
 * before the end of its symbolic pass (an error, or no CSR product).  No
 * reference counterpart. */
uint32_t    ias_last_diag(void);
#define IAS_DIAG_CBM_GLOBAL_OWN    1u   /* minima table in the row's work space */
#define IAS_DIAG_CBM_UNLISTED_KEEP 2u   /* duplicate sweep, duplicates kept for the fix-ups */
#define IAS_DIAG_CBM_UNLISTED_DROP 4u   /* duplicate sweep, row left to the table path */
#define IAS_DIAG_CBM_GLOBAL_WORDS  8u   /* first-touch words built in global memory */
#define IAS_DIAG_CBM_LISTED_KEEP  16u   /* duplicate list, duplicates kept */
#define IAS_DIAG_CBM_LISTED_DROP  32u   /* duplicate list, row left to the table path */
#define IAS_DIAG_CBM_LDS_OWN      64u   /* minima table in LDS */
ias_status  ias_device_count(int32_t *count);
void        ias_opts_default(ias_opts *opts);

/* Workspace/stream holder; the analogue of the cuSPARSE handle the reference
 * creates per call (GPU/detail/cusparse/common_cusparse.h:44-72). */
ias_status ias_plan_create(ias_plan **plan, int32_t device, void *stream);
ias_status ias_plan_destroy(ias_plan *plan);
/* Memory the library keeps on a device between calls: the block cache of
 * freed output blocks and the workspace of the per-device default plan (the
 * plan of calls made without one).  Both are released by themselves when a
 * device allocation of the library runs out of memory; a caller about to
 * allocate a lot of its own can release them first.  (No reference
 * counterpart: the reference creates a cuSPARSE handle per call,
 * GPU/detail/cusparse/common_cusparse.h:44, and keeps nothing between
 * calls.)  released_bytes may be NULL. */
ias_status ias_device_release(int32_t device, int64_t *released_bytes);
ias_status ias_device_cached_bytes(int32_t device, int64_t *bytes);

/* ---------------------------------------------------------------- memory */
ias_status ias_csr_alloc(ias_csr *m, int64_t rows, int64_t cols, int64_t nnz,
                         int32_t memory, int32_t device);
ias_status ias_csr_copy(const ias_csr *src, ias_csr *dst, int32_t memory, int32_t device);
/* Device arrays go back to a per-device block cache (reused by later calls
 * on that device) instead of hipFree; finish your own work on them first. */
ias_status ias_csr_free(ias_csr *m);   /* FreeCsrMatrix  csr/common_csr.h:307-317 */
ias_status ias_coo_free(ias_coo *m);   /* FreeCooMatrix  coo/common_coo.h:185-195 */
ias_status ias_ell_free(ias_ell *m);   /* FreeEllMatrix  ell/common_ell.h:232-244 */
ias_status ias_dia_free(ias_dia *m);   /* FreeDiaMatrix  dia/common_dia.h:236-249 */
ias_status ias_coo_copy(const ias_coo *src, ias_coo *dst, int32_t memory, int32_t device);
ias_status ias_ell_copy(const ias_ell *src, ias_ell *dst, int32_t memory, int32_t device);
ias_status ias_dia_copy(const ias_dia *src, ias_dia *dst, int32_t memory, int32_t device);

/* ---------------------------------------------------------------- Matrix-Market I/O
 * Reader semantics of main.cpp:143-458 + mmio.h:254-367: banner typecode,
 * comment skipping, 1-based -> 0-based, pattern -> 1.0, integer -> double,
 * symmetric/hermitian mirrored with the same value (skew NOT mirrored),
 * stable counting sort by row in file order, duplicates kept, columns unsorted.
 * Result is on the host. */
ias_status ias_mtx_read(const char *path, ias_csr *A, ias_mtx_info *info);
/* Two-file read exactly as main.cpp:139-458: B's row count is forced to A's
 * column count (main.cpp:482) and B's own row count is ignored. */
ias_status ias_mtx_read_pair(const char *path_a, const char *path_b, ias_csr *A, ias_csr *B,
                             ias_mtx_info *info_a, ias_mtx_info *info_b);
/* mm_write_mtx_crd (mmio.h:445-486): "%%MatrixMarket matrix coordinate real general". */
ias_status ias_mtx_write(const char *path, const ias_csr *A);

/* ---------------------------------------------------------------- format layer
 * gate: the reference feasibility threshold (50 on CPU: coo/common_coo.h:37,
 * dia/common_dia.h:56, ell/common_ell.h:47; 20 on GPU: GPU/detail/dia/
 * common_dia.h:51 etc.); <= 0 disables the gate.  When the gate fails the
 * output has choice = 0, no arrays, and IAS_ERROR_INFEASIBLE is returned.
 * Inputs may be host or device; outputs land in the same memory.  A device
 * CSR is converted on its device (no host round trip), byte-identical to the
 * host conversion. */
ias_status ias_csr_to_coo(const ias_csr *A, ias_coo *out, double gate); /* CSRtoCOO coo:29-66 */
ias_status ias_csr_to_ell(const ias_csr *A, ias_ell *out, double gate); /* CSRtoELL ell:30-77 */
ias_status ias_csr_to_dia(const ias_csr *A, ias_dia *out, double gate); /* CSRtoDIA dia:29-96 */
ias_status ias_coo_to_csr(const ias_coo *A, ias_csr *out);
ias_status ias_ell_to_csr(const ias_ell *A, ias_csr *out);
/* Every stored DIA position that is in range (explicit zeros included). */
ias_status ias_dia_to_csr(const ias_dia *A, ias_csr *out);
/* B = A^T, as mkl_dcsrcsc(job={0,0,0,0,0,1}) in GPU/main.cu:260-269; columns of
 * each output row ascend (stable by source row).  A device CSR is transposed
 * on its device (stable radix sort), byte-identical to the host path. */
ias_status ias_csr_transpose(const ias_csr *A, ias_csr *AT);

/* size models of the report's memory_size column */
double ias_sizeof_csr(const ias_csr *A); /* sizeofcsr csr/common_csr.h:196-202 */
double ias_sizeof_coo(const ias_coo *A); /* sizeofcoo coo/common_coo.h:20-26 */
double ias_sizeof_ell(const ias_ell *A); /* sizeofell ell/common_ell.h:21-27 */
double ias_sizeof_dia(const ias_dia *A); /* sizeofdia dia/common_dia.h:20-26 */

/* ---------------------------------------------------------------- SpGEMM hot path
 * C = A * B.  C must be zero-initialised by the caller; the library allocates
 * its arrays (memory per opts->output_memory) and the caller frees them.
 * opts and report may be NULL. */
ias_status ias_csr_mul_csr(const ias_csr *A, const ias_csr *B, ias_csr *C,
                           const ias_opts *opts, ias_report *report);  /* CSR_MUL_CSR csr:85-193 */
ias_status ias_coo_mul_coo(const ias_coo *A, const ias_coo *B, ias_coo *C,
                           const ias_opts *opts, ias_report *report);  /* COO_MUL_COO coo:72-161 */
ias_status ias_ell_mul_ell(const ias_ell *A, const ias_ell *B, ias_ell *C,
                           const ias_opts *opts, ias_report *report);  /* ELL_MUL_ELL ell:80-189 */
/* DIA: bitwise the reference for narrow bands (LDS-tiled VALU kernel); bands
 * with nd_A * nd_B >= 256 use f64 MFMA dense blocks (fused sums: within the
 * north-star 1e-10 relative tolerance, not bitwise); IAS_DIA_MFMA=0/1 in the
 * environment forces either kernel. */
ias_status ias_dia_mul_dia(const ias_dia *A, const ias_dia *B, ias_dia *C,
                           const ias_opts *opts, ias_report *report);  /* DIA_mul_DIA dia:101-195 */
/* The same into caller-provided device arrays (no allocation in the call; the
 * reference's GPU DIA path, GPU/detail/dia_dev/common_dia_dev.h:85-122, writes
 * into C arrays allocated before its kernels): C->memory = device, C->device
 * the compute device, C->num_diagonals = the capacity in diagonals,
 * diagonal_offsets >= capacity entries, diagonal_ind >= rows + cols - 1, val >=
 * rows x capacity.  On success C->num_diagonals = nd_C and val is rows x nd_C
 * row-major; a capacity below nd_C returns IAS_ERROR_INSUFFICIENT_CAPACITY with
 * C->num_diagonals = nd_C.  C's arrays must not share memory with A's or B's
 * (C is written while they are read): IAS_ERROR_INVALID_ARGUMENT.
 * ias_dia_mul_dia_ndiag gives nd_C from the offsets alone (dia:107-140's
 * reachability rule; IAS_ERROR_INFEASIBLE for an infeasible operand, as the
 * product itself). */
ias_status ias_dia_mul_dia_into(const ias_dia *A, const ias_dia *B, ias_dia *C,
                                const ias_opts *opts, ias_report *report);
ias_status ias_dia_mul_dia_ndiag(const ias_dia *A, const ias_dia *B, int32_t *nd_c);

/* Two-phase form on device-resident CSR, the split the reference's GPU path
 * uses (cusparseXcsrgemmNnz + cusparseDcsrgemm, GPU/detail/cusparse/
 * common_cusparse.h:78-91).  nnz: analysis + symbolic + scan; the row pointer
 * of C is written to row_ptr_c (device, rows+1) when non-NULL and kept in the
 * plan otherwise.  compute: numeric phase into caller-provided device arrays
 * C->row_ptr/col/val with capacity C->nnz (>= the nnz returned); it must
 * follow an nnz call on the same plan with the same A and B.  Both calls
 * return only when their device work is complete (C may be read or freed
 * from any stream right away). */
ias_status ias_csr_mul_csr_nnz(ias_plan *plan, const ias_csr *A, const ias_csr *B,
                               int64_t *nnz_c, int64_t *row_ptr_c, ias_report *report);
ias_status ias_csr_mul_csr_compute(ias_plan *plan, const ias_csr *A, const ias_csr *B,
                                   ias_csr *C, int32_t order, ias_report *report);

/* Single-call form on device-resident CSR (no separate nnz call): the two
 * loops of CSR_MUL_CSR (csr/common_csr.h:95-189) as the two-phase engine
 * behind one call.  (A row-block pipeline — each block's symbolic pass beside
 * the previous block's numeric pass — was measured 4-40% slower on K2/K3/K3'/
 * K4 and dropped)
 * C->row_ptr
 * (rows+1), C->col and C->val are caller-provided device arrays of capacity
 * C->nnz; nnz(C) <= flops(A*B) (ias_flops), so that capacity always suffices.
 * On success C->nnz = nnz(C).  With less capacity than nnz(C), nothing is
 * written beyond it, C->row_ptr is complete, C->nnz is set to the nnz needed
 * and IAS_ERROR_INSUFFICIENT_CAPACITY is returned.  Returns when C is
 * complete.  order: ias_order. */
ias_status ias_csr_mul_csr_into(ias_plan *plan, const ias_csr *A, const ias_csr *B, ias_csr *C,
                                int32_t order, ias_report *report);

/* ---------------------------------------------------------------- input-aware selector
 * The "IA" of IA-SpGEMM (main.cpp:512-704; GPU/main.cu:272-460): matrix
 * features and two 128x128 density images (A's and B's) go to MatNet, a small
 * Keras CNN (MatNet.py Pred), whose argmax names the algorithm to run.  Host
 * code (device matrices are copied to the host), off the timed path. */
#define IAS_IMAGE_SIDE 128
typedef struct ias_matnet ias_matnet;
/* nfeatures 26 (the CPU program, main.cpp:651-679): GetInfo1(A) [0..8],
 * GetInfo1(B) [9..17] (csr:257-287), GetInfo2(DIA(A)) [18..20], GetInfo2(DIA(B))
 * [21..23] (dia:222-233), GetInfo3(ELL(A)) [24], GetInfo3(ELL(B)) [25]
 * (ell:222-229); nfeatures 18 (the GPU program, GPU/main.cu:434-444):
 * GetInfo1(A), GetInfo1(B).  Integer products the reference forms in `int`
 * (row*col) are formed in double (the reference overflows beyond 2^31). */
ias_status ias_features(const ias_csr *A, const ias_csr *B, int32_t nfeatures, double *features);
/* main.cpp:516-565: image[k*128 + m] = number of A's entries mapped to cell
 * (k, m) (rows/cols scaled to 128; sides under 128 spread over several cells). */
ias_status ias_density_image(const ias_csr *A, int64_t *image);
/* weights: "intel" / "amd" (the CPU program's sets: 26 features, 5 classes =
 * algorithms {MKL, CSR, DIA, ELL, COO}), "p100" (the GPU program's: 18
 * features, 3 classes = {CUSP, cuSPARSE, NSPARSE}), or a path to a blob made
 * by tools/matnet_export.py; named sets are read from $IAS_MATNET_DIR or
 * <dir of libias.so>/data. */
ias_status ias_matnet_load(const char *weights, ias_matnet **net);
ias_status ias_matnet_free(ias_matnet *net);
ias_status ias_matnet_shape(const ias_matnet *net, int32_t *nfeatures, int32_t *nclasses);
/* MatNet.py Pred: images scaled to 255*count/max, float32 forward pass,
 * softmax into probs (nclasses, may be NULL); *chosen = argmax, 0-based. */
ias_status ias_matnet_predict(const ias_matnet *net, const int64_t *image_a, const int64_t *image_b,
                              const double *features, float *probs, int32_t *chosen);

/* ---------------------------------------------------------------- verification */
/* GetFlop (csr/common_csr.h:290-304): sum over stored A(i,j) of nnz(B row j). */
ias_status ias_flops(const ias_csr *A, const ias_csr *B, int64_t *flops);
/* verified_sum (main.cpp:753-755 etc.): sum of all stored values (sequential
 * order on the host; DIA/ELL sum their padded arrays as the reference). */
ias_status ias_sum_csr(const ias_csr *A, double *sum);
ias_status ias_sum_coo(const ias_coo *A, double *sum);
ias_status ias_sum_ell(const ias_ell *A, double *sum);
ias_status ias_sum_dia(const ias_dia *A, double *sum);

/* ---------------------------------------------------------------- multi-GPU helpers
 * Row-block view [r0, r1) of A without copying (row_ptr is an offset view;
 * kernels address col/val absolutely, so no rebasing is needed). */
ias_status ias_csr_row_view(const ias_csr *A, int64_t r0, int64_t r1, ias_csr *view);
/* Split A's rows into nparts contiguous blocks of near-equal estimated device
 * cost (a flops prefix, not rows; each row weighted by a fixed
 * per-row cost plus its products, products of hash-partitioned rows counted
 * 3.4x, calibrated on MI355X); bounds has nparts+1 entries.
 * Host or device A. */
ias_status ias_partition_rows(const ias_csr *A, const ias_csr *B, int32_t nparts,
                              int64_t *bounds);
/* Add `offset` to every entry of a device row pointer (allgatherv fix-up). */
ias_status ias_row_ptr_shift(int64_t *row_ptr, int64_t count, int64_t offset,
                             int32_t device, void *stream);

/* One process, N devices (the reference is single-device, its
 * CPU kernels split rows the same way over OpenMP threads,
 * csr/common_csr.h:95-189): A's rows split by ias_partition_rows, one host
 * thread + plan per device computes its block of C = A*B (host or device
 * operands; B staged on every device), the blocks concatenated in row order
 * into C (library-allocated; opts->output_memory host (default) or device =
 * devices[0]).  devices may be NULL (0..ndev-1); a device may repeat.
 * report: flops / nnz summed, times = the slowest device. */
ias_status ias_csr_mul_csr_multi(const ias_csr *A, const ias_csr *B, ias_csr *C, int32_t ndev,
                                 const int32_t *devices, const ias_opts *opts, ias_report *report);

/* One process per GPU over RCCL (xGMI).  librccl is opened at first use.
 * ias_dist_unique_id: rank 0 makes the id (>= 128 bytes) and shares it out of
 * band; every rank then calls ias_dist_create with it. */
typedef struct ias_dist ias_dist;
ias_status ias_dist_unique_id(char *id, int32_t id_len);
ias_status ias_dist_create(ias_dist **dist, const char *id, int32_t nranks, int32_t rank, int32_t device);
/* The same rank handle over the in-process loopback transport (SURVEY.md
 * §4.4): nranks ranks of ONE process, each driven by its own host thread, meet
 * under the name `group`; the collectives are host barriers + hipMemcpyAsync
 * of the peers' buffers.  Ranks may share a device (RCCL allows one rank per
 * device), so the sharded path and the allgatherv fix-up run at P > 1 on one
 * GPU.  Every other ias_dist_* entry point takes either kind of handle. */
ias_status ias_dist_create_loopback(ias_dist **dist, const char *group, int32_t nranks, int32_t rank,
                                    int32_t device);
ias_status ias_dist_destroy(ias_dist *dist);
/* Concatenate the row-sharded C on every rank: C_local (device, this rank's
 * rows, row pointer from 0) -> C_full (library-allocated on the rank's
 * device): per-rank counts by ncclAllGather, then one ncclBroadcast per root
 * into its slice (one group), row pointers shifted by the global nnz offset. */
ias_status ias_dist_allgatherv_csr(ias_dist *dist, const ias_csr *C_local, ias_csr *C_full, void *stream);
/* This rank's row block of C = A*B (A, B replicated, host or device): C is the
 * block (gather = 0) or the whole C on every rank (gather = 1), on the rank's
 * device, library-allocated. */
ias_status ias_dist_csr_mul_csr(ias_dist *dist, const ias_csr *A, const ias_csr *B, ias_csr *C,
                                int32_t gather, int32_t order, ias_report *report);

/* ---------------------------------------------------------------- synthetic inputs
 * Deterministic host generators (counter-based splitmix64; identical on every
 * machine).  value_mode 0: U(-1,1); 1: integers 1..9 (exact fp64 sums). */
ias_status ias_gen_rmat(int32_t scale, double edge_factor, double a, double b, double c,
                        uint64_t seed, int32_t value_mode, ias_csr *out);
ias_status ias_gen_band(int64_t n, int32_t half_width, uint64_t seed, int32_t value_mode,
                        ias_csr *out);
ias_status ias_gen_ell(int64_t n, int32_t per_row, uint64_t seed, int32_t value_mode,
                       ias_csr *out);

/* ---------------------------------------------------------------- CPU baseline
 * The reference's Algorithm 1, MKL_MUL_MKL (csr/common_csr.h:18-47):
 * mkl_sparse_d_create_csr x2 + mkl_sparse_sp2m(FULL_MULT) + export, timed as
 * main.cpp:746-748.  MKL is loaded at run time (dlopen libmkl_rt, GNU threading
 * layer); IAS_ERROR_UNAVAILABLE if absent.  A, B on the host; C on the host
 * (library-allocated); int32 (LP64) unless nnz needs ILP64, which is used then. */
ias_status ias_mkl_available(int32_t *available, char *version, int32_t version_len);
ias_status ias_mkl_sp2m(const ias_csr *A, const ias_csr *B, ias_csr *C, int32_t threads,
                        double *ms);

#ifdef __cplusplus
}
#endif

#endif /* IAS_H */
