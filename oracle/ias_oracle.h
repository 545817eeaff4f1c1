/*
 * ias_oracle.h — CPU restatement of the reference's SpGEMM path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libias.so, the CLIs)
 * links or calls this; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, and only as the checker.
 *
 * Every function restates one reference function (paths relative to
 * /root/reference/IA-SPGEMM-CPU_release/):
 *   ora_mtx_read       main.cpp:143-458 + mmio.h:254-367
 *   ora_flops          detail/csr/common_csr.h:290-304 (GetFlop)
 *   ora_csr_mul_csr    detail/csr/common_csr.h:85-193  (CSR_MUL_CSR)
 *   ora_csr_to_coo     detail/coo/common_coo.h:29-66   (CSRtoCOO)
 *   ora_coo_mul_coo    detail/coo/common_coo.h:72-161  (COO_MUL_COO)
 *   ora_csr_to_ell     detail/ell/common_ell.h:30-77   (CSRtoELL)
 *   ora_ell_mul_ell    detail/ell/common_ell.h:80-189  (ELL_MUL_ELL)
 *   ora_csr_to_dia     detail/dia/common_dia.h:29-96   (CSRtoDIA)
 *   ora_dia_mul_dia    detail/dia/common_dia.h:101-195 (DIA_mul_DIA)
 *   ora_sizeof_*       sizeofcsr/coo/ell/dia
 *   ora_features       main.cpp:651-679 (GetInfo1/2/3: the selector's input)
 *   ora_density_image  main.cpp:516-565 (MatNet's density images)
 *
 * Integer products the reference forms in `int` (row*col in GetInfo1/2,
 * row*max_nnz_per_row in GetInfo3, old_i*128 in the image) overflow there for
 * large inputs (undefined behaviour); here they are formed in int64/double,
 * which agrees with the reference wherever it is defined.  The features are
 * pinned by the reference's own printout for Inputs/dia.mtx (CPU/1.jpg,
 * GPU/2.jpg: tests/golden/matnet_known_answers.json).
 *
 * Parity pinning: the reference kernels cannot be built in this image (every
 * detail/<fmt>/common_<fmt>.h includes "mkl.h", which the image lacks), so this restatement is
 * pinned by (1) the known answers recorded from the reference in SURVEY.md §4
 * (tests/golden/), and (2) MKL mkl_sparse_sp2m, the third-party routine behind
 * the reference's Algorithm 1, run on the same inputs (tests/test_oracle.py).
 *
 * Struct layouts equal the product's ias_* structs (include/ias.h) so one set
 * of ctypes definitions serves both.
 */
#ifndef IAS_ORACLE_H
#define IAS_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ora_csr {
    int64_t rows, cols, nnz;
    int64_t *row_ptr; int32_t *col; double *val;
    int32_t memory, device;
} ora_csr;

typedef struct ora_coo {
    int64_t rows, cols, nnz;
    int64_t *row_offset; int32_t *row; int32_t *col; double *val;
    int32_t memory, device, choice, reserved;
} ora_coo;

typedef struct ora_ell {
    int64_t rows, cols, nnz;
    int32_t max_nnz_per_row, choice;
    int32_t *nnz_row; int32_t *col; double *val;
    int32_t memory, device;
} ora_ell;

typedef struct ora_dia {
    int64_t rows, cols;
    int32_t num_diagonals, choice;
    int32_t *diagonal_offsets; int32_t *diagonal_ind; double *val;
    int32_t memory, device;
} ora_dia;

/* returns 0 on success, <0 as the reference's main() return codes */
int     ora_mtx_read(const char *path, ora_csr *A, int32_t flags[4]);
int64_t ora_flops(const ora_csr *A, const ora_csr *B);
void    ora_csr_mul_csr(const ora_csr *A, const ora_csr *B, ora_csr *C);
/* CSR_MUL_CSR folded into per-row nnz and an order-sensitive digest of C
   (row, position, column, value bits), without storing C (full-size pins) */
void    ora_csr_mul_csr_digest(const ora_csr *A, const ora_csr *B, int64_t *row_nnz, uint64_t *digest);
/* the same digest of C with every row sorted by column (IAS_ORDER_SORTED) */
void    ora_csr_mul_csr_digest_sorted(const ora_csr *A, const ora_csr *B, int64_t *row_nnz, uint64_t *digest);
int     ora_csr_to_coo(const ora_csr *A, ora_coo *out, double gate);
void    ora_coo_mul_coo(const ora_coo *A, const ora_coo *B, ora_coo *C);
int     ora_csr_to_ell(const ora_csr *A, ora_ell *out, double gate);
void    ora_ell_mul_ell(const ora_ell *A, const ora_ell *B, ora_ell *C);
int     ora_csr_to_dia(const ora_csr *A, ora_dia *out, double gate);
void    ora_dia_mul_dia(const ora_dia *A, const ora_dia *B, ora_dia *C);
double  ora_sizeof_csr(const ora_csr *A);
double  ora_sizeof_coo(const ora_coo *A);
double  ora_sizeof_ell(const ora_ell *A);
double  ora_sizeof_dia(const ora_dia *A);
/* features[0..25] in main.cpp:651-679's layout (nfeatures 26) or GPU/main.cu:
   434-444's (18): GetInfo1 of A and B (csr/common_csr.h:257-287), GetInfo2 of
   DIA(A), DIA(B) (dia/common_dia.h:222-233; num_diagonals as CSRtoDIA counts
   it, :32-49), GetInfo3 of ELL(A), ELL(B) (ell/common_ell.h:222-229;
   max_nnz_per_row as CSRtoELL, :33-39). */
void    ora_features(const ora_csr *A, const ora_csr *B, int32_t nfeatures, double *features);
/* 128x128 density image, main.cpp:516-565 (row-major, image[k*128+m]) */
void    ora_density_image(const ora_csr *A, int64_t *image);
void    ora_free_csr(ora_csr *A);
void    ora_free_coo(ora_coo *A);
void    ora_free_ell(ora_ell *A);
void    ora_free_dia(ora_dia *A);

#ifdef __cplusplus
}
#endif
#endif
