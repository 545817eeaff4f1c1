/*
 * ias_oracle.c — CPU restatement of the reference SpGEMM path.
 * TEST INFRASTRUCTURE ONLY (see ias_oracle.h).  Compiled with
 * -ffp-contract=off so every a*b and s+p rounds separately, as the reference
 * does when built for x86-64 without FMA (CPU/Makefile:13: icc -O3, no -x).
 */
#include "ias_oracle.h"

#include <ctype.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

static void *zalloc(size_t n, size_t sz) {
    void *p = calloc(n ? n : 1, sz);
    if (!p) { fprintf(stderr, "oracle: out of memory\n"); abort(); }
    return p;
}

/* ------------------------------------------------------------------ reader
 * main.cpp:143-458: banner via mm_read_banner (mmio.h:254-337), size line via
 * mm_read_mtx_crd_size (mmio.h:339-367, skips '%' lines), entries read as
 * "%d %d %lg" / "%d %d %d" / "%d %d", 1-based -> 0-based, then a stable
 * counting sort by row in file order; symmetric/hermitian files also place the
 * mirrored (col,row) entry when row != col (main.cpp:317-332, 372-447). */
static void lower(char *s) { for (; *s; ++s) *s = (char)tolower((unsigned char)*s); }

int ora_mtx_read(const char *path, ora_csr *A, int32_t flags[4]) {
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    char line[1100], b0[64], b1[64], b2[64], b3[64], b4[64];
    if (!fgets(line, sizeof line, f) ||
        sscanf(line, "%63s %63s %63s %63s %63s", b0, b1, b2, b3, b4) != 5) { fclose(f); return -2; }
    lower(b1); lower(b2); lower(b3); lower(b4);
    if (strncmp(b0, "%%MatrixMarket", 14) != 0 || strcmp(b1, "matrix") != 0) { fclose(f); return -2; }
    if (strcmp(b2, "coordinate") != 0) { fclose(f); return -2; } /* dense arrays never worked in main.cpp */
    int is_real = !strcmp(b3, "real"), is_int = !strcmp(b3, "integer"), is_pat = !strcmp(b3, "pattern");
    if (!strcmp(b3, "complex")) { fclose(f); return -3; }
    if (!is_real && !is_int && !is_pat) { fclose(f); return -2; }
    int is_sym = !strcmp(b4, "symmetric") || !strcmp(b4, "hermitian");
    if (!is_sym && strcmp(b4, "general") && strcmp(b4, "skew-symmetric")) { fclose(f); return -2; }

    long long m = 0, n = 0, nz = 0;
    do { if (!fgets(line, sizeof line, f)) { fclose(f); return -4; } } while (line[0] == '%');
    if (sscanf(line, "%lld %lld %lld", &m, &n, &nz) != 3) {
        int got;
        do { got = fscanf(f, "%lld %lld %lld", &m, &n, &nz); if (got == EOF) { fclose(f); return -4; } } while (got != 3);
    }
    int64_t *ri = (int64_t *)zalloc((size_t)nz, sizeof(int64_t));
    int64_t *ci = (int64_t *)zalloc((size_t)nz, sizeof(int64_t));
    double *vv = (double *)zalloc((size_t)nz, sizeof(double));
    for (long long e = 0; e < nz; ++e) {
        long long r = 0, c = 0; double v = 1.0; int iv = 0;
        if (is_real) { if (fscanf(f, "%lld %lld %lg", &r, &c, &v) != 3) break; }
        else if (is_int) { if (fscanf(f, "%lld %lld %d", &r, &c, &iv) != 3) break; v = iv; }
        else { if (fscanf(f, "%lld %lld", &r, &c) != 2) break; v = 1.0; }
        ri[e] = r - 1; ci[e] = c - 1; vv[e] = v;
    }
    fclose(f);

    int64_t *cnt = (int64_t *)zalloc((size_t)m + 1, sizeof(int64_t));
    for (long long e = 0; e < nz; ++e) {
        cnt[ri[e]]++;
        if (is_sym && ri[e] != ci[e]) cnt[ci[e]]++;
    }
    A->rows = m; A->cols = n;
    A->row_ptr = (int64_t *)zalloc((size_t)m + 1, sizeof(int64_t));
    for (long long i = 0; i < m; ++i) A->row_ptr[i + 1] = A->row_ptr[i] + cnt[i];
    A->nnz = A->row_ptr[m];
    A->col = (int32_t *)zalloc((size_t)A->nnz, sizeof(int32_t));
    A->val = (double *)zalloc((size_t)A->nnz, sizeof(double));
    memset(cnt, 0, (size_t)(m + 1) * sizeof(int64_t));
    for (long long e = 0; e < nz; ++e) {
        int64_t r = ri[e], c = ci[e];
        int64_t at = A->row_ptr[r] + cnt[r]++;
        A->col[at] = (int32_t)c; A->val[at] = vv[e];
        if (is_sym && r != c) {
            at = A->row_ptr[c] + cnt[c]++;
            A->col[at] = (int32_t)r; A->val[at] = vv[e];
        }
    }
    A->memory = 0; A->device = 0;
    free(cnt); free(ri); free(ci); free(vv);
    if (flags) { flags[0] = is_pat; flags[1] = is_real; flags[2] = is_int; flags[3] = is_sym; }
    return 0;
}

/* ------------------------------------------------------------------ GetFlop */
int64_t ora_flops(const ora_csr *A, const ora_csr *B) {
    int64_t total = 0;
    for (int64_t i = 0; i < A->rows; ++i)
        for (int64_t p = A->row_ptr[i]; p < A->row_ptr[i + 1]; ++p) {
            int32_t j = A->col[p];
            total += B->row_ptr[j + 1] - B->row_ptr[j];
        }
    return total;
}

/* ------------------------------------------------------------------ generic
 * Gustavson over "row views": row i of X is (start, length).  The reference
 * runs the same two passes for CSR and ELL (csr:95-189, ell:89-187):
 *   pass 1: count distinct columns per row with a per-thread stamp array;
 *   pass 2: accumulate s[k] = s[k] + a*b in product order (A entries in row
 *           order, then B entries in row order) from s[k] = 0.0, remember the
 *           discovery order, and emit it reversed (linked-list head insert). */
typedef struct rowview {
    const int64_t *ptr;   /* CSR: start = ptr[i], len = ptr[i+1]-ptr[i] */
    const int32_t *len;   /* ELL: start = i*stride, len = len[i] */
    int64_t stride;
    const int32_t *col; const double *val;
} rowview;

static inline void rv_row(const rowview *v, int64_t i, int64_t *s, int64_t *n) {
    if (v->ptr) { *s = v->ptr[i]; *n = v->ptr[i + 1] - v->ptr[i]; }
    else { *s = i * v->stride; *n = v->len[i]; }
}

static void gustavson_count(const rowview *a, const rowview *b, int64_t rows, int64_t cols,
                            int64_t *count) {
#pragma omp parallel
    {
        int64_t *stamp = (int64_t *)malloc((size_t)(cols ? cols : 1) * sizeof(int64_t));
        for (int64_t k = 0; k < cols; ++k) stamp[k] = -1;
#pragma omp for schedule(dynamic, 64)
        for (int64_t i = 0; i < rows; ++i) {
            int64_t as, an, distinct = 0;
            rv_row(a, i, &as, &an);
            for (int64_t p = as; p < as + an; ++p) {
                int64_t bs, bn;
                rv_row(b, a->col[p], &bs, &bn);
                for (int64_t q = bs; q < bs + bn; ++q) {
                    int32_t k = b->col[q];
                    if (stamp[k] != i) { stamp[k] = i; ++distinct; }
                }
            }
            count[i] = distinct;
        }
        free(stamp);
    }
}

/* order: 0 = reverse discovery (CSR/ELL), 1 = forward discovery (COO).
 * first_assign: 1 = first product assigned (COO: values[pos] = a*b),
 *               0 = accumulated from 0.0 (CSR/ELL: sums[k] = sums[k] + v*b). */
static void gustavson_numeric(const rowview *a, const rowview *b, int64_t rows, int64_t cols,
                              const int64_t *out_start, int32_t *out_col, double *out_val,
                              int order, int first_assign) {
#pragma omp parallel
    {
        double *acc = (double *)malloc((size_t)(cols ? cols : 1) * sizeof(double));
        char *seen = (char *)calloc((size_t)(cols ? cols : 1), 1);
        int32_t *disc = (int32_t *)malloc((size_t)(cols ? cols : 1) * sizeof(int32_t));
#pragma omp for schedule(dynamic, 64)
        for (int64_t i = 0; i < rows; ++i) {
            int64_t as, an, nd = 0;
            rv_row(a, i, &as, &an);
            for (int64_t p = as; p < as + an; ++p) {
                double av = a->val[p];
                int64_t bs, bn;
                rv_row(b, a->col[p], &bs, &bn);
                for (int64_t q = bs; q < bs + bn; ++q) {
                    int32_t k = b->col[q];
                    double prod = av * b->val[q];
                    if (!seen[k]) {
                        seen[k] = 1; disc[nd++] = k;
                        acc[k] = first_assign ? prod : 0.0 + prod;
                    } else {
                        acc[k] = acc[k] + prod;
                    }
                }
            }
            int64_t o = out_start[i];
            for (int64_t t = 0; t < nd; ++t) {
                int32_t k = order == 0 ? disc[nd - 1 - t] : disc[t];
                out_col[o + t] = k; out_val[o + t] = acc[k];
            }
            for (int64_t t = 0; t < nd; ++t) seen[disc[t]] = 0;
        }
        free(acc); free(seen); free(disc);
    }
}

void ora_csr_mul_csr(const ora_csr *A, const ora_csr *B, ora_csr *C) {
    rowview a = {A->row_ptr, NULL, 0, A->col, A->val};
    rowview b = {B->row_ptr, NULL, 0, B->col, B->val};
    C->rows = A->rows; C->cols = B->cols;
    C->row_ptr = (int64_t *)zalloc((size_t)C->rows + 1, sizeof(int64_t));
    int64_t *cnt = (int64_t *)zalloc((size_t)C->rows + 1, sizeof(int64_t));
    gustavson_count(&a, &b, A->rows, B->cols, cnt);
    for (int64_t i = 0; i < C->rows; ++i) C->row_ptr[i + 1] = C->row_ptr[i] + cnt[i];
    C->nnz = C->row_ptr[C->rows];
    C->col = (int32_t *)zalloc((size_t)C->nnz, sizeof(int32_t));
    C->val = (double *)zalloc((size_t)C->nnz, sizeof(double));
    gustavson_numeric(&a, &b, A->rows, B->cols, C->row_ptr, C->col, C->val, 0, 0);
    C->memory = 0; C->device = 0;
    free(cnt);
}

/* ------------------------------------------------------------------ digest
 * CSR_MUL_CSR (csr:85-193) at sizes whose C does not fit host memory (K3:
 * 2.28e9 entries): each row is formed exactly as gustavson_numeric forms it
 * (reverse discovery order, sums from 0.0 in product order) and folded into
 * an order-sensitive digest instead of being stored.  row_nnz[i] = nnz of row
 * i; digest = sum over entries of ora_mix(row, position in row, column, value
 * bits) mod 2^64 (addition commutes, so the thread split does not matter).
 * tests/fulldigest.py computes the same sum on the GPU's C. */
static inline uint64_t ora_mix(uint64_t row, uint64_t pos, uint64_t col, uint64_t vbits) {
    uint64_t x = vbits ^ (col * 0x9E3779B97F4A7C15ull) ^ (pos * 0xC2B2AE3D27D4EB4Full) ^
                 (row * 0x165667B19E3779F9ull);
    x *= 0xD6E8FEB86659FD93ull;
    return x ^ (x >> 32);
}

static int ora_cmp_i32(const void *x, const void *y) {
    const int32_t a = *(const int32_t *)x, b = *(const int32_t *)y;
    return (a > b) - (a < b);
}

/* sorted = 0: the reference's order (reverse discovery); 1: every row by
 * ascending column (IAS_ORDER_SORTED, the cuSPARSE-like order of
 * GPU/detail/cusparse/common_cusparse.h:78-91) — same sums, positions by
 * column. */
static void csr_digest(const ora_csr *A, const ora_csr *B, int sorted, int64_t *row_nnz, uint64_t *digest) {
    const int64_t cols = B->cols;
    uint64_t total = 0;
#pragma omp parallel reduction(+ : total)
    {
        double *acc = (double *)malloc((size_t)(cols ? cols : 1) * sizeof(double));
        char *seen = (char *)calloc((size_t)(cols ? cols : 1), 1);
        int32_t *disc = (int32_t *)malloc((size_t)(cols ? cols : 1) * sizeof(int32_t));
#pragma omp for schedule(dynamic, 64)
        for (int64_t i = 0; i < A->rows; ++i) {
            int64_t nd = 0;
            for (int64_t p = A->row_ptr[i]; p < A->row_ptr[i + 1]; ++p) {
                const double av = A->val[p];
                const int32_t j = A->col[p];
                for (int64_t q = B->row_ptr[j]; q < B->row_ptr[j + 1]; ++q) {
                    const int32_t k = B->col[q];
                    const double prod = av * B->val[q];
                    if (!seen[k]) { seen[k] = 1; disc[nd++] = k; acc[k] = 0.0 + prod; }
                    else acc[k] = acc[k] + prod;
                }
            }
            if (sorted) qsort(disc, (size_t)nd, sizeof(int32_t), ora_cmp_i32);
            for (int64_t t = 0; t < nd; ++t) {
                const int32_t k = sorted ? disc[t] : disc[nd - 1 - t];
                uint64_t vb;
                memcpy(&vb, &acc[k], sizeof vb);
                total += ora_mix((uint64_t)i, (uint64_t)t, (uint64_t)(uint32_t)k, vb);
                seen[k] = 0;
            }
            row_nnz[i] = nd;
        }
        free(acc); free(seen); free(disc);
    }
    *digest = total;
}

void ora_csr_mul_csr_digest(const ora_csr *A, const ora_csr *B, int64_t *row_nnz, uint64_t *digest) {
    csr_digest(A, B, 0, row_nnz, digest);
}
void ora_csr_mul_csr_digest_sorted(const ora_csr *A, const ora_csr *B, int64_t *row_nnz, uint64_t *digest) {
    csr_digest(A, B, 1, row_nnz, digest);
}

/* ------------------------------------------------------------------ sizes */
double ora_sizeof_csr(const ora_csr *A) { return 4.0 * (double)(A->rows + 1 + A->nnz + 3) + 8.0 * (double)A->nnz; }
double ora_sizeof_coo(const ora_coo *A) { return 4.0 * (double)(A->rows + 1 + 2 * A->nnz + 3) + 8.0 * (double)A->nnz; }
double ora_sizeof_ell(const ora_ell *A) {
    double rk = (double)A->rows * (double)A->max_nnz_per_row;
    return 4.0 * ((double)A->rows + rk + 4.0) + 8.0 * rk;
}
double ora_sizeof_dia(const ora_dia *A) {
    return 4.0 * (double)(A->rows + A->cols - 1 + A->num_diagonals + 3) +
           8.0 * (double)A->rows * (double)A->num_diagonals;
}

/* ------------------------------------------------------------------ COO */
int ora_csr_to_coo(const ora_csr *A, ora_coo *out, double gate) {
    memset(out, 0, sizeof *out);
    out->rows = A->rows; out->cols = A->cols; out->nnz = A->nnz; out->choice = 1;
    if (gate > 0 && !(ora_sizeof_coo(out) < gate * ora_sizeof_csr(A))) { out->choice = 0; return 1; }
    out->row_offset = (int64_t *)zalloc((size_t)A->rows + 1, sizeof(int64_t));
    out->row = (int32_t *)zalloc((size_t)A->nnz, sizeof(int32_t));
    out->col = (int32_t *)zalloc((size_t)A->nnz, sizeof(int32_t));
    out->val = (double *)zalloc((size_t)A->nnz, sizeof(double));
    int64_t at = 0;
    for (int64_t i = 0; i < A->rows; ++i) {
        out->row_offset[i] = at;
        for (int64_t p = A->row_ptr[i]; p < A->row_ptr[i + 1]; ++p, ++at) {
            out->row[at] = (int32_t)i; out->col[at] = A->col[p]; out->val[at] = A->val[p];
        }
    }
    out->row_offset[A->rows] = at;
    return 0;
}

/* COO_MUL_COO: distinct count with a stamp array, then (serially in the
 * reference: the numeric `omp for` is orphaned) each product is placed in the
 * first free slot of its row or added to the slot already holding its column:
 * forward first-touch order, first value assigned (not added to 0.0). */
void ora_coo_mul_coo(const ora_coo *A, const ora_coo *B, ora_coo *C) {
    rowview a = {A->row_offset, NULL, 0, A->col, A->val};
    rowview b = {B->row_offset, NULL, 0, B->col, B->val};
    memset(C, 0, sizeof *C);
    C->rows = A->rows; C->cols = B->cols; C->choice = 1;
    C->row_offset = (int64_t *)zalloc((size_t)C->rows + 1, sizeof(int64_t));
    int64_t *cnt = (int64_t *)zalloc((size_t)C->rows + 1, sizeof(int64_t));
    gustavson_count(&a, &b, A->rows, B->cols, cnt);
    for (int64_t i = 0; i < C->rows; ++i) C->row_offset[i + 1] = C->row_offset[i] + cnt[i];
    C->nnz = C->row_offset[C->rows];
    C->row = (int32_t *)zalloc((size_t)C->nnz, sizeof(int32_t));
    C->col = (int32_t *)zalloc((size_t)C->nnz, sizeof(int32_t));
    C->val = (double *)zalloc((size_t)C->nnz, sizeof(double));
    gustavson_numeric(&a, &b, A->rows, B->cols, C->row_offset, C->col, C->val, 1, 1);
    for (int64_t i = 0; i < C->rows; ++i)
        for (int64_t p = C->row_offset[i]; p < C->row_offset[i + 1]; ++p) C->row[p] = (int32_t)i;
    free(cnt);
}

/* ------------------------------------------------------------------ ELL */
int ora_csr_to_ell(const ora_csr *A, ora_ell *out, double gate) {
    memset(out, 0, sizeof *out);
    int32_t K = 0;
    for (int64_t i = 0; i < A->rows; ++i) {
        int64_t n = A->row_ptr[i + 1] - A->row_ptr[i];
        if (n > K) K = (int32_t)n;
    }
    out->rows = A->rows; out->cols = A->cols; out->nnz = A->nnz; out->max_nnz_per_row = K;
    out->choice = 1;
    if (gate > 0 && !(ora_sizeof_ell(out) < gate * ora_sizeof_csr(A))) { out->choice = 0; return 1; }
    out->nnz_row = (int32_t *)zalloc((size_t)A->rows, sizeof(int32_t));
    out->col = (int32_t *)zalloc((size_t)A->rows * (size_t)K, sizeof(int32_t));
    out->val = (double *)zalloc((size_t)A->rows * (size_t)K, sizeof(double));
    for (int64_t i = 0; i < A->rows; ++i) {
        int64_t t = 0;
        for (int64_t p = A->row_ptr[i]; p < A->row_ptr[i + 1]; ++p, ++t) {
            out->col[i * K + t] = A->col[p]; out->val[i * K + t] = A->val[p];
        }
        out->nnz_row[i] = (int32_t)t;
    }
    return 0;
}

void ora_ell_mul_ell(const ora_ell *A, const ora_ell *B, ora_ell *C) {
    rowview a = {NULL, A->nnz_row, A->max_nnz_per_row, A->col, A->val};
    rowview b = {NULL, B->nnz_row, B->max_nnz_per_row, B->col, B->val};
    memset(C, 0, sizeof *C);
    C->rows = A->rows; C->cols = B->cols; C->choice = 1;
    int64_t *cnt = (int64_t *)zalloc((size_t)C->rows + 1, sizeof(int64_t));
    gustavson_count(&a, &b, A->rows, B->cols, cnt);
    int32_t K = 0; int64_t nnz = 0;
    C->nnz_row = (int32_t *)zalloc((size_t)C->rows, sizeof(int32_t));
    for (int64_t i = 0; i < C->rows; ++i) {
        C->nnz_row[i] = (int32_t)cnt[i]; nnz += cnt[i];
        if (cnt[i] > K) K = (int32_t)cnt[i];
    }
    C->nnz = nnz; C->max_nnz_per_row = K;
    C->col = (int32_t *)zalloc((size_t)C->rows * (size_t)K, sizeof(int32_t));
    C->val = (double *)zalloc((size_t)C->rows * (size_t)K, sizeof(double));
    int64_t *start = (int64_t *)zalloc((size_t)C->rows + 1, sizeof(int64_t));
    for (int64_t i = 0; i < C->rows; ++i) start[i] = i * (int64_t)K;
    gustavson_numeric(&a, &b, A->rows, B->cols, start, C->col, C->val, 0, 0);
    free(start); free(cnt);
}

/* ------------------------------------------------------------------ DIA
 * CSRtoDIA: a diagonal exists when any stored entry lies on it; offsets
 * ascend; val[i][slot] = A(i,j) — a later duplicate entry overwrites an
 * earlier one (dia:73-83).  diagonal_ind[off + rows - 1] = slot, 0 if absent. */
int ora_csr_to_dia(const ora_csr *A, ora_dia *out, double gate) {
    memset(out, 0, sizeof *out);
    int64_t span = A->rows + A->cols;      /* map index (rows - i) + j in [1, span) */
    int32_t *map = (int32_t *)zalloc((size_t)span, sizeof(int32_t));
    int32_t nd = 0;
    for (int64_t i = 0; i < A->rows; ++i)
        for (int64_t p = A->row_ptr[i]; p < A->row_ptr[i + 1]; ++p) {
            int64_t idx = (A->rows - i) + A->col[p];
            if (!map[idx]) { map[idx] = 1; ++nd; }
        }
    out->rows = A->rows; out->cols = A->cols; out->num_diagonals = nd; out->choice = 1;
    if (gate > 0 && !(ora_sizeof_dia(out) < gate * ora_sizeof_csr(A))) {
        out->choice = 0; free(map); return 1;
    }
    out->diagonal_ind = (int32_t *)zalloc((size_t)(A->rows + A->cols - 1), sizeof(int32_t));
    out->diagonal_offsets = (int32_t *)zalloc((size_t)nd, sizeof(int32_t));
    out->val = (double *)zalloc((size_t)A->rows * (size_t)nd, sizeof(double));
    for (int64_t idx = 0, d = 0; idx < span; ++idx)
        if (map[idx]) { map[idx] = (int32_t)d; out->diagonal_offsets[d] = (int32_t)(idx - A->rows); ++d; }
    for (int64_t i = 0; i < A->rows; ++i)
        for (int64_t p = A->row_ptr[i]; p < A->row_ptr[i + 1]; ++p) {
            int64_t slot = map[(A->rows - i) + A->col[p]];
            out->val[i * nd + slot] = A->val[p];
        }
    for (int64_t idx = 1; idx < span; ++idx) out->diagonal_ind[idx - 1] = map[idx];
    free(map);
    return 0;
}

/* DIA_mul_DIA: C diagonal off_a + off_b exists when some row i has both
 * i+off_a in [0, A.cols) and i+off_a+off_b in [0, B.cols) (dia:107-140, no
 * look at the stored values); C[i][slot] += A[i][ja] * B[i+off_a][kb] in
 * (ja, kb) loop order starting from the zero-filled array (dia:162-193). */
void ora_dia_mul_dia(const ora_dia *A, const ora_dia *B, ora_dia *C) {
    memset(C, 0, sizeof *C);
    int64_t span = A->rows + B->cols - 1;   /* out index = off + rows - 1 */
    char *flag = (char *)zalloc((size_t)span, 1);
    int32_t nd = 0;
    for (int32_t ja = 0; ja < A->num_diagonals; ++ja)
        for (int32_t kb = 0; kb < B->num_diagonals; ++kb) {
            int64_t oa = A->diagonal_offsets[ja], ob = B->diagonal_offsets[kb];
            /* rows i with 0 <= i < A.rows, 0 <= i+oa < A.cols, 0 <= i+oa+ob < B.cols */
            int64_t lo = 0, hi = A->rows;                 /* [lo, hi) */
            if (-oa > lo) lo = -oa;
            if (A->cols - oa < hi) hi = A->cols - oa;
            if (-oa - ob > lo) lo = -oa - ob;
            if (B->cols - oa - ob < hi) hi = B->cols - oa - ob;
            if (lo < hi) {
                int64_t idx = oa + ob + A->rows - 1;
                if (!flag[idx]) { flag[idx] = 1; ++nd; }
            }
        }
    C->rows = A->rows; C->cols = B->cols; C->num_diagonals = nd; C->choice = 1;
    C->diagonal_ind = (int32_t *)zalloc((size_t)span, sizeof(int32_t));
    C->diagonal_offsets = (int32_t *)zalloc((size_t)nd, sizeof(int32_t));
    C->val = (double *)zalloc((size_t)C->rows * (size_t)nd, sizeof(double));
    for (int64_t idx = 0, d = 0; idx < span; ++idx)
        if (flag[idx]) { C->diagonal_ind[idx] = (int32_t)d; C->diagonal_offsets[d] = (int32_t)(idx + 1 - C->rows); ++d; }
    for (int64_t i = 0; i < A->rows; ++i)
        for (int32_t ja = 0; ja < A->num_diagonals; ++ja) {
            int64_t acol = i + A->diagonal_offsets[ja];
            if (acol < 0 || acol >= A->cols) continue;
            double av = A->val[i * A->num_diagonals + ja];
            for (int32_t kb = 0; kb < B->num_diagonals; ++kb) {
                int64_t bcol = acol + B->diagonal_offsets[kb];
                if (bcol < 0 || bcol >= B->cols) continue;
                int64_t slot = C->diagonal_ind[bcol - i + C->rows - 1];
                double prod = av * B->val[acol * B->num_diagonals + kb];
                C->val[i * nd + slot] = C->val[i * nd + slot] + prod;
            }
        }
    free(flag);
}

/* ------------------------------------------------------------------ free */
void ora_free_csr(ora_csr *A) { free(A->row_ptr); free(A->col); free(A->val); memset(A, 0, sizeof *A); }
void ora_free_coo(ora_coo *A) { free(A->row_offset); free(A->row); free(A->col); free(A->val); memset(A, 0, sizeof *A); }
void ora_free_ell(ora_ell *A) { free(A->nnz_row); free(A->col); free(A->val); memset(A, 0, sizeof *A); }
void ora_free_dia(ora_dia *A) { free(A->diagonal_offsets); free(A->diagonal_ind); free(A->val); memset(A, 0, sizeof *A); }

/* ------------------------------------------------------------------ selector inputs
 * GetInfo1 (csr:257-287): param5/6 start from row 0's length (csr:263-264),
 * param7 = nnz/row, param8 = sum (n - param7)^2 / (row - 1), param9 =
 * sqrt(param8) / param7. */
static void ora_info1(const ora_csr *A, double *f) {
    int64_t m = A->rows;
    double p7 = (A->nnz + 0.0) / (double)m;
    int64_t p5 = m > 0 ? A->row_ptr[1] - A->row_ptr[0] : 0, p6 = p5;
    double p8 = 0.0;
    for (int64_t i = 0; i < m; ++i) {
        int64_t n = A->row_ptr[i + 1] - A->row_ptr[i];
        p5 = p5 > n ? p5 : n;
        p6 = p6 < n ? p6 : n;
        p8 += ((double)n - p7) * ((double)n - p7);
    }
    p8 = p8 / (double)(m - 1);
    f[0] = (double)A->rows; f[1] = (double)A->cols; f[2] = (double)A->nnz;
    f[3] = (A->nnz + 0.0) / ((double)A->rows * (double)A->cols);
    f[4] = (double)p5; f[5] = (double)p6; f[6] = p7; f[7] = p8; f[8] = sqrt(p8) / p7;
}

void ora_features(const ora_csr *A, const ora_csr *B, int32_t nfeatures, double *f) {
    const ora_csr *M[2] = {A, B};
    for (int i = 0; i < nfeatures; ++i) f[i] = 0.0;
    ora_info1(A, f);
    ora_info1(B, f + 9);
    if (nfeatures != 26) return;
    for (int t = 0; t < 2; ++t) {
        ora_dia d;
        ora_csr_to_dia(M[t], &d, 1e-300);   /* counts the diagonals, builds nothing */
        f[18 + 3 * t] = d.num_diagonals;
        f[19 + 3 * t] = (d.num_diagonals + 0.0) / (double)(M[t]->rows + M[t]->cols - 1);
        f[20 + 3 * t] = ((double)d.num_diagonals * (double)M[t]->rows) / ((double)M[t]->rows * (double)M[t]->cols);
        ora_free_dia(&d);
        ora_ell e;
        ora_csr_to_ell(M[t], &e, 1e-300);
        f[24 + t] = (M[t]->nnz + 0.0) / ((double)M[t]->rows * (double)e.max_nnz_per_row);
        ora_free_ell(&e);
    }
}

/* main.cpp:520-565: cells [i*128/row, + 128/row] x [j*128/col, + 128/col]
 * when a side is under 128, one cell when over, the identity at 128. */
void ora_density_image(const ora_csr *A, int64_t *img) {
    memset(img, 0, sizeof(int64_t) * 128 * 128);
    for (int64_t i = 0; i < A->rows; ++i)
        for (int64_t jj = A->row_ptr[i]; jj < A->row_ptr[i + 1]; ++jj) {
            int64_t old_i = i, old_j = A->col[jj];
            int64_t is = 0, ie = 0, js = 0, je = 0;
            if (A->rows > 128) { is = old_i * 128 / A->rows; ie = is; }
            else if (A->rows < 128) { is = old_i * 128 / A->rows; ie = is + 128 / A->rows; }
            else { is = old_i; ie = old_i; }
            if (A->cols > 128) { js = old_j * 128 / A->cols; je = js; }
            else if (A->cols < 128) { js = old_j * 128 / A->cols; je = js + 128 / A->cols; }
            else { js = old_j; je = old_j; }
            for (int64_t k = is; k <= ie; ++k)
                for (int64_t m = js; m <= je; ++m)
                    if (k < 128 && m < 128) img[k * 128 + m]++;
        }
}
