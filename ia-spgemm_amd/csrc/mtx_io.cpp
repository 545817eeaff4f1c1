// mtx_io.cpp — Matrix-Market reader/writer with the reference's semantics
// (IA-SPGEMM-CPU_release/main.cpp:143-458, mmio.h:254-367 and 445-486).
//
//   * banner: "%%MatrixMarket matrix coordinate <real|integer|pattern>
//     <general|symmetric|hermitian|skew-symmetric>" (case-insensitive tokens
//     after the banner word, as mm_read_banner lower-cases them); complex is
//     rejected (main.cpp:164-168); dense "array" files are rejected (the
//     reference would misparse them as coordinate entries);
//   * size line: the first line not starting with '%' (mm_read_mtx_crd_size);
//   * entries: "i j v" / "i j v(int)" / "i j" -> 0-based, pattern -> 1.0;
//   * symmetric and hermitian files also get the mirrored (j,i) entry with the
//     same value when i != j; skew-symmetric is NOT mirrored (main.cpp:317-332
//     tests mm_is_symmetric || mm_is_hermitian only);
//   * CSR assembly is a stable counting sort by row in file order: columns stay
//     unsorted and duplicate (i,j) entries are kept (main.cpp:334-447).
// Parsing works on the whole file in memory (strtoll/strtod), not fscanf per
// entry, so a 200M-entry file reads at disk speed.
#include "ias.h"
#include "ias_internal.hpp"

#include <cctype>
#include <cerrno>
#include <string>
#include <vector>

using namespace ias;

namespace {

struct Parsed {
    ias_mtx_info info{};
    std::vector<int64_t> r, c;
    std::vector<double> v;
};

ias_status slurp(const char *path, std::string &buf) {
    FILE *f = fopen(path, "rb");
    if (!f) {
        set_last_error("cannot open %s: %s", path, strerror(errno));
        return IAS_ERROR_IO;
    }
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    if (n < 0) {
        fclose(f);
        return IAS_ERROR_IO;
    }
    buf.resize((size_t)n);
    size_t got = n ? fread(&buf[0], 1, (size_t)n, f) : 0;
    fclose(f);
    if (got != (size_t)n) return IAS_ERROR_IO;
    return IAS_SUCCESS;
}

std::string lower(std::string s) {
    for (auto &ch : s) ch = (char)tolower((unsigned char)ch);
    return s;
}

ias_status parse(const char *path, Parsed &P) {
    std::string buf;
    IAS_TRY(slurp(path, buf));
    const char *p = buf.c_str();
    const char *end = p + buf.size();
    // banner line
    const char *eol = (const char *)memchr(p, '\n', (size_t)(end - p));
    if (!eol) eol = end;
    std::string line(p, eol);
    char t0[64] = {0}, t1[64] = {0}, t2[64] = {0}, t3[64] = {0}, t4[64] = {0};
    if (sscanf(line.c_str(), "%63s %63s %63s %63s %63s", t0, t1, t2, t3, t4) != 5) {
        set_last_error("%s: could not process Matrix Market banner", path);
        return IAS_ERROR_FORMAT;
    }
    if (strncmp(t0, "%%MatrixMarket", 14) != 0 || lower(t1) != "matrix") {
        set_last_error("%s: not a Matrix Market matrix", path);
        return IAS_ERROR_FORMAT;
    }
    const std::string fmt = lower(t2), type = lower(t3), sym = lower(t4);
    if (fmt != "coordinate") {
        set_last_error("%s: only coordinate format is supported", path);
        return fmt == "array" ? IAS_ERROR_UNSUPPORTED : IAS_ERROR_FORMAT;
    }
    if (type == "complex") {
        set_last_error("%s: data type 'COMPLEX' is not supported", path);
        return IAS_ERROR_UNSUPPORTED;
    }
    ias_mtx_info &I = P.info;
    I.is_real = type == "real";
    I.is_integer = type == "integer";
    I.is_pattern = type == "pattern";
    if (!I.is_real && !I.is_integer && !I.is_pattern) return IAS_ERROR_FORMAT;
    if (sym != "general" && sym != "symmetric" && sym != "hermitian" && sym != "skew-symmetric")
        return IAS_ERROR_FORMAT;
    I.is_symmetric = (sym == "symmetric" || sym == "hermitian");
    p = eol < end ? eol + 1 : end;
    // skip comment lines
    while (p < end && *p == '%') {
        const char *e2 = (const char *)memchr(p, '\n', (size_t)(end - p));
        p = e2 ? e2 + 1 : end;
    }
    char *q;
    errno = 0;
    long long m = strtoll(p, &q, 10);
    if (q == p) return IAS_ERROR_FORMAT;
    p = q;
    long long n = strtoll(p, &q, 10);
    if (q == p) return IAS_ERROR_FORMAT;
    p = q;
    long long nz = strtoll(p, &q, 10);
    if (q == p) return IAS_ERROR_FORMAT;
    p = q;
    if (m < 0 || n < 0 || nz < 0) return IAS_ERROR_FORMAT;
    if (m > INT32_MAX || n > INT32_MAX) return IAS_ERROR_OVERFLOW;
    I.rows = m;
    I.cols = n;
    I.nnz_file = nz;
    P.r.resize((size_t)nz);
    P.c.resize((size_t)nz);
    P.v.resize((size_t)nz);
    for (long long e = 0; e < nz; ++e) {
        long long i = strtoll(p, &q, 10);
        if (q == p) {
            set_last_error("%s: premature end of entries at %lld of %lld", path, e, nz);
            return IAS_ERROR_FORMAT;
        }
        p = q;
        long long j = strtoll(p, &q, 10);
        if (q == p) return IAS_ERROR_FORMAT;
        p = q;
        double v = 1.0;
        if (I.is_real) {
            v = strtod(p, &q);
            if (q == p) return IAS_ERROR_FORMAT;
            p = q;
        } else if (I.is_integer) {
            long long iv = strtoll(p, &q, 10);
            if (q == p) return IAS_ERROR_FORMAT;
            p = q;
            v = (double)(int)iv;   // "%d" then fval = ival (main.cpp:223-224)
        }
        if (i < 1 || i > m || j < 1 || j > n) {
            set_last_error("%s: entry %lld (%lld,%lld) outside %lldx%lld", path, e, i, j, m, n);
            return IAS_ERROR_FORMAT;
        }
        P.r[(size_t)e] = i - 1;
        P.c[(size_t)e] = j - 1;
        P.v[(size_t)e] = v;
    }
    return IAS_SUCCESS;
}

// Stable counting sort by row in file order (+ mirrored entries).
ias_status assemble(const Parsed &P, int64_t rows, ias_csr *A) {
    const bool sym = P.info.is_symmetric != 0;
    const size_t nz = P.r.size();
    std::vector<int64_t> cnt((size_t)rows + 1, 0);
    for (size_t e = 0; e < nz; ++e) {
        if (P.r[e] >= rows) return IAS_ERROR_DIMENSION_MISMATCH;
        cnt[(size_t)P.r[e]]++;
        if (sym && P.r[e] != P.c[e]) {
            if (P.c[e] >= rows) return IAS_ERROR_DIMENSION_MISMATCH;
            cnt[(size_t)P.c[e]]++;
        }
    }
    int64_t total = 0;
    for (int64_t i = 0; i < rows; ++i) total += cnt[(size_t)i];
    ias_csr M{};
    IAS_TRY(ias_csr_alloc(&M, rows, P.info.cols, total, IAS_MEMORY_HOST, 0));
    M.row_ptr[0] = 0;
    for (int64_t i = 0; i < rows; ++i) M.row_ptr[i + 1] = M.row_ptr[i] + cnt[(size_t)i];
    std::fill(cnt.begin(), cnt.end(), 0);
    for (size_t e = 0; e < nz; ++e) {
        const int64_t r = P.r[e], c = P.c[e];
        int64_t at = M.row_ptr[r] + cnt[(size_t)r]++;
        M.col[at] = (int32_t)c;
        M.val[at] = P.v[e];
        if (sym && r != c) {
            at = M.row_ptr[c] + cnt[(size_t)c]++;
            M.col[at] = (int32_t)r;
            M.val[at] = P.v[e];
        }
    }
    *A = M;
    return IAS_SUCCESS;
}

}  // namespace

extern "C" ias_status ias_mtx_read(const char *path, ias_csr *A, ias_mtx_info *info) {
    if (!path || !A) return IAS_ERROR_INVALID_ARGUMENT;
    Parsed P;
    IAS_TRY(parse(path, P));
    IAS_TRY(assemble(P, P.info.rows, A));
    if (info) *info = P.info;
    return IAS_SUCCESS;
}

extern "C" ias_status ias_mtx_read_pair(const char *path_a, const char *path_b, ias_csr *A,
                                        ias_csr *B, ias_mtx_info *info_a, ias_mtx_info *info_b) {
    if (!path_a || !path_b || !A || !B) return IAS_ERROR_INVALID_ARGUMENT;
    Parsed PA, PB;
    IAS_TRY(parse(path_a, PA));
    IAS_TRY(parse(path_b, PB));
    ias_csr a{}, b{};
    IAS_TRY(assemble(PA, PA.info.rows, &a));
    // B.row = A.col (main.cpp:482); B's own row count only printed.
    ias_status s = assemble(PB, PA.info.cols, &b);
    if (s != IAS_SUCCESS) {
        ias_csr_free(&a);
        return s;
    }
    *A = a;
    *B = b;
    if (info_a) *info_a = PA.info;
    if (info_b) *info_b = PB.info;
    return IAS_SUCCESS;
}

extern "C" ias_status ias_mtx_write(const char *path, const ias_csr *A) {
    if (!path || !A) return IAS_ERROR_INVALID_ARGUMENT;
    ias_csr H{};
    const ias_csr *M = A;
    if (A->memory == IAS_MEMORY_DEVICE) {
        IAS_TRY(ias_csr_copy(A, &H, IAS_MEMORY_HOST, 0));
        M = &H;
    }
    FILE *f = strcmp(path, "stdout") == 0 ? stdout : fopen(path, "w");
    if (!f) {
        if (M == &H) ias_csr_free(&H);
        return IAS_ERROR_IO;
    }
    fprintf(f, "%%%%MatrixMarket matrix coordinate real general\n");
    fprintf(f, "%lld %lld %lld\n", (long long)M->rows, (long long)M->cols, (long long)M->nnz);
    for (int64_t i = 0; i < M->rows; ++i)
        for (int64_t p = M->row_ptr[i]; p < M->row_ptr[i + 1]; ++p)
            fprintf(f, "%lld %d %20.16g\n", (long long)(i + 1), M->col[p] + 1, M->val[p]);
    if (f != stdout) fclose(f);
    if (M == &H) ias_csr_free(&H);
    return IAS_SUCCESS;
}
