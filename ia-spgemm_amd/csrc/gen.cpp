// gen.cpp — deterministic synthetic inputs for the benchmark configs
// (SURVEY.md §8d): R-MAT power-law, banded, uniform-ELL.  Counter-based
// (splitmix64 of (seed, item, level)), so every thread count and machine
// produces the same matrix.  Values depend only on (seed, row, col), so
// duplicate R-MAT edges collapse to one entry with a well-defined value.
#include "ias.h"
#include "ias_internal.hpp"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

using namespace ias;

namespace {

inline uint64_t mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

inline uint64_t h2(uint64_t seed, uint64_t a, uint64_t b) {
    return mix(mix(seed ^ (a * 0xD1B54A32D192ED03ull)) + b);
}

inline double entry_value(uint64_t seed, int64_t r, int64_t c, int mode) {
    const uint64_t h = h2(seed ^ 0x5BD1E9955BD1E995ull, (uint64_t)r, (uint64_t)c);
    if (mode == 1) return (double)(1 + (int)(h % 9u));
    return (double)(h >> 11) * (2.0 / 9007199254740992.0) - 1.0;   // U(-1,1)
}

inline uint64_t thresh(double p) {
    if (p <= 0) return 0;
    if (p >= 1) return ~0ull;
    return (uint64_t)(p * 18446744073709551616.0);
}

// rows' column lists (sorted, duplicates removed) -> CSR with hashed values
ias_status finish(int64_t rows, int64_t cols, std::vector<int64_t> &ptr, std::vector<int32_t> &cidx,
                  uint64_t seed, int mode, ias_csr *out) {
    // sort + unique per row, in place
    std::vector<int64_t> cnt((size_t)rows, 0);
#pragma omp parallel for schedule(dynamic, 256)
    for (int64_t i = 0; i < rows; ++i) {
        int32_t *b = cidx.data() + ptr[(size_t)i], *e = cidx.data() + ptr[(size_t)i + 1];
        std::sort(b, e);
        cnt[(size_t)i] = std::unique(b, e) - b;
    }
    int64_t nnz = 0;
    for (int64_t i = 0; i < rows; ++i) nnz += cnt[(size_t)i];
    ias_csr M{};
    IAS_TRY(ias_csr_alloc(&M, rows, cols, nnz, IAS_MEMORY_HOST, 0));
    M.row_ptr[0] = 0;
    for (int64_t i = 0; i < rows; ++i) M.row_ptr[i + 1] = M.row_ptr[i] + cnt[(size_t)i];
#pragma omp parallel for schedule(dynamic, 256)
    for (int64_t i = 0; i < rows; ++i) {
        const int32_t *src = cidx.data() + ptr[(size_t)i];
        for (int64_t k = 0; k < cnt[(size_t)i]; ++k) {
            const int64_t at = M.row_ptr[i] + k;
            M.col[at] = src[k];
            M.val[at] = entry_value(seed, i, src[k], mode);
        }
    }
    *out = M;
    return IAS_SUCCESS;
}

}  // namespace

extern "C" ias_status ias_gen_rmat(int32_t scale, double edge_factor, double a, double b, double c,
                                   uint64_t seed, int32_t value_mode, ias_csr *out) {
    if (!out || scale < 0 || scale > 30 || edge_factor < 0 || a < 0 || b < 0 || c < 0 ||
        a + b + c > 1.0)
        return IAS_ERROR_INVALID_ARGUMENT;
    const int64_t n = 1ll << scale;
    const int64_t E = (int64_t)std::llround(edge_factor * (double)n);
    const uint64_t ta = thresh(a), tab = thresh(a + b), tabc = thresh(a + b + c);
    auto edge = [&](int64_t e, int64_t &r, int64_t &cc) {
        const uint64_t base = mix(seed ^ ((uint64_t)e * 0xD1B54A32D192ED03ull));
        r = 0;
        cc = 0;
        for (int l = 0; l < scale; ++l) {
            const uint64_t u = mix(base + (uint64_t)l);
            const int q = u < ta ? 0 : u < tab ? 1 : u < tabc ? 2 : 3;
            r = (r << 1) | (q >> 1);
            cc = (cc << 1) | (q & 1);
        }
    };
    std::vector<std::atomic<int64_t>> cnt((size_t)n);
    for (auto &x : cnt) x.store(0, std::memory_order_relaxed);
#pragma omp parallel for schedule(static)
    for (int64_t e = 0; e < E; ++e) {
        int64_t r, cc;
        edge(e, r, cc);
        cnt[(size_t)r].fetch_add(1, std::memory_order_relaxed);
    }
    std::vector<int64_t> ptr((size_t)n + 1, 0);
    for (int64_t i = 0; i < n; ++i) ptr[(size_t)i + 1] = ptr[(size_t)i] + cnt[(size_t)i].load();
    for (auto &x : cnt) x.store(0, std::memory_order_relaxed);
    std::vector<int32_t> cidx((size_t)E);
#pragma omp parallel for schedule(static)
    for (int64_t e = 0; e < E; ++e) {
        int64_t r, cc;
        edge(e, r, cc);
        const int64_t at = ptr[(size_t)r] + cnt[(size_t)r].fetch_add(1, std::memory_order_relaxed);
        cidx[(size_t)at] = (int32_t)cc;
    }
    return finish(n, n, ptr, cidx, seed, value_mode, out);
}

extern "C" ias_status ias_gen_band(int64_t n, int32_t half_width, uint64_t seed, int32_t value_mode,
                                   ias_csr *out) {
    if (!out || n < 0 || n > INT32_MAX || half_width < 0) return IAS_ERROR_INVALID_ARGUMENT;
    std::vector<int64_t> ptr((size_t)n + 1, 0);
    for (int64_t i = 0; i < n; ++i) {
        const int64_t lo = std::max<int64_t>(0, i - half_width), hi = std::min<int64_t>(n - 1, i + half_width);
        ptr[(size_t)i + 1] = ptr[(size_t)i] + (hi - lo + 1);
    }
    std::vector<int32_t> cidx((size_t)ptr[(size_t)n]);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        const int64_t lo = std::max<int64_t>(0, i - half_width), hi = std::min<int64_t>(n - 1, i + half_width);
        for (int64_t j = lo; j <= hi; ++j) cidx[(size_t)(ptr[(size_t)i] + j - lo)] = (int32_t)j;
    }
    return finish(n, n, ptr, cidx, seed, value_mode, out);
}

extern "C" ias_status ias_gen_ell(int64_t n, int32_t per_row, uint64_t seed, int32_t value_mode,
                                  ias_csr *out) {
    if (!out || n < 0 || n > INT32_MAX || per_row < 0 || per_row > n) return IAS_ERROR_INVALID_ARGUMENT;
    std::vector<int64_t> ptr((size_t)n + 1, 0);
    for (int64_t i = 0; i < n; ++i) ptr[(size_t)i + 1] = ptr[(size_t)i] + per_row;
    std::vector<int32_t> cidx((size_t)ptr[(size_t)n]);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        int32_t *row = cidx.data() + ptr[(size_t)i];
        int got = 0;
        for (uint64_t t = 0; got < per_row; ++t) {     // distinct columns by rejection
            const int32_t c = (int32_t)(h2(seed, (uint64_t)i, t) % (uint64_t)n);
            bool dup = false;
            for (int k = 0; k < got; ++k) dup |= row[k] == c;
            if (!dup) row[got++] = c;
        }
    }
    return finish(n, n, ptr, cidx, seed, value_mode, out);
}
