// report.hpp — shared pieces of the drop-in CLIs: timers, the reference's
// print_csr layout (csr/common_csr.h:213-233) and its per-algorithm report
// block (main.cpp:968-1000), plus the format selector.
#pragma once

#include "ias.h"

#include <sys/time.h>

#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

namespace cli {

inline double now_ms() {
    timeval t;
    gettimeofday(&t, nullptr);
    return t.tv_sec * 1000.0 + t.tv_usec / 1000.0;
}

inline void die(const char *what, ias_status s) {
    fprintf(stderr, "%s: %s (%s)\n", what, ias_status_string(s), ias_last_error());
    exit(1);
}

#define CLI_TRY(what, expr)                 \
    do {                                    \
        ias_status _s = (expr);             \
        if (_s != IAS_SUCCESS) cli::die(what, _s); \
    } while (0)

// print_csr: "row:%d col:%d nnz:%d", then row pointers, columns, "%.2lf," values.
inline void print_csr(const ias_csr &m) {
    ias_csr h{};
    const ias_csr *p = &m;
    if (m.memory == IAS_MEMORY_DEVICE) {
        CLI_TRY("copy", ias_csr_copy(&m, &h, IAS_MEMORY_HOST, 0));
        p = &h;
    }
    printf("row:%lld col:%lld nnz:%lld\n", (long long)p->rows, (long long)p->cols, (long long)p->nnz);
    for (int64_t i = 0; i <= p->rows; ++i) printf("%lld,", (long long)p->row_ptr[i]);
    printf("\n");
    for (int64_t i = 0; i < p->nnz; ++i) printf("%d,", p->col[i]);
    printf("\n");
    for (int64_t i = 0; i < p->nnz; ++i) printf("%.2lf,", p->val[i]);
    printf("\n");
    if (p == &h) ias_csr_free(&h);
}

struct AlgResult {
    double run_ms = 0, trans_ms = 0, mem = 0, sum = 0;
};

// The reference's timeout harness (main.cpp:43-93, 770-775): each algorithm
// runs on a pthread that is cancelled after time_scale (20) x the MKL time;
// an algorithm still running then reports run_time, memory_size and
// verified_sum as 0 (and so drops out of the speedup ranking).  A device
// kernel cannot be cancelled mid-flight, so the verdict is applied to the
// measured time after the run instead: same report, no cancellation.
// scale <= 0 or no MKL time disables it.
inline bool over_deadline(AlgResult &x, double mkl_ms, double scale) {
    if (scale <= 0 || mkl_ms <= 0 || !(x.run_ms > scale * mkl_ms)) return false;
    x.run_ms = x.mem = x.sum = 0.0;
    return true;
}

// main.cpp:968-1000 (trans_time printed from defined values; the reference
// indexes a 3-element array out of bounds there).
inline int report(const std::vector<AlgResult> &r, long long flops, bool speedup, bool trans) {
    std::vector<double> sp(r.size(), 0.0);
    double best = 0.0;
    int best_i = -1;
    for (size_t i = 0; i < r.size(); ++i) {
        sp[i] = r[i].run_ms == 0.0 ? 0.0 : r[0].run_ms / r[i].run_ms;
        if (best < sp[i]) {
            best = sp[i];
            best_i = (int)i;
        }
    }
    for (size_t i = 0; i < r.size(); ++i) {
        printf("------------------------------\n");
        printf("Algorithm %d:\n", (int)i + 1);
        printf("run_time: %lf\n", r[i].run_ms);
        if (trans) printf("trans_time: %lf\n", r[i].trans_ms);
        printf("memory_size: %lf\n", r[i].mem);
        printf("verified_sum: %lf\n", r[i].sum);
        printf("Gflops: %lf\n", r[i].run_ms == 0.0 ? 0.0 : (flops * 2.0) / (r[i].run_ms * 1000000));
        if (speedup) printf("Speedup: %lf\n", sp[i]);
    }
    printf("------------------------------\n");
    return best_i;
}

// Python's repr of a float (MatNet.py:27 prints the features as a list).
inline std::string py_float(double v) {
    char buf[64];
    auto r = std::to_chars(buf, buf + sizeof buf, v);
    std::string s(buf, r.ptr);
    if (s.find_first_of(".en") == std::string::npos) s += ".0";
    return s;
}

// The input-aware choice (main.cpp:651-704, GPU/main.cu:434-460):
// features + density images of A and B into MatNet with the reference's own
// weights (libias: ias_features, ias_density_image, ias_matnet_*).  Prints
// MatNet.py's "matrix features" and "Prediction cost" lines.  $IAS_MATNET
// overrides the weight set (a name or a blob path).  Returns the 0-based
// class, or `fallback` when the weights cannot be loaded.
inline int matnet_choose(const ias_csr &A, const ias_csr &B, int nfeatures, const char *weights, int fallback) {
    const char *env = getenv("IAS_MATNET");
    if (env && *env) weights = env;
    std::vector<double> f((size_t)nfeatures);
    std::vector<int64_t> ia(IAS_IMAGE_SIDE * IAS_IMAGE_SIDE), ib(IAS_IMAGE_SIDE * IAS_IMAGE_SIDE);
    CLI_TRY("features", ias_features(&A, &B, nfeatures, f.data()));
    CLI_TRY("image", ias_density_image(&A, ia.data()));
    CLI_TRY("image", ias_density_image(&B, ib.data()));
    printf("matrix features: [");
    for (int i = 0; i < nfeatures; ++i) printf("%s%s", i ? ", " : "", py_float(f[i]).c_str());
    printf("]\n");
    ias_matnet *net = nullptr;
    ias_status s = ias_matnet_load(weights, &net);
    if (s != IAS_SUCCESS) {
        printf("MatNet weights unavailable (%s): fallback choice\n", ias_last_error());
        return fallback;
    }
    int32_t nf = 0, chosen = fallback;
    ias_matnet_shape(net, &nf, nullptr);
    const double t = now_ms();
    if (nf == nfeatures) CLI_TRY("matnet", ias_matnet_predict(net, ia.data(), ib.data(), f.data(), nullptr, &chosen));
    printf("Prediction cost: %f seconds\n", (now_ms() - t) / 1000.0);
    ias_matnet_free(net);
    return chosen;
}

// Deterministic fallback when no weights are available: banded -> DIA,
// uniform rows -> ELL, else the CSR hash path (0-based into {MKL, CSR, DIA,
// ELL, COO}).
inline int select_format(bool dia_ok, double dia_fill, bool ell_ok, double ell_fill) {
    if (dia_ok && dia_fill >= 0.5) return 2;
    if (ell_ok && ell_fill >= 0.9) return 3;
    return 1;
}

}  // namespace cli
