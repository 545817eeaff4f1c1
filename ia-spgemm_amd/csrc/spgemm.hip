// spgemm.hip — kernels and host engine of the row-wise SpGEMM hot path
// (replaces CSR_MUL_CSR / COO_MUL_COO / ELL_MUL_ELL of the reference and the
// CUSP / cuSPARSE calls of GPU/main.cu:467-523).  See spgemm_kernels.hpp for
// the per-row algorithm and DESIGN.md for the pipeline and its roofline.
#include "spgemm_kernels.hpp"
#include "spgemm_engine.hpp"
#include "ias_internal.hpp"

#include <algorithm>
#include <vector>

namespace ias {
namespace dev {

// ---------------------------------------------------------------- analysis
// Products per row (GetFlop per row).  A block owns 256 consecutive rows and
// spreads their A entries over its threads (a hub row does not serialise on
// one lane).  Also accumulates total flops and the max products per row.
constexpr int AN_BLOCK = 256;

__global__ __launch_bounds__(AN_BLOCK) void k_row_products(Rows A, Rows B, int64_t rows,
                                                           int32_t *prod,
                                                           unsigned long long *flops,
                                                           int32_t *max_prod) {
    __shared__ int64_t start[AN_BLOCK];
    __shared__ int64_t pref[AN_BLOCK + 1];
    __shared__ unsigned long long acc[AN_BLOCK];
    __shared__ int scratch[8];
    const int t = threadIdx.x;
    const int64_t r0 = (int64_t)blockIdx.x * AN_BLOCK;
    const int64_t r = r0 + t;
    int64_t s = 0;
    int32_t n = 0;
    if (r < rows) A.row(r, s, n);
    start[t] = s;
    acc[t] = 0;
    // block exclusive scan of n (int64 to be safe)
    {
        int tot;
        const int ex = Team<AN_BLOCK>::excl_sum(n, tot, scratch);
        pref[t] = ex;
        if (t == 0) pref[AN_BLOCK] = tot;
    }
    __syncthreads();
    const int64_t E = pref[AN_BLOCK];
    for (int64_t e = t; e < E; e += AN_BLOCK) {
        // row of entry e: last k with pref[k] <= e
        int lo = 0, hi = AN_BLOCK;
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (pref[mid] <= e) lo = mid;
            else hi = mid;
        }
        const int32_t j = A.col[start[lo] + (e - pref[lo])];
        int64_t bs;
        int32_t bn;
        B.row(j, bs, bn);
        atomicAdd(&acc[lo], (unsigned long long)bn);
    }
    __syncthreads();
    unsigned long long mine = acc[t];
    if (r < rows) prod[r] = (int32_t)min(mine, (unsigned long long)INT32_MAX);
    // block reductions
    __shared__ unsigned long long red_sum[AN_BLOCK / WAVE];
    __shared__ int red_max[AN_BLOCK / WAVE];
    unsigned long long sm = (r < rows) ? mine : 0ull;
    int mx = (r < rows) ? (int)min(mine, (unsigned long long)INT32_MAX) : 0;
    for (int d = WAVE / 2; d > 0; d >>= 1) {
        sm += __shfl_down(sm, d);
        mx = max(mx, __shfl_down(mx, d));
    }
    if ((t & (WAVE - 1)) == 0) {
        red_sum[t / WAVE] = sm;
        red_max[t / WAVE] = mx;
    }
    __syncthreads();
    if (t == 0) {
        unsigned long long S = 0;
        int MX = 0;
        for (int i = 0; i < AN_BLOCK / WAVE; ++i) {
            S += red_sum[i];
            MX = max(MX, red_max[i]);
        }
        atomicAdd(flops, S);
        atomicMax(max_prod, MX);
    }
}

// ---------------------------------------------------------------- binning
constexpr int BIN_BLOCK = 256;

// key[i] -> bin; bin 0 = key 0 (no list, zero_out[i] = 0 when given);
// bins 1..nbins-2 = LDS bins by upper bound; bin nbins-1 = global table,
// whose rows also get a workspace offset of nextpow2(ceil(key*3/2)) slots.
__global__ __launch_bounds__(BIN_BLOCK) void k_bin_rows(const int32_t *key, int64_t rows,
                                                        BinSpec spec, int32_t *lists,
                                                        int32_t *counts,
                                                        unsigned long long *ws_slots,
                                                        int64_t *ws_off, int32_t *zero_out) {
    __shared__ int hist[MAX_BINS];
    __shared__ int base[MAX_BINS];
    const int t = threadIdx.x;
    if (t < MAX_BINS) hist[t] = 0;
    __syncthreads();
    const int64_t r = (int64_t)blockIdx.x * BIN_BLOCK + t;
    int b = -1, local = 0;
    int32_t k = 0;
    if (r < rows) {
        k = key[r];
        if (k <= 0) {
            b = 0;
            if (zero_out) zero_out[r] = 0;
        } else {
            b = spec.nbins - 1;
            for (int i = 1; i < spec.nbins - 1; ++i)
                if (k <= spec.upper[i]) { b = i; break; }
            local = atomicAdd(&hist[b], 1);
        }
    }
    __syncthreads();
    if (t < spec.nbins && t > 0 && hist[t] > 0) base[t] = atomicAdd(&counts[t], hist[t]);
    __syncthreads();
    if (b > 0) {
        const int pos = base[b] + local;
        lists[(int64_t)b * rows + pos] = (int32_t)r;
        if (b == spec.nbins - 1) {
            const unsigned long long need = (unsigned long long)k + ((unsigned long long)k + 1) / 2;
            unsigned long long S = 1;
            while (S < need) S <<= 1;
            ws_off[pos] = (int64_t)atomicAdd(ws_slots, S);
        }
    }
}

// ---------------------------------------------------------------- per-bin kernels
template <int TEAM, int LOG2S, int TPW>
__global__ __launch_bounds__(TEAM *TPW) void k_symbolic_lds(Rows A, Rows B, const int32_t *list,
                                                             int32_t count, int32_t *nnz_row) {
    static_assert(TEAM <= 64 || TPW == 1, "multi-wave teams own their workgroup");
    __shared__ int32_t keys[TPW][1 << LOG2S];
    __shared__ Seg<TEAM, false> seg[TPW];
    __shared__ int scratch[TPW][16];
    const int team = (TPW == 1) ? 0 : (int)(threadIdx.x / TEAM);
    const int64_t idx = (int64_t)blockIdx.x * TPW + team;
    const int64_t row = idx < count ? list[idx] : -1;
    KeyTable tb{keys[team], (uint32_t)LOG2S};
    const int32_t n = symbolic_row<TEAM>(A, B, row, tb, seg[team], scratch[team]);
    if (row >= 0 && Team<TEAM>::lane() == 0) nnz_row[row] = n;
}

template <int TEAM>
__global__ __launch_bounds__(TEAM) void k_symbolic_global(Rows A, Rows B, const int32_t *list,
                                                          const int64_t *ws_off,
                                                          const int32_t *prod, int32_t count,
                                                          int32_t *ws, int32_t *nnz_row) {
    __shared__ Seg<TEAM, false> seg;
    __shared__ int scratch[16];
    const int64_t idx = blockIdx.x;
    if (idx >= count) return;
    const int64_t row = list[idx];
    const unsigned long long need =
        (unsigned long long)prod[row] + ((unsigned long long)prod[row] + 1) / 2;
    uint32_t l2 = 0;
    while ((1ull << l2) < need) ++l2;
    KeyTable tb{ws + ws_off[idx], l2};
    const int32_t n = symbolic_row<TEAM>(A, B, row, tb, seg, scratch);
    if (threadIdx.x == 0) nnz_row[row] = n;
}

template <int TEAM, int LOG2S, int TPW>
__global__ __launch_bounds__(TEAM *TPW) void k_numeric_lds(Rows A, Rows B, const int32_t *list,
                                                            int32_t count, Out out) {
    static_assert(TEAM <= 64 || TPW == 1, "multi-wave teams own their workgroup");
    __shared__ int32_t keys[TPW][1 << LOG2S];
    __shared__ uint32_t meta[TPW][1 << LOG2S];
    __shared__ double vals[TPW][1 << LOG2S];
    __shared__ Seg<TEAM, true> seg[TPW];
    __shared__ int scratch[TPW][16];
    const int team = (TPW == 1) ? 0 : (int)(threadIdx.x / TEAM);
    const int64_t idx = (int64_t)blockIdx.x * TPW + team;
    const int64_t row = idx < count ? list[idx] : -1;
    NumTable<false> tb{keys[team], meta[team], vals[team], (uint32_t)LOG2S};
    numeric_row<TEAM, false>(A, B, row, tb, seg[team], scratch[team], out);
}

template <int TEAM>
__global__ __launch_bounds__(TEAM) void k_numeric_global(Rows A, Rows B, const int32_t *list,
                                                         const int64_t *ws_off,
                                                         const int32_t *nnz_row, int32_t count,
                                                         char *ws, Out out) {
    __shared__ Seg<TEAM, true> seg;
    __shared__ int scratch[16];
    const int64_t idx = blockIdx.x;
    if (idx >= count) return;
    const int64_t row = list[idx];
    const unsigned long long k = (unsigned long long)nnz_row[row];
    const unsigned long long need = k + (k + 1) / 2;
    uint32_t l2 = 0;
    while ((1ull << l2) < need) ++l2;
    // slot layout inside the row's region of 16-byte words: [keys | meta | vals]
    // region = S * 16 bytes: keys S*4, pad to 8, meta S*8 ... kept simple:
    const uint64_t S = 1ull << l2;
    char *base = ws + (uint64_t)ws_off[idx] * 20ull;
    NumTable<true> tb{(int32_t *)base, (unsigned long long *)(base + S * 4ull),
                      (double *)(base + S * 12ull), l2};
    numeric_row<TEAM, true>(A, B, row, tb, seg, scratch, out);
}

// ---------------------------------------------------------------- scan
constexpr int SCAN_BLOCK = 256;
constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;

__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_reduce(const int32_t *in, int64_t n,
                                                            int64_t *partial, int32_t *max_out) {
    const int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
    int64_t s = 0;
    int mx = 0;
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        const int64_t k = base + (int64_t)i * SCAN_BLOCK + threadIdx.x;
        if (k < n) {
            s += in[k];
            mx = max(mx, in[k]);
        }
    }
    for (int d = WAVE / 2; d > 0; d >>= 1) {
        s += __shfl_down(s, d);
        mx = max(mx, __shfl_down(mx, d));
    }
    __shared__ int64_t ws[SCAN_BLOCK / WAVE];
    __shared__ int wm[SCAN_BLOCK / WAVE];
    if ((threadIdx.x & (WAVE - 1)) == 0) {
        ws[threadIdx.x / WAVE] = s;
        wm[threadIdx.x / WAVE] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t S = 0;
        int M = 0;
        for (int i = 0; i < SCAN_BLOCK / WAVE; ++i) {
            S += ws[i];
            M = max(M, wm[i]);
        }
        partial[blockIdx.x] = S;
        if (max_out) atomicMax(max_out, M);
    }
}

// single block: exclusive scan of partial[0..nb) in place; total -> partial[nb]
__global__ __launch_bounds__(1024) void k_scan_partials(int64_t *partial, int64_t nb) {
    __shared__ int64_t wsum[16];
    __shared__ int64_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int64_t b0 = 0; b0 < nb; b0 += 1024) {
        const int64_t k = b0 + threadIdx.x;
        const int64_t v = k < nb ? partial[k] : 0;
        int64_t x = v;
        const int l = threadIdx.x & (WAVE - 1);
        for (int d = 1; d < WAVE; d <<= 1) {
            const int64_t t = __shfl_up(x, d);
            if (l >= d) x += t;
        }
        if (l == WAVE - 1) wsum[threadIdx.x / WAVE] = x;
        __syncthreads();
        int64_t before = 0, tot = 0;
        for (int i = 0; i < 16; ++i) {
            before += (i < (int)(threadIdx.x / WAVE)) ? wsum[i] : 0;
            tot += wsum[i];
        }
        const int64_t c = carry;
        if (k < nb) partial[k] = c + before + x - v;
        __syncthreads();
        if (threadIdx.x == 0) carry = c + tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[nb] = carry;
}

__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_apply(const int32_t *in, int64_t n,
                                                           const int64_t *partial,
                                                           int64_t *out) {
    __shared__ int64_t wsum[SCAN_BLOCK / WAVE];
    const int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
    int64_t carry = partial[blockIdx.x];
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        const int64_t k = base + (int64_t)i * SCAN_BLOCK + threadIdx.x;
        const int64_t v = k < n ? in[k] : 0;
        int64_t x = v;
        const int l = threadIdx.x & (WAVE - 1);
        for (int d = 1; d < WAVE; d <<= 1) {
            const int64_t t = __shfl_up(x, d);
            if (l >= d) x += t;
        }
        if (l == WAVE - 1) wsum[threadIdx.x / WAVE] = x;
        __syncthreads();
        int64_t before = 0, tot = 0;
        for (int w = 0; w < SCAN_BLOCK / WAVE; ++w) {
            before += (w < (int)(threadIdx.x / WAVE)) ? wsum[w] : 0;
            tot += wsum[w];
        }
        if (k < n) out[k] = carry + before + x - v;
        __syncthreads();
        carry += tot;
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) out[n] = partial[gridDim.x];
}

__global__ void k_shift(int64_t *p, int64_t n, int64_t off) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] += off;
}

__global__ void k_fill_rows(const int64_t *ptr, int64_t rows, int32_t *row_idx) {
    // one wave per row: row index of every entry (COO output)
    const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
    if (r >= rows) return;
    for (int64_t e = ptr[r] + (threadIdx.x & (WAVE - 1)); e < ptr[r + 1]; e += WAVE)
        row_idx[e] = (int32_t)r;
}


// ---------------------------------------------------------------- row sort
// IAS_ORDER_SORTED: bitonic sort of (col, val) per row, in LDS up to 8192
// entries, in a per-row global workspace beyond.  Columns of a row are
// distinct, so the order is unique.
template <int TEAM>
__device__ __forceinline__ void bitonic(int32_t *sk, double *sv, uint32_t cap) {
    const int lane = Team<TEAM>::lane();
    for (uint32_t k = 2; k <= cap; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = lane; i < cap; i += TEAM) {
                const uint32_t ixj = i ^ j;
                if (ixj > i) {
                    const bool up = (i & k) == 0;
                    const int32_t a = sk[i], b = sk[ixj];
                    if ((a > b) == up) {
                        sk[i] = b;
                        sk[ixj] = a;
                        const double t = sv[i];
                        sv[i] = sv[ixj];
                        sv[ixj] = t;
                    }
                }
            }
            Team<TEAM>::sync();
        }
    }
}

__device__ __forceinline__ void sort_row_span(const int64_t *ptr, const int32_t *len, int64_t stride,
                                              int64_t row, int64_t &o, int32_t &n) {
    if (ptr) {
        o = ptr[row];
        n = (int32_t)(ptr[row + 1] - o);
    } else {
        o = row * stride;
        n = len[row];
    }
}

template <int TEAM, int CAP, int TPW>
__global__ __launch_bounds__(TEAM *TPW) void k_sort_lds(const int32_t *list, int32_t count,
                                                         const int64_t *ptr, const int32_t *len,
                                                         int64_t stride, int32_t *col, double *val) {
    static_assert(TEAM <= 64 || TPW == 1, "multi-wave teams own their workgroup");
    __shared__ int32_t sk[TPW][CAP];
    __shared__ double sv[TPW][CAP];
    const int team = (TPW == 1) ? 0 : (int)(threadIdx.x / TEAM);
    const int lane = Team<TEAM>::lane();
    const int64_t idx = (int64_t)blockIdx.x * TPW + team;
    const int64_t row = idx < count ? list[idx] : -1;
    int64_t o = 0;
    int32_t n = 0;
    if (row >= 0) sort_row_span(ptr, len, stride, row, o, n);
    for (int e = lane; e < CAP; e += TEAM) {
        sk[team][e] = e < n ? col[o + e] : INT32_MAX;
        sv[team][e] = e < n ? val[o + e] : 0.0;
    }
    Team<TEAM>::sync();
    bitonic<TEAM>(sk[team], sv[team], CAP);
    for (int e = lane; e < n; e += TEAM) {
        col[o + e] = sk[team][e];
        val[o + e] = sv[team][e];
    }
}

__global__ __launch_bounds__(1024) void k_sort_global(const int32_t *list, int32_t count,
                                                      const int64_t *ws_off, const int64_t *ptr,
                                                      const int32_t *len, int64_t stride,
                                                      int32_t *col, double *val, char *ws) {
    const int64_t idx = blockIdx.x;
    if (idx >= count) return;
    const int64_t row = list[idx];
    int64_t o;
    int32_t n;
    sort_row_span(ptr, len, stride, row, o, n);
    uint32_t cap = 1;
    while (cap < (uint32_t)n) cap <<= 1;
    double *sv = (double *)(ws + (uint64_t)ws_off[idx] * 12ull);
    int32_t *sk = (int32_t *)(sv + cap);
    for (uint32_t e = threadIdx.x; e < cap; e += 1024) {
        sk[e] = e < (uint32_t)n ? col[o + e] : INT32_MAX;
        sv[e] = e < (uint32_t)n ? val[o + e] : 0.0;
    }
    __syncthreads();
    bitonic<1024>(sk, sv, cap);
    for (uint32_t e = threadIdx.x; e < (uint32_t)n; e += 1024) {
        col[o + e] = sk[e];
        val[o + e] = sv[e];
    }
}

__global__ void k_row_len(const int64_t *ptr, int64_t rows, int32_t *len) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < rows) len[i] = (int32_t)(ptr[i + 1] - ptr[i]);
}

}  // namespace dev
}  // namespace ias

// =================================================================== host engine
using namespace ias;
using namespace ias::dev;
using Plan = ias_plan;

// Bin tables.  Symbolic bins by products, numeric bins by nnz; the table of a
// bin holds up to `upper` keys at load <= 2/3 (S >= 1.5 * upper).
static const int SYM_UPPER[] = {0, 40, 170, 680, 2730, 10920, 21840};   // + global
static const int NUM_UPPER[] = {0, 20, 85, 340, 1365, 2730, 5460};     // + global

static BinSpec make_spec(const int *upper, int n_lds) {
    BinSpec s{};
    s.nbins = n_lds + 2;
    for (int i = 0; i <= n_lds; ++i) s.upper[i] = upper[i];
    return s;
}

static inline unsigned grid_for(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }

#define HIPC(x)                                                                   \
    do {                                                                          \
        hipError_t _e = (x);                                                      \
        if (_e != hipSuccess) {                                                   \
            set_last_error("%s failed: %s", #x, hipGetErrorString(_e));           \
            return _e == hipErrorOutOfMemory ? IAS_ERROR_OUT_OF_MEMORY : IAS_ERROR_DEVICE; \
        }                                                                         \
    } while (0)

ias_status Plan::reserve(void **buf, size_t *cap, size_t bytes) {
    if (*cap >= bytes && *buf) return IAS_SUCCESS;
    if (*buf) HIPC(hipFree(*buf));
    *buf = nullptr;
    *cap = 0;
    const size_t want = std::max<size_t>(bytes + bytes / 8, 256);
    HIPC(hipMalloc(buf, want));
    *cap = want;
    return IAS_SUCCESS;
}

ias_plan::~ias_plan() {
    hipSetDevice(device);
    for (auto &b : bufs)
        if (b.p) hipFree(b.p);
    for (auto &e : ev)
        if (e) hipEventDestroy(e);
    if (host_counters) hipHostFree(host_counters);
    if (own_stream && stream) hipStreamDestroy((hipStream_t)stream);
}

ias_status Plan::init(int dev, void *strm) {
    device = dev;
    HIPC(hipSetDevice(device));
    if (strm) {
        stream = strm;
        own_stream = false;
    } else {
        hipStream_t s;
        HIPC(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        stream = s;
        own_stream = true;
    }
    for (auto &e : ev) HIPC(hipEventCreate(&e));
    HIPC(hipHostMalloc(&host_counters, sizeof(Counters)));
    return IAS_SUCCESS;
}

template <typename T>
static T *as(Plan::Buf &b) { return (T *)b.p; }

ias_status Plan::symbolic(const Rows &A, const Rows &B, int64_t rows, int64_t cols,
                          ias_report *rep) {
    (void)cols;
    hipStream_t s = (hipStream_t)stream;
    HIPC(hipSetDevice(device));
    n_rows = rows;
    const BinSpec sspec = make_spec(SYM_UPPER, 6);
    const BinSpec nspec = make_spec(NUM_UPPER, 6);
    IAS_TRY(reserve(&bufs[B_PROD].p, &bufs[B_PROD].cap, sizeof(int32_t) * (rows + 1)));
    IAS_TRY(reserve(&bufs[B_NNZ].p, &bufs[B_NNZ].cap, sizeof(int32_t) * (rows + 1)));
    IAS_TRY(reserve(&bufs[B_SLIST].p, &bufs[B_SLIST].cap, sizeof(int32_t) * rows * MAX_BINS + 4));
    IAS_TRY(reserve(&bufs[B_NLIST].p, &bufs[B_NLIST].cap, sizeof(int32_t) * rows * MAX_BINS + 4));
    IAS_TRY(reserve(&bufs[B_SOFF].p, &bufs[B_SOFF].cap, sizeof(int64_t) * (rows + 1)));
    IAS_TRY(reserve(&bufs[B_NOFF].p, &bufs[B_NOFF].cap, sizeof(int64_t) * (rows + 1)));
    IAS_TRY(reserve(&bufs[B_CNT].p, &bufs[B_CNT].cap, sizeof(Counters)));
    IAS_TRY(reserve(&bufs[B_PTR].p, &bufs[B_PTR].cap, sizeof(int64_t) * (rows + 1)));
    const int64_t nb = (rows + SCAN_TILE - 1) / SCAN_TILE;
    IAS_TRY(reserve(&bufs[B_PART].p, &bufs[B_PART].cap, sizeof(int64_t) * (nb + 2)));
    Counters *dc = as<Counters>(bufs[B_CNT]);

    HIPC(hipEventRecord(ev[0], s));
    HIPC(hipMemsetAsync(dc, 0, sizeof(Counters), s));
    if (rows > 0) {
        k_row_products<<<grid_for(rows, AN_BLOCK), AN_BLOCK, 0, s>>>(
            A, B, rows, as<int32_t>(bufs[B_PROD]), &dc->flops, &dc->max_prod);
        k_bin_rows<<<grid_for(rows, BIN_BLOCK), BIN_BLOCK, 0, s>>>(
            as<int32_t>(bufs[B_PROD]), rows, sspec, as<int32_t>(bufs[B_SLIST]), dc->sym_count,
            &dc->sym_ws, as<int64_t>(bufs[B_SOFF]), as<int32_t>(bufs[B_NNZ]));
    }
    HIPC(hipEventRecord(ev[1], s));
    HIPC(hipMemcpyAsync(host_counters, dc, sizeof(Counters), hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    Counters hc = *(Counters *)host_counters;
    flops = (int64_t)hc.flops;
    max_prod = hc.max_prod;

    // workspace for global-table rows (keys only, 4 B per slot)
    if (hc.sym_count[sspec.nbins - 1] > 0)
        IAS_TRY(reserve(&bufs[B_WS].p, &bufs[B_WS].cap, sizeof(int32_t) * hc.sym_ws));
    const int32_t *L = as<int32_t>(bufs[B_SLIST]);
    int32_t *nnz = as<int32_t>(bufs[B_NNZ]);
    auto lst = [&](int b) { return L + (int64_t)b * rows; };
    int c;
    if ((c = hc.sym_count[1]) > 0)
        k_symbolic_lds<32, 6, 8><<<grid_for(c, 8), 256, 0, s>>>(A, B, lst(1), c, nnz);
    if ((c = hc.sym_count[2]) > 0)
        k_symbolic_lds<64, 8, 4><<<grid_for(c, 4), 256, 0, s>>>(A, B, lst(2), c, nnz);
    if ((c = hc.sym_count[3]) > 0)
        k_symbolic_lds<128, 10, 1><<<c, 128, 0, s>>>(A, B, lst(3), c, nnz);
    if ((c = hc.sym_count[4]) > 0)
        k_symbolic_lds<256, 12, 1><<<c, 256, 0, s>>>(A, B, lst(4), c, nnz);
    if ((c = hc.sym_count[5]) > 0)
        k_symbolic_lds<512, 14, 1><<<c, 512, 0, s>>>(A, B, lst(5), c, nnz);
    if ((c = hc.sym_count[6]) > 0)
        k_symbolic_lds<1024, 15, 1><<<c, 1024, 0, s>>>(A, B, lst(6), c, nnz);
    if ((c = hc.sym_count[7]) > 0)
        k_symbolic_global<1024><<<c, 1024, 0, s>>>(A, B, lst(7), as<int64_t>(bufs[B_SOFF]),
                                                    as<int32_t>(bufs[B_PROD]), c,
                                                    as<int32_t>(bufs[B_WS]), nnz);
    // row pointer of C
    int64_t *ptr = as<int64_t>(bufs[B_PTR]);
    if (rows > 0) {
        k_scan_reduce<<<(unsigned)nb, SCAN_BLOCK, 0, s>>>(nnz, rows, as<int64_t>(bufs[B_PART]),
                                                          &dc->max_nnz);
        k_scan_partials<<<1, 1024, 0, s>>>(as<int64_t>(bufs[B_PART]), nb);
        k_scan_apply<<<(unsigned)nb, SCAN_BLOCK, 0, s>>>(nnz, rows, as<int64_t>(bufs[B_PART]),
                                                         ptr);
        k_bin_rows<<<grid_for(rows, BIN_BLOCK), BIN_BLOCK, 0, s>>>(
            nnz, rows, nspec, as<int32_t>(bufs[B_NLIST]), dc->num_count, &dc->num_ws,
            as<int64_t>(bufs[B_NOFF]), nullptr);
    } else {
        HIPC(hipMemsetAsync(ptr, 0, sizeof(int64_t), s));
    }
    HIPC(hipEventRecord(ev[2], s));
    HIPC(hipMemcpyAsync(host_counters, dc, sizeof(Counters), hipMemcpyDeviceToHost, s));
    HIPC(hipMemcpyAsync(&nnz_total, ptr + rows, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    hc = *(Counters *)host_counters;
    std::copy(hc.num_count, hc.num_count + MAX_BINS, num_count);
    num_ws = hc.num_ws;
    max_nnz = hc.max_nnz;
    if (rep) {
        float a = 0, b = 0;
        hipEventElapsedTime(&a, ev[0], ev[1]);
        hipEventElapsedTime(&b, ev[1], ev[2]);
        rep->ms_analysis = a;
        rep->ms_symbolic = b;
        rep->flops = flops;
        rep->nnz_c = nnz_total;
        rep->max_row_products = max_prod;
        rep->max_row_nnz = max_nnz;
    }
    return IAS_SUCCESS;
}

ias_status Plan::numeric(const Rows &A, const Rows &B, const Out &out, ias_report *rep) {
    hipStream_t s = (hipStream_t)stream;
    HIPC(hipSetDevice(device));
    const int64_t rows = n_rows;
    const int nglob = MAX_BIN_LDS + 1;
    if (num_count[nglob] > 0) IAS_TRY(reserve(&bufs[B_WS].p, &bufs[B_WS].cap, 20ull * num_ws));
    const int32_t *L = as<int32_t>(bufs[B_NLIST]);
    auto lst = [&](int b) { return L + (int64_t)b * rows; };
    HIPC(hipEventRecord(ev[3], s));
    int c;
    if ((c = num_count[1]) > 0)
        k_numeric_lds<32, 5, 8><<<grid_for(c, 8), 256, 0, s>>>(A, B, lst(1), c, out);
    if ((c = num_count[2]) > 0)
        k_numeric_lds<64, 7, 4><<<grid_for(c, 4), 256, 0, s>>>(A, B, lst(2), c, out);
    if ((c = num_count[3]) > 0)
        k_numeric_lds<128, 9, 1><<<c, 128, 0, s>>>(A, B, lst(3), c, out);
    if ((c = num_count[4]) > 0)
        k_numeric_lds<256, 11, 1><<<c, 256, 0, s>>>(A, B, lst(4), c, out);
    if ((c = num_count[5]) > 0)
        k_numeric_lds<512, 12, 1><<<c, 512, 0, s>>>(A, B, lst(5), c, out);
    if ((c = num_count[6]) > 0)
        k_numeric_lds<1024, 13, 1><<<c, 1024, 0, s>>>(A, B, lst(6), c, out);
    if ((c = num_count[nglob]) > 0)
        k_numeric_global<1024><<<c, 1024, 0, s>>>(A, B, lst(nglob), as<int64_t>(bufs[B_NOFF]),
                                                   as<int32_t>(bufs[B_NNZ]), c,
                                                   (char *)bufs[B_WS].p, out);
    if (out.row_idx && rows > 0)
        k_fill_rows<<<grid_for(rows * WAVE, 256), 256, 0, s>>>(out.ptr, rows, out.row_idx);
    HIPC(hipGetLastError());
    HIPC(hipEventRecord(ev[4], s));
    if (rep) {
        HIPC(hipEventSynchronize(ev[4]));
        float a = 0, t = 0;
        hipEventElapsedTime(&a, ev[3], ev[4]);
        hipEventElapsedTime(&t, ev[0], ev[4]);
        rep->ms_numeric = a;
        rep->ms_total = t;
    }
    return IAS_SUCCESS;
}

ias_status Plan::shift(int64_t *p, int64_t n, int64_t off) {
    if (n <= 0 || off == 0) return IAS_SUCCESS;
    k_shift<<<grid_for(n, 256), 256, 0, (hipStream_t)stream>>>(p, n, off);
    HIPC(hipGetLastError());
    return IAS_SUCCESS;
}


// ------------------------------------------------------------------ row sort host
static const int SORT_UPPER[] = {0, 32, 128, 512, 2048, 4096, 8192};

static ias_status sort_rows_impl(ias_plan *plan, const int64_t *ptr, const int32_t *len_in,
                                 int64_t stride, int64_t rows, int32_t *col, double *val) {
    if (rows <= 0) return IAS_SUCCESS;
    hipStream_t s = (hipStream_t)plan->stream;
    HIPC(hipSetDevice(plan->device));
    IAS_TRY(plan->reserve(&plan->bufs[ias_plan::B_TMP0].p, &plan->bufs[ias_plan::B_TMP0].cap,
                          sizeof(int32_t) * (rows + 1)));
    IAS_TRY(plan->reserve(&plan->bufs[ias_plan::B_TMP1].p, &plan->bufs[ias_plan::B_TMP1].cap,
                          sizeof(int32_t) * rows * MAX_BINS + 4));
    IAS_TRY(plan->reserve(&plan->bufs[ias_plan::B_TMP2].p, &plan->bufs[ias_plan::B_TMP2].cap,
                          sizeof(int64_t) * (rows + 1)));
    IAS_TRY(plan->reserve(&plan->bufs[ias_plan::B_TMP3].p, &plan->bufs[ias_plan::B_TMP3].cap,
                          sizeof(Counters)));
    const int32_t *len = len_in;
    if (ptr) {
        k_row_len<<<grid_for(rows, 256), 256, 0, s>>>(ptr, rows, (int32_t *)plan->bufs[ias_plan::B_TMP0].p);
        len = (const int32_t *)plan->bufs[ias_plan::B_TMP0].p;
    }
    Counters *dc = (Counters *)plan->bufs[ias_plan::B_TMP3].p;
    HIPC(hipMemsetAsync(dc, 0, sizeof(Counters), s));
    const BinSpec spec = make_spec(SORT_UPPER, 6);
    int32_t *lists = (int32_t *)plan->bufs[ias_plan::B_TMP1].p;
    int64_t *offs = (int64_t *)plan->bufs[ias_plan::B_TMP2].p;
    k_bin_rows<<<grid_for(rows, BIN_BLOCK), BIN_BLOCK, 0, s>>>(len, rows, spec, lists, dc->num_count,
                                                                &dc->num_ws, offs, nullptr);
    Counters hc;
    HIPC(hipMemcpyAsync(&hc, dc, sizeof(Counters), hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    if (hc.num_count[7] > 0)
        IAS_TRY(plan->reserve(&plan->bufs[ias_plan::B_TMP4].p, &plan->bufs[ias_plan::B_TMP4].cap,
                              12ull * hc.num_ws + 16));
    auto lst = [&](int b) { return lists + (int64_t)b * rows; };
    int c;
    if ((c = hc.num_count[1]) > 0)
        k_sort_lds<32, 32, 8><<<grid_for(c, 8), 256, 0, s>>>(lst(1), c, ptr, len, stride, col, val);
    if ((c = hc.num_count[2]) > 0)
        k_sort_lds<64, 128, 4><<<grid_for(c, 4), 256, 0, s>>>(lst(2), c, ptr, len, stride, col, val);
    if ((c = hc.num_count[3]) > 0)
        k_sort_lds<256, 512, 1><<<c, 256, 0, s>>>(lst(3), c, ptr, len, stride, col, val);
    if ((c = hc.num_count[4]) > 0)
        k_sort_lds<512, 2048, 1><<<c, 512, 0, s>>>(lst(4), c, ptr, len, stride, col, val);
    if ((c = hc.num_count[5]) > 0)
        k_sort_lds<1024, 4096, 1><<<c, 1024, 0, s>>>(lst(5), c, ptr, len, stride, col, val);
    if ((c = hc.num_count[6]) > 0)
        k_sort_lds<1024, 8192, 1><<<c, 1024, 0, s>>>(lst(6), c, ptr, len, stride, col, val);
    if ((c = hc.num_count[7]) > 0)
        k_sort_global<<<c, 1024, 0, s>>>(lst(7), c, offs, ptr, len, stride, col, val,
                                         (char *)plan->bufs[ias_plan::B_TMP4].p);
    HIPC(hipGetLastError());
    return IAS_SUCCESS;
}

ias_status ias::ias_sort_rows_device(ias_plan *plan, const int64_t *ptr, int64_t rows, int32_t *col,
                                     double *val, int32_t max_nnz) {
    (void)max_nnz;
    return sort_rows_impl(plan, ptr, nullptr, 0, rows, col, val);
}

ias_status ias::ias_sort_rows_ell_device(ias_plan *plan, const int32_t *nnz_row, int64_t rows,
                                         int32_t K, int32_t *col, double *val) {
    return sort_rows_impl(plan, nullptr, nnz_row, K, rows, col, val);
}

ias_status ias::ias_shift_device(int64_t *p, int64_t n, int64_t off, void *stream) {
    if (n <= 0 || off == 0) return IAS_SUCCESS;
    k_shift<<<grid_for(n, 256), 256, 0, (hipStream_t)stream>>>(p, n, off);
    HIPC(hipGetLastError());
    return IAS_SUCCESS;
}
