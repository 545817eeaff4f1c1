// spgemm.hip — kernels and host engine of the row-wise SpGEMM hot path
// (replaces CSR_MUL_CSR / COO_MUL_COO / ELL_MUL_ELL of the reference and the
// CUSP / cuSPARSE calls of GPU/main.cu:467-523).  See spgemm_kernels.hpp for
// the per-row algorithm and DESIGN.md §4 for the pipeline and its roofline.
#include <hipcub/hipcub.hpp>
#include "spgemm_kernels.hpp"
#include "sym2_kernels.hpp"
#include "sym3_kernels.hpp"
#include "sym4_kernels.hpp"
#include "sym5_kernels.hpp"
#include "num2_kernels.hpp"
#include "short_kernels.hpp"
#include "spgemm_engine.hpp"
#include "ias_internal.hpp"

#include <algorithm>
#include <functional>
#include <map>
#include <mutex>
#include <set>
#include <tuple>
#include <type_traits>
#include <vector>

namespace ias {
namespace dev {

// ---------------------------------------------------------------- binning
// Bin of a row with key k (products for symbolic, nnz for numeric/sort) and
// products `prod` (numeric class test).  Bin numbering: 0 = nothing to do,
// 1..nval = value LDS bins, nval+1 = hash partitions, nval+2 = global table,
// nval+3.. = direct-write LDS bins.
__device__ __forceinline__ uint32_t nparts_of(int32_t key, int32_t cap) {
    return (uint32_t)((key + cap - 1) / cap);
}

// stv: the row's streaming state (-2: none given; >= 0: a streaming row with
// stv duplicates -> the fix-up bin when it has any, nothing to do otherwise;
// -3: a table-path row without a first-touch bitmap too long for the LDS
// bins -> the per-row global table; -5: a short row (<= SHORT_MAX products,
// short_kernels.hpp) -> its numeric bin by products).
__device__ __forceinline__ int bin_of(const BinSpec &sp, int32_t k, int32_t prod, int32_t stv, int32_t ent2 = 0) {
    if (k <= 0) return 0;
    if (stv == -3) return sp.nval + 2;
    if (stv == -5 && sp.short_base > 0) return sp.short_base + (prod <= 64 ? 0 : (prod <= 128 ? 1 : 2));
    if (stv >= 0 && sp.nst > 0) {   // fix-up bins: <= 16 (one lane), <= 256 (one wave), then the
                                    // sorted fix-ups by list length: <= 1024, <= 4096, longer
        if (stv == 0) return 0;
        return sp.nval + 3 + sp.ndw + (stv > 4096 ? 4 : (stv > 1024 ? 3 : (stv > 256 ? 2 : (stv > 16 ? 1 : 0))));
    }
    if (sp.wide_min > 0 && k >= sp.wide_min) return sp.nval + 2;
    const bool val_class =
        sp.ratio_den == 0 || (int64_t)prod * sp.ratio_den > (int64_t)k * sp.ratio_num;
    if (val_class)
        for (int i = 1; i <= sp.nval; ++i)
            if (k <= sp.upper[i] && ent2 <= sp.upper[i]) return i;
    for (int i = 0; i < sp.ndw; ++i)
        if (k <= sp.upper[sp.nval + 3 + i]) return sp.nval + 3 + i;
    return sp.nval + 1;
}

// duplicate-list capacity of a row in bin b with key k
__device__ __forceinline__ int32_t dcap_of(const BinSpec &sp, int b, int32_t k) {
    if (b == sp.nval + 1 && sp.part_dcap_div > 0) return min(k / sp.part_dcap_div, sp.part_dcap_max);
    return sp.dcap[b];
}

// Block-wide exclusive prefix of a 64-bit value (BLOCK threads); every
// thread gets the block total.  Two barriers; `red` holds BLOCK/WAVE words.
template <int BLOCK>
__device__ __forceinline__ unsigned long long block_excl_u64(unsigned long long v, unsigned long long &total,
                                                             unsigned long long *red) {
    const int l = (int)(threadIdx.x & (WAVE - 1)), w = (int)(threadIdx.x / WAVE);
    unsigned long long x = v;
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
        const unsigned long long t = __shfl_up(x, d);
        if (l >= d) x += t;
    }
    if (l == WAVE - 1) red[w] = x;
    __syncthreads();
    unsigned long long before = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < BLOCK / WAVE; ++i) {
        before += i < w ? red[i] : 0ull;
        tot += red[i];
    }
    __syncthreads();
    total = tot;
    return before + x - v;
}

// Per-row allocation sizes of a binned row: bitmap words, duplicate slots,
// partition items, global-table slots.
constexpr int NQ = 5;   // per-row allocations: bitmap words, duplicate slots, partition items,
                        // global-table slots, partition-bucket pairs
__device__ __forceinline__ void bin_needs(const BinSpec &sp, int b, int32_t k, unsigned long long (&q)[NQ]) {
    q[0] = q[1] = q[2] = q[3] = q[4] = 0ull;
    if (b <= 0) return;
    if (sp.ft) q[0] = (unsigned long long)((k + 31) / 32);
    const int32_t dc = dcap_of(sp, b, k);
    if (dc > 0) q[1] = (unsigned long long)dc;
    if (b == sp.nval + 1) {
        q[2] = (unsigned long long)nparts_of(k, sp.part_cap);
        if (sp.ft) q[4] = (unsigned long long)k;   // symbolic: the row's products, bucketed by partition
    } else if (b == sp.nval + 2) {
        const unsigned long long need = (unsigned long long)k + ((unsigned long long)k + 1) / 2;
        unsigned long long S = 1;
        while (S < need) S <<= 1;
        q[3] = S;
    }
}

// Block-level count of rows per bin (+ the allocation totals) into the
// Counters, R rows per thread: one global atomic per block and counter.  The
// counters share a few cache lines, so atomics on them serialise: blocks of
// BLOCK*R rows keep their number small.
template <int BLOCK, int R>
__device__ __forceinline__ void count_bins(const BinSpec &sp, const int (&b)[R], const int32_t (&k)[R],
                                           Counters *cnt) {
    __shared__ int hist[MAX_BINS];
    __shared__ unsigned long long red[NQ][BLOCK / WAVE];
    for (int i = threadIdx.x; i < MAX_BINS; i += BLOCK) hist[i] = 0;
    __syncthreads();
    unsigned long long q[NQ] = {0ull, 0ull, 0ull, 0ull, 0ull};   // bin_needs order
#pragma unroll
    for (int i = 0; i < R; ++i) {
        if (b[i] > 0) {
            atomicAdd(&hist[b[i]], 1);
            unsigned long long n[NQ];
            bin_needs(sp, b[i], k[i], n);
#pragma unroll
            for (int j = 0; j < NQ; ++j) q[j] += n[j];
        }
    }
#pragma unroll
    for (int j = 0; j < NQ; ++j)
#pragma unroll
        for (int d = WAVE / 2; d > 0; d >>= 1) q[j] += __shfl_xor(q[j], d);
    if ((threadIdx.x & (WAVE - 1)) == 0)
#pragma unroll
        for (int j = 0; j < NQ; ++j) red[j][threadIdx.x / WAVE] = q[j];
    __syncthreads();
    if (threadIdx.x < NQ) {
        unsigned long long t = 0;
        for (int i = 0; i < BLOCK / WAVE; ++i) t += red[threadIdx.x][i];
        unsigned long long *dst[NQ] = {&cnt->bm_words, &cnt->dup_slots, &cnt->items, &cnt->ws_slots,
                                       &cnt->part_prod};
        if (t) atomicAdd(dst[threadIdx.x], t);
    }
    for (int i = threadIdx.x; i < MAX_BINS; i += BLOCK)
        if (i > 0 && hist[i] > 0) atomicAdd(&cnt->count[i], hist[i]);
}

// ---------------------------------------------------------------- analysis
// Two passes, load-balanced: flat over A entries the expanded A (B-row start and
// length, A value) — independent of how entries spread over rows, so R-MAT
// hub rows do not serialise a block — and, after the scan of the B-row
// lengths, per row: products (GetFlop per row, csr/common_csr.h:290-304) =
// difference of the product offsets, the symbolic bin counts, total flops
// and the max products per row.
constexpr int AN_BLOCK = 256;
constexpr int AN_U = 8;   // entries per thread: a block is one scan tile (SCAN_TILE = AN_BLOCK * AN_U)

// Expanded A, flat over entries (ELL, A.ptr null: padding entries beyond
// len[row] get no products); each block also writes its tile's sum of B-row
// lengths into `partial` — the reduce step of the product-offset scan
// (k_scan_partials + k_scan_apply finish it), so the lengths are not read back.
__global__ __launch_bounds__(AN_BLOCK) void k_an_entries(Rows A, Rows B, int64_t a_entries, AxOut ax,
                                                         int64_t *partial) {
    const int64_t abase = A.base();
    const int64_t q0 = (int64_t)blockIdx.x * AN_BLOCK * AN_U + threadIdx.x;
    int32_t j[AN_U], bn[AN_U];
    int64_t bs[AN_U];
    double av[AN_U];
    bool ok[AN_U];
#pragma unroll
    for (int u = 0; u < AN_U; ++u) {
        const int64_t q = q0 + (int64_t)u * AN_BLOCK;
        ok[u] = q < a_entries;
        if (ok[u] && !A.ptr) ok[u] = (q % A.stride) < A.len[q / A.stride];
        j[u] = ok[u] ? A.col[abase + q] : 0;
    }
    int64_t sum = 0;
#pragma unroll
    for (int u = 0; u < AN_U; ++u) {   // all loads before any store (no alias ordering)
        bn[u] = 0;
        bs[u] = 0;
        av[u] = 0.0;
        if (ok[u]) {
            B.row(j[u], bs[u], bn[u]);
            if (ax.aval) av[u] = A.val[abase + q0 + (int64_t)u * AN_BLOCK];
        }
        sum += bn[u];
    }
    if (ax.wide_b) {
        bool wide = false, widev = false;
#pragma unroll
        for (int u = 0; u < AN_U; ++u) {
            wide |= bs[u] + bn[u] > (1ll << 30);
            widev |= bs[u] + bn[u] > (1ll << 29);
        }
        if (wide) *ax.wide_b = 1;
        if (widev && ax.wide_v) *ax.wide_v = 1;
    }
#pragma unroll
    for (int u = 0; u < AN_U; ++u) {
        const int64_t q = q0 + (int64_t)u * AN_BLOCK;
        if (q >= a_entries) continue;
        ax.bstart[q] = bs[u];
        ax.blen[q] = bn[u];
        if (ax.aval) ax.aval[q] = av[u];
    }
    // the tile's sum
#pragma unroll
    for (int d = WAVE / 2; d > 0; d >>= 1) sum += __shfl_down(sum, d);
    __shared__ int64_t ws[AN_BLOCK / WAVE];
    if ((threadIdx.x & (WAVE - 1)) == 0) ws[threadIdx.x / WAVE] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t t = 0;
#pragma unroll
        for (int i = 0; i < AN_BLOCK / WAVE; ++i) t += ws[i];
        partial[blockIdx.x] = t;
    }
}

constexpr int BIN_BLOCK = 256;
constexpr int BIN_RPT = 8;   // rows per thread of the row passes
constexpr int BIN_ROWS = BIN_BLOCK * BIN_RPT;    // rows per block
// Small row counts use BIN_RPT / 2 rows per thread (twice the blocks: K1's
// 256k rows 128 -> 256 blocks; its binning 0.354 -> 0.337 ms per step); from
// BIN_RPT_BIG_ROWS rows on BIN_RPT (K2 / K3': 4 measured 1 % slower).
constexpr int BIN_RPT_BIG_ROWS = (1 << 20);
constexpr int BIN_RPT_SMALL = BIN_RPT > 1 ? BIN_RPT / 2 : 1;
#define BIN_LAUNCH(kern, nrows, strm, ...)                                                                       \
    do {                                                                                                         \
        if ((nrows) < BIN_RPT_BIG_ROWS)                                                                          \
            kern<BIN_RPT_SMALL><<<grid_for((nrows), BIN_BLOCK * BIN_RPT_SMALL), BIN_BLOCK, 0, (strm)>>>(__VA_ARGS__); \
        else                                                                                                     \
            kern<BIN_RPT><<<grid_for((nrows), BIN_ROWS), BIN_BLOCK, 0, (strm)>>>(__VA_ARGS__);                   \
    } while (0)

__device__ __forceinline__ int32_t ent2_of(const BinSpec &sp, const Rows &A, int64_t r) {
    if (!sp.ent_key) return 0;
    int64_t s;
    int32_t n;
    A.row(r, s, n);
    return n > INT32_MAX / sp.ent_key ? INT32_MAX : sp.ent_key * n;
}

// A row's first entry in the expanded A (clamped; a row pointer that
// disagrees with the declared entry count sets the overflow flag).
__device__ __forceinline__ int64_t row_q(const Rows &A, int64_t r, int64_t n_entries, Counters *cnt) {
    int64_t s;
    int32_t n;
    A.row(r, s, n);
    int64_t q = s - A.base();
    if (q < 0 || n < 0 || q + n > n_entries) {
        cnt->overflow = 1;
        q = q < 0 ? 0 : (q > n_entries ? n_entries : q);
    }
    return q;
}

// Per row: the product offset poff (from axp at the row's first entry), the
// products, the symbolic bin histogram, max products, flops.
template <int RPT>
__global__ __launch_bounds__(BIN_BLOCK) void k_an_rows(const int64_t *axp, int64_t n_entries, int64_t *poff,
                                                       int64_t rows, int32_t *prod, BinSpec spec, Counters *cnt,
                                                       Rows A) {
    int b[RPT];
    int32_t k[RPT];
    int mx = 0;
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
        const int64_t r = (int64_t)blockIdx.x * (BIN_BLOCK * RPT) + i * BIN_BLOCK + threadIdx.x;
        b[i] = -1;
        k[i] = 0;
        if (r < rows) {
            const int64_t p0 = axp[row_q(A, r, n_entries, cnt)];
            const int64_t p1 = r + 1 < rows ? axp[row_q(A, r + 1, n_entries, cnt)] : axp[n_entries];
            poff[r] = p0;
            if (r + 1 == rows) poff[rows] = p1;
            const int64_t p = p1 - p0;
            k[i] = (int32_t)min(p, (int64_t)INT32_MAX);
            prod[r] = k[i];
            b[i] = bin_of(spec, k[i], k[i], -2, ent2_of(spec, A, r));
            mx = max(mx, k[i]);
        }
    }
    count_bins<BIN_BLOCK, RPT>(spec, b, k, cnt);
#pragma unroll
    for (int d = WAVE / 2; d > 0; d >>= 1) mx = max(mx, __shfl_xor(mx, d));
    __shared__ int wmx[BIN_BLOCK / WAVE];
    if ((threadIdx.x & (WAVE - 1)) == 0) wmx[threadIdx.x / WAVE] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 0; i < BIN_BLOCK / WAVE; ++i) mx = max(mx, wmx[i]);
        if (mx > 0) atomicMax(&cnt->max_prod, mx);
        if (blockIdx.x == 0) {
            cnt->flops = (unsigned long long)(axp[n_entries] - axp[row_q(A, 0, n_entries, cnt)]);
            cnt->a_base = (long long)A.base();
        }
    }
}

// Counting pass of a binning (numeric and sort binnings; the symbolic one is
// fused into k_an_rows).  prod may be null (class test off); a row is
// streaming-class when stn is given and stn[r] >= 0.
template <int RPT>
__global__ __launch_bounds__(BIN_BLOCK) void k_bin_count(const int32_t *key, const int32_t *prod,
                                                         const int32_t *stn, int64_t rows,
                                                         BinSpec spec, Counters *cnt,
                                                         const int64_t *total = nullptr) {
    if (total && blockIdx.x == 0 && threadIdx.x == 0) cnt->nnz_total = (unsigned long long)*total;
    int b[RPT];
    int32_t k[RPT];
    unsigned long long sp = 0, sn = 0;
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
        const int64_t r = (int64_t)blockIdx.x * (BIN_BLOCK * RPT) + i * BIN_BLOCK + threadIdx.x;
        b[i] = -1;
        k[i] = 0;
        if (r < rows) {
            k[i] = key[r];
            const int32_t st = stn ? stn[r] : -2;
            const int32_t pr = prod ? prod[r] : k[i];
            b[i] = bin_of(spec, k[i], pr, st);
            if (stn && st >= 0 && k[i] > 0) {   // a streaming row: its work in the flat pass
                sp += (unsigned long long)pr;
                sn += (unsigned long long)k[i];
            }
        }
    }
    count_bins<BIN_BLOCK, RPT>(spec, b, k, cnt);
    if (stn) {   // block sums, one pair of atomics per block
        __shared__ unsigned long long red[2][BIN_BLOCK / WAVE];
        for (int d = WAVE / 2; d > 0; d >>= 1) {
            sp += __shfl_down(sp, d);
            sn += __shfl_down(sn, d);
        }
        if ((threadIdx.x & (WAVE - 1)) == 0) {
            red[0][threadIdx.x / WAVE] = sp;
            red[1][threadIdx.x / WAVE] = sn;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long a = 0, c = 0;
            for (int i = 0; i < BIN_BLOCK / WAVE; ++i) {
                a += red[0][i];
                c += red[1][i];
            }
            if (a | c) {
                atomicAdd(&cnt->st_prod, a);
                atomicAdd(&cnt->st_nnz, c);
            }
        }
    }
}

// Scatter pass: every listed row gets a RowRef in its bin's compact list
// (bins laid out in bin order, offsets = prefix of the counted totals);
// partitioned rows get one PartItem per partition (+ a bitmap offset when
// FT); global-table rows a workspace offset of nextpow2(ceil(k*3/2)) slots.
// R rows per thread; per-row allocations come from a block prefix and one
// cursor atomic per block and counter.
template <int RPT>
__global__ __launch_bounds__(BIN_BLOCK) void k_bin_scatter(const int32_t *key, const int32_t *prod,
                                                           const int32_t *stn, int64_t rows,
                                                           BinSpec spec, Rows A, RowRef *lists,
                                                           PartItem *items, int64_t *bm_off,
                                                           int64_t *ws_off, int64_t *dup_off,
                                                           int32_t *dupn, int32_t *nnz_row,
                                                           const int64_t *qstart, Counters *cnt,
                                                           int64_t *pfirst, int64_t *pboff, int sym2) {
    __shared__ int hist[MAX_BINS];
    __shared__ int64_t base[MAX_BINS];
    __shared__ int64_t bin_start[MAX_BINS];
    __shared__ unsigned long long red[BIN_BLOCK / WAVE];
    __shared__ unsigned long long cbase[NQ];
    const int t = threadIdx.x;
    if (t < MAX_BINS) hist[t] = 0;
    if (t == 0) {
        int64_t acc = 0;
        for (int i = 0; i < MAX_BINS; ++i) {
            bin_start[i] = acc;
            acc += i > 0 ? cnt->count[i] : 0;
        }
    }
    __syncthreads();
    const int part_bin = spec.nval + 1, wide_bin = spec.nval + 2;
    int b[RPT], local[RPT];
    int32_t k[RPT];
    unsigned long long mine[NQ] = {0ull, 0ull, 0ull, 0ull, 0ull};
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
        const int64_t r = (int64_t)blockIdx.x * (BIN_BLOCK * RPT) + i * BIN_BLOCK + t;
        b[i] = -1;
        local[i] = 0;
        k[i] = 0;
        if (r < rows) {
            k[i] = key[r];
            b[i] = bin_of(spec, k[i], prod ? prod[r] : k[i], stn ? stn[r] : -2, ent2_of(spec, A, r));
            if (b[i] == 0 && spec.zero_nnz) nnz_row[r] = 0;
            if (b[i] == 0 && dupn) dupn[r] = 0;
            if (b[i] > 0) local[i] = atomicAdd(&hist[b[i]], 1);
            unsigned long long n[NQ];
            bin_needs(spec, b[i], k[i], n);
#pragma unroll
            for (int j = 0; j < NQ; ++j) mine[j] += n[j];
        }
    }
    __syncthreads();
    if (t > 0 && t < MAX_BINS && hist[t] > 0) base[t] = atomicAdd(&cnt->cursor[t], hist[t]);
    unsigned long long at[NQ], tot[NQ];
#pragma unroll
    for (int j = 0; j < NQ; ++j) at[j] = block_excl_u64<BIN_BLOCK>(mine[j], tot[j], red);
    if (t < NQ) {
        unsigned long long *cur[NQ] = {&cnt->bm_cur, &cnt->dup_cur, &cnt->items_cur, &cnt->ws_cur, &cnt->pb_cur};
        cbase[t] = tot[t] ? atomicAdd(cur[t], tot[t]) : 0ull;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NQ; ++j) at[j] += cbase[j];
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
        if (b[i] <= 0) continue;
        const int64_t r = (int64_t)blockIdx.x * (BIN_BLOCK * RPT) + i * BIN_BLOCK + t;
        unsigned long long n[NQ];
        bin_needs(spec, b[i], k[i], n);
        const int64_t within = base[b[i]] + local[i];
        RowRef ref;
        ref.row = (int32_t)r;
        if (sym2) {     // sym2 bins: the row's A entries; partitioned rows: their products in the
                        // compact expansion of the partitioned rows (at the bucket offset)
            if (b[i] == part_bin) {
                ref.q0 = (int64_t)at[4];
                ref.n = k[i];
            } else {
                int64_t s;
                int32_t nn;
                A.row(r, s, nn);
                ref.q0 = s - A.base();
                ref.n = nn;
            }
        } else if (qstart) {   // products of the row in the expansion
            ref.q0 = qstart[r];
            ref.n = k[i];
        } else {        // entries of the row in the expanded A
            int64_t s;
            int32_t nn;
            A.row(r, s, nn);
            ref.q0 = s - A.base();
            ref.n = nn;
        }
        lists[bin_start[b[i]] + within] = ref;
        if (spec.ft) bm_off[r] = (int64_t)at[0];
        if (n[1]) dup_off[r] = (int64_t)at[1];
        if (b[i] == part_bin) {
            const uint32_t np = (uint32_t)n[2];
            for (uint32_t q = 0; q < np; ++q) items[at[2] + q] = PartItem{ref, q, np};
            if (pfirst) pfirst[r] = (int64_t)at[2];
            if (pboff) pboff[r] = (int64_t)at[4];
            if (spec.zero_nnz) nnz_row[r] = 0;
            // partitioned rows: a duplicate counter (k_dup_place decides the path)
            if (dupn) dupn[r] = spec.part_dcap_div > 0 ? 0 : -1;
        } else if (b[i] == wide_bin) {
            ws_off[within] = (int64_t)at[3];
        }
#pragma unroll
        for (int j = 0; j < NQ; ++j) at[j] += n[j];
    }
}

// ---------------------------------------------------------------- symbolic kernels
// LDS tables are sized per bin at launch (dynamic LDS, any slot count), so a
// row costs only the bytes its bin needs and more rows are resident per CU.

__host__ __device__ constexpr size_t round16(size_t b) { return (b + 15) & ~size_t(15); }

template <int SEG, bool NUMERIC>
__host__ __device__ constexpr size_t team_fixed_bytes() {
    return round16(sizeof(Seg<SEG, NUMERIC>)) + 256;   // segment + 64-int scratch
}
template <int SEG>
__host__ __device__ constexpr size_t val_team_bytes(uint32_t S) {
    return round16(8ull * S) + 2 * round16(4ull * S) + team_fixed_bytes<SEG, true>();
}
template <int SEG>
__host__ __device__ constexpr size_t dw_team_bytes(uint32_t S) {
    return 2 * round16(4ull * S) + team_fixed_bytes<SEG, true>();
}

__device__ __forceinline__ RowRef ref_at(const RowRef *list, int64_t idx, int32_t count) {
    if (idx < count) return list[idx];
    return RowRef{0, -1, 0};
}

// One workgroup per (row, hash partition): distinct columns of the partition
// (added to nnz_row) and the first-touch bits of the row's bitmap.
// Partition buckets: one workgroup per partitioned row gathers its products'
// columns from B (one wave per A entry, lanes along the entry's B row) and
// scatters (column, product) pairs into per-partition buckets (count, scan,
// scatter in LDS; the scatter pass gathers again, from the caches), so that
// each partition's workgroup reads only its own products.  Rows with more
// than PB_MAXP partitions keep the rescan of their expansion (span len -1;
// k_expand_part writes it for those rows only).  Measured on K3 (14,470 rows
// beyond 16,384 products): the expansion pass + a bucket pass over it took
// 1.28 + 2.58 ms.
constexpr int PB_BLOCK = 1024;
constexpr int PB_MAXP = 4096;
__global__ __launch_bounds__(PB_BLOCK) void k_part_bucket(Rows A, AxView ax, const int64_t *axp,
                                                          const int64_t *poff, const int32_t *bcol,
                                                          const RowRef *list, int32_t count,
                                                          const int64_t *pfirst, const int64_t *pboff,
                                                          int32_t part_cap, uint2 *bucket, PartSpan *spans) {
    __shared__ uint32_t cnt[PB_MAXP];
    __shared__ int scratch[32];
    const RowRef ref = list[blockIdx.x];
    const uint32_t np = nparts_of(ref.n, part_cap);
    const int64_t it0 = pfirst[ref.row];
    const int tid = threadIdx.x;
    if (np > (uint32_t)PB_MAXP) {
        for (uint32_t q = tid; q < np; q += PB_BLOCK) spans[it0 + q] = PartSpan{0, -1, 0};
        return;
    }
    for (uint32_t q = tid; q < np; q += PB_BLOCK) cnt[q] = 0u;
    int64_t rs;
    int32_t ne;
    A.row(ref.row, rs, ne);
    const int64_t q0 = rs - A.base();
    const int64_t p0 = poff[ref.row];
    const int w = tid / WAVE, lane = tid & (WAVE - 1);
    constexpr int NW = PB_BLOCK / WAVE;
    __syncthreads();
    // wave-aggregated LDS atomics: one per (wave, partition present), not per
    // product (a row has few partitions, so per-product atomics all collide)
    const bool direct = np >= 4;   // several partitions: plain LDS atomics (np >= 32 before: K3 33.6 vs 33.8 ms, K3' 1 %)
    auto wave_add = [&](bool active, uint32_t q) -> uint32_t {
        if (direct) return active ? atomicAdd(&cnt[q], 1u) : 0u;
        uint32_t rank = 0;
        uint64_t todo = __ballot(active);
        while (todo) {
            const uint32_t q1 = (uint32_t)__shfl((int)q, __builtin_ctzll(todo));
            const uint64_t same = __ballot(active && q == q1);
            const int leader = __builtin_ctzll(same);
            uint32_t base = 0;
            if (__lane_id() == (uint32_t)leader) base = atomicAdd(&cnt[q1], (uint32_t)__popcll(same));
            base = (uint32_t)__shfl((int)base, leader);
            if (active && q == q1) rank = base + (uint32_t)__popcll(same & ((1ull << __lane_id()) - 1ull));
            todo &= ~same;
        }
        return rank;
    };
    // the row's products, entry by entry: U B-row positions per lane in flight
    constexpr int U = 4;
    auto sweep = [&](auto &&visit) {
        for (int32_t e = w; e < ne; e += NW) {
            const int32_t bl = ax.blen[q0 + e];
            const int64_t bs = ax.bstart[q0 + e];
            const int32_t pe = (int32_t)(axp[q0 + e] - p0);
            for (int32_t j0 = 0; j0 < bl; j0 += U * WAVE) {
                int32_t c[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int32_t j = j0 + u * WAVE + lane;
                    c[u] = j < bl ? bcol[bs + j] : 0;
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int32_t j = j0 + u * WAVE + lane;
                    visit(j < bl, c[u], pe + j);
                }
            }
        }
    };
    sweep([&](bool act, int32_t c, int32_t) { wave_add(act, act ? part_of(c, np) : 0u); });
    __syncthreads();
    // exclusive scan of the counts (np <= PB_MAXP: PB_MAXP / PB_BLOCK per thread)
    constexpr int PER = PB_MAXP / PB_BLOCK;
    uint32_t v[PER], sum = 0;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const uint32_t q = (uint32_t)(tid * PER + i);
        v[i] = q < np ? cnt[q] : 0u;
        sum += v[i];
    }
    int tot;
    const int ex = Team<PB_BLOCK>::excl_sum((int)sum, tot, scratch);
    __syncthreads();
    const int64_t base = pboff[ref.row];
    uint32_t run = (uint32_t)ex;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const uint32_t q = (uint32_t)(tid * PER + i);
        if (q < np) {
            spans[it0 + q] = PartSpan{base + run, (int32_t)v[i], 0};
            cnt[q] = run;   // cursor
        }
        run += v[i];
    }
    __syncthreads();
    sweep([&](bool act, int32_t c, int32_t p) {
        const uint32_t at = wave_add(act, act ? part_of(c, np) : 0u);
        if (act) bucket[base + at] = make_uint2((uint32_t)c, (uint32_t)p);
    });
}

template <int TEAM, int K, int LOG2S>
__global__ __launch_bounds__(TEAM) void k_symbolic_part(const int32_t *tcol, const PartItem *items,
                                                        Bitmap bm, int32_t *nnz_row, uint2 *gpairs,
                                                        const int64_t *dup_off, int32_t *dupn,
                                                        int32_t div, int32_t dmax, int *overflow,
                                                        const uint2 *bucket, const PartSpan *spans) {
    __shared__ __attribute__((aligned(16))) int32_t keys[1 << LOG2S];
    __shared__ __attribute__((aligned(16))) uint32_t minp[1 << LOG2S];
    __shared__ int scratch[64];
    __shared__ uint32_t lbits[LBITS_WORDS];
    const PartItem it = items[blockIdx.x];
    const int64_t row = it.ref.row;
    Timer tmr;
    tmr.start();
    for (int w = threadIdx.x; w < LBITS_WORDS; w += TEAM) lbits[w] = 0u;
    SymTable<true> tb{keys, minp, 1u << LOG2S};
    uint32_t *gbits = bm.bits + bm.off[row];
    const uint32_t cap = div > 0 ? (uint32_t)min(it.ref.n / div, dmax) : 0u;
    const PartSpan sp = spans ? spans[blockIdx.x] : PartSpan{0, -1, 0};
    const int32_t n =
        sp.len >= 0 ? symbolic_bucket_row<TEAM, K>(bucket + sp.start, sp.len, tb, scratch, lbits, gbits,
                                                   cap > 0 ? gpairs + dup_off[row] : nullptr, dupn + row, cap,
                                                   overflow, tmr)
                    : symbolic_part_row<TEAM, K>(tcol, it.ref, tb, it.part, it.nparts, scratch, lbits, gbits,
                                                 cap > 0 ? gpairs + dup_off[row] : nullptr, dupn + row, cap,
                                                 overflow);
    // publish this partition's first-touch words (one atomic per non-zero word)
    const int64_t W = min<int64_t>(LBITS_WORDS, ((int64_t)it.ref.n + 31) / 32);
    for (int64_t w = threadIdx.x; w < W; w += TEAM)
        if (lbits[w]) atomicOr(&gbits[w], lbits[w]);
    if (threadIdx.x == 0 && n > 0) atomicAdd(&nnz_row[row], n);
    tmr.mark(6);
    tmr.flush(29, threadIdx.x == 0);   // slot 29: symbolic partitions
}

// Exclusive popcount prefix of each partitioned row's first-touch bitmap.
__global__ __launch_bounds__(256) void k_bitmap_prefix(const RowRef *list, int32_t count,
                                                       const int32_t *prod, Bitmap bm) {
    __shared__ int scratch[8];
    const int64_t row = list[blockIdx.x].row;
    const int64_t W = (prod[row] + 31) / 32;
    const uint32_t *bits = bm.bits + bm.off[row];
    uint32_t *pref = bm.pref + bm.off[row];
    int carry = 0;
    for (int64_t w0 = 0; w0 < W; w0 += 256) {
        const int64_t w = w0 + threadIdx.x;
        const int c = w < W ? __popc(bits[w]) : 0;
        int tot;
        const int ex = Team<256>::excl_sum(c, tot, scratch);
        if (w < W) pref[w] = (uint32_t)(carry + ex);
        carry += tot;
    }
}

// Partitioned rows: place the unordered duplicate pairs at their product-
// order index d = p - rank(p) (bitmap complete), or send the row to the
// table path when its duplicates overflowed its list.
__global__ __launch_bounds__(256) void k_dup_place(const RowRef *list, int32_t count, Bitmap bm,
                                                   const uint2 *gpairs, const int64_t *dup_off,
                                                   int32_t *dupn, int32_t *gdupt, int32_t div,
                                                   int32_t dmax) {
    const RowRef ref = list[blockIdx.x];
    const int64_t row = ref.row;
    const int32_t cnt = dupn[row];
    const int32_t cap = div > 0 ? min(ref.n / div, dmax) : 0;
    if (cnt > cap) {
        if (threadIdx.x == 0) dupn[row] = -1;
        return;
    }
    const uint32_t *bits = bm.bits + bm.off[row];
    const uint32_t *pref = bm.pref + bm.off[row];
    const uint2 *pr = gpairs + dup_off[row];
    int32_t *dt = gdupt + dup_off[row];
    for (int32_t i = threadIdx.x; i < cnt; i += 256) {
        const uint2 e = pr[i];
        const uint32_t rk = pref[e.x >> 5] + (uint32_t)__popc(bits[e.x >> 5] & ((1u << (e.x & 31)) - 1u));
        dt[e.x - rk] = (int32_t)e.y;
    }
}

// Column-bitmap symbolic of the partitioned rows (> SYM2_MAX products) when
// B's columns fit one LDS bitmap (ncw words, n_cols <= 32 * CBM_MAXW): one
// 1024-lane workgroup per row, no partitions, no bucket pass.
//  1. every product sets its column's bit: the products that find it clear
//     are the row's distinct columns (nnz = products - the others); the
//     others (duplicates) list their column;
//  2. the bitmap is rebuilt from the list: the columns with more than one
//     product, ranked by a superblock popcount prefix;
//  3. the products of those columns take the smallest product index per
//     column (atomicMin on a compact table indexed by rank: in the LDS left
//     beyond the bitmap when it fits, else in the row's work space): the
//     first touch, as the sequential loop of CSR_MUL_CSR finds it
//     (IA-SPGEMM-CPU_release/detail/csr/common_csr.h:133-189), and are
//     listed (product, rank);
//  4. first-touch bitmap = every product but the duplicates (built in the
//     LDS over the dead column bitmap when it fits), its word prefixes, and
//     the duplicates' first touches at their product-order index when the
//     row's list holds them (else dupn = -1: table path).
// Outputs are those of k_symbolic_part + k_bitmap_prefix + k_dup_place.
constexpr int CBM_BLOCK = 1024;
constexpr int CBM_SB = 8;            // bitmap words per rank superblock
constexpr int32_t CBM_MAXW = 36096;  // 4.5 B per word of LDS (bitmap + superblock prefix)
constexpr int CBM_U = 8;             // product columns per lane per block of a sweep
constexpr int CBM_L = 4;             // list items per lane per step of the duplicate pass
__host__ __device__ constexpr int32_t cbm_words(int64_t cols) {
    return (int32_t)(((cols + 31) / 32 + CBM_SB - 1) / CBM_SB * CBM_SB);
}
__host__ __device__ constexpr size_t cbm_lds_bytes(int32_t ncw) { return 4ull * ncw + 4ull * (ncw / CBM_SB); }
static_assert(cbm_lds_bytes(CBM_MAXW) + 512 <= 160 * 1024, "column bitmap beyond the LDS");
static_assert(32ll * CBM_MAXW == CBM_MAX_COLS && cbm_words(CBM_MAX_COLS) == CBM_MAXW, "ias_internal.hpp's limit");

struct CbmArgs {
    const int32_t *tcol;   // the rows' product columns (k_expand_part, every row)
    const RowRef *list;   // ref.q0: the row's work space (2 words per product), ref.n: products
    int32_t ncw;
    uint2 *work;
    Bitmap bm;
    int32_t *nnz_row;
    const int64_t *dup_off;
    int32_t *dupn, *gdupt;
    int32_t div, dmax;
    int32_t own_cap;   // LDS words beyond the bitmap + prefixes (the minima table when it fits)
    int32_t force;     // test knob (IAS_CBM_FORCE): CBM_NO_LIST / CBM_NO_LWORDS force those branches
    uint32_t *hits;    // test knob: the branches the rows took (CBM_HIT_*, OR-ed), or nullptr
    // column slices (k_sym_cbm<true>, C wider than one bitmap): slices per
    // row, the rows listed, each row's work-space cursor (zeroed) and the
    // duplicate pairs' list (k_dup_place places them)
    int32_t nslice;
    int32_t nrows;
    unsigned long long *wcur;
    uint2 *gpairs;
};
// IAS_CBM_FORCE bits (own_cap = 0 forces the global minima table) and the
// branch flags k_sym_cbm ORs into CbmArgs::hits
constexpr int32_t CBM_GLOBAL_OWN = 1, CBM_NO_LIST = 2, CBM_NO_LWORDS = 4;
constexpr uint32_t CBM_HIT_GLOBAL_OWN = 1, CBM_HIT_UNLISTED_KEEP = 2, CBM_HIT_UNLISTED_DROP = 4,
                   CBM_HIT_GLOBAL_WORDS = 8, CBM_HIT_LISTED_KEEP = 16, CBM_HIT_LISTED_DROP = 32,
                   CBM_HIT_LDS_OWN = 64;
static_assert(CBM_HIT_GLOBAL_OWN == IAS_DIAG_CBM_GLOBAL_OWN && CBM_HIT_UNLISTED_KEEP == IAS_DIAG_CBM_UNLISTED_KEEP &&
                  CBM_HIT_UNLISTED_DROP == IAS_DIAG_CBM_UNLISTED_DROP &&
                  CBM_HIT_GLOBAL_WORDS == IAS_DIAG_CBM_GLOBAL_WORDS && CBM_HIT_LISTED_KEEP == IAS_DIAG_CBM_LISTED_KEEP &&
                  CBM_HIT_LISTED_DROP == IAS_DIAG_CBM_LISTED_DROP && CBM_HIT_LDS_OWN == IAS_DIAG_CBM_LDS_OWN,
              "ias_last_diag flags");

// Workgroup-only sharing in k_sym_cbm: plain stores and loads meet in the
// CU's L1 after a barrier; values changed by global atomics (performed in
// L2) are read past the L1 with this load.  No device-scope fence: on gfx950
// one writes back and invalidates the XCD's L2.
__device__ __forceinline__ uint32_t ld_agent(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// SL (round 6): C wider than one LDS bitmap (K4: 8.4 M columns).  One
// workgroup per (row, column slice of 32 * ncw columns): the passes above
// restricted to the products whose column falls in the slice (every sweep
// reads the row's whole expansion, L2-resident: a row's slices share an XCD
// and run together), the slice's part of the row's work space reserved by a
// count pass, the duplicate bits cleared in the row's global first-touch
// words (preset to all ones by k_expand_flat), nnz and the duplicate pairs
// added to the row's (k_bitmap_prefix and k_dup_place finish, as for the
// hash partitions).  No hash partitions, no bucket pass.
template <bool SL>
__global__ __launch_bounds__(CBM_BLOCK) void k_sym_cbm(CbmArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t cbm[];
    __shared__ int scratch[64];
    __shared__ int ncnt[3];
    __shared__ unsigned long long sl_base[2];
    const int NCW = a.ncw;
    uint32_t *spre = cbm + NCW;
    // SL: workgroup b -> (row index, slice); the slices of a row are b, b + 8,
    // ... (one XCD by the dispatcher's round robin, its L2 keeps the row's
    // expansion), eight rows interleaved
    int32_t ridx = (int32_t)blockIdx.x, slice = 0;
    if constexpr (SL) {
        const int32_t per = 8 * a.nslice;
        const int32_t g = (int32_t)blockIdx.x / per, rem = (int32_t)blockIdx.x % per;
        slice = rem / 8;
        ridx = g * 8 + rem % 8;
        if (ridx >= a.nrows) return;
    }
    const RowRef ref = a.list[ridx];
    const int32_t row = ref.row;
    const int32_t P = ref.n;
    const int32_t cbase = slice * 32 * NCW;   // the slice's first column
    const int tid = (int)threadIdx.x, lane = tid & (WAVE - 1);
    const uint64_t lt = (1ull << lane) - 1ull;
    uint32_t *wk = (uint32_t *)(a.work + ref.q0);   // 2 P words (SL: 2 PS words of them, below)
    Timer tmr;   // phases (IAS_TIMING builds): 0 pass 1, 1 multi bitmap, 2 ranks, 3 pass 2, 4 pass 3, 5 prefixes, 6 placement
    tmr.start();
    for (int i = tid; i < NCW / 4; i += CBM_BLOCK) ((uint4 *)cbm)[i] = make_uint4(0u, 0u, 0u, 0u);
    if (tid < 3) ncnt[tid] = 0;
    __syncthreads();
    // the row's product columns from its expansion (k_expand_part): flat,
    // coalesced, lanes on consecutive products; blocks of U per lane, the
    // next block's loads issued before this block's work (2U in flight)
    constexpr int U = CBM_U;
    const int32_t *tc = a.tcol + ref.q0;
    // SL: columns relative to the slice; a product of another slice reads as
    // -1 and takes no part (insl)
    const uint32_t sw = 32u * (uint32_t)NCW;
    auto load = [&](int32_t b0, int32_t(&c)[U]) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int32_t p = b0 + u * CBM_BLOCK + tid;
            c[u] = p < P ? tc[p] : 0;
            if constexpr (SL) c[u] = p < P && (uint32_t)(c[u] - cbase) < sw ? c[u] - cbase : -1;
        }
    };
    auto insl = [&](int32_t c) -> bool { return !SL || c >= 0; };
    // blockwise: work(b0, c) gets U columns per lane (products b0 + u *
    // CBM_BLOCK + tid), so its LDS operations are issued U at a time
    auto sweep = [&](auto &&work) {
        int32_t ca[U], cb[U];
        constexpr int32_t STEP = U * CBM_BLOCK;
        load(0, ca);
        for (int32_t b0 = 0; b0 < P; b0 += 2 * STEP) {
            if (b0 + STEP < P) load(b0 + STEP, cb);
            work(b0, ca);
            if (b0 + STEP >= P) break;
            if (b0 + 2 * STEP < P) load(b0 + 2 * STEP, ca);
            work(b0 + STEP, cb);
        }
    };
    // wave-aggregated append of up to N items per lane (item j present when
    // on[j]) to LDS counter k: item j of all lanes takes consecutive slots,
    // lane order, so each item's stores are one contiguous run (a lane's own
    // run of slots would scatter every store instruction over 64 lines)
    auto append = [&](auto const &on, auto &at, int k) {
        constexpr int N = sizeof(on) / sizeof(on[0]);
        uint64_t m[N];
        int tot = 0, off[N];
#pragma unroll
        for (int j = 0; j < N; ++j) {
            m[j] = __ballot(on[j]);
            off[j] = tot;
            tot += (int)__popcll(m[j]);
        }
        int base = 0;
        if (lane == 0 && tot > 0) base = atomicAdd(&ncnt[k], tot);
        base = __shfl(base, 0);
#pragma unroll
        for (int j = 0; j < N; ++j) at[j] = base + off[j] + (int)__popcll(m[j] & lt);
    };
    // wave-aggregated slot of an LDS counter
    auto slot = [&](bool on, int k) -> int {
        const uint64_t m = __ballot(on);
        int at = 0;
        if (m) {
            if (lane == 0) at = atomicAdd(&ncnt[k], (int)__popcll(m));
            at = __shfl(at, 0) + (int)__popcll(m & lt);
        }
        return at;
    };
    // SL: the slice's products (PS) and its 2 PS words of the row's work space
    int32_t PS = P;
    if constexpr (SL) {
        int cnt = 0;
        sweep([&](int32_t b0, const int32_t(&c)[U]) {
#pragma unroll
            for (int u = 0; u < U; ++u) cnt += (b0 + u * CBM_BLOCK + tid < P && c[u] >= 0) ? 1 : 0;
        });
        int tot;
        (void)Team<CBM_BLOCK>::excl_sum(cnt, tot, scratch);
        PS = tot;
        if (tid == 0) sl_base[0] = PS > 0 ? atomicAdd(&a.wcur[ridx], 2ull * (unsigned long long)PS) : 0ull;
        __syncthreads();
        if (PS == 0) return;
        wk += sl_base[0];
    }
    // ---- 1. distinct columns; the duplicates list their column
    sweep([&](int32_t b0, const int32_t(&c)[U]) {
        uint32_t old[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            old[u] = 0u;
            if (b0 + u * CBM_BLOCK + tid < P && insl(c[u])) old[u] = atomicOr(&cbm[c[u] >> 5], 1u << (c[u] & 31));
        }
        bool dup[U];
        int at[U];
#pragma unroll
        for (int u = 0; u < U; ++u) dup[u] = insl(c[u]) && ((old[u] >> (c[u] & 31)) & 1u);
        append(dup, at, 0);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (dup[u]) wk[at[u]] = (uint32_t)c[u];
    });
    __syncthreads();
    tmr.mark(0);
    const int32_t nd = ncnt[0];
    const int32_t nnz = PS - nd;
    const int32_t W = (P + 31) >> 5;
    uint32_t *gbits = a.bm.bits + a.bm.off[row];
    uint32_t *gpref = a.bm.pref + a.bm.off[row];
    const int32_t cap = a.div > 0 ? min(P / a.div, a.dmax) : 0;
    // SL: the slice's pairs go to the row's list at a reserved offset (the
    // row's count, dupn, decides the path in k_dup_place); kept while they fit
    bool keep = nd <= cap;
    if constexpr (SL) {
        if (tid == 0) sl_base[1] = (nd > 0 && cap > 0) ? (unsigned long long)atomicAdd(&a.dupn[row], nd) : 0ull;
        __syncthreads();
        keep = cap > 0 && (int64_t)sl_base[1] + nd <= cap;
    }
    int M = 0;   // columns of more than one product
    uint2 *pairs = nullptr;   // the duplicates (product, first touch) when kept
    bool lwords = false;      // first-touch words in LDS (over the dead column bitmap)
    uint32_t hit = 0u;        // branches taken (test knob)
    auto full_word = [&](int32_t i) -> uint32_t {
        return (i < W - 1 || (P & 31) == 0) ? ~0u : ((1u << (P & 31)) - 1u);
    };
    if (nd > 0) {
        // ---- 2. columns of more than one product + their ranks
        for (int i = tid; i < NCW / 4; i += CBM_BLOCK) ((uint4 *)cbm)[i] = make_uint4(0u, 0u, 0u, 0u);
        __syncthreads();
        for (int32_t i = tid; i < nd; i += CBM_BLOCK) {
            const uint32_t c = wk[i];
            atomicOr(&cbm[c >> 5], 1u << (c & 31));
        }
        __syncthreads();
        tmr.mark(1);
        const int nsb = NCW / CBM_SB;
        constexpr int SPT = (CBM_MAXW / CBM_SB + CBM_BLOCK - 1) / CBM_BLOCK;   // superblocks per thread
        int v[SPT], sum = 0;
#pragma unroll
        for (int k = 0; k < SPT; ++k) {
            const int sb = tid * SPT + k;
            v[k] = 0;
            if (sb < nsb) {
                const uint4 x = ((const uint4 *)cbm)[2 * sb], y = ((const uint4 *)cbm)[2 * sb + 1];
                v[k] = __popc(x.x) + __popc(x.y) + __popc(x.z) + __popc(x.w) + __popc(y.x) + __popc(y.y) +
                       __popc(y.z) + __popc(y.w);
            }
            sum += v[k];
        }
        int run = Team<CBM_BLOCK>::excl_sum(sum, M, scratch);
#pragma unroll
        for (int k = 0; k < SPT; ++k) {
            const int sb = tid * SPT + k;
            if (sb < nsb) spre[sb] = (uint32_t)run;
            run += v[k];
        }
        // own[0, M): the smallest product per multi column — in the LDS beyond
        // the bitmap when it fits, else over the (dead) list in the work space
        // (two instantiations: a pointer that may be either compiles to flat
        // instructions, which wait on both the LDS and the memory counters)
        const bool own_l = M <= a.own_cap;
#if IAS_TIMING
        if (!own_l) tmr.acc[7] += 100;   // phase 7 reads as the share of rows with the global minima table
#endif
        auto multi = [&](int32_t c) -> bool { return (cbm[c >> 5] >> (c & 31)) & 1u; };
        // rank of a multi column from its superblock's 8 words and prefix
        auto rank_of = [&](int32_t c, const uint4 &x, const uint4 &y, uint32_t sp) -> uint32_t {
            const int kw = (c >> 5) & (CBM_SB - 1);
            const uint32_t wv[CBM_SB] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
            uint32_t r = sp;
#pragma unroll
            for (int i = 0; i < CBM_SB; ++i)
                r += (uint32_t)__popc(i < kw ? wv[i] : (i == kw ? wv[i] & ((1u << (c & 31)) - 1u) : 0u));
            return r;
        };
        auto rank = [&](int32_t c) -> uint32_t {   // three independent LDS reads
            const int sb = c >> 8;
            return rank_of(c, ((const uint4 *)cbm)[2 * sb], ((const uint4 *)cbm)[2 * sb + 1], spre[sb]);
        };
        auto passes = [&](auto tag) {
        constexpr bool OL = decltype(tag)::value;
        uint32_t *own = OL ? spre + nsb : wk;
        for (int32_t i = tid; i < M; i += CBM_BLOCK) own[i] = 0x7fffffffu;
        __syncthreads();
        tmr.mark(2);
        // ---- 3. first touch of each multi column; its products listed (p,
        // rank) when the list fits the work space.  Global own: products in
        // order, one above the column's current minimum issues no atomic (a
        // hub column's later products do not queue on one L2 address).
        const int32_t m0 = OL ? 0 : (M + 1) & ~1;
        const int32_t mcap = (2 * PS - m0) / 2;
        uint2 *ml = (uint2 *)(wk + m0);
        sweep([&](int32_t b0, const int32_t(&c)[U]) {
            bool on[U];
            uint32_t r[U];
#pragma unroll
            for (int u = 0; u < U; ++u) on[u] = b0 + u * CBM_BLOCK + tid < P && insl(c[u]) && multi(c[u]);
            // ranks of the multi products only: their superblocks' loads
            // first (masked to those lanes, all in flight), then the sums
            uint4 x[U], y[U];
            uint32_t sp[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                x[u] = y[u] = make_uint4(0u, 0u, 0u, 0u);
                sp[u] = 0u;
                if (on[u]) {
                    const int sb = c[u] >> 8;
                    x[u] = ((const uint4 *)cbm)[2 * sb];
                    y[u] = ((const uint4 *)cbm)[2 * sb + 1];
                    sp[u] = spre[sb];
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) r[u] = rank_of(c[u], x[u], y[u], sp[u]);
            uint32_t cur[U];   // global own: the current minima, all loads in flight
#pragma unroll
            for (int u = 0; u < U; ++u) cur[u] = (!OL && on[u]) ? ld_agent(&own[r[u]]) : ~0u;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t p = (uint32_t)(b0 + u * CBM_BLOCK + tid);
                if (on[u] && cur[u] > p) atomicMin(&own[r[u]], p);
            }
            int at[U];
            append(on, at, 2);
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (on[u] && at[u] < mcap) ml[at[u]] = make_uint2((uint32_t)(b0 + u * CBM_BLOCK + tid), r[u]);
        });
        __syncthreads();
        tmr.mark(3);
        // ---- 4. duplicates: clear their first-touch bits, list (product, first touch)
        const int32_t nml = ncnt[2];
        const bool listed = !(a.force & CBM_NO_LIST) && nml + ((keep && !SL) ? nd : 0) <= mcap;   // + room for the pairs
        pairs = SL ? a.gpairs + a.dup_off[row] + sl_base[1] : (uint2 *)(wk + (listed ? m0 + 2 * nml : m0));
        lwords = !SL && listed && W <= NCW && !(a.force & CBM_NO_LWORDS);
        hit = (OL ? CBM_HIT_LDS_OWN : CBM_HIT_GLOBAL_OWN) | (lwords ? 0u : CBM_HIT_GLOBAL_WORDS) |
              (listed ? (keep ? CBM_HIT_LISTED_KEEP : CBM_HIT_LISTED_DROP)
                      : (keep ? CBM_HIT_UNLISTED_KEEP : CBM_HIT_UNLISTED_DROP));
        if (lwords) {
            for (int32_t i = tid; i < W; i += CBM_BLOCK) cbm[i] = full_word(i);
            __syncthreads();
        } else if (!SL) {   // SL: preset by k_expand_flat (the row's slices share the words)
            for (int32_t i = tid; i < W; i += CBM_BLOCK) gbits[i] = full_word(i);
            __syncthreads();
        }
        if (listed) {   // CBM_L items per lane per step, each stage's loads in flight together
            for (int32_t i0 = 0; i0 < nml; i0 += CBM_L * CBM_BLOCK) {
                uint2 e[CBM_L];
                uint32_t f[CBM_L];
#pragma unroll
                for (int j = 0; j < CBM_L; ++j) {
                    const int32_t i = i0 + j * CBM_BLOCK + tid;
                    e[j] = i < nml ? ml[i] : make_uint2(0u, 0u);
                }
#pragma unroll
                for (int j = 0; j < CBM_L; ++j) {
                    const bool in = i0 + j * CBM_BLOCK + tid < nml;
                    f[j] = !in ? 0u : (OL ? own[e[j].y] : ld_agent(&own[e[j].y]));
                }
                bool dup[CBM_L];
#pragma unroll
                for (int j = 0; j < CBM_L; ++j) {
                    dup[j] = i0 + j * CBM_BLOCK + tid < nml && f[j] != e[j].x;
                    if (dup[j]) {
                        const uint32_t m = ~(1u << (e[j].x & 31));
                        if (lwords) atomicAnd(&cbm[e[j].x >> 5], m);
                        else atomicAnd(&gbits[e[j].x >> 5], m);
                    }
                }
                if (keep) {
                    int at[CBM_L];
                    append(dup, at, 1);
#pragma unroll
                    for (int j = 0; j < CBM_L; ++j)
                        if (dup[j]) pairs[at[j]] = make_uint2(e[j].x, f[j]);
                }
            }
        } else {
            sweep([&](int32_t b0, const int32_t(&c)[U]) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int32_t p = b0 + u * CBM_BLOCK + tid;
                    uint32_t f = 0u;
                    bool dup = false;
                    if (p < P && insl(c[u]) && multi(c[u])) {
                        const uint32_t r = rank(c[u]);
                        f = OL ? own[r] : ld_agent(&own[r]);
                        dup = f != (uint32_t)p;
                    }
                    // the lanes' products are consecutive: one atomic per bitmap word
                    const uint64_t dm = __ballot(dup);
                    if (dup) {
                        const int32_t pb = p - lane, wi = p >> 5;
                        const int lo = max(0, wi * 32 - pb), hi = min(WAVE - 1, wi * 32 + 31 - pb);
                        const uint64_t mine = dm & (((1ull << (hi - lo + 1)) - 1ull) << lo);
                        if (lane == __builtin_ctzll(mine))
                            atomicAnd(&gbits[wi], ~((uint32_t)(mine >> lo) << ((pb + lo) & 31)));
                    }
                    if (keep) {
                        const int at = slot(dup, 1);
                        if (dup) pairs[at] = make_uint2((uint32_t)p, f);
                    }
                }
            });
        }
        };
        if (own_l) passes(std::true_type{});
        else passes(std::false_type{});
    }
    __syncthreads();
    tmr.mark(4);
    if constexpr (SL) {   // prefixes and placement: k_bitmap_prefix, k_dup_place
        if (tid == 0) {
            atomicAdd(&a.nnz_row[row], nnz);
            if (a.hits && hit) atomicOr(a.hits, hit);
        }
        return;
    }
    // ---- words (from the LDS, or all ones without duplicates) and their
    // prefixes, tiles of CBM_BLOCK words, carried
    auto word = [&](int32_t i) -> uint32_t {
        return nd == 0 ? full_word(i) : (lwords ? cbm[i] : ld_agent(&gbits[i]));
    };
    int carry = 0;
    for (int32_t w0 = 0; w0 < W; w0 += CBM_BLOCK) {
        const int32_t i = w0 + tid;
        const uint32_t wv = i < W ? word(i) : 0u;
        int tot;
        const int ex = Team<CBM_BLOCK>::excl_sum(__popc(wv), tot, scratch);
        if (i < W) {
            gpref[i] = (uint32_t)(carry + ex);
            if (nd == 0 || lwords) gbits[i] = wv;
        }
        carry += tot;
    }
    tmr.mark(5);
    if (nd > 0 && keep) {   // duplicates at their product-order index d = p - rank(p)
        __syncthreads();
        int32_t *dt = a.gdupt + a.dup_off[row];
        for (int32_t i = tid; i < nd; i += CBM_BLOCK) {
            const uint2 e = pairs[i];
            const uint32_t wi = e.x >> 5;
            const uint32_t rk = gpref[wi] + (uint32_t)__popc(word((int32_t)wi) & ((1u << (e.x & 31)) - 1u));
            dt[e.x - rk] = (int32_t)e.y;
        }
    }
    if (tid == 0) {
        a.nnz_row[row] = nnz;
        a.dupn[row] = keep ? nd : -1;
        if (a.hits && hit) atomicOr(a.hits, hit);
    }
    tmr.mark(6);
    tmr.flush(28, tid == 0);   // slot 28: column-bitmap symbolic
}

// ---------------------------------------------------------------- numeric kernels
// Value bins: LDS layout per team [vals 8S | keys 4S | meta 4S | segment | scratch].
template <int TEAM, int K, int SEG, int TPW, int PER>
__global__ __launch_bounds__(TEAM *TPW) void k_numeric_val(AxView ax, Rows B, const RowRef *list,
                                                            int32_t count, uint32_t S, Out out) {
    static_assert(TEAM <= 64 || TPW == 1, "multi-wave teams own their workgroup");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int team = (TPW == 1) ? 0 : (int)(threadIdx.x / TEAM);
    unsigned char *base = smem + (size_t)team * val_team_bytes<SEG>(S);
    double *vals = (double *)base;
    int32_t *keys = (int32_t *)(base + round16(8ull * S));
    uint32_t *meta = (uint32_t *)(base + round16(8ull * S) + round16(4ull * S));
    unsigned char *fixed = base + round16(8ull * S) + 2 * round16(4ull * S);
    auto &seg = *(Seg<SEG, true> *)fixed;
    int *scratch = (int *)(fixed + round16(sizeof(Seg<SEG, true>)));
    const RowRef ref = ref_at(list, (int64_t)blockIdx.x * TPW + team, count);
    NumTable<false> tb{keys, meta, vals, S};
    numeric_row<TEAM, K, SEG, M_VAL, PER>(ax, B, ref, tb, 0, 1, nullptr, nullptr, seg, scratch, out,
                                          nullptr);
}

// Direct-write bins: LDS layout per team [keys 4S | meta 4S | segment | scratch].
template <int TEAM, int K, int SEG, int TPW>
__global__ __launch_bounds__(TEAM *TPW) void k_numeric_dw(AxView ax, Rows B, const RowRef *list,
                                                           int32_t count, uint32_t S, Out out) {
    static_assert(TEAM <= 64 || TPW == 1, "multi-wave teams own their workgroup");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int team = (TPW == 1) ? 0 : (int)(threadIdx.x / TEAM);
    unsigned char *base = smem + (size_t)team * dw_team_bytes<SEG>(S);
    int32_t *keys = (int32_t *)base;
    uint32_t *meta = (uint32_t *)(base + round16(4ull * S));
    unsigned char *fixed = base + 2 * round16(4ull * S);
    auto &seg = *(Seg<SEG, true> *)fixed;
    int *scratch = (int *)(fixed + round16(sizeof(Seg<SEG, true>)));
    const RowRef ref = ref_at(list, (int64_t)blockIdx.x * TPW + team, count);
    NumTable<false> tb{keys, meta, nullptr, S};
    numeric_row<TEAM, K, SEG, M_DW, 1>(ax, B, ref, tb, 0, 1, nullptr, nullptr, seg, scratch, out,
                                       nullptr);
}

// One workgroup per (row, hash partition), direct write, ranks from the bitmap.
template <int TEAM, int K, int LOG2S, int SEG>
__global__ __launch_bounds__(TEAM) void k_numeric_part(AxView ax, Rows B, const PartItem *items,
                                                       Bitmap bm, Out out, int *overflow) {
    __shared__ __attribute__((aligned(16))) int32_t keys[1 << LOG2S];
    __shared__ uint32_t meta[1 << LOG2S];
    __shared__ Seg<SEG, true> seg;
    __shared__ int scratch[64];
    const PartItem it = items[blockIdx.x];
    const int64_t row = it.ref.row;
    NumTable<false> tb{keys, meta, nullptr, 1u << LOG2S};
    numeric_row<TEAM, K, SEG, M_DWPART, 1>(ax, B, it.ref, tb, it.part, it.nparts, bm.bits + bm.off[row],
                                           bm.pref + bm.off[row], seg, scratch, out, overflow);
}

// Duplicate fix-up of streaming rows with 17 - 256 duplicates: one wave per row,
// the list sorted in LDS (numeric_fixup_lds; the head scan it replaced was O(n^2)).
constexpr int FIX_TPW = 4;
__global__ __launch_bounds__(WAVE *FIX_TPW) void k_fixup(const RowRef *list, int32_t count, Bitmap bm,
                                                        const int64_t *dup_off, const int32_t *dupn,
                                                        const int32_t *gdupt, const double *gdupval,
                                                        Out out) {
    __shared__ unsigned long long key[FIX_TPW][2 * 256 + 256 / 64];
    const int team = threadIdx.x / WAVE;
    const int64_t idx = (int64_t)blockIdx.x * FIX_TPW + team;
    if (idx >= count) return;
    const int64_t row = list[idx].row;
    const int32_t nd = dupn[row];
    if (nd <= 0 || nd > 256) return;
    const int64_t off = bm.off[row];
    numeric_fixup_lds<WAVE, 256>(row, bm.bits + off, bm.pref + off, gdupt + dup_off[row],
                                 gdupval + dup_off[row], nd, key[team], out);
}

// Duplicate fix-up of streaming rows with short lists (<= 16): one lane per
// row, the list in registers, each column's products added in list order.
constexpr int FIX_TINY = 16;
__global__ __launch_bounds__(256) void k_fixup_tiny(const RowRef *list, int32_t count, Bitmap bm,
                                                    const int64_t *dup_off, const int32_t *dupn,
                                                    const int32_t *gdupt, const double *gdupval, Out out) {
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= count) return;
    const int64_t row = list[idx].row;
    const int32_t nd = dupn[row];
    if (nd <= 0 || nd > FIX_TINY) return;
    const int64_t off = dup_off[row];
    const uint32_t *bits = bm.bits + bm.off[row];
    const uint32_t *pref = bm.pref + bm.off[row];
    int32_t t[FIX_TINY];
    double v[FIX_TINY];
#pragma unroll
    for (int i = 0; i < FIX_TINY; ++i)
        if (i < nd) {
            t[i] = gdupt[off + i];
            v[i] = gdupval[off + i];
        }
    const int64_t st = out.start(row);
    const uint32_t nnz = (uint32_t)out.len[row];
#pragma unroll
    for (int i = 0; i < FIX_TINY; ++i) {
        if (i >= nd) break;
        bool head = true;
#pragma unroll
        for (int j = 0; j < FIX_TINY; ++j)
            if (j < i && t[j] == t[i]) head = false;
        if (!head) continue;
        const uint32_t p = (uint32_t)t[i];
        const uint32_t rk = pref[p >> 5] + (uint32_t)__popc(bits[p >> 5] & ((1u << (p & 31)) - 1u));
        const int64_t pos = st + (out.order == 0 ? (int64_t)(nnz - 1u - rk) : (int64_t)rk);
        double a = out.val[pos];
#pragma unroll
        for (int j = 0; j < FIX_TINY; ++j)
            if (j >= i && j < nd && t[j] == t[i]) a = a + v[j];
        out.val[pos] = a;
    }
}

// Duplicate fix-up of streaming rows with long duplicate lists (sort-based).
// keys (then values) in dynamic LDS: 8 B each, + run-head bits (16384, 128 KB
// of LDS and one block per CU: K3 37.3 vs 36.0 ms)
constexpr int FIXBIG_CAP = 8192;
constexpr size_t FIXBIG_LDS = 8ull * FIXBIG_CAP + FIXBIG_CAP / 8;
// Lists of at most FIXMID_CAP: 256 lanes and 16 KB of LDS, so several rows per
// CU (and room beside the streaming pass's waves); longer lists: k_fixup_large
// / k_fixup_big.
constexpr int FIXMID_CAP = 1024;
__global__ __launch_bounds__(256) void k_fixup_mid(const RowRef *list, int32_t count, Bitmap bm,
                                                  const int64_t *dup_off, const int32_t *dupn,
                                                  const int32_t *gdupt, const double *gdupval, Out out) {
    __shared__ unsigned long long key[2 * FIXMID_CAP + FIXMID_CAP / 64];
    const int64_t row = list[blockIdx.x].row;
    const int32_t nd = dupn[row];
    if (nd <= 0 || nd > FIXMID_CAP) return;
    const int64_t off = bm.off[row];
    numeric_fixup_lds<256, FIXMID_CAP>(row, bm.bits + off, bm.pref + off, gdupt + dup_off[row],
                                       gdupval + dup_off[row], nd, key, out);
}
// Lists of FIXMID_CAP+1 .. FIXLARGE_CAP: 256 lanes and 64 KB, small enough to
// sit beside the streaming pass's waves on a CU.
constexpr int FIXLARGE_CAP = 4096;
constexpr size_t FIXLARGE_LDS = 8ull * (2 * FIXLARGE_CAP + FIXLARGE_CAP / 64);
__global__ __launch_bounds__(256) void k_fixup_large(const RowRef *list, int32_t count, Bitmap bm,
                                                    const int64_t *dup_off, const int32_t *dupn,
                                                    const int32_t *gdupt, const double *gdupval, Out out) {
    extern __shared__ unsigned long long key[];   // FIXLARGE_LDS bytes (dynamic: > 64 KB)
    const int64_t row = list[blockIdx.x].row;
    const int32_t nd = dupn[row];
    if (nd <= FIXMID_CAP || nd > FIXLARGE_CAP) return;
    const int64_t off = bm.off[row];
    numeric_fixup_lds<256, FIXLARGE_CAP>(row, bm.bits + off, bm.pref + off, gdupt + dup_off[row],
                                         gdupval + dup_off[row], nd, key, out);
}
__global__ __launch_bounds__(1024) void k_fixup_big(const RowRef *list, int32_t count, Bitmap bm,
                                                   const int64_t *dup_off, const int32_t *dupn,
                                                   const int32_t *gdupt, const double *gdupval, Out out) {
    extern __shared__ unsigned long long key[];
    const int64_t row = list[blockIdx.x].row;
    const int32_t nd = dupn[row];
    if (nd <= FIXLARGE_CAP || nd > FIXBIG_CAP) return;
    const int64_t off = bm.off[row];
    numeric_fixup_big<1024, FIXBIG_CAP>(row, bm.bits + off, bm.pref + off, gdupt + dup_off[row],
                                        gdupval + dup_off[row], nd, key, out);
}

// Row-wise analysis helpers: product offset of every row, and the expansion
// of every A entry's products into tcol (one wave per FLAT_CHUNK entries,
// lanes over the chunk's products: coalesced B-row reads, contiguous writes).
__global__ void k_row_poff(Rows A, int64_t rows, const int64_t *axp, int64_t n_entries, int64_t *poff,
                           Counters *cnt) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r > rows) return;
    if (r == rows) {
        poff[r] = axp[n_entries];
        return;
    }
    int64_t s;
    int32_t n;
    A.row(r, s, n);
    int64_t q = s - A.base();
    if (q < 0 || n < 0 || q + n > n_entries) {   // row pointer disagrees with the declared entry count
        cnt->overflow = 1;
        q = q < 0 ? 0 : (q > n_entries ? n_entries : q);
    }
    poff[r] = axp[q];
}


template <int TEAM, int K, int SEG>
__global__ __launch_bounds__(TEAM) void k_numeric_global(AxView ax, Rows B, const RowRef *list,
                                                         const int64_t *ws_off, int32_t count,
                                                         char *ws, Out out) {
    __shared__ Seg<SEG, true> seg;
    __shared__ int scratch[64];
    const int64_t idx = blockIdx.x;
    if (idx >= count) return;
    const RowRef ref = list[idx];
    const unsigned long long k = (unsigned long long)out.len[ref.row];
    const unsigned long long need = k + (k + 1) / 2;
    uint32_t l2 = 0;
    while ((1ull << l2) < need) ++l2;
    // region of S * 20 bytes: keys (4 S) | meta (8 S) | vals (8 S)
    const uint64_t S = 1ull << l2;
    char *base = ws + (uint64_t)ws_off[idx] * 20ull;
    NumTable<true> tb{(int32_t *)base, (unsigned long long *)(base + S * 4ull),
                      (double *)(base + S * 12ull), (uint32_t)S};
    numeric_row<TEAM, K, SEG, M_WIDE, 1>(ax, B, ref, tb, 0, 1, nullptr, nullptr, seg, scratch, out,
                                         nullptr);
}

// ---------------------------------------------------------------- scan
constexpr int SCAN_BLOCK = 256;
constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;
static_assert(SCAN_TILE == AN_BLOCK * AN_U, "k_an_entries blocks are scan tiles");

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

// single block: exclusive scan of partial[0..nb) in place; total -> partial[nb].
// Eight consecutive partials per thread (a chunk of 8,192 per pass: K3''s
// 10,234 tiles in two passes instead of ten, three barriers each).
__global__ __launch_bounds__(1024) void k_scan_partials(int64_t *partial, int64_t nb) {
    constexpr int PT = 8;
    __shared__ int64_t wsum[16];
    const int l = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
    int64_t carry = 0;
    for (int64_t b0 = 0; b0 < nb; b0 += 1024 * PT) {
        const int64_t k0 = b0 + (int64_t)threadIdx.x * PT;
        int64_t v[PT], run = 0;
#pragma unroll
        for (int j = 0; j < PT; ++j) v[j] = k0 + j < nb ? partial[k0 + j] : 0;
#pragma unroll
        for (int j = 0; j < PT; ++j) {
            const int64_t t = v[j];
            v[j] = run;
            run += t;
        }
        int64_t x = run;
#pragma unroll
        for (int d = 1; d < WAVE; d <<= 1) {
            const int64_t t = __shfl_up(x, d);
            if (l >= d) x += t;
        }
        if (l == WAVE - 1) wsum[w] = x;
        __syncthreads();
        int64_t before = 0, tot = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            before += i < w ? wsum[i] : 0;
            tot += wsum[i];
        }
        const int64_t b = carry + before + x - run;
#pragma unroll
        for (int j = 0; j < PT; ++j)
            if (k0 + j < nb) partial[k0 + j] = b + v[j];
        __syncthreads();   // wsum is rewritten by the next pass
        carry += tot;
    }
    if (threadIdx.x == 0) partial[nb] = carry;
}

// Thread t of a tile scans its SCAN_ITEMS consecutive entries in registers
// (two 16-byte loads when they are in range and aligned), the tile's thread
// sums are scanned once, and the results leave through LDS in lane order (an
// 8-byte lane each, 512 contiguous bytes per wave instruction).  The
// item-by-item form it replaces waited on one load and two barriers per item
// (K3' 72 us for 21 M entries, 3.5 TB/s).  LDS slot of entry e: e + e / 8
// (two dwords of padding per thread's run: 2-way bank conflicts at most).
static_assert(SCAN_ITEMS == 8, "k_scan_apply: two 16-byte loads per thread");
__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_apply(const int32_t *in, int64_t n,
                                                           const int64_t *partial,
                                                           int64_t *out) {
    __shared__ int64_t st[SCAN_TILE + SCAN_TILE / SCAN_ITEMS];
    __shared__ int64_t wsum[SCAN_BLOCK / WAVE];
    const int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
    const int t = (int)threadIdx.x, l = t & (WAVE - 1);
    const int64_t k0 = base + (int64_t)t * SCAN_ITEMS;
    int32_t v[SCAN_ITEMS];
    if (k0 + SCAN_ITEMS <= n && ((uintptr_t)in & 15u) == 0) {
        const int4 a = *(const int4 *)(in + k0), b = *(const int4 *)(in + k0 + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
        v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
#pragma unroll
        for (int j = 0; j < SCAN_ITEMS; ++j) v[j] = k0 + j < n ? in[k0 + j] : 0;
    }
    int64_t run = 0;
    int64_t loc[SCAN_ITEMS];
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        loc[j] = run;
        run += v[j];
    }
    int64_t x = run;
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
        const int64_t u = __shfl_up(x, d);
        if (l >= d) x += u;
    }
    if (l == WAVE - 1) wsum[t / WAVE] = x;
    __syncthreads();
    int64_t before = partial[blockIdx.x] + x - run;
#pragma unroll
    for (int w = 0; w < SCAN_BLOCK / WAVE; ++w) before += w < t / WAVE ? wsum[w] : 0;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) st[t * (SCAN_ITEMS + 1) + j] = before + loc[j];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        const int e = i * SCAN_BLOCK + t;
        if (base + e < n) out[base + e] = st[e + e / SCAN_ITEMS];
    }
    if (blockIdx.x == gridDim.x - 1 && t == 0) out[n] = partial[gridDim.x];
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
// IAS_ORDER_SORTED: rows up to `wide_min` - 1 entries (8,192 by default,
// IAS_SORT_WIDE_MIN lowers it) get a bucket sort in LDS (k_sort_bucket).
// Longer rows: the column bitmap sort (k_sort_bitmap) when C has at most 2^20
// columns, else one segmented radix sort over a compact workspace
// (k_wide_gather), or, when that workspace cannot be had (or
// IAS_SORT_GLOBAL=1), a bitonic sort per row in a global workspace
// (k_sort_global).  Columns of a row are distinct, so the order is unique.
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

// a bucket of more keys than this sends the row to the bitonic sort: its m^2 / TEAM
// rank loop then costs about what the bitonic sort does (32 = 8x the mean of
// 4 sent most of K3's R-MAT rows there: sorted K3' 19.5 -> 41.7 ms)
constexpr uint32_t SORTB_HEAVY = 256;

// A listed row's extent from its list entry (the sort binning stores the
// row's start relative to ptr[0] and its length): no dependent row-pointer
// load after the list entry's.
__device__ __forceinline__ void sort_ref_span(const RowRef &ref, const int64_t *ptr, int64_t &o, int32_t &n) {
    o = ref.q0 + (ptr ? ptr[0] : 0);
    n = ref.n;
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

__host__ __device__ constexpr int sort_pow2_floor(int x) { return x < 2 ? 1 : 2 * sort_pow2_floor(x / 2); }

// A team barrier for LDS only: waits for this wave's LDS operations, not for
// its global loads in flight (a workgroup fence waits for both, which would
// stall the sort's prefetch at the next barrier).  The "memory" clobber keeps
// the compiler from moving memory operations across it.
template <bool MULTI>
__device__ __forceinline__ void lds_sync() {
    if constexpr (MULTI) {
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    } else {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// Rows of up to TEAM * E entries sorted by a bucket pass in LDS: the row's
// columns are distinct, so an entry's sorted position is the number of the
// row's columns below it.  Buckets split the row's columns into nb ~ n/2 ..
// n/4 parts by a monotone map (bucket order is key order); an entry's
// position = its bucket's start (a scan of the bucket counts) + the keys of
// its bucket below it (values never leave registers).
//   * The map is equalised: R-MAT rows crowd their low columns (~n^0.74 of a
//     row's keys below column x^0.74), so equal-width buckets held 10 - 14
//     keys per key on average and a wave waited on its fullest lane.  A
//     coarse histogram (G equal-width bins) and its scan give each coarse bin
//     fine buckets in proportion to its keys: 6 - 7 keys per key.
//   * A lane's E bucket walks go in lockstep, the E reads of a step issued
//     together: one LDS round trip per step of the longest walk, not one per
//     key of every walk (modelled on K3''s rows: 217 -> 16 round trips per
//     wave on the 4,097 - 8,192-entry rows).
// Every team stages the sorted row in LDS and writes it out contiguously (the
// 1,024-lane teams in two halves of values, 72 KB: their scattered stores
// touched a cache line per lane).
template <int TEAM, int E, int TPW>
__global__ __launch_bounds__(TEAM *TPW) void k_sort_bucket(const RowRef *list, int32_t count,
                                                           const int64_t *ptr, int32_t *col, double *val) {
    static_assert(TEAM <= 64 || TPW == 1, "multi-wave teams own their workgroup");
    using TM = Team<TEAM>;
    constexpr int CAP = TEAM * E;
    constexpr int NBM = TEAM < 1024 ? CAP : CAP / 2;        // most buckets
    constexpr int NBT = (NBM + TEAM - 1) / TEAM;            // bucket counts per thread in the scan
    constexpr int SVC = TEAM < 1024 ? CAP : CAP / 2;        // values staged per round
    // coarse bins: as many as fit beside the bucket counts in the staging
    // area, at most 1,024 (finer bins equalise better: modelled on K3''s
    // rows, 256 -> 1,024 bins takes the walks 10.3 -> 8.4 steps per wave)
    constexpr int G = sort_pow2_floor((2 * SVC - NBM - 2) < 1024 ? (2 * SVC - NBM - 2) : 1024);
    constexpr int GT = (G + TEAM - 1) / TEAM;
    static_assert(2 * SVC >= NBM + G + 2, "the bucket counts and the coarse bins overlay the value staging");
    __shared__ int32_t sk[TPW][CAP];
    __shared__ double sv[TPW][SVC];
    __shared__ int scratch[TPW][64];
    const int team = (TPW == 1) ? 0 : (int)(threadIdx.x / TEAM);
    // the bucket counts / starts and the coarse bins live in the value
    // staging area, which is dead until the ranks are known
    uint32_t *const hist = (uint32_t *)sv[team];
    uint32_t *const gh = hist + NBM + 1;
    const int lane = TM::lane();
    // persistent teams: row i + 1's list entry is loaded at the top of row
    // i and its columns (with row i's values) once row i's buckets are
    // counted, so they arrive while row i is ranked and written (the load
    // chain was ~6 of a row's 13 - 20 us)
    const int64_t rstride = (int64_t)gridDim.x * TPW;
    int64_t idx = (int64_t)blockIdx.x * TPW + team;
    Timer tm;   // timing builds only (phases: 0 loads + range, 1 coarse bins, 2 fine buckets, 3 bucket scan,
                // 4 ranks, 5 staging, 6 stores issued)
    tm.start();
    RowRef ref = idx < count ? list[idx] : RowRef{0, -1, 0};
    int64_t o = 0;
    int32_t n = 0;
    if (ref.row >= 0) sort_ref_span(ref, ptr, o, n);
    int32_t c[E];
#pragma unroll
    for (int k = 0; k < E; ++k) {
        const int e = k * TEAM + lane;
        c[k] = e < n ? col[o + e] : 0;
    }
    while (ref.row >= 0) {   // uniform over the team
    const RowRef nref = idx + rstride < count ? list[idx + rstride] : RowRef{0, -1, 0};
    int32_t lo = INT32_MAX, hi = INT32_MIN;
#pragma unroll
    for (int k = 0; k < E; ++k)
        if (k * TEAM + lane < n) {
            lo = min(lo, c[k]);
            hi = max(hi, c[k]);
        }
    // the row's column range (team min / max)
    {
        constexpr int W = TEAM < WAVE ? TEAM : WAVE;
#pragma unroll
        for (int d = W / 2; d > 0; d >>= 1) {
            lo = min(lo, __shfl_xor(lo, d, W));
            hi = max(hi, __shfl_xor(hi, d, W));
        }
        if constexpr (TM::MULTI) {
            const int w = lane / WAVE;
            if ((lane & (WAVE - 1)) == 0) {
                scratch[0][2 * w] = lo;
                scratch[0][2 * w + 1] = hi;
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < TM::NWAVES; ++i) {
                lo = min(lo, scratch[0][2 * i]);
                hi = max(hi, scratch[0][2 * i + 1]);
            }
        }
    }
    tm.mark(0);
    // nb: a power of two in (n / 2, n] (at least 1, at most NBM): ~1.5 keys
    // per bucket (K3''s rows, equalised: 5 - 11 lockstep steps per wave)
    int nb = 1;
    while (nb < NBM && 2 * nb <= n) nb <<= 1;
    // coarse bins of 2^sh columns, fewer than G of them over [lo, hi]
    const uint32_t range = n > 0 ? (uint32_t)(hi - lo) : 0u;
    int sh = 0;
    while ((range >> sh) >= (uint32_t)G) ++sh;
    for (int i = lane; i <= nb; i += TEAM) hist[i] = 0u;
    for (int i = lane; i <= G; i += TEAM) gh[i] = 0u;
    TM::sync();   // (multi-wave: also every wave's min / max read before scratch is reused)
#pragma unroll
    for (int k = 0; k < E; ++k)
        if (k * TEAM + lane < n) atomicAdd(&gh[(uint32_t)(c[k] - lo) >> sh], 1u);
    TM::sync();
    {
        uint32_t cnt[GT], sum = 0;
#pragma unroll
        for (int j = 0; j < GT; ++j) {
            const int i = lane * GT + j;
            cnt[j] = i < G ? gh[i] : 0u;
            sum += cnt[j];
        }
        int tot;
        uint32_t run = (uint32_t)TM::excl_sum((int)sum, tot, scratch[team]);
        TM::sync();   // every count read before the starts overwrite them
#pragma unroll
        for (int j = 0; j < GT; ++j) {
            const int i = lane * GT + j;
            if (i < G) gh[i] = run;
            run += cnt[j];
        }
        if (lane == 0) gh[G] = (uint32_t)n;
    }
    TM::sync();
    tm.mark(1);
    // fine bucket: nb / n * (keys of the coarse bins below + the key's share
    // of its own bin's keys) — non-decreasing in the column (float products
    // and sums of non-negative terms round monotonically; a bin's share stays
    // at most its count, where the next bin starts)
    const float fnb = n > 0 ? (float)nb / (float)n : 0.0f;
    const float winv = 1.0f / (float)(1u << sh);
    int b[E];
    uint32_t pib[E];
#pragma unroll
    for (int k = 0; k < E; ++k) {
        const int e = k * TEAM + lane;
        b[k] = 0;
        pib[k] = 0u;
        if (e < n) {
            const uint32_t d = (uint32_t)(c[k] - lo), g = d >> sh;
            const uint32_t g0 = gh[g], g1 = gh[g + 1];
            const float t = (float)g0 + (float)(d & ((1u << sh) - 1u)) * ((float)(g1 - g0) * winv);
            b[k] = min((int)(t * fnb), nb - 1);
            pib[k] = atomicAdd(&hist[b[k]], 1u);
        }
    }
    TM::sync();
    tm.mark(2);
    // bucket starts: exclusive scan of the counts (NBT per thread, in order);
    // bits 16+ of the scanned value count the lanes holding a bucket of more
    // than SORTB_HEAVY keys (the in-bucket rank walk is quadratic)
    bool heavy;
    {
        uint32_t cnt[NBT], sum = 0;
        bool big = false;
#pragma unroll
        for (int j = 0; j < NBT; ++j) {
            const int i = lane * NBT + j;
            cnt[j] = i < nb ? hist[i] : 0u;
            sum += cnt[j];
            big = big || cnt[j] > SORTB_HEAVY;
        }
        int tot;
        uint32_t run = (uint32_t)TM::excl_sum((int)(sum | (big ? 1u << 16 : 0u)), tot, scratch[team]) & 0xffffu;
        heavy = (tot >> 16) != 0;
        TM::sync();   // every count read before the starts overwrite them
#pragma unroll
        for (int j = 0; j < NBT; ++j) {
            const int i = lane * NBT + j;
            if (i < nb) hist[i] = run;
            run += cnt[j];
        }
        if (lane == 0) hist[nb] = (uint32_t)n;
    }
    TM::sync();
    tm.mark(3);
    // this row's values and the next row's columns, in flight from here
    // (the values are first needed by the staging)
    int64_t no = 0;
    int32_t nn = 0;
    if (nref.row >= 0) sort_ref_span(nref, ptr, no, nn);
    double v[E];
    int32_t cn[E];
#pragma unroll
    for (int k = 0; k < E; ++k) {
        const int e = k * TEAM + lane;
        v[k] = e < n ? val[o + e] : 0.0;
        cn[k] = e < nn ? col[no + e] : 0;
    }
    uint32_t r[E];
    if (!heavy) {
        // each bucket's start and size read once: for the key's slot and its walk
        uint32_t s0[E], sz[E], mx = 0u;
#pragma unroll
        for (int k = 0; k < E; ++k) {
            s0[k] = 0u;
            sz[k] = 0u;
            if (k * TEAM + lane < n) {
                s0[k] = hist[b[k]];
                sz[k] = hist[b[k] + 1] - s0[k];
                sk[team][s0[k] + pib[k]] = c[k];
            }
            r[k] = s0[k];
            mx = max(mx, sz[k]);
        }
        lds_sync<TM::MULTI>();
        // lockstep steps: the E reads of a step are issued before any compare;
        // a finished walk's lanes are masked off its read (the walks are
        // LDS-bound: a clamped read still took its bank cycles)
        for (uint32_t j = 0; j < mx; ++j) {
            int32_t kj[E];
#pragma unroll
            for (int k = 0; k < E; ++k) {
                kj[k] = INT32_MAX;
                if (j < sz[k]) kj[k] = sk[team][s0[k] + j];
            }
#pragma unroll
            for (int k = 0; k < E; ++k) r[k] += kj[k] < c[k] ? 1u : 0u;
        }
    } else {
        // skewed buckets: the keys alone sorted in LDS (bitonic, padded to a
        // power of two), each entry's rank by a binary search of its key —
        // the keys are distinct, so the rank is exact
        uint32_t cap = 1;
        while (cap < (uint32_t)n) cap <<= 1;
#pragma unroll
        for (int k = 0; k < E; ++k) {
            const int e = k * TEAM + lane;
            if ((uint32_t)e < cap) sk[team][e] = e < n ? c[k] : INT32_MAX;
        }
        lds_sync<TM::MULTI>();
        bitonic_lds<TEAM, CAP>(sk[team], cap);
#pragma unroll
        for (int k = 0; k < E; ++k) {
            r[k] = 0u;
            if (k * TEAM + lane >= n) continue;
            uint32_t lo2 = 0, hi2 = (uint32_t)n;   // first key >= c[k]
            while (lo2 < hi2) {
                const uint32_t mid = (lo2 + hi2) >> 1;
                if (sk[team][mid] < c[k]) lo2 = mid + 1;
                else hi2 = mid;
            }
            r[k] = lo2;
        }
    }
    // the entries land at their ranks in LDS, then leave in order (a lane's
    // scattered global store touched its own cache line)
    lds_sync<TM::MULTI>();   // every rank read of sk done
    tm.mark(4);
#pragma unroll
    for (int k = 0; k < E; ++k)
        if (k * TEAM + lane < n) {
            sk[team][r[k]] = c[k];
            if (r[k] < (uint32_t)SVC) sv[team][r[k]] = v[k];
        }
    lds_sync<TM::MULTI>();
    tm.mark(5);
    for (int e = lane; e < n; e += TEAM) {
        col[o + e] = sk[team][e];
        if (e < SVC) val[o + e] = sv[team][e];
    }
    if constexpr (SVC < CAP) {
        if (n > SVC) {   // uniform: one team per workgroup here
            lds_sync<TM::MULTI>();
#pragma unroll
            for (int k = 0; k < E; ++k)
                if (k * TEAM + lane < n && r[k] >= (uint32_t)SVC) sv[team][r[k] - SVC] = v[k];
            lds_sync<TM::MULTI>();
            for (int e = SVC + lane; e < n; e += TEAM) val[o + e] = sv[team][e - SVC];
        }
    }
    lds_sync<TM::MULTI>();   // the staging read out before the next row's counts overwrite it
    tm.mark(6);
    tm.done();
#pragma unroll
    for (int k = 0; k < E; ++k) c[k] = cn[k];
    ref = nref;
    o = no;
    n = nn;
    idx += rstride;
    }
    tm.flush(TEAM == 64 ? (E == 8 ? 12 : 11) : 6 + ilog2(TEAM), lane == 0 && team == 0);   // slots 11 - 16
}

__global__ __launch_bounds__(1024) void k_sort_global(const RowRef *list, int32_t count,
                                                      const int64_t *ws_off, const int64_t *ptr,
                                                      const int32_t *len, int64_t stride,
                                                      int32_t *col, double *val, char *ws) {
    const int64_t idx = blockIdx.x;
    if (idx >= count) return;
    const int64_t row = list[idx].row;
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

// Rows beyond the LDS bins: sorted by a column bitmap when C has at most
// SORTBM_COLS columns (C's columns are distinct within a row): every entry
// sets its column's bit in LDS, a prefix of popcounts (per 8 words) gives
// each column its sorted position.  O(n + cols/32) per row against a
// segmented radix sort's passes over its keys.  Bitmap: 128 KB of LDS + 16 KB
// of prefixes.
constexpr int SORTBM_T = 1024;
constexpr int32_t SORTBM_COLS = 1 << 20;
static_assert(SORTBM_COLS / 256 <= SORTBM_T * 4, "bitmap_prefix8: at most four groups per thread");
// k_sort_bitmap stages SORTBM_W sorted positions at a time over the dead
// bitmap (12 B each: 120 KB)
constexpr int SORTBM_W = 10240;
constexpr size_t sortbm_area(int32_t cols) {
    const size_t bm = 4ull * (((size_t)cols + 255) / 256 * 8);
    const size_t st = 12ull * SORTBM_W;
    return bm > st ? bm : st;
}
constexpr size_t sortbm_lds(int32_t cols) {
    return sortbm_area(cols) + 4ull * (((size_t)cols + 255) / 256 + 1) + 4ull * 64;
}
// Sorted position of column c from the row's bitmap: the exclusive prefix of
// its 8-word group plus the popcounts of the group's words below it, the
// group read as two 16-byte loads (one LDS round trip; the word-by-word loop
// it replaces waited on up to seven).
__device__ __forceinline__ int bitmap_rank(const uint32_t *bits, const int32_t *pre8, uint32_t c) {
    const uint32_t wi = c >> 5, g = wi >> 3, j = wi & 7u;
    const uint4 a = ((const uint4 *)bits)[2 * g], b = ((const uint4 *)bits)[2 * g + 1];
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    int p = pre8[g];
#pragma unroll
    for (uint32_t q = 0; q < 8; ++q) {
        const uint32_t m = q < j ? ~0u : (q == j ? (1u << (c & 31)) - 1u : 0u);
        p += __popc(w[q] & m);
    }
    return p;
}

// Exclusive popcount prefix of every 8-word group of the bitmap (pre8[g]):
// whole groups per thread, each read as two 16-byte loads, the group sums
// kept in registers for the second half (one pass over the bitmap, where a
// word-by-word count pass and a prefix pass read it twice, one word per wait)
constexpr int SORTBM_GPT = 4;   // groups per thread: 2^20 columns = 4,096 groups
__device__ __forceinline__ void bitmap_prefix8(const uint32_t *bits, int32_t *pre8, int NW, int *scratch) {
    const int tid = (int)threadIdx.x, ng = NW / 8;
    const int gpt = (ng + SORTBM_T - 1) / SORTBM_T;
    int gs[SORTBM_GPT], cnt = 0;
#pragma unroll
    for (int j = 0; j < SORTBM_GPT; ++j) {
        const int g = tid * gpt + j;
        gs[j] = 0;
        if (j < gpt && g < ng) {
            const uint4 a = ((const uint4 *)bits)[2 * g], b = ((const uint4 *)bits)[2 * g + 1];
            gs[j] = __popc(a.x) + __popc(a.y) + __popc(a.z) + __popc(a.w) + __popc(b.x) + __popc(b.y) +
                    __popc(b.z) + __popc(b.w);
        }
        cnt += gs[j];
    }
    int tot;
    int run = Team<SORTBM_T>::excl_sum(cnt, tot, scratch);
#pragma unroll
    for (int j = 0; j < SORTBM_GPT; ++j) {
        const int g = tid * gpt + j;
        if (j < gpt && g < ng) pre8[g] = run;
        run += gs[j];
    }
}

// Rows longer than k_sort_bitmap16's (more than fit the registers): a pass
// sets the bitmap, the next ranks every entry and copies it with its
// position into the row's slot of a compact workspace (coalesced: the
// scattered 4- and 8-byte stores of every entry to its sorted slot it
// replaces took ~96 of a row's 120 us, one cache line per lane), then the
// sorted row is assembled SORTBM_W positions at a time in LDS over the dead
// bitmap and written out contiguously in place.  Passes take SORTBM_B
// entries per thread at a time, their loads issued together.
constexpr int SORTBM_B = 8;
__global__ __launch_bounds__(SORTBM_T) void k_sort_bitmap(const RowRef *list, int32_t count, const int64_t *ws_off,
                                                         const int64_t *ptr, int32_t *col, double *val,
                                                         int32_t ncols, int32_t *wcol, double *wval,
                                                         int32_t *wpos) {
    extern __shared__ __attribute__((aligned(16))) uint32_t sbm[];
    const int NW = (ncols + 255) / 256 * 8;   // bitmap words, a multiple of 8
    uint32_t *bits = sbm;
    int32_t *skey = (int32_t *)sbm;               // staging (after the bitmap is dead)
    double *sval = (double *)(sbm + SORTBM_W);
    int32_t *pre8 = (int32_t *)((char *)sbm + sortbm_area(ncols));   // exclusive popcount prefix per 8 words
    int *scratch = pre8 + NW / 8 + 1;
    const int tid = (int)threadIdx.x;
    constexpr int BT = SORTBM_B * SORTBM_T;
    Timer tm;   // timing builds only (phases: 0 row + clear, 1 bitmap, 2 prefix, 3 ranks + workspace, 4 windows)
    tm.start();
    for (int64_t idx = blockIdx.x; idx < count; idx += gridDim.x) {
        int64_t o;
        int32_t n;
        sort_ref_span(list[idx], ptr, o, n);
        const int64_t w0 = ws_off[idx];
        for (int i = tid; i < NW / 4; i += SORTBM_T) ((uint4 *)bits)[i] = make_uint4(0u, 0u, 0u, 0u);
        __syncthreads();
        tm.mark(0);
        for (int32_t e0 = 0; e0 < n; e0 += BT) {
            uint32_t c[SORTBM_B];
#pragma unroll
            for (int k = 0; k < SORTBM_B; ++k) {
                const int32_t e = e0 + k * SORTBM_T + tid;
                c[k] = e < n ? (uint32_t)col[o + e] : 0u;
            }
#pragma unroll
            for (int k = 0; k < SORTBM_B; ++k)
                if (e0 + k * SORTBM_T + tid < n) atomicOr(&bits[c[k] >> 5], 1u << (c[k] & 31));
        }
        __syncthreads();
        tm.mark(1);
        bitmap_prefix8(bits, pre8, NW, scratch);
        __syncthreads();
        tm.mark(2);
        for (int32_t e0 = 0; e0 < n; e0 += BT) {
            uint32_t c[SORTBM_B];
            double v[SORTBM_B];
#pragma unroll
            for (int k = 0; k < SORTBM_B; ++k) {
                const int32_t e = e0 + k * SORTBM_T + tid;
                c[k] = e < n ? (uint32_t)col[o + e] : 0u;
                v[k] = e < n ? val[o + e] : 0.0;
            }
#pragma unroll
            for (int k = 0; k < SORTBM_B; ++k) {
                const int32_t e = e0 + k * SORTBM_T + tid;
                if (e < n) {
                    wpos[w0 + e] = bitmap_rank(bits, pre8, c[k]);
                    wcol[w0 + e] = (int32_t)c[k];
                    wval[w0 + e] = v[k];
                }
            }
        }
        __threadfence_block();
        __syncthreads();   // the workspace written; the bitmap is dead
        tm.mark(3);
        for (int32_t lo = 0; lo < n; lo += SORTBM_W) {
            const uint32_t m = (uint32_t)min(SORTBM_W, n - lo);
            for (int32_t e0 = 0; e0 < n; e0 += BT) {
                uint32_t q[SORTBM_B];
                int32_t c[SORTBM_B];
                double v[SORTBM_B];
#pragma unroll
                for (int k = 0; k < SORTBM_B; ++k) {
                    const int32_t e = e0 + k * SORTBM_T + tid;
                    q[k] = e < n ? (uint32_t)(wpos[w0 + e] - lo) : ~0u;
                    c[k] = e < n ? wcol[w0 + e] : 0;
                    v[k] = e < n ? wval[w0 + e] : 0.0;
                }
#pragma unroll
                for (int k = 0; k < SORTBM_B; ++k)
                    if (q[k] < m) {
                        skey[q[k]] = c[k];
                        sval[q[k]] = v[k];
                    }
            }
            __syncthreads();
            for (uint32_t e = tid; e < m; e += SORTBM_T) {
                col[o + lo + e] = skey[e];
                val[o + lo + e] = sval[e];
            }
            __syncthreads();
        }
        tm.mark(4);
        tm.done();
    }
    tm.flush(18, tid == 0);
}

// Rows of 8,193 .. 16,384 entries (C has at most SORTBM_COLS columns): the
// column bitmap sort with the row held in registers (16 entries per lane,
// loaded once — the loop form above reloads them per phase, a global round
// trip each) and the sorted row staged in LDS over the dead bitmap, 8,192
// entries at a time, then written out contiguously in place.
constexpr int SORTB2_E = 16, SORTB2_CH = 8192;
constexpr size_t sortb2_lds(int32_t cols) {
    const size_t bm = 4ull * (((size_t)cols + 255) / 256 * 8);
    const size_t st = 12ull * SORTB2_CH;
    return (bm > st ? bm : st) + 4ull * (((size_t)cols + 255) / 256 + 1) + 4ull * 64;
}
__global__ __launch_bounds__(SORTBM_T) void k_sort_bitmap16(const RowRef *list, int32_t count, const int64_t *ptr,
                                                           const int32_t *len, int64_t stride, int32_t *col,
                                                           double *val, int32_t ncols) {
    extern __shared__ __attribute__((aligned(16))) uint32_t sbm[];
    const int NW = (ncols + 255) / 256 * 8;   // bitmap words, a multiple of 8
    const size_t area = sortb2_lds(ncols) - 4ull * (NW / 8 + 1) - 4ull * 64;   // bitmap / staging bytes
    uint32_t *bits = sbm;
    int32_t *skey = (int32_t *)sbm;                       // staging (after the bitmap is dead)
    double *sval = (double *)(sbm + SORTB2_CH);
    int32_t *pre8 = (int32_t *)((char *)sbm + area);
    int *scratch = pre8 + NW / 8 + 1;
    const int tid = (int)threadIdx.x;
    Timer tm;   // timing builds only (phases: 0 loads + clear, 1 bitmap, 2 prefix, 3 ranks, 4 staging + stores)
    tm.start();
    for (int64_t idx = blockIdx.x; idx < count; idx += gridDim.x) {
        int64_t o;
        int32_t n;
        sort_ref_span(list[idx], ptr, o, n);
        int32_t *const rc = col + o;
        double *const rv = val + o;
        int32_t c[SORTB2_E];
        double v[SORTB2_E];
#pragma unroll
        for (int k = 0; k < SORTB2_E; ++k) {
            const int e = k * SORTBM_T + tid;
            c[k] = e < n ? rc[e] : 0;
            v[k] = e < n ? rv[e] : 0.0;
        }
        for (int i = tid; i < NW / 4; i += SORTBM_T) ((uint4 *)bits)[i] = make_uint4(0u, 0u, 0u, 0u);
        __syncthreads();
        tm.mark(0);
#pragma unroll
        for (int k = 0; k < SORTB2_E; ++k)
            if (k * SORTBM_T + tid < n) atomicOr(&bits[(uint32_t)c[k] >> 5], 1u << (c[k] & 31));
        __syncthreads();
        tm.mark(1);
        bitmap_prefix8(bits, pre8, NW, scratch);
        __syncthreads();
        tm.mark(2);
        int32_t pos[SORTB2_E];
#pragma unroll
        for (int k = 0; k < SORTB2_E; ++k) {
            pos[k] = 0;
            if (k * SORTBM_T + tid < n) pos[k] = bitmap_rank(bits, pre8, (uint32_t)c[k]);
        }
        __syncthreads();   // every bitmap read done: the area becomes the staging row
        tm.mark(3);
        for (int32_t lo = 0; lo < n; lo += SORTB2_CH) {
            const int32_t m = min(SORTB2_CH, n - lo);
#pragma unroll
            for (int k = 0; k < SORTB2_E; ++k)
                if (k * SORTBM_T + tid < n && pos[k] >= lo && pos[k] < lo + m) {
                    skey[pos[k] - lo] = c[k];
                    sval[pos[k] - lo] = v[k];
                }
            __syncthreads();
            for (int e = tid; e < m; e += SORTBM_T) {
                rc[lo + e] = skey[e];
                rv[lo + e] = sval[e];
            }
            __syncthreads();
        }
        tm.mark(4);
        tm.done();
    }
    tm.flush(17, tid == 0);
}

__global__ __launch_bounds__(256) void k_wide_gather(const RowRef *list, int32_t count,
                                                     const int64_t *ws_off, const int64_t *ptr,
                                                     const int32_t *len, int64_t stride,
                                                     const int32_t *col, const double *val,
                                                     int32_t *kin, double *vin, int64_t *beg,
                                                     int64_t *end, bool back) {
    const int64_t idx = blockIdx.x;
    if (idx >= count) return;
    int64_t o;
    int32_t n;
    sort_row_span(ptr, len, stride, list[idx].row, o, n);
    const int64_t w = ws_off[idx];
    if (!back && blockIdx.y == 0 && threadIdx.x == 0) {
        beg[idx] = w;
        end[idx] = w + n;
    }
    for (int64_t e = (int64_t)blockIdx.y * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.y * 256) {
        if (back) {
            ((int32_t *)col)[o + e] = kin[w + e];
            ((double *)val)[o + e] = vin[w + e];
        } else {
            kin[w + e] = col[o + e];
            vin[w + e] = val[o + e];
        }
    }
}

// Compact expansion of the partitioned rows only (sym2): the product columns
// of each listed row at tcol[ref.q0 + p] (ref.q0 = the row's offset in the
// compact space), for the partition bucketing; the LDS-bin rows gather their
// columns from B themselves.  Workgroups (row, y) take the row's A entries
// y*4 + wave, y*4 + wave + 4*gridDim.y, ...; lanes over the entry's B row.
__global__ __launch_bounds__(256) void k_expand_part(Rows A, AxView ax, const int64_t *axp, const int64_t *poff,
                                                     const RowRef *list, const int32_t *bcol, int32_t *tcol,
                                                     int32_t part_cap) {
    const RowRef ref = list[blockIdx.x];
    if (nparts_of(ref.n, part_cap) <= (uint32_t)PB_MAXP) return;   // bucketed from B instead
    int64_t s;
    int32_t n;
    A.row(ref.row, s, n);
    const int64_t q0 = s - A.base();
    const int64_t p0 = poff[ref.row];
    const int w = (int)(threadIdx.x / WAVE), lane = (int)(threadIdx.x & (WAVE - 1));
    for (int32_t e = (int32_t)blockIdx.y * 4 + w; e < n; e += 4 * (int32_t)gridDim.y) {
        const int64_t q = q0 + e;
        const int32_t bl = ax.blen[q];
        const int64_t bs = ax.bstart[q];
        int32_t *dst = tcol + ref.q0 + (axp[q] - p0);
        for (int32_t j = lane; j < bl; j += WAVE) dst[j] = bcol[bs + j];
    }
}

// The same expansion for k_sym_cbm, flat over products: a wave takes 64 A
// entries of the row at a time (lane = entry: B-row start, length; a DPP
// scan gives each its first product), then walks their products in windows
// of 64 — product t of the group finds its entry by a 6-step binary search
// over the lanes' starts — so every gather slot carries a product and each
// window's stores are one contiguous run (R-MAT's B rows hold ~20 - 30
// entries: a wave per entry left half its lanes idle).
// words (k_sym_cbm<true>: the sliced rows) non-null: it also presets each
// row's first-touch words to all ones (its products; the slices clear their
// duplicates' bits).
__global__ __launch_bounds__(256) void k_expand_flat(Rows A, AxView ax, const int64_t *axp, const int64_t *poff,
                                                     const RowRef *list, const int32_t *bcol, int32_t *tcol,
                                                     Bitmap words) {
    const RowRef ref = list[blockIdx.x];
    if (words.bits && blockIdx.y == 0) {
        uint32_t *g = words.bits + words.off[ref.row];
        const int32_t W = (ref.n + 31) >> 5;
        for (int32_t i = (int32_t)threadIdx.x; i < W; i += (int32_t)blockDim.x)
            g[i] = (i < W - 1 || (ref.n & 31) == 0) ? ~0u : ((1u << (ref.n & 31)) - 1u);
    }
    int64_t s;
    int32_t n;
    A.row(ref.row, s, n);
    const int64_t q0 = s - A.base();
    const int64_t p0 = poff[ref.row];
    const int w = (int)(threadIdx.x / WAVE), lane = (int)(threadIdx.x & (WAVE - 1));
    const int nw = 4 * (int)gridDim.y;
    for (int32_t g = ((int32_t)blockIdx.y * 4 + w) * WAVE; g < n; g += nw * WAVE) {
        const int32_t e = g + lane;
        int32_t bl = 0;
        int64_t bs = 0;
        if (e < n) {
            bl = ax.blen[q0 + e];
            bs = ax.bstart[q0 + e];
        }
        const int incl = wave_incl_sum(bl);
        const int excl = incl - bl;
        const int total = __shfl(incl, WAVE - 1);
        int32_t *dst = tcol + ref.q0 + (axp[q0 + g] - p0);   // the group's products are contiguous
        for (int t0 = 0; t0 < total; t0 += WAVE) {
            const int t = t0 + lane;
            int j = 0;
#pragma unroll
            for (int step = WAVE / 2; step >= 1; step >>= 1) {
                const int ex = __shfl(excl, j + step);
                if (ex <= t) j += step;
            }
            const int64_t bsj = __shfl(bs, j);
            const int exj = __shfl(excl, j);
            if (t < total) dst[t] = bcol[bsj + (t - exj)];
        }
    }
}

// entries of every listed wide row (the compact radix workspace is their scan)
__global__ void k_wide_len(const RowRef *list, int32_t count, const int64_t *ptr, const int32_t *len,
                           int64_t stride, int32_t *wl) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    int64_t o;
    int32_t n;
    sort_row_span(ptr, len, stride, list[i].row, o, n);
    wl[i] = n;
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

// Bin tables.
//  * Symbolic: rows by products (SYM2_BINS: short / sym3 / sym2 kernels);
//    beyond SYM2_MAX products a row is hash-partitioned (SYM_PART_CAP
//    products per partition) and gets a first-touch bitmap.
//  * Numeric: rows by nnz.  Rows with many duplicate products (products >
//    1.5 nnz) and nnz <= VAL_MAX use value tables (16 B/slot, LDS-staged
//    emission); all others use direct-write tables (8 B/slot) up to DW_MAX;
//    beyond DW_MAX a row is hash-partitioned (direct write, bitmap ranks);
//    rows at >= 2^19 - 1 nnz (beyond the 19-bit rank field) use a per-row
//    table in global memory.  Every row above DW_MAX nnz has more than
//    SYM2_MAX products, so every partitioned numeric row has a bitmap.
static inline unsigned grid_for(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }

constexpr int32_t VAL_MAX = 5460;
constexpr int32_t DW_MAX = 10922;
constexpr int SYM_PART_LOG2S = 14; // table slots of a symbolic partition (2^14 = 128 KB of LDS)
constexpr int32_t SYM_PART_CAP = ((1 << SYM_PART_LOG2S) * 2) / 3;   // products per symbolic partition
constexpr int32_t NUM_PART_CAP = 10922;   // nnz per numeric partition (16384-slot table)
constexpr int32_t WIDE_MIN = (1 << 19) - 1;
// IAS_SYM_CBM=0: the partitioned rows take the hash partitions (A/B)
static bool retry_print() {
    static const bool on = [] {
        const char *e = getenv("IAS_RETRY_PRINT");
        return e && *e == '1';
    }();
    return on;
}
constexpr int32_t RETRY_GRID_MIN = 16;   // retry teams at least (history-sized grids)
// IAS_SYM_BIG: 0 = rows beyond SYM2_MAX take the hash partitions / column
// bitmap (A/B), 1 (default) = the sym5<32768> bins when B is too wide for the
// column bitmap, 2 = also when it is not
static int big_mode() {
    static const int m = [] {
        const char *e = getenv("IAS_SYM_BIG");
        return e && *e ? atoi(e) : 1;
    }();
    return m;
}
static bool cbm_enabled() {
    static const bool on = [] {
        const char *e = getenv("IAS_SYM_CBM");
        return !(e && *e == '0');
    }();
    return on;
}
// Column slices of the column-bitmap symbolic when C is wider than one bitmap
// (k_sym_cbm<true>), up to CBS_MAXS of them, with IAS_SYM_CBS=1 (read per
// call); otherwise the hash partitions.  Opt-in: on K4 (8 slices) every slice
// sweeps its row's whole expansion, and the slices measured slower than the
// hash partitions (whole-K4 symbolic 59.1 vs 42.0 ms)
// Slices of 2^20 columns (32,768 words): 3,968 LDS minima slots beside the
// bitmap, as for a 2^20-column C; K4's 2^23 columns are 8 slices
constexpr int32_t CBS_MAXS = 16;
constexpr int32_t CBS_W = 32768;   // bitmap words per slice
static int32_t cbs_slices(int64_t cols) { return (int32_t)((cols + 32ll * CBS_W - 1) / (32ll * CBS_W)); }
static bool cbs_on(int64_t cols) {
    const char *e = getenv("IAS_SYM_CBS");
    return cbm_enabled() && e && *e == '1' && cbs_slices(cols) <= CBS_MAXS;
}

// LDS bins: upper bound of the key and kernel configuration; table slots
// S = ceil(1.5 * upper).
struct BinCfg {
    int32_t upper;
    int32_t cfg;
};
// value-table config of the <= 16-entry bin: 8-lane teams, 4 products per
// lane (K1: 101 vs 130 us with 16-lane teams; 32- / 64-lane teams 214 / 254
// us; 8 products per lane 171 us)
constexpr int VAL_CFG16 = 9;
static constexpr BinCfg VAL_BINS[] = {{16, VAL_CFG16},   {32, 0},   {64, 1},   {128, 2},  {256, 3},
                                      {512, 4},  {768, 5},  {1024, 5}, {1365, 5}, {1820, 6},
                                      {2430, 6}, {3240, 7}, {4320, 7}, {VAL_MAX, 7}};
static constexpr BinCfg DW_BINS[] = {{16, 0},   {32, 0},   {64, 1},   {128, 2},   {256, 3},
                                     {512, 4},  {768, 5},  {1024, 5}, {1536, 6},  {2048, 6},
                                     {3072, 7}, {4096, 7}, {6144, 7}, {8192, 7},  {DW_MAX, 7}};
// sym2 (sym2_kernels.hpp): rows up to SYM2_MAX products whose
// entry count fits (8 * entries <= bound) gather from B; the rest are
// hash-partitioned.  cfg: 0..3 = one-wave teams (K = 1 .. 8 products per
// lane, 4 teams per workgroup: no workgroup barrier per row), 4..7 = 128- to
// 1024-lane teams with K = 8 (one-wave teams with K = 16 / 32 measured slower:
// 160-256 VGPRs, 2-3 waves per SIMD).
constexpr int32_t SYM2_MAX = 16384;
constexpr int SYM2_WAVE_CFG_MAX = 3;
constexpr int SYM2_CFG_WIDE = 8;   // 16 products per lane of a 1024-lane team, one-wave (compact) layout
// 16,385 .. 32,768 products (round 5), only when B's columns do not fit the
// column bitmap: k_sym5<32768, 8>, its retries (and all of them when B's
// entries exceed 32-bit offsets) k_sym_gtab; no sym2 team takes them
constexpr int SYM_CFG_BIG = 9;
static constexpr BinCfg SYM2_BINS[] = {{64, 0},    {128, 1},  {256, 2},  {512, 3},  {768, 4},
                                       {1024, 4},  {1536, 5}, {2048, 5}, {3072, 6}, {4096, 6},
                                       {6144, 7},  {8192, 7},
                                       {12288, SYM2_CFG_WIDE}, {SYM2_MAX, SYM2_CFG_WIDE},
                                       {24576, SYM_CFG_BIG}, {GT_U, SYM_CFG_BIG}
};
constexpr int N_SYM2 = sizeof(SYM2_BINS) / sizeof(SYM2_BINS[0]);
constexpr int N_SYM2_LDS = N_SYM2 - 2;   // the bins up to SYM2_MAX
static_assert(SYM2_BINS[N_SYM2_LDS - 1].upper == SYM2_MAX, "bins");
static void scan_i32(const int32_t *in, int64_t n, int64_t *part, int64_t *out, hipStream_t s);
constexpr int N_VAL = sizeof(VAL_BINS) / sizeof(VAL_BINS[0]);
constexpr int N_DW = sizeof(DW_BINS) / sizeof(DW_BINS[0]);
static_assert(N_SYM2 + 3 <= MAX_BINS && N_VAL + N_DW + 6 <= MAX_BINS, "bins");

// table slots of an LDS bin: 1.5 x its bound, a whole number of 4-slot buckets
constexpr int SLOT_NUM = 3; // slots per bound: SLOT_NUM / 2
static constexpr uint32_t slots_for(int32_t upper) {
    return (uint32_t)(((SLOT_NUM * (long long)upper + 1) / 2 + 3) / 4 * 4);
}
// duplicate-list capacity of a symbolic bin: rows with more duplicate
// products than this take the table path in the numeric pass
static constexpr int32_t dcap_for(int32_t upper) {
    return upper / 8 < 8 ? 8 : (upper / 8 > 2048 ? 2048 : upper / 8);
}
constexpr int PART_DCAP_DIV = 4; // partitioned rows: list of min(products / PART_DCAP_DIV, FIXBIG_CAP); 8: K3 38.96 vs 36.27 ms

// TEAM * PER of each value configuration in val_bin(): the emission loop
// visits that many slots, so it must cover every bin's S.
static constexpr uint32_t VAL_CFG_EMIT[] = {48, 96, 192, 384, 768, 2048, 4096, 8192, 48, 48, 48};
static constexpr bool val_bins_covered() {
    for (int i = 0; i < N_VAL; ++i)
        if (VAL_CFG_EMIT[VAL_BINS[i].cfg] < slots_for(VAL_BINS[i].upper)) return false;
    return true;
}
static_assert(val_bins_covered(), "value-bin emission does not cover a bin's table");

// Symbolic LDS bins in use: when the column-bitmap symbolic applies, those
// up to SYM2_MAX: the longer rows join
// the partitioned bin (k_sym_cbm); otherwise also the two bins to 32,768
// products (sym5<32768>; K4: 4.6 vs 31.5 ps per product in the hash
// partitions), the longer rows hash-partitioned.
// wide: B's selected rows end beyond 2^30 entries (32-bit offsets fail): the
// rows beyond SYM5_MAX take the hash partitions, not the 8-wave sym5 bins
// (whose every row would go through the global tables: K4 forced that way,
// symbolic 115.5 ms at one workgroup per CU against 53.0 ms through the hash
// partitions; round 6, profiles/r06/gtab/)
static int sym_nval(bool cbm, bool wide = false) {
    return cbm ? (big_mode() == 2 ? N_SYM2 : N_SYM2_LDS) : (big_mode() && !wide ? N_SYM2 : N_SYM2_LDS);
}

static BinSpec sym_spec(int nval = N_SYM2) {
    BinSpec s{};
    s.ndw = 0;
    s.nval = nval;
    for (int i = 0; i < nval; ++i) {
        s.upper[i + 1] = SYM2_BINS[i].upper;
        s.dcap[i + 1] = dcap_for(SYM2_BINS[i].upper);
    }
    s.ent_key = 8;   // the row's non-empty entries are staged in LDS, upper/8 of them
    s.ratio_num = 0;
    s.ratio_den = 0;
    s.part_cap = SYM_PART_CAP;
    s.part_dcap_div = PART_DCAP_DIV;
    s.part_dcap_max = FIXBIG_CAP;
    s.wide_min = 0;
    s.ft = 1;
    s.zero_nnz = 1;
    return s;
}

static BinSpec num_spec() {
    BinSpec s{};
    s.nval = N_VAL;
    s.ndw = N_DW;
    for (int i = 0; i < N_VAL; ++i) s.upper[i + 1] = VAL_BINS[i].upper;
    for (int i = 0; i < N_DW; ++i) s.upper[N_VAL + 3 + i] = DW_BINS[i].upper;
    // streaming rows: the rows that need a duplicate fix-up (by list length)
    s.nst = 5;
    s.ratio_num = 3;   // value tables when products * 2 > nnz * 3
    s.ratio_den = 2;
    s.part_cap = NUM_PART_CAP;
    s.wide_min = WIDE_MIN;
    s.ft = 0;
    s.zero_nnz = 0;
    s.short_base = N_VAL + 3 + N_DW + 5;   // after the fix-up bins
    return s;
}
static_assert(N_VAL + 3 + N_DW + 5 + 3 <= MAX_BINS, "short bins beyond MAX_BINS");

// Rows of at most SHORT_MAX products take the short path (short_kernels.hpp:
// one wave per row, exact LDS table, no bitmap) in both passes.
constexpr int32_t SHORT_MAX = 256;

// Dynamic LDS beyond 64 KiB is requested per kernel (once per instantiation:
// the callers below are templates, so each has its own flag).
template <typename F>
static void allow_lds(F kernel, bool &done, size_t bytes) {
    (void)done;
    if (bytes <= 65536) return;
    // once per kernel and device; thread-safe (ias_csr_mul_csr_multi runs one
    // host thread per device)
    static std::mutex mu;
    static std::set<std::pair<const void *, int>> seen;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> g(mu);
    if (seen.insert({(const void *)kernel, dev}).second) {
        hipFuncSetAttribute((const void *)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipGetLastError();   // a refusal shows up at launch
    }
}

// Workgroups of `kernel` resident on the whole device at once (cached per
// kernel, block size, LDS bytes and device).
template <typename F>
static int64_t resident_blocks(F kernel, int threads, size_t lds) {
    static std::mutex mu;
    static std::map<std::tuple<const void *, int, size_t, int>, int64_t> cache;
    int dev = 0;
    hipGetDevice(&dev);
    const auto key = std::make_tuple((const void *)kernel, threads, lds, dev);
    {
        std::lock_guard<std::mutex> g(mu);
        auto it = cache.find(key);
        if (it != cache.end()) return it->second;
    }
    int per_cu = 0, cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)kernel, threads, lds) != hipSuccess ||
        per_cu < 1)
        per_cu = 1;
    (void)hipGetLastError();
    const int64_t v = (int64_t)per_cu * std::max(cus, 1);
    std::lock_guard<std::mutex> g(mu);
    cache[key] = v;
    return v;
}

// One wave per row (the kernels' grid-stride loop then runs once): measured
// faster than persistent waves capped at the resident count with the next
// row prefetched (K2: 0.99 / 1.46 ms vs 1.16 / 1.56 ms symbolic / numeric).
static unsigned short_grid(int32_t count, int rows_per_wave = 1) {
    const int64_t per = (int64_t)SH_WPB * rows_per_wave;
    return (unsigned)std::max<int64_t>(1, ((int64_t)count + per - 1) / per);
}
// The short symbolic pass: two rows per wave for rows of <= 128 products; rows
// of 129..256 products one per wave with the 4-slots-per-product table.
static void short_sym_launch(int32_t upper, const ShortArgs &a, hipStream_t t) {
    constexpr int R = 2;
    if (upper <= 64) k_short_sym_r<1, R><<<short_grid(a.count, R), 64 * SH_WPB, 0, t>>>(a);
    else if (upper <= 128) k_short_sym_r<2, R><<<short_grid(a.count, R), 64 * SH_WPB, 0, t>>>(a);
    else k_short_sym<4><<<short_grid(a.count), 64 * SH_WPB, 0, t>>>(a);
}
static void short_num_launch(int i, const ShortArgs &a, const Out &out, hipStream_t t) {
    if (i == 0) k_short_num<1><<<short_grid(a.count), 64 * SH_WPB, 0, t>>>(a, out);
    else if (i == 1) k_short_num<2><<<short_grid(a.count), 64 * SH_WPB, 0, t>>>(a, out);
    else k_short_num<4><<<short_grid(a.count), 64 * SH_WPB, 0, t>>>(a, out);
}

struct Launch {
    int c;
    uint32_t S;
    hipStream_t s;
    const AxView &ax;
    const Rows &B;
    const RowRef *list;
};

// duplicate lists and bitmap of the streaming path
struct StArgs {
    Bitmap bm;
    int64_t *dup_off;
    int32_t *dupn;
    int32_t *dupt;
};

static Sym2Layout sym2_layout(int32_t upper, int cfg) {
    if (cfg == SYM_CFG_BIG) return sym2_layout(SYM2_MAX, SYM2_CFG_WIDE);   // unused: no sym2 team takes these rows
    // 8 filter bits keep the widest bin's team within one CU's LDS
    return Sym2Layout::for_bound((uint32_t)upper, cfg == SYM2_CFG_WIDE     ? Sym2Layout::WIDE
                                                  : cfg <= SYM2_WAVE_CFG_MAX ? Sym2Layout::ONE_WAVE
                                                                             : Sym2Layout::TEAM_LAYOUT);
}

template <int TEAM, int K, int TPW, int WPE = 1>
static void sym2_launch(Sym2Args a, hipStream_t s) {
    auto kern = k_sym2<TEAM, K, TPW, WPE>;
    static bool done = false;
    const size_t lds = (size_t)TPW * a.lay.bytes();
    allow_lds(kern, done, lds);
    int64_t grid = grid_for(a.count, TPW);
    grid = std::min<int64_t>(grid, resident_blocks(kern, TEAM * TPW, lds));
    kern<<<(unsigned)std::max<int64_t>(grid, 1), TEAM * TPW, lds, s>>>(a);
}

constexpr int SYM2_WPE_TEAM = 1; // waves per SIMD the multi-wave teams' registers must allow (1: no cap)
static void sym2_bin(int cfg, const Sym2Args &a, hipStream_t s) {
    switch (cfg) {
        case 0: sym2_launch<64, 1, 4>(a, s); break;
        case 1: sym2_launch<64, 2, 4>(a, s); break;
        case 2: sym2_launch<64, 4, 4>(a, s); break;
        case 3: sym2_launch<64, 8, 4>(a, s); break;
        case 4: sym2_launch<128, 8, 1, SYM2_WPE_TEAM>(a, s); break;   // one-wave K=16 measured 30 % slower
        case 5: sym2_launch<256, 8, 1, SYM2_WPE_TEAM>(a, s); break;
        case 6: sym2_launch<512, 8, 1, SYM2_WPE_TEAM>(a, s); break;
        case 7: sym2_launch<1024, 8, 1, SYM2_WPE_TEAM>(a, s); break;
        default: sym2_launch<1024, 16, 1, SYM2_WPE_TEAM>(a, s); break;   // SYM2_CFG_WIDE
    }
}


// sym3's one-wave rows (sym3_kernels.hpp): rows of SYM3_MIN .. SYM3_MAX products
constexpr int32_t SYM3_MIN = 257, SYM3_MAX = 2048;   // sym4<2048> on 1,025 - 2,048: 0.98 vs 0.79 ms (K3', serial)
constexpr int SYM3_WPB = 4;
constexpr int SYM3_DB_MAXK = 4;   // K up to which the next row's columns are gathered during a row (K = 8: 298 vs 309 us on K3')
template <int K>
static void sym3_launch(const Sym3Args &a, hipStream_t s) {
    auto kern = k_sym3<K, SYM3_WPB, (K <= SYM3_DB_MAXK)>;
    const int64_t want = ((int64_t)a.count + SYM3_WPB - 1) / SYM3_WPB;
    const int64_t grid = std::min<int64_t>(want, resident_blocks(kern, 64 * SYM3_WPB, 0));
    kern<<<(unsigned)std::max<int64_t>(grid, 1), 64 * SYM3_WPB, 0, s>>>(a);
}
// a sym3 bin (upper in SYM3_MIN .. SYM3_MAX); the rows it hands back go to
// sym2's 128- / 256-lane teams (retry_cfg, launched by the caller)
static void sym3_bin(int32_t upper, const Sym3Args &a, hipStream_t s) {
    if (upper <= 512) sym3_launch<8>(a, s);
    else if (upper <= 768) sym3_launch<12>(a, s);
    else if (upper <= 1024) sym3_launch<16>(a, s);
    else if (upper <= 1536) sym3_launch<24>(a, s);
    else sym3_launch<32>(a, s);
}

// sym4's one-wave long rows (sym4_kernels.hpp): rows of SYM3_MAX+1 .. SYM4_MAX
// products; the rows it hands back go to the bin's own sym2 teams.  K3'
// serial: 2,049 - 4,096 products 0.89 ms (sym2's 512-lane teams 1.2 ms);
// 4,097 - 8,192 1.0 ms (sym2's 1024-lane teams 0.96 ms: kept).
constexpr int32_t SYM4_MAX = 4096;
constexpr int SYM4_WPB = 2;
// (its retries: sym2's 512-lane teams, cfg 6)
template <int U>
static void sym4_launch(const Sym3Args &a, hipStream_t s) {
    auto kern = k_sym4<U, 16, 8, SYM4_WPB>;
    const int64_t want = ((int64_t)a.count + SYM4_WPB - 1) / SYM4_WPB;
    const int64_t grid = std::min<int64_t>(want, resident_blocks(kern, 64 * SYM4_WPB, 0));
    kern<<<(unsigned)std::max<int64_t>(grid, 1), 64 * SYM4_WPB, 0, s>>>(a);
}

// sym5 (sym5_kernels.hpp): SYM4_MAX+1 .. SYM5_MAX products, NW waves per row
constexpr int32_t SYM5_MAX = 16384;
template <int U, int NW>
static void sym5_launch(const Sym3Args &a, hipStream_t s) {
    auto kern = k_sym5<U, NW, 8>;
    static bool done = false;
    const size_t lds = sizeof(Sym5Lds<U, NW>);
    allow_lds(kern, done, lds);
    const int64_t grid = std::min<int64_t>(a.count, resident_blocks(kern, 64 * NW, lds));
    kern<<<(unsigned)std::max<int64_t>(grid, 1), 64 * NW, lds, s>>>(a);
}
// k_sym_gtab over a row list (device count a.retry_count), `grid`
// workgroups each with GT_SLOTS table slots of `keys` / `own`
// workgroups: GT_GRID_MAX for sym5's hand-backs (rare rows), GT_GRID_ALL
// (one per CU) when every row of the bins comes here (B beyond 32-bit
// offsets): K4 with every 16,385 - 32,768-product row forced here
// (IAS_GTAB_ALL=1), symbolic 134.9 ms at 64 workgroups (advisor, round 5)
constexpr int GT_GRID_MAX = 64;
constexpr int GT_GRID_ALL = 256;
static bool gtab_all(int32_t wide_b) {   // IAS_GTAB_ALL=1: test knob, read per call
    const char *ga = getenv("IAS_GTAB_ALL");
    return wide_b || (ga && *ga == '1');
}
static void gtab_launch(const Sym3Args &a, int64_t grid, int32_t *keys, uint32_t *own, hipStream_t s, int gmax) {
    grid = std::max<int64_t>(1, std::min<int64_t>(grid, gmax));
    k_sym_gtab<<<(unsigned)grid, GT_BLOCK, 0, s>>>(a, keys, own);
}
// (its retries: sym2's 1024-lane teams, cfg 7 / SYM2_CFG_WIDE)
static void sym5_bin(int32_t upper, const Sym3Args &a, hipStream_t s) {
    if (upper <= 8192) sym5_launch<8192, 2>(a, s);
    else sym5_launch<16384, 4>(a, s);
}

template <int TEAM, int K, int SEG, int TPW, int PER>
static void val_launch(const Launch &l, const Out &out) {
    auto kern = k_numeric_val<TEAM, K, SEG, TPW, PER>;
    static bool done = false;
    const size_t lds = (size_t)TPW * val_team_bytes<SEG>(l.S);
    allow_lds(kern, done, lds);
    kern<<<grid_for(l.c, TPW), TEAM * TPW, lds, l.s>>>(l.ax, l.B, l.list, l.c, l.S, out);
}

static void val_bin(int cfg, const Launch &l, const Out &out) {
    switch (cfg) {
        case 0: val_launch<16, 4, 16, 16, 3>(l, out); break;
        case 1: val_launch<32, 4, 32, 8, 3>(l, out); break;
        case 2: val_launch<64, 4, 64, 4, 3>(l, out); break;
        case 3: val_launch<64, 4, 64, 2, 6>(l, out); break;
        case 4: val_launch<128, 4, 128, 1, 6>(l, out); break;
        case 5: val_launch<256, 4, 256, 1, 8>(l, out); break;
        case 6: val_launch<512, 4, 256, 1, 8>(l, out); break;
        case 8: val_launch<8, 8, 8, 32, 6>(l, out); break;   // VAL_CFG16 A/B: 8-lane teams
        case 9: val_launch<8, 4, 8, 32, 6>(l, out); break;
        case 10: val_launch<4, 4, 4, 64, 12>(l, out); break;
        default: val_launch<1024, 2, 256, 1, 8>(l, out); break;
    }
}

template <int TEAM, int K, int SEG, int TPW>
static void dw_launch(const Launch &l, const Out &out) {
    auto kern = k_numeric_dw<TEAM, K, SEG, TPW>;
    static bool done = false;
    const size_t lds = (size_t)TPW * dw_team_bytes<SEG>(l.S);
    allow_lds(kern, done, lds);
    kern<<<grid_for(l.c, TPW), TEAM * TPW, lds, l.s>>>(l.ax, l.B, l.list, l.c, l.S, out);
}

static void dw_bin(int cfg, const Launch &l, const Out &out) {
    switch (cfg) {
        case 0: dw_launch<16, 4, 16, 16>(l, out); break;
        case 1: dw_launch<32, 4, 32, 8>(l, out); break;
        case 2: dw_launch<64, 4, 64, 4>(l, out); break;
        case 3: dw_launch<64, 4, 64, 2>(l, out); break;
        case 4: dw_launch<128, 4, 128, 1>(l, out); break;
        case 5: dw_launch<256, 4, 256, 1>(l, out); break;
        case 6: dw_launch<512, 4, 256, 1>(l, out); break;
        default: dw_launch<1024, 2, 256, 1>(l, out); break;
    }
}

// start of each bin's compact list (bins in numeric order; bin 0 unlisted)
static void bin_starts(const Counters &c, int64_t *start) {
    int64_t acc = 0;
    for (int i = 0; i < MAX_BINS; ++i) {
        start[i] = acc;
        acc += i > 0 ? c.count[i] : 0;
    }
}

#define HIPC(x)                                                                   \
    do {                                                                          \
        hipError_t _e = (x);                                                      \
        if (_e != hipSuccess) {                                                   \
            set_last_error("%s failed: %s", #x, hipGetErrorString(_e));           \
            return _e == hipErrorOutOfMemory ? IAS_ERROR_OUT_OF_MEMORY : IAS_ERROR_DEVICE; \
        }                                                                         \
    } while (0)

// IAS_DEBUG_SYNC=1: synchronise and check after every launch group, naming
// the group in ias_last_error() (diagnostics only; off by default).
static bool debug_sync() {
    static const bool on = [] {
        const char *e = getenv("IAS_DEBUG_SYNC");
        return e && *e && *e != '0';
    }();
    return on;
}
#define CHECK_LAUNCH(what, strm)                                                          \
    do {                                                                                 \
        if (debug_sync()) {                                                              \
            hipError_t _e = hipGetLastError();                                           \
            if (_e == hipSuccess) _e = hipStreamSynchronize(strm);                       \
            if (_e != hipSuccess) {                                                      \
                set_last_error("%s: %s", what, hipGetErrorString(_e));                   \
                return IAS_ERROR_DEVICE;                                                 \
            }                                                                            \
        }                                                                                \
    } while (0)

ias_status ias_plan::reserve(void **buf, size_t *cap, size_t bytes) {
    if (*cap >= bytes && *buf) return IAS_SUCCESS;
    if (*buf) HIPC(hipFree(*buf));
    *buf = nullptr;
    *cap = 0;
    const size_t want = std::max<size_t>(bytes + bytes / 8, 256);
    hipError_t e = hipMalloc(buf, want);
    if (e == hipErrorOutOfMemory) {
        // the block cache and an idle default plan may hold what is missing
        (void)hipGetLastError();
        release_device_memory(device, this);
        e = hipMalloc(buf, want);
    }
    if (e != hipSuccess) *buf = nullptr;
    HIPC(e);
    *cap = want;
    return IAS_SUCCESS;
}

size_t ias_plan::release_workspace() {
    hipSetDevice(device);
    if (stream) hipStreamSynchronize((hipStream_t)stream);
    for (int i = 0; i < NSIDE; ++i)
        if (side[i]) hipStreamSynchronize((hipStream_t)side[i]);
    size_t b = 0;
    for (auto &x : bufs) {
        if (x.p) {
            hipFree(x.p);
            b += x.cap;
        }
        x = Buf{};
    }
    last_a = last_b = nullptr;   // a compute() after this needs a new nnz()
    return b;
}

size_t ias_plan::workspace_bytes() const {
    size_t b = 0;
    for (const auto &x : bufs) b += x.p ? x.cap : 0;
    return b;
}

ias_plan::~ias_plan() {
    hipSetDevice(device);
    if (stream) hipStreamSynchronize((hipStream_t)stream);
    for (auto &b : bufs)
        if (b.p) hipFree(b.p);
    for (auto &e : ev)
        if (e) hipEventDestroy(e);
    for (int i = 0; i < NSIDE; ++i) {
        if (side[i]) {
            hipStreamSynchronize((hipStream_t)side[i]);
            hipStreamDestroy((hipStream_t)side[i]);
        }
        if (join_ev[i]) hipEventDestroy(join_ev[i]);
    }
    if (fork_ev) hipEventDestroy(fork_ev);
    for (auto &e : fix_ev)
        if (e) hipEventDestroy(e);
    for (auto &e : n2_ev)
        if (e) hipEventDestroy(e);
    for (auto &e : bin_ev)
        if (e) hipEventDestroy(e);
    if (host_counters) hipHostFree(host_counters);
    if (own_stream && stream) hipStreamDestroy((hipStream_t)stream);
}

ias_status ias_plan::init(int dev, void *strm) {
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
    for (int i = 0; i < NSIDE; ++i) {
        hipStream_t t;
        HIPC(hipStreamCreateWithFlags(&t, hipStreamNonBlocking));
        side[i] = t;
        HIPC(hipEventCreateWithFlags(&join_ev[i], hipEventDisableTiming));
    }
    HIPC(hipEventCreateWithFlags(&fork_ev, hipEventDisableTiming));
    for (auto &e : fix_ev) HIPC(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (auto &e : n2_ev) HIPC(hipEventCreate(&e));
    const char *e = getenv("IAS_SERIAL");
    serial = e && *e && *e != '0';
    HIPC(hipHostMalloc(&host_counters, 3 * sizeof(Counters)));   // [0], [1]: counters; [2]: A's base
    return IAS_SUCCESS;
}

ias_status ias_plan::fork() {
    if (serial || small) return IAS_SUCCESS;
    HIPC(hipEventRecord(fork_ev, (hipStream_t)stream));
    for (int i = 0; i < NSIDE; ++i) HIPC(hipStreamWaitEvent((hipStream_t)side[i], fork_ev, 0));
    return IAS_SUCCESS;
}

ias_status ias_plan::join() {
    if (serial || small) return IAS_SUCCESS;
    for (int i = 0; i < NSIDE; ++i) {
        HIPC(hipEventRecord(join_ev[i], (hipStream_t)side[i]));
        HIPC(hipStreamWaitEvent((hipStream_t)stream, join_ev[i], 0));
    }
    return IAS_SUCCESS;
}

template <typename T>
static T *as(ias_plan::Buf &b) { return (T *)b.p; }

// The A value of expanded entry q is A.val[base + q] (CSR: base = the view's
// first row pointer, read back with the analysis counters; ELL: 0), so the
// expanded A carries no copy of the values.
AxView ias_plan::ax_view() {
    return AxView{as<int64_t>(bufs[B_AXS]), as<int32_t>(bufs[B_AXL]), ax_aval};
}

// Analysis (queued, no host wait): products per row, expanded A, product
// offsets per entry and per row, symbolic bin counts into the B_CNT counters.
ias_status ias_plan::analysis_launch(const Rows &A, const Rows &B, int64_t rows, int64_t a_entries) {
    hipStream_t s = (hipStream_t)stream;
    HIPC(hipSetDevice(device));
    n_rows = rows;
    n_entries = a_entries;
    cbm_path = cbm_words(n_cols) <= CBM_MAXW && cbm_enabled();
    const BinSpec ss = sym_spec(sym_nval(cbm_path, wide_redo));
    const size_t ae = (size_t)std::max<int64_t>(a_entries, 1);
    IAS_TRY(reserve(B_AXS, sizeof(int64_t) * ae));
    IAS_TRY(reserve(B_AXL, sizeof(int32_t) * ae));
    IAS_TRY(reserve(B_AXP, sizeof(int64_t) * (ae + 1)));
    IAS_TRY(reserve(B_POFF, sizeof(int64_t) * (rows + 1)));
    const int64_t nbe = (a_entries + SCAN_TILE - 1) / SCAN_TILE;
    IAS_TRY(reserve(B_PART2, sizeof(int64_t) * (nbe + 2)));
    IAS_TRY(reserve(B_PROD, sizeof(int32_t) * (rows + 1)));
    IAS_TRY(reserve(B_NNZ, sizeof(int32_t) * (rows + 1)));
    IAS_TRY(reserve(B_SLIST, sizeof(RowRef) * (rows + 1)));
    IAS_TRY(reserve(B_NLIST, sizeof(RowRef) * (rows + 1)));
    IAS_TRY(reserve(B_BMOFF, sizeof(int64_t) * (rows + 1)));
    IAS_TRY(reserve(B_WSOFF, sizeof(int64_t) * (rows + 1)));
    IAS_TRY(reserve(B_DUPOFF, sizeof(int64_t) * (rows + 1)));
    IAS_TRY(reserve(B_DUPN, sizeof(int32_t) * (rows + 1)));
    IAS_TRY(reserve(B_CNT, 2 * sizeof(Counters)));   // [0]: analysis / symbolic, [1]: numeric binning
    IAS_TRY(reserve(B_PTR, sizeof(int64_t) * (rows + 1)));
    const int64_t nb = (rows + SCAN_TILE - 1) / SCAN_TILE;
    IAS_TRY(reserve(B_PART, sizeof(int64_t) * (3 * nb + 4)));   // also the 3*rows scan of the num2 units
    Counters *dc = as<Counters>(bufs[B_CNT]);

    // ---- analysis: products per row, expanded A (+ product offsets), symbolic bin counts
    HIPC(hipEventRecord(ev[0], s));
    HIPC(hipMemsetAsync(dc, 0, 2 * sizeof(Counters), s));   // dc, dc2
    int32_t *axl = as<int32_t>(bufs[B_AXL]);
    int64_t *axp = as<int64_t>(bufs[B_AXP]);
    int64_t *poff = as<int64_t>(bufs[B_POFF]);
    if (a_entries > 0)   // one block per scan tile (its B-row length sum -> B_PART2)
        k_an_entries<<<(unsigned)nbe, AN_BLOCK, 0, s>>>(A, B, a_entries,
                                                        AxOut{as<int64_t>(bufs[B_AXS]), axl, nullptr, &dc->wide_b, &dc->wide_v},
                                                        as<int64_t>(bufs[B_PART2]));
    CHECK_LAUNCH("expanded A", s);
    if (a_entries > 0) {
        k_scan_partials<<<1, 1024, 0, s>>>(as<int64_t>(bufs[B_PART2]), nbe);
        k_scan_apply<<<(unsigned)nbe, SCAN_BLOCK, 0, s>>>(axl, a_entries, as<int64_t>(bufs[B_PART2]), axp);
    } else {
        HIPC(hipMemsetAsync(axp, 0, sizeof(int64_t), s));
    }
    if (rows > 0)
        BIN_LAUNCH(k_an_rows, rows, s, axp, a_entries, poff, rows, as<int32_t>(bufs[B_PROD]), ss, dc, A);
    else
        k_row_poff<<<1, 64, 0, s>>>(A, rows, axp, a_entries, poff, dc);
    CHECK_LAUNCH("product offsets", s);
    HIPC(hipGetLastError());
    return IAS_SUCCESS;
}

ias_status ias_plan::symbolic(const Rows &A, const Rows &B, int64_t rows, int64_t cols,
                              int64_t a_entries, ias_report *rep) {
    n_cols = cols;
    set_last_diag(0);   // ias_last_diag(): this call's branches, or none if it stops early
    wide_redo = false;
    IAS_TRY(analysis_launch(A, B, rows, a_entries));
    hipStream_t s = (hipStream_t)stream;
    // the previous call's symbolic bins are done: their durations for this
    // call's balance, read while the analysis kernels run
    for (int b = 0; b < MAX_BINS; ++b)
        if (bin_rec[b]) {
            bin_rec[b] = false;
            float ms = 0.f;
            if (sym_est_prev[b] > 0.0 && hipEventElapsedTime(&ms, bin_ev[2 * b], bin_ev[2 * b + 1]) == hipSuccess &&
                ms > 0.f)
                sym_w[b] = 1e6 * (double)ms / sym_est_prev[b];
            (void)hipGetLastError();
        }
    Counters *dc = as<Counters>(bufs[B_CNT]);
    Counters *dc2 = as<Counters>(bufs[B_CNT]) + 1;
    Counters *hc = (Counters *)host_counters;
    int64_t *poff = as<int64_t>(bufs[B_POFF]);
    const int64_t *axp = as<int64_t>(bufs[B_AXP]);
    const int64_t nb = (rows + SCAN_TILE - 1) / SCAN_TILE;
    HIPC(hipMemcpyAsync(hc, dc, sizeof(Counters), hipMemcpyDeviceToHost, s));   // + A's base entry
    HIPC((hipError_t)host_wait(s));
    bool big_rows = false;   // rows in the 8-wave sym5 bins (numbered N_SYM2_LDS + 1 ..)
    for (int b = N_SYM2_LDS + 1; b <= N_SYM2 && sym_nval(cbm_path) == N_SYM2; ++b) big_rows |= hc->count[b] > 0;
    if (hc->wide_b && big_rows && sym_nval(cbm_path, true) != sym_nval(cbm_path)) {
        // B beyond 32-bit offsets: the analysis again with the bins of that
        // case (its binning needs the flag the analysis itself raises)
        wide_redo = true;
        IAS_TRY(analysis_launch(A, B, rows, a_entries));
        HIPC(hipMemcpyAsync(hc, dc, sizeof(Counters), hipMemcpyDeviceToHost, s));
        HIPC((hipError_t)host_wait(s));
    }
    const BinSpec ss = sym_spec(sym_nval(cbm_path, wide_redo)), ns = num_spec();
    const Counters c1 = *hc;
    ax_aval = A.val + (rows > 0 ? c1.a_base : 0);
    const AxView ax = ax_view();
    if (c1.overflow) {
        set_last_error("A's row pointer addresses entries beyond its nnz (%lld)", (long long)a_entries);
        return IAS_ERROR_INVALID_ARGUMENT;
    }
    flops = (int64_t)c1.flops;
    wide_v = c1.wide_v != 0;
    if (!wide_v) {   // IAS_WIDE_V=1: test knob, the 64-bit-address streaming pass on any input
        const char *e = getenv("IAS_WIDE_V");
        wide_v = e && *e == '1';
    }
    small = flops < SMALL_FLOPS;
    max_prod = c1.max_prod;

    // ---- expansion of the partitioned rows' product columns (in their
    // compact space; the other bins gather from B)
    // the partitioned rows: one LDS column bitmap per row when B's columns
    // fit it (k_sym_cbm), else hash partitions (expansion + buckets)
    const int32_t ncw = cbm_words(cols);
    const bool cbm = cbm_path;
    const bool cbs = !cbm_path && cbs_on(cols);
    IAS_TRY(reserve(B_TCOL, sizeof(int32_t) * (size_t)std::max<int64_t>((int64_t)c1.part_prod, 1)));
    const int32_t *tcol = as<int32_t>(bufs[B_TCOL]);

    // ---- symbolic binning + symbolic
    IAS_TRY(reserve(B_SITEM, sizeof(PartItem) * (size_t)(c1.items + 1)));
    IAS_TRY(reserve(B_PFIRST, sizeof(int64_t) * (size_t)(rows + 1)));
    IAS_TRY(reserve(B_PBOFF, sizeof(int64_t) * (size_t)(rows + 1)));
    IAS_TRY(reserve(B_PSPAN, sizeof(PartSpan) * (size_t)(c1.items + 1)));
    IAS_TRY(reserve(B_PBKT, sizeof(uint2) * (size_t)(c1.part_prod + 1)));
    if (!c1.wide_b) IAS_TRY(reserve(B_S3RETRY, sizeof(RowRef) * (size_t)(rows + 1)));
    if (ss.nval > N_SYM2_LDS && (c1.count[N_SYM2_LDS + 1] > 0 || c1.count[N_SYM2_LDS + 2] > 0)) {
        const size_t tab = (size_t)(N_SYM2 - N_SYM2_LDS) * (gtab_all(c1.wide_b) ? GT_GRID_ALL : GT_GRID_MAX) * GT_SLOTS;
        IAS_TRY(reserve(B_GTKEY, sizeof(int32_t) * tab));
        IAS_TRY(reserve(B_GTOWN, sizeof(uint32_t) * tab));
    }
    const int sym_part = ss.nval + 1;
    // every listed row gets a first-touch bitmap; LDS-bin rows a duplicate list
    IAS_TRY(reserve(B_BITS, sizeof(uint32_t) * (c1.bm_words + 1)));
    IAS_TRY(reserve(B_BPREF, sizeof(uint32_t) * (c1.bm_words + 1)));
    IAS_TRY(reserve(B_DUPT, sizeof(int32_t) * (c1.dup_slots + 1)));
    IAS_TRY(reserve(B_DUPV, sizeof(double) * (c1.dup_slots + 1)));
    IAS_TRY(reserve(B_DUPP, sizeof(uint2) * (c1.dup_slots + 1)));
    Bitmap bm{as<uint32_t>(bufs[B_BITS]), as<uint32_t>(bufs[B_BPREF]), as<int64_t>(bufs[B_BMOFF])};
    const StArgs sa{bm, as<int64_t>(bufs[B_DUPOFF]), as<int32_t>(bufs[B_DUPN]), as<int32_t>(bufs[B_DUPT])};
    if (c1.count[sym_part] > 0 && !cbm) HIPC(hipMemsetAsync(bm.bits, 0, sizeof(uint32_t) * c1.bm_words, s));
    RowRef *SL = as<RowRef>(bufs[B_SLIST]);
    int32_t *nnz = as<int32_t>(bufs[B_NNZ]);
    if (rows > 0)
        BIN_LAUNCH(k_bin_scatter, rows, s, 
            as<int32_t>(bufs[B_PROD]), nullptr, nullptr, rows, ss, A, SL, as<PartItem>(bufs[B_SITEM]),
            as<int64_t>(bufs[B_BMOFF]), nullptr, sa.dup_off, sa.dupn, nnz, poff, dc, as<int64_t>(bufs[B_PFIRST]),
            as<int64_t>(bufs[B_PBOFF]), 1);
    CHECK_LAUNCH("k_bin_scatter(symbolic)", s);
    HIPC(hipEventRecord(ev[1], s));
    int64_t st[MAX_BINS];
    bin_starts(c1, st);
    int c;
    std::fill(retry_upper_cur, retry_upper_cur + 16, 0);   // set per launched bin below
    IAS_TRY(fork());
    // Streams by estimated cost, largest first onto the least loaded stream:
    // pairs of side streams share a hardware queue, so four balanced streams
    // keep both queues balanced whatever the pairing (round robin left one
    // queue 1 ms behind the other on K3').  Cost = estimated products x the
    // kernel's serial ns per product on K3' (short 5, sym3 3.5, sym4 4.2,
    // sym5 7, bucketed partitions 40: their whole-CU workgroups wait beside
    // the other bins).
    // From the second call of a plan on, each bin's weight is its measured
    // duration beside the others per estimated product (the serial weights
    // left the two queues 0.55 ms apart on K3').
    int sym_lane[MAX_BINS] = {};
    double *sym_est = sym_est_prev;   // read back with the bins' durations by the next call
    std::fill(sym_est, sym_est + MAX_BINS, 0.0);
    const bool fb = !serial && !small;
    if (fb && !bin_ev[0])
        for (auto &e : bin_ev) HIPC(hipEventCreate(&e));
    {
        double load[NSIDE] = {};
        std::vector<std::pair<double, int>> jobs;
        auto weight = [&](int b, double serial_w) { return fb && sym_w[b] > 0.0 ? sym_w[b] : serial_w; };
        // the partitioned rows (one workgroup per row or partition, grids far
        // beyond residency) run on the plan stream: on a side stream their
        // dispatch held its hardware queue, and the bins of the stream sharing
        // that queue waited behind it (K3: 3.2 ms of one queue idle at the
        // end of the symbolic phase; round 5)
        if (c1.count[sym_part] > 0) sym_est[sym_part] = (double)c1.part_prod;
        for (int b = 1; b <= ss.nval; ++b)
            if (c1.count[b] > 0) {
                const int32_t u = SYM2_BINS[b - 1].upper, l = b > 1 ? SYM2_BINS[b - 2].upper : 0;
                const double w = u <= SHORT_MAX ? 5.0 : u <= SYM3_MAX ? 3.5 : u <= SYM4_MAX ? 4.2 : 7.0;
                sym_est[b] = c1.count[b] * 0.5 * (double)(l + u);
                jobs.push_back({weight(b, w) * sym_est[b], b});
            }
        std::stable_sort(jobs.begin(), jobs.end(), [](const auto &x, const auto &y) { return x.first > y.first; });
        for (const auto &j : jobs) {
            const int i = (int)(std::min_element(load, load + NSIDE) - load);
            load[i] += j.first;
            sym_lane[j.second] = i;
        }
    }
    auto bin_mark = [&](int b, hipStream_t t, int end) {
        if (!fb) return;
        (void)hipEventRecord(bin_ev[2 * b + end], t);
        bin_rec[b] = true;
    };
    if ((c = c1.count[sym_part]) > 0) {
        hipStream_t t = s;
        bin_mark(sym_part, t, 0);
        if (cbm) {
            static bool cbm_done = false;
            // the minima table takes the LDS left beyond the bitmap (3,968
            // entries at 2^20 columns); IAS_CBM_FORCE (test knob, read per
            // call): forced branches (CBM_GLOBAL_OWN: no LDS table) and the
            // branch flags collected for ias_last_diag()
            const char *fe = getenv("IAS_CBM_FORCE");
            const int32_t force = fe && *fe ? (int32_t)atoi(fe) : 0;
            const int32_t own_lds = (int32_t)std::max<int64_t>(0, ((int64_t)160 * 1024 - 512 - (int64_t)cbm_lds_bytes(ncw)) / 4);
            const int32_t own_cap = (force & CBM_GLOBAL_OWN) ? 0 : own_lds;
            const size_t lds = cbm_lds_bytes(ncw) + 4ull * own_lds;
            allow_lds(k_sym_cbm<false>, cbm_done, lds);
            k_expand_flat<<<dim3((unsigned)c, 4), 256, 0, t>>>(A, ax, axp, poff, SL + st[sym_part], B.col,
                                                               as<int32_t>(bufs[B_TCOL]), Bitmap{});
            const CbmArgs ca{tcol, SL + st[sym_part], ncw, as<uint2>(bufs[B_PBKT]), bm, nnz,
                             sa.dup_off, sa.dupn, sa.dupt, PART_DCAP_DIV, FIXBIG_CAP, own_cap, force,
                             fe && *fe ? (uint32_t *)&dc2->cbm_hits : nullptr, 1, c, nullptr, nullptr};
            k_sym_cbm<false><<<c, CBM_BLOCK, lds, t>>>(ca);
            CHECK_LAUNCH("k_sym_cbm", t);
        } else if (cbs) {
            // wider C (round 6): the same passes per column slice of 2^20
            // columns, a workgroup per (row, slice)
            static bool cbs_done = false;
            const char *fe = getenv("IAS_CBM_FORCE");
            const int32_t force = fe && *fe ? (int32_t)atoi(fe) : 0;
            const int32_t own_lds = (int32_t)std::max<int64_t>(0, ((int64_t)160 * 1024 - 512 - (int64_t)cbm_lds_bytes(CBS_W)) / 4);
            const int32_t own_cap = (force & CBM_GLOBAL_OWN) ? 0 : own_lds;
            const size_t lds = cbm_lds_bytes(CBS_W) + 4ull * own_lds;
            allow_lds(k_sym_cbm<true>, cbs_done, lds);
            IAS_TRY(reserve(B_CBSCUR, sizeof(unsigned long long) * (size_t)c));
            unsigned long long *wcur = as<unsigned long long>(bufs[B_CBSCUR]);
            HIPC(hipMemsetAsync(wcur, 0, sizeof(unsigned long long) * (size_t)c, t));
            k_expand_flat<<<dim3((unsigned)c, 4), 256, 0, t>>>(A, ax, axp, poff, SL + st[sym_part], B.col,
                                                               as<int32_t>(bufs[B_TCOL]), bm);
            const CbmArgs ca{tcol, SL + st[sym_part], CBS_W, as<uint2>(bufs[B_PBKT]), bm, nnz,
                             sa.dup_off, sa.dupn, sa.dupt, PART_DCAP_DIV, FIXBIG_CAP, own_cap, force,
                             fe && *fe ? (uint32_t *)&dc2->cbm_hits : nullptr, cbs_slices(cols), c, wcur,
                             as<uint2>(bufs[B_DUPP])};
            k_sym_cbm<true><<<(unsigned)((c + 7) / 8 * 8 * ca.nslice), CBM_BLOCK, lds, t>>>(ca);
            k_bitmap_prefix<<<c, 256, 0, t>>>(SL + st[sym_part], c, as<int32_t>(bufs[B_PROD]), bm);
            k_dup_place<<<c, 256, 0, t>>>(SL + st[sym_part], c, bm, as<uint2>(bufs[B_DUPP]), sa.dup_off, sa.dupn,
                                          sa.dupt, PART_DCAP_DIV, FIXBIG_CAP);
            CHECK_LAUNCH("k_sym_cbm<true>", t);
        } else {
            k_expand_part<<<dim3((unsigned)c, 8), 256, 0, t>>>(A, ax, axp, poff, SL + st[sym_part], B.col,
                                                                   as<int32_t>(bufs[B_TCOL]), SYM_PART_CAP);
            k_part_bucket<<<c, PB_BLOCK, 0, t>>>(A, ax, axp, poff, B.col, SL + st[sym_part], c, as<int64_t>(bufs[B_PFIRST]),
                                                     as<int64_t>(bufs[B_PBOFF]), SYM_PART_CAP, as<uint2>(bufs[B_PBKT]),
                                                     as<PartSpan>(bufs[B_PSPAN]));
            k_symbolic_part<1024, 12, SYM_PART_LOG2S><<<(unsigned)c1.items, 1024, 0, t>>>(
                tcol, as<PartItem>(bufs[B_SITEM]), bm, nnz, as<uint2>(bufs[B_DUPP]), sa.dup_off, sa.dupn,
                PART_DCAP_DIV, FIXBIG_CAP, &dc2->overflow, as<uint2>(bufs[B_PBKT]), as<PartSpan>(bufs[B_PSPAN]));
            k_bitmap_prefix<<<c, 256, 0, t>>>(SL + st[sym_part], c, as<int32_t>(bufs[B_PROD]), bm);
            k_dup_place<<<c, 256, 0, t>>>(SL + st[sym_part], c, bm, as<uint2>(bufs[B_DUPP]), sa.dup_off, sa.dupn,
                                          sa.dupt, PART_DCAP_DIV, FIXBIG_CAP);
            CHECK_LAUNCH("k_symbolic_part", t);
        }
        bin_mark(sym_part, t, 1);
    }
    // The rows a sym3 / sym4 / sym5 bin hands back (list overflow, too many
    // entries) are finished by sym2's teams, launched right after the bin in
    // its stream (launched after the join instead, on the main stream, they
    // ran last and serially: K3' symbolic +0.1 - 0.25 ms, rounds 4 and 5)
    auto retry = [&](int cfg, const Sym3Args &a3, Sym2Args r2, hipStream_t t) {
        r2.list = a3.retry;
        r2.count_dev = a3.retry_count;   // r2.count bounds the grid; the device count decides
        sym2_bin(cfg, r2, t);
    };
    auto launch_sym = [&](int b, int c, hipStream_t t) -> ias_status {
        const int32_t u = SYM2_BINS[b - 1].upper;
        if (u <= SHORT_MAX) {
            const ShortArgs sh{A, ax, B.col, B.val, SL + st[b], c, nnz, sa.dupn};
            short_sym_launch(u, sh, t);
            CHECK_LAUNCH("k_short_sym", t);
            return IAS_SUCCESS;
        }
        Sym2Args a2{ax, B.col, SL + st[b], c, as<int32_t>(bufs[B_PROD]), sym2_layout(u, SYM2_BINS[b - 1].cfg), nnz, bm,
                    sa.dup_off, sa.dupn, sa.dupt, dcap_for(u), DW_MAX, nullptr};
        // the retry teams' grid (persistent: any grid finishes the list): a
        // bin hands back few rows, and a full grid of LDS-heavy workgroups
        // waits for whole CUs beside the other bins (K3': 50 - 260 us per
        // retry launch for ~no rows) — so twice the rows this bin handed back
        // on the plan's last call, when known
        // (history only from a call that launched this bin — retry_prev is
        // -1 otherwise; at least RETRY_GRID_MIN teams, so an input that
        // crowds a bin the last call found clean still spreads its retries)
        retry_upper_cur[b & 15] = u;
        Sym2Args r2 = a2;
        if (retry_prev[b & 15] >= 0 && retry_upper[b & 15] == u)
            r2.count = std::min<int32_t>(c, std::max<int32_t>(2 * retry_prev[b & 15] + 2, RETRY_GRID_MIN));
        if (u > SYM5_MAX) {   // SYM_CFG_BIG: sym5<32768>, its retries through the global tables
            const bool all = gtab_all(c1.wide_b);
            const size_t tab = (size_t)(b - N_SYM2_LDS - 1) * (all ? GT_GRID_ALL : GT_GRID_MAX) * GT_SLOTS;
            int32_t *gk = as<int32_t>(bufs[B_GTKEY]) + tab;
            uint32_t *go = as<uint32_t>(bufs[B_GTOWN]) + tab;
            Sym3Args a5{ax, B.col, SL + st[b], c, as<int32_t>(bufs[B_PROD]), nnz, bm, sa.dup_off,
                        sa.dupn, sa.dupt, dcap_for(u), DW_MAX, as<RowRef>(bufs[B_S3RETRY]) + st[b],
                        &dc->s3_retry[b & 15]};
            if (!all) {
                sym5_launch<GT_U, 8>(a5, t);
                CHECK_LAUNCH("k_sym5", t);
                gtab_launch(a5, r2.count, gk, go, t, GT_GRID_MAX);
            } else {   // B beyond 32-bit offsets: every row of the bin through the global tables
                a5.retry = SL + st[b];
                a5.retry_count = &dc->count[b];
                gtab_launch(a5, c, gk, go, t, GT_GRID_ALL);
            }
            CHECK_LAUNCH("k_sym_gtab", t);
            return IAS_SUCCESS;
        }
        if (!c1.wide_b && u > SYM4_MAX && u <= SYM5_MAX) {
            const Sym3Args a5{ax, B.col, SL + st[b], c, as<int32_t>(bufs[B_PROD]), nnz, bm, sa.dup_off,
                              sa.dupn, sa.dupt, dcap_for(u), DW_MAX, as<RowRef>(bufs[B_S3RETRY]) + st[b],
                              &dc->s3_retry[b & 15]};
            sym5_bin(u, a5, t);
            retry(SYM2_BINS[b - 1].cfg, a5, r2, t);
            CHECK_LAUNCH("k_sym5", t);
            return IAS_SUCCESS;
        }
        if (!c1.wide_b && u > SYM3_MAX && u <= SYM4_MAX) {
            const Sym3Args a4{ax, B.col, SL + st[b], c, as<int32_t>(bufs[B_PROD]), nnz, bm, sa.dup_off,
                              sa.dupn, sa.dupt, dcap_for(u), DW_MAX, as<RowRef>(bufs[B_S3RETRY]) + st[b],
                              &dc->s3_retry[b & 15]};
            sym4_launch<SYM4_MAX>(a4, t);
            retry(SYM2_BINS[b - 1].cfg, a4, r2, t);
            CHECK_LAUNCH("k_sym4", t);
            return IAS_SUCCESS;
        }
        if (!c1.wide_b && u >= SYM3_MIN && u <= SYM3_MAX) {
            const Sym3Args a3{ax, B.col, SL + st[b], c, as<int32_t>(bufs[B_PROD]), nnz, bm, sa.dup_off,
                              sa.dupn, sa.dupt, dcap_for(u), DW_MAX, as<RowRef>(bufs[B_S3RETRY]) + st[b],
                              &dc->s3_retry[b & 15]};   // a counter per bin (bins run concurrently)
            r2.lay = sym2_layout(u, u <= 1024 ? 4 : 5);   // the 128- / 256-lane team layout of this bound
            sym3_bin(u, a3, t);
            retry(u <= 1024 ? 4 : 5, a3, r2, t);
            CHECK_LAUNCH("k_sym3", t);
            return IAS_SUCCESS;
        }
        sym2_bin(SYM2_BINS[b - 1].cfg, a2, t);
        CHECK_LAUNCH("k_sym2", t);
        return IAS_SUCCESS;
    };
    for (int b = ss.nval; b >= 1; --b)
        if ((c = c1.count[b]) > 0) {
            hipStream_t t = (hipStream_t)side_stream(sym_lane[b]);
            bin_mark(b, t, 0);
            IAS_TRY(launch_sym(b, c, t));
            bin_mark(b, t, 1);
        }
    HIPC(hipGetLastError());
    IAS_TRY(join());

    // ---- row pointer of C, numeric binning by nnz (and products / nnz)
    int64_t *ptr = as<int64_t>(bufs[B_PTR]);
    IAS_TRY(reserve(B_NITEM, sizeof(PartItem) * (size_t)(rows + flops / NUM_PART_CAP + 2)));
    n2_units = n2_bunits = n2_dunits = 0;
    if (rows > 0) {
        k_scan_reduce<<<(unsigned)nb, SCAN_BLOCK, 0, s>>>(nnz, rows, as<int64_t>(bufs[B_PART]),
                                                          &dc2->max_nnz);
        k_scan_partials<<<1, 1024, 0, s>>>(as<int64_t>(bufs[B_PART]), nb);
        k_scan_apply<<<(unsigned)nb, SCAN_BLOCK, 0, s>>>(nnz, rows, as<int64_t>(bufs[B_PART]), ptr);
    CHECK_LAUNCH("scan", s);
        BIN_LAUNCH(k_bin_count, rows, s, nnz, as<int32_t>(bufs[B_PROD]), sa.dupn,
                                                                    rows, ns, dc2, ptr + rows);
        BIN_LAUNCH(k_bin_scatter, rows, s, 
            nnz, as<int32_t>(bufs[B_PROD]), sa.dupn, rows, ns, A, as<RowRef>(bufs[B_NLIST]),
            as<PartItem>(bufs[B_NITEM]), nullptr, as<int64_t>(bufs[B_WSOFF]), nullptr, nullptr, nullptr,
            nullptr, dc2, nullptr, nullptr, 0);
    CHECK_LAUNCH("numeric binning", s);
        // streaming rows exist only in the sym2 / partitioned bins (all rows
        // short, as K1 / K2: no unit lists to build)
        bool any_stream = c1.count[sym_part] > 0;
        for (int b = 1; b <= ss.nval; ++b) {
            if (c1.count[b] > 0 && SYM2_BINS[b - 1].upper > SHORT_MAX) any_stream = true;
        }
        if (any_stream) {
            // work units of the row-unit numeric pass: 64 A entries of a streaming row
            // (ordered by class: rows with > 256 duplicates, with fewer,
            // without — each class's fix-ups can start once its units are done)
            IAS_TRY(reserve(B_N2CNT, sizeof(int32_t) * (size_t)(3 * rows)));
            IAS_TRY(reserve(B_N2OFF, sizeof(int64_t) * (size_t)(3 * rows + 3)));
            IAS_TRY(reserve(B_N2UNIT, sizeof(Num2Unit) * (size_t)(rows + a_entries / N2_ENT + 1)));
            int32_t *cnt = as<int32_t>(bufs[B_N2CNT]);
            int64_t *uoff = as<int64_t>(bufs[B_N2OFF]);
            k_num2_count<<<grid_for(rows, 256), 256, 0, s>>>(A, rows, sa.dupn, as<int32_t>(bufs[B_PROD]), cnt);
            scan_i32(cnt, 3 * rows, as<int64_t>(bufs[B_PART]), uoff, s);
            k_num2_fill<<<grid_for(3 * rows, 256), 256, 0, s>>>(rows, cnt, uoff, as<Num2Unit>(bufs[B_N2UNIT]),
                                                                 dc2);
            CHECK_LAUNCH("k_num2_fill", s);
        }
    } else {
        HIPC(hipMemsetAsync(ptr, 0, sizeof(int64_t), s));
    }
    HIPC(hipGetLastError());
    HIPC(hipEventRecord(ev[2], s));
    // both counter sets: [1] nnz(C), unit counts; [0] the bins' retry counts
    HIPC(hipMemcpyAsync(hc, dc, 2 * sizeof(Counters), hipMemcpyDeviceToHost, s));
    HIPC((hipError_t)host_wait(s));
    // a bin's count is history only if this call launched it (retry_upper_cur
    // set): an empty or skipped bin says nothing about its retries
    for (int i = 0; i < 16; ++i) retry_prev[i] = (c1.wide_b || retry_upper_cur[i] == 0) ? -1 : hc[0].s3_retry[i];
    std::copy(retry_upper_cur, retry_upper_cur + 16, retry_upper);
    if (retry_print())   // IAS_RETRY_PRINT=1: rows each bin handed to sym2 (stderr)
        for (int i = 0; i < 16; ++i)
            if (retry_upper[i] > 0) fprintf(stderr, "ias retry: bin <= %d products: %d rows\n", retry_upper[i], retry_prev[i]);
    // the bins' durations are read by the next call, while its analysis runs
    // (here they would delay the return by ~60 us of event queries)
    const Counters c2 = hc[1];
    nnz_total = rows > 0 ? (int64_t)c2.nnz_total : 0;
    n2_units = (int64_t)c2.n2_units;
    n2_bunits = (int64_t)c2.n2_bunits;
    n2_dunits = (int64_t)c2.n2_dunits;
    if (c2.overflow) {
        set_last_error("hash partition table overflow in the symbolic pass");
        return IAS_ERROR_OVERFLOW;
    }
    std::copy(c2.count, c2.count + MAX_BINS, num_count);
    num_items = c2.items;
    num_ws = c2.ws_slots;
    st_prod = (int64_t)c2.st_prod;
    st_nnz = (int64_t)c2.st_nnz;
    max_nnz = c2.max_nnz;
    set_last_diag((uint32_t)c2.cbm_hits);
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

ias_status ias_plan::numeric(const Rows &A, const Rows &B, const Out &out_in, ias_report *rep) {
    hipStream_t s = (hipStream_t)stream;
    HIPC(hipSetDevice(device));
    const int64_t rows = n_rows;
    const BinSpec ns = num_spec();
    const int part_bin = ns.nval + 1, wide_bin = ns.nval + 2;
    if (num_count[wide_bin] > 0) IAS_TRY(reserve(B_WS, 20ull * num_ws));
    Out out = out_in;
    out.len = as<int32_t>(bufs[B_NNZ]);
    const RowRef *NL = as<RowRef>(bufs[B_NLIST]);
    Counters cc{};
    std::copy(num_count, num_count + MAX_BINS, cc.count);
    int64_t st[MAX_BINS];
    bin_starts(cc, st);
    Counters *dc2 = as<Counters>(bufs[B_CNT]) + 1;
    const AxView ax = ax_view();
    Bitmap bm{as<uint32_t>(bufs[B_BITS]), as<uint32_t>(bufs[B_BPREF]), as<int64_t>(bufs[B_BMOFF])};
    const StArgs sa{bm, as<int64_t>(bufs[B_DUPOFF]), as<int32_t>(bufs[B_DUPN]), as<int32_t>(bufs[B_DUPT])};
    HIPC(hipEventRecord(ev[3], s));
    int c;
    std::function<ias_status(hipStream_t, int)> launch_fix;   // part 0: sorted fix-ups, 1: the others, 2: all
    bool fix_split = false;
    int fix_lane = 0, n2_launches = 0, n2_mask = 0;
    // big bins first: their long rows start early and the small bins fill in
    // behind.  The table bins (partitioned, wide, direct-write) take the first
    // side streams and the streaming pass the next (at least the third), but
    // the streaming pass — the phase's critical path — is launched first: the
    // host issues ~30 API calls for the others (~60 us on K3')
    IAS_TRY(fork());
    int lane_no = num_count[wide_bin] > 0 ? 1 : 0;
    for (int i = 0; i < N_DW; ++i) lane_no += num_count[ns.nval + 3 + i] > 0 ? 1 : 0;
    auto launch_tables = [&]() -> ias_status {
        int tl = 0;
        // the partition tables (one workgroup per (row, partition), grids far
        // beyond residency) on the plan stream: on a side stream their
        // dispatch held the hardware queue, and the fix-ups and short rows of
        // the stream sharing it waited behind (K3: 3.9 ms of fix-ups after
        // the last streaming launch; round 5)
        if (num_count[part_bin] > 0) {
            hipStream_t t = s;
            k_numeric_part<1024, 4, 14, 256><<<(unsigned)num_items, 1024, 0, t>>>(
                ax, B, as<PartItem>(bufs[B_NITEM]), bm, out, &dc2->overflow);
            CHECK_LAUNCH("k_numeric_part", t);
        }
        if ((c = num_count[wide_bin]) > 0) {
            hipStream_t t = (hipStream_t)side_stream(tl++);
            k_numeric_global<1024, 2, 256><<<c, 1024, 0, t>>>(ax, B, NL + st[wide_bin], as<int64_t>(bufs[B_WSOFF]),
                                                              c, (char *)bufs[B_WS].p, out);
            CHECK_LAUNCH("k_numeric_global", t);
        }
        for (int i = N_DW - 1; i >= 0; --i) {
            const int b = ns.nval + 3 + i;
            if ((c = num_count[b]) > 0) {
                hipStream_t t = (hipStream_t)side_stream(tl++);
                dw_bin(DW_BINS[i].cfg, Launch{c, slots_for(DW_BINS[i].upper), t, ax, B, NL + st[b]}, out);
                CHECK_LAUNCH("k_numeric_dw", t);
            }
        }
        return IAS_SUCCESS;
    };
    // streaming rows: flat pass, then the duplicate fix-up (same stream, ordered).
    // Fixed lanes (side stream 2 for the pass, 3 for its fix-ups and the short
    // rows), whatever the bins before it: measured, the schedule is sensitive
    // to which streams share a hardware queue (K3' numeric 5.33 vs 5.90 ms when
    // an empty direct-write bin shifted the pass one stream down).
    if (n_entries > 0) {
        if (!serial && !small && lane_no < 2) lane_no = 2;
        hipStream_t t = (hipStream_t)side_stream(lane_no++);
        // fix-ups of the rows with duplicates: on the pass's stream after it,
        // or (split) the 1024-lane sorted fix-ups (> 4096 duplicates) on the
        // pass's stream right after their rows' units (they need whole CUs:
        // beside the pass they would starve), the others on the next side
        // stream once their class's units are done, beside the later units
        const int fb = ns.nval + 3 + N_DW;
        const bool fixups = num_count[fb] + num_count[fb + 1] + num_count[fb + 2] + num_count[fb + 3] +
                                num_count[fb + 4] > 0;
        // part 0: lists > 4096 (1024 lanes, whole CUs); 1: 1025 .. 4096; 2: the
        // rest; 3: all
        launch_fix = [&, fb](hipStream_t f, int part) -> ias_status {
            int cf;
            if ((part == 0 || part == 3) && (cf = num_count[fb + 4]) > 0) {
                static bool fb_done = false;
                allow_lds(k_fixup_big, fb_done, FIXBIG_LDS);
                k_fixup_big<<<cf, 1024, FIXBIG_LDS, f>>>(NL + st[fb + 4], cf, bm, sa.dup_off, sa.dupn, sa.dupt,
                                                         as<double>(bufs[B_DUPV]), out);
                CHECK_LAUNCH("k_fixup_big", f);
            }
            if ((part == 1 || part == 3) && (cf = num_count[fb + 3]) > 0) {
                static bool fl_done = false;
                allow_lds(k_fixup_large, fl_done, FIXLARGE_LDS);
                k_fixup_large<<<cf, 256, FIXLARGE_LDS, f>>>(NL + st[fb + 3], cf, bm, sa.dup_off, sa.dupn,
                                                            sa.dupt, as<double>(bufs[B_DUPV]), out);
                CHECK_LAUNCH("k_fixup_large", f);
            }
            if ((part == 2 || part == 3) && (cf = num_count[fb + 2]) > 0) {
                k_fixup_mid<<<cf, 256, 0, f>>>(NL + st[fb + 2], cf, bm, sa.dup_off, sa.dupn, sa.dupt,
                                               as<double>(bufs[B_DUPV]), out);
                CHECK_LAUNCH("k_fixup_mid", f);
            }
            if ((part == 2 || part == 3) && (cf = num_count[fb]) > 0) {
                k_fixup_tiny<<<grid_for(cf, 256), 256, 0, f>>>(NL + st[fb], cf, bm, sa.dup_off, sa.dupn, sa.dupt,
                                                               as<double>(bufs[B_DUPV]), out);
                CHECK_LAUNCH("k_fixup_tiny", f);
            }
            if ((part == 2 || part == 3) && (cf = num_count[fb + 1]) > 0) {
                k_fixup<<<grid_for(cf, FIX_TPW), WAVE * FIX_TPW, 0, f>>>(NL + st[fb + 1], cf, bm, sa.dup_off,
                                                                        sa.dupn, sa.dupt, as<double>(bufs[B_DUPV]),
                                                                        out);
                CHECK_LAUNCH("k_fixup", f);
            }
            return IAS_SUCCESS;
        };
        HIPC(hipEventRecord(ev[5], t));
        {
            if (n2_units > 0) {
                Num2Args na{A, ax, as<int64_t>(bufs[B_AXP]), as<int64_t>(bufs[B_POFF]), B.col, B.val,
                            as<Num2Unit>(bufs[B_N2UNIT]), n2_units, bm, sa.dup_off, as<double>(bufs[B_DUPV])};
                fix_split = fixups && !serial && !small;
                // units by class: [0, bunits) rows with > 1024 duplicates,
                // [bunits, dunits) with fewer, [dunits, units) without
                const int64_t cut[4] = {0, fix_split ? n2_bunits : 0, fix_split ? n2_dunits : 0, n2_units};
                for (int k = 0; k < 3; ++k) {
                    const int64_t nu = cut[k + 1] - cut[k];
                    if (nu > 0) {
                        Num2Args nk = na;
                        nk.units += cut[k];
                        nk.nunits = nu;
                        if (rep) HIPC(hipEventRecord(n2_ev[2 * k], t));
                        const unsigned g = (unsigned)((nu + N2_WPB - 1) / N2_WPB);
                        if (wide_v) {
                            if (out.order == 0) k_num2<true, 0><<<g, 64 * N2_WPB, 0, t>>>(nk, out);
                            else k_num2<true, 1><<<g, 64 * N2_WPB, 0, t>>>(nk, out);
                        } else {
                            if (out.order == 0) k_num2<false, 0><<<g, 64 * N2_WPB, 0, t>>>(nk, out);
                            else k_num2<false, 1><<<g, 64 * N2_WPB, 0, t>>>(nk, out);
                        }
                        if (rep) HIPC(hipEventRecord(n2_ev[2 * k + 1], t));
                        ++n2_launches;
                        n2_mask |= 1 << k;
                    }
                    if (fix_split && k < 2) HIPC(hipEventRecord(fix_ev[k], t));

                }
                fix_lane = lane_no;   // the fix-ups: the stream after this one
            }
        }
        HIPC(hipEventRecord(ev[6], t));
        CHECK_LAUNCH("k_num2", t);
        if (!fix_split) IAS_TRY(launch_fix(t, 3));
    }
    IAS_TRY(launch_tables());
    // short rows: all on the fix-up stream when the pass is split (ahead of
    // its waits; not behind the streaming pass on a shared queue)
    const int short_lane = fix_split ? fix_lane : -1;
    for (int i = 2; i >= 0 && ns.short_base > 0; --i)
        if ((c = num_count[ns.short_base + i]) > 0) {
            hipStream_t t = (hipStream_t)side_stream(short_lane >= 0 ? short_lane : lane_no++);
            const ShortArgs sh{A, ax, B.col, B.val, NL + st[ns.short_base + i], c, nullptr, nullptr};
            short_num_launch(i, sh, out, t);
            CHECK_LAUNCH("k_short_num", t);
        }
    for (int b = ns.nval; b >= 1; --b)
        if ((c = num_count[b]) > 0) {
            hipStream_t t = (hipStream_t)side_stream(lane_no++);
            val_bin(VAL_BINS[b - 1].cfg, Launch{c, slots_for(VAL_BINS[b - 1].upper), t, ax, B, NL + st[b]}, out);
            CHECK_LAUNCH("k_numeric_val", t);
        }
    if (fix_split) {
        hipStream_t f = (hipStream_t)side_stream(fix_lane);
        HIPC(hipStreamWaitEvent(f, fix_ev[0], 0));
        IAS_TRY(launch_fix(f, 0));
        IAS_TRY(launch_fix(f, 1));
        HIPC(hipStreamWaitEvent(f, fix_ev[1], 0));
        IAS_TRY(launch_fix(f, 2));
    }
    HIPC(hipGetLastError());
    IAS_TRY(join());
    if (out.row_idx && rows > 0)
        k_fill_rows<<<grid_for(rows * WAVE, 256), 256, 0, s>>>(out.ptr, rows, out.row_idx);
    HIPC(hipGetLastError());
    HIPC(hipEventRecord(ev[4], s));
    if (num_count[part_bin] > 0) {
        int32_t of = 0;
        HIPC(hipMemcpyAsync(&of, &dc2->overflow, sizeof(int32_t), hipMemcpyDeviceToHost, s));
        HIPC((hipError_t)host_wait(s));
        if (of) {
            set_last_error("hash partition table overflow in the numeric pass");
            return IAS_ERROR_OVERFLOW;
        }
    }
    if (rep) {
        HIPC(hipEventSynchronize(ev[4]));
        float a = 0, t = 0;
        hipEventElapsedTime(&a, ev[3], ev[4]);
        hipEventElapsedTime(&t, ev[0], ev[4]);
        rep->ms_numeric = a;
        rep->ms_total = t;
        float f = 0;
        if (n_entries > 0 && hipEventElapsedTime(&f, ev[5], ev[6]) == hipSuccess) rep->ms_stream = f;
        // split pass: the k_num2 launches alone (the class-0 fix-ups run
        // between them on the same stream)
        if (n2_mask) {
            float sum = 0;
            for (int k = 0; k < 3; ++k)
                if ((n2_mask >> k) & 1) {
                    float g = 0;
                    if (hipEventElapsedTime(&g, n2_ev[2 * k], n2_ev[2 * k + 1]) == hipSuccess) sum += g;
                }
            rep->ms_stream = sum;
        }
        rep->stream_products = st_prod;
        rep->stream_nnz = st_nnz;
        rep->stream_launches = n2_launches;
    }
    return IAS_SUCCESS;
}


// =================================================================== scan
// Exclusive scan of n int32 values into out[0..n] (out[n] = total), on `s`.
static void scan_i32(const int32_t *in, int64_t n, int64_t *part, int64_t *out, hipStream_t s) {
    const int64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
    k_scan_reduce<<<(unsigned)nb, SCAN_BLOCK, 0, s>>>(in, n, part, nullptr);
    k_scan_partials<<<1, 1024, 0, s>>>(part, nb);
    k_scan_apply<<<(unsigned)nb, SCAN_BLOCK, 0, s>>>(in, n, part, out);
}

// ------------------------------------------------------------------ row sort host
// A bucket-sort bin: persistent teams, one workgroup per resident slot at most.
template <int TEAM, int E, int TPW>
static void sort_bucket(const RowRef *list, int32_t c, const int64_t *ptr, int32_t *col, double *val,
                        hipStream_t t) {
    auto kern = k_sort_bucket<TEAM, E, TPW>;
    const int64_t grid = std::min<int64_t>(grid_for(c, TPW), resident_blocks(kern, TEAM * TPW, 0));
    kern<<<(unsigned)std::max<int64_t>(grid, 1), TEAM * TPW, 0, t>>>(list, c, ptr, col, val);
}

static ias_status sort_rows_impl(ias_plan *plan, const int64_t *ptr, const int32_t *len_in,
                                 int64_t stride, int64_t rows, int32_t *col, double *val) {
    if (rows <= 0) return IAS_SUCCESS;
    hipStream_t s = (hipStream_t)plan->stream;
    HIPC(hipSetDevice(plan->device));
    IAS_TRY(plan->reserve(ias_plan::B_TMP0, sizeof(int32_t) * (rows + 1)));
    IAS_TRY(plan->reserve(ias_plan::B_TMP1, sizeof(RowRef) * (rows + 1)));
    IAS_TRY(plan->reserve(ias_plan::B_TMP2, sizeof(int64_t) * (rows + 1)));
    IAS_TRY(plan->reserve(ias_plan::B_TMP3, sizeof(Counters)));
    const int32_t *len = len_in;
    if (ptr) {
        k_row_len<<<grid_for(rows, 256), 256, 0, s>>>(ptr, rows, (int32_t *)plan->bufs[ias_plan::B_TMP0].p);
        len = (const int32_t *)plan->bufs[ias_plan::B_TMP0].p;
    }
    Counters *dc = (Counters *)plan->bufs[ias_plan::B_TMP3].p;
    HIPC(hipMemsetAsync(dc, 0, sizeof(Counters), s));
    BinSpec spec{};
    spec.nval = 8;
    const int32_t u[] = {0, 64, 256, 512, 1024, 2048, 4096, 8192, 16384};
    for (int i = 0; i <= 8; ++i) spec.upper[i] = u[i];
    spec.part_cap = 1;
    // rows of at least this many entries -> the wide path (column bitmap /
    // segmented radix sort); IAS_SORT_WIDE_MIN: A/B knob
    static const int32_t wide_min_env = [] {
        const char *e = getenv("IAS_SORT_WIDE_MIN");
        const int v = e ? atoi(e) : 0;
        return v > 0 && v <= 16385 ? (int32_t)v : 16385;
    }();
    // the 8,193 .. 16,384 bin is the register bitmap sort: C's columns must fit
    // its bitmap, else those rows go to the wide path too
    spec.wide_min = plan->n_cols > 0 && plan->n_cols <= SORTBM_COLS ? wide_min_env : std::min(wide_min_env, 8193);
    RowRef *lists = (RowRef *)plan->bufs[ias_plan::B_TMP1].p;
    int64_t *offs = (int64_t *)plan->bufs[ias_plan::B_TMP2].p;
    // the scatter's row extents are not used by the sort kernels (they read ptr/len)
    const Rows span{ptr, len, stride, nullptr, nullptr};
    BIN_LAUNCH(k_bin_count, rows, s, len, nullptr, nullptr, rows, spec, dc);
    BIN_LAUNCH(k_bin_scatter, rows, s, len, nullptr, nullptr, rows, spec, span,
                                                                  lists, nullptr, nullptr, offs, nullptr,
                                                                  nullptr, nullptr, nullptr, dc, nullptr, nullptr, 0);
    Counters hc;
    HIPC(hipMemcpyAsync(&hc, dc, sizeof(Counters), hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    const int wide = spec.nval + 2;
    const int32_t nwide = hc.count[wide];
    int64_t st[MAX_BINS];
    bin_starts(hc, st);
    auto lst = [&](int b) { return lists + st[b]; };
    // wide rows: compact radix workspace (their entries, scanned), else the
    // padded per-row bitonic workspace (12 B per binning slot)
    const char *fg = getenv("IAS_SORT_GLOBAL");   // read per call: a test knob
    const bool force_global = fg && *fg == '1';
    bool radix = false;
    size_t rtmp = 0, slots = 0;
    int64_t *coff = nullptr;
    if (nwide > 0 && !force_global) {
        const int64_t nb = (nwide + SCAN_TILE - 1) / SCAN_TILE;
        IAS_TRY(plan->reserve(ias_plan::B_TMP5, 4ull * nwide + 8ull * (nwide + 1) + 8ull * (nb + 2) + 64));
        int32_t *wl = (int32_t *)plan->bufs[ias_plan::B_TMP5].p;
        coff = (int64_t *)(((uintptr_t)(wl + nwide) + 7) & ~(uintptr_t)7);
        int64_t *part = coff + nwide + 1;
        k_wide_len<<<grid_for(nwide, 256), 256, 0, s>>>(lst(wide), nwide, ptr, len, stride, wl);
        scan_i32(wl, nwide, part, coff, s);
        int64_t total = 0;
        HIPC(hipMemcpyAsync(&total, coff + nwide, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        HIPC(hipStreamSynchronize(s));
        slots = (size_t)total;
        if (total < (int64_t)INT32_MAX) {
            HIPC(hipcub::DeviceSegmentedRadixSort::SortPairs(
                nullptr, rtmp, (const int32_t *)nullptr, (int32_t *)nullptr, (const double *)nullptr,
                (double *)nullptr, (int)slots, nwide, (const int64_t *)nullptr, (const int64_t *)nullptr,
                0, 31, s));
            radix = plan->reserve(ias_plan::B_TMP4, 24ull * slots + 16ull * nwide + rtmp + 256) == IAS_SUCCESS;
            if (!radix) (void)hipGetLastError();   // allocation failure: take the bitonic workspace
        }
    }
    // wide rows by the column bitmap when C's columns fit it (the compact
    // workspace of the radix path, 12 B per entry, is its staging)
    const bool bitmap_sort = nwide > 0 && !force_global && plan->n_cols > 0 && plan->n_cols <= SORTBM_COLS;
    if (bitmap_sort && !radix) IAS_TRY(plan->reserve(ias_plan::B_TMP4, 16ull * slots + 16ull * nwide + 256));
    if (nwide > 0 && !radix && !bitmap_sort) IAS_TRY(plan->reserve(ias_plan::B_TMP4, 12ull * hc.ws_slots + 16));
    // one wave per row up to 512 entries (4 rows per workgroup, wave
    // barriers only), then teams sized so a row fills ~half their slots.
    // The bins run on the forked side streams, largest estimated work (rows x
    // mean entries) first onto the least-loaded stream, as the symbolic bins:
    // serially they summed to the whole sort pass (K3' 9.9 ms), the
    // column-bitmap kernels holding one workgroup per CU.
    auto launch = [&](int b, hipStream_t t) -> hipError_t {
        int c;
        switch (b) {
        case 1: c = hc.count[1]; sort_bucket<64, 1, 4>(lst(1), c, ptr, col, val, t); break;
        case 2: c = hc.count[2]; sort_bucket<64, 4, 4>(lst(2), c, ptr, col, val, t); break;
        case 3: c = hc.count[3]; sort_bucket<64, 8, 4>(lst(3), c, ptr, col, val, t); break;
        case 4: c = hc.count[4]; sort_bucket<128, 8, 1>(lst(4), c, ptr, col, val, t); break;
        case 5: c = hc.count[5]; sort_bucket<256, 8, 1>(lst(5), c, ptr, col, val, t); break;
        case 6: c = hc.count[6]; sort_bucket<512, 8, 1>(lst(6), c, ptr, col, val, t); break;
        case 7: c = hc.count[7]; sort_bucket<1024, 8, 1>(lst(7), c, ptr, col, val, t); break;
        case 8: {
            c = hc.count[8];
            const size_t lds = sortb2_lds((int32_t)plan->n_cols);
            static bool b2_done = false;
            allow_lds(k_sort_bitmap16, b2_done, lds);
            const int64_t grid = std::min<int64_t>(c, resident_blocks(k_sort_bitmap16, SORTBM_T, lds));
            k_sort_bitmap16<<<(unsigned)std::max<int64_t>(grid, 1), SORTBM_T, lds, t>>>(
                lst(8), c, ptr, len, stride, col, val, (int32_t)plan->n_cols);
            break;
        }
        default: {   // the wide rows
            c = nwide;
            if (bitmap_sort) {
                char *bp = (char *)plan->bufs[ias_plan::B_TMP4].p;
                double *wv = (double *)bp;   // 16 B per slot: value, column, position
                int32_t *wc = (int32_t *)(wv + slots);
                int32_t *wp = wc + slots;
                const size_t lds = sortbm_lds((int32_t)plan->n_cols);
                static bool sb_done = false;
                allow_lds(k_sort_bitmap, sb_done, lds);
                const int64_t grid = std::min<int64_t>(c, resident_blocks(k_sort_bitmap, SORTBM_T, lds));
                k_sort_bitmap<<<(unsigned)std::max<int64_t>(grid, 1), SORTBM_T, lds, t>>>(
                    lst(wide), c, coff, ptr, col, val, (int32_t)plan->n_cols, wc, wv, wp);
            } else if (radix) {
                char *bp = (char *)plan->bufs[ias_plan::B_TMP4].p;
                double *vin = (double *)bp;
                double *vout = vin + slots;
                int64_t *beg = (int64_t *)(vout + slots);
                int64_t *end = beg + c;
                int32_t *kin = (int32_t *)(end + c);
                int32_t *kout = kin + slots;
                void *tmp = (void *)(((uintptr_t)(kout + slots) + 255) & ~(uintptr_t)255);
                const dim3 g(c, 16);
                k_wide_gather<<<g, 256, 0, t>>>(lst(wide), c, coff, ptr, len, stride, col, val, kin, vin, beg,
                                                end, false);
                const hipError_t e = hipcub::DeviceSegmentedRadixSort::SortPairs(
                    tmp, rtmp, (const int32_t *)kin, kout, (const double *)vin, vout, (int)slots, c,
                    (const int64_t *)beg, (const int64_t *)end, 0, 31, t);
                if (e != hipSuccess) return e;
                k_wide_gather<<<g, 256, 0, t>>>(lst(wide), c, coff, ptr, len, stride, col, val, kout, vout,
                                                beg, end, true);
            } else {
                k_sort_global<<<c, 1024, 0, t>>>(lst(wide), c, offs, ptr, len, stride, col, val,
                                                 (char *)plan->bufs[ias_plan::B_TMP4].p);
            }
        }
        }
        return hipGetLastError();
    };
    std::vector<std::pair<double, int>> jobs;
    for (int b = 1; b <= 8; ++b)
        if (hc.count[b] > 0) jobs.push_back({(double)hc.count[b] * 0.5 * (double)(u[b - 1] + u[b]), b});
    if (nwide > 0) jobs.push_back({slots > 0 ? (double)slots : (double)nwide * 16384.0, wide});
    std::stable_sort(jobs.begin(), jobs.end(), [](const auto &x, const auto &y) { return x.first > y.first; });
    IAS_TRY(plan->fork());
    double load[ias_plan::NSIDE] = {};
    hipError_t le = hipSuccess;
    for (const auto &j : jobs) {
        const int i = (int)(std::min_element(load, load + ias_plan::NSIDE) - load);
        load[i] += j.first;
        if (le == hipSuccess) le = launch(j.second, (hipStream_t)plan->side_stream(i));
    }
    IAS_TRY(plan->join());   // the side streams join the plan stream even after a failed launch
    if (le != hipSuccess) {
        set_last_error("row sort launch failed: %s", hipGetErrorString(le));
        return le == hipErrorOutOfMemory ? IAS_ERROR_OUT_OF_MEMORY : IAS_ERROR_DEVICE;
    }
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

// Timing builds only: copy out (and reset) the per-phase cycle sums,
// TIMING_SLOTS x (TIMING_PHASES + 1) values (last = rows timed).
extern "C" int ias_debug_timing(unsigned long long *out, int n) {
#if IAS_TIMING
    const int total = TIMING_SLOTS * (TIMING_PHASES + 1);
    if (n < total) return -1;
    hipDeviceSynchronize();
    static unsigned long long all[TIMING_REPS * TIMING_SLOTS * (TIMING_PHASES + 1)];
    if (hipMemcpyFromSymbol(all, HIP_SYMBOL(g_timing), sizeof all) != hipSuccess) return -1;
    for (int i = 0; i < total; ++i) {
        out[i] = 0;
        for (int r = 0; r < TIMING_REPS; ++r) out[i] += all[r * total + i];
    }
    static unsigned long long zero[TIMING_REPS * TIMING_SLOTS * (TIMING_PHASES + 1)] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_timing), zero, sizeof zero) != hipSuccess) return -1;
    return total;
#else
    (void)out;
    (void)n;
    return 0;
#endif
}

ias_status ias::ias_shift_device(int64_t *p, int64_t n, int64_t off, void *stream) {
    if (n <= 0 || off == 0) return IAS_SUCCESS;
    k_shift<<<grid_for(n, 256), 256, 0, (hipStream_t)stream>>>(p, n, off);
    HIPC(hipGetLastError());
    return IAS_SUCCESS;
}
