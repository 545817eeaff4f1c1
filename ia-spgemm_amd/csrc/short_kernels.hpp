// short_kernels.hpp — rows of at most 64*K products (K = 1, 2, 4: the
// ELL-shaped and banded inputs, most R-MAT rows), one wave per row, no
// first-touch bitmap and no duplicate list: the symbolic pass counts the
// row's distinct columns in an LDS table, the numeric pass rebuilds the table
// with each column's first product and writes the row.
//
// Restates CSR_MUL_CSR (IA-SPGEMM-CPU_release/detail/csr/common_csr.h:95-189)
// and ELL_MUL_ELL (detail/ell/common_ell.h:80-189) for such rows: the
// column set of row i is the union of B's rows selected by A's row; the
// output lists the columns in reverse first-touch order (the reference's
// linked-list head insertion) — or forward for COO_MUL_COO
// (detail/coo/common_coo.h:136-156) — each value the sequential sum of its
// products in product order starting from 0.0 (or from the first product).
//
// Per row (wave): the row's A entries, 64 at a time, give each entry its
// first product (a DPP prefix sum of the B-row lengths) and set that product's
// bit in per-window start masks; product p = 64k + lane then finds its entry
// by a popcount (the flat/num2 mapping) and gathers B's column (and value).
// Columns go into an open-addressing LDS table (2 slots per product bound,
// CAS on the key); the numeric pass also keeps each column's smallest product
// (atomicMin) — that product is the first touch.  Ranks of the first touches
// in product order come from one ballot per window; duplicates (rare in these
// rows) are added to their column's value one lane at a time in product
// order; the row leaves LDS as one contiguous, coalesced store per array.
#pragma once

#include "spgemm_kernels.hpp"

namespace ias {
namespace dev {

constexpr int SH_WPB = 4;   // waves (rows) per workgroup
// table slots per product bound: symbolic K = 1, 2 rows; numeric K = 4 rows;
// symbolic K = 4 rows
constexpr int SH_SYM_SF12 = 2;
constexpr int SH_NUM_SF4 = 2;
constexpr int SH_SYM_SF4 = 4;
typedef int32_t sh_i32x4 __attribute__((ext_vector_type(4)));
typedef double sh_f64x2 __attribute__((ext_vector_type(2)));
constexpr int SH_ENT = 64;  // A entries per short row at most (the sym2 bins hold 8 * entries <= bound)
constexpr int32_t SH_EMPTY = -1;

struct ShortArgs {
    Rows A;
    AxView ax;
    const int32_t *bcol;
    const double *bval;
    const RowRef *list;   // rows of the bin (q0 = first A entry relative to A's base, n = A entries)
    int32_t count;
    int32_t *nnz_row;     // symbolic: nnz per row
    int32_t *dupn;        // symbolic: -5 marks the row for the short numeric pass
};

template <int K, bool NUM>
struct ShortLds {
    static constexpr int P = 64 * K;   // product bound
    // table slots: 2 per product bound; the symbolic pass's 256-product rows
    // 4 (shorter probe chains: K2 symbolic 1.01 -> 0.79 ms with one row per
    // wave — two rows per wave then need 8.5 KB of LDS per wave, 1.05 ms)
    static constexpr int S = (NUM ? (K >= 4 ? SH_NUM_SF4 : 2) : (K >= 4 ? SH_SYM_SF4 : SH_SYM_SF12)) * P;
    __attribute__((aligned(16))) int32_t keys[S];
    __attribute__((aligned(16))) int32_t minp[NUM ? S : 4];   // numeric: first product of the slot's column
    int64_t ebs[SH_ENT];         // non-empty entries: B-row start - row-relative first product
    double eav[NUM ? SH_ENT : 1];
    unsigned long long wmask[K];
    // the numeric pass stages a row's C values (up to P doubles) over minp
    static_assert(!NUM || sizeof(int32_t) * S >= sizeof(double) * P, "staged C values overflow minp");
};

__device__ __forceinline__ void sh_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One row's A entries in the lanes (entry `lane`, n <= 64): B-row length,
// start and A value, loaded one row ahead by the persistent loops below.
struct ShEnt {
    int32_t bl;
    int64_t bs;
    double av;
};
template <bool NUM>
__device__ __forceinline__ ShEnt sh_load(const ShortArgs &a, const RowRef &ref, bool valid) {
    const int lane = (int)(threadIdx.x & (WAVE - 1));
    ShEnt e{0, 0, 0.0};
    if (valid && lane < ref.n) {
        e.bl = a.ax.blen[ref.q0 + lane];
        e.bs = a.ax.bstart[ref.q0 + lane];
        if (NUM) e.av = a.ax.aval[ref.q0 + lane];
    }
    return e;
}
__device__ __forceinline__ RowRef sh_ref(const ShortArgs &a, int64_t idx) {
    RowRef r{0, -1, 0};
    if (idx < a.count) r = a.list[idx];
    return r;
}

// Stage the row's non-empty entries (bases, A values, start bits) and gather
// the columns (and products a*b when NUM) of p = 64k + lane < P; returns P,
// the row's products.
template <int K, bool NUM>
__device__ __forceinline__ int32_t short_gather(const ShortArgs &a, ShortLds<K, NUM> &L, const ShEnt &en,
                                                int32_t (&c)[K], double (&pv)[K]) {
    const int lane = (int)(threadIdx.x & (WAVE - 1));
    if (lane < K) L.wmask[lane] = 0ull;
    const int incl = wave_incl_sum(en.bl);
    const int rel = incl - en.bl;
    const int32_t P = __builtin_amdgcn_readlane(incl, WAVE - 1);
    const uint64_t ne = __ballot(en.bl > 0);
    sh_wave_sync();   // wmask cleared
    if (en.bl > 0) {
        const int o = __popcll(ne & ((1ull << lane) - 1ull));
        L.ebs[o] = en.bs - rel;
        if (NUM) L.eav[o] = en.av;
        atomicOr(&L.wmask[rel >> 6], 1ull << (rel & 63));
    }
    sh_wave_sync();
    const uint64_t upto = (2ull << lane) - 1ull;
    int before = 0;   // non-empty entries starting before window k
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const unsigned long long m = L.wmask[k];
        const int32_t p = 64 * k + lane;
        const int e = max(before + __popcll(m & upto) - 1, 0);
        const bool in = p < P;
        const int64_t kb = in ? L.ebs[e] + p : 0;
        c[k] = in ? a.bcol[kb] : SH_EMPTY;
        pv[k] = 0.0;
        if (NUM) pv[k] = in ? L.eav[e] * a.bval[kb] : 0.0;
        before += __popcll(m);
    }
    return P;
}

__device__ __forceinline__ uint32_t sh_hash(int32_t c, int lg) { return ((uint32_t)c * 0x9E3779B1u) >> (32 - lg); }

// Insert the K columns; slot[k] = the column's slot, made = new columns.  The
// first probe of all K items is issued back to back (items beyond P issue
// none: their CAS of the empty key into its home slot, one address for every
// idle lane, serialised in one bank); collisions then probe on.
template <int S, int K>
__device__ __forceinline__ int sh_insert(int32_t *keys, const int32_t (&c)[K], uint32_t (&slot)[K]) {
    constexpr int LG = __builtin_ctz(S);
    int made = 0;
    int32_t g[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        slot[k] = sh_hash(c[k], LG);
        int32_t o = SH_EMPTY;
        if (c[k] != SH_EMPTY) o = atomicCAS(&keys[slot[k]], SH_EMPTY, c[k]);
        g[k] = o;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        if (c[k] == SH_EMPTY) continue;
        if (g[k] == SH_EMPTY) {
            ++made;
            continue;
        }
        uint32_t s = slot[k];
        for (int probe = 1; probe < S && g[k] != c[k]; ++probe) {
            s = (s + 1) & (S - 1);
            g[k] = atomicCAS(&keys[s], SH_EMPTY, c[k]);
            if (g[k] == SH_EMPTY) {
                ++made;
                break;
            }
        }
        slot[k] = s;
    }
    return made;
}

// Rows with more duplicates than this take the table path (dupn -1: the
// numeric LDS value / direct-write bins), which adds them in parallel; the
// short numeric pass adds duplicates one at a time.
constexpr int SH_DUP_MAX = 8;   // K1 numeric 0.097 vs 0.103 ms with 16 (32: 0.103); K3' within noise

// Persistent waves (grid-stride over the bin's rows); the next row's list
// entry and A entries are loaded while this row is resolved.
template <int K>
__global__ __launch_bounds__(64 * SH_WPB) void k_short_sym(ShortArgs a) {
    using LDS = ShortLds<K, false>;
    __shared__ LDS lds[SH_WPB];
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / WAVE));
    const int lane = (int)(threadIdx.x & (WAVE - 1));
    const int64_t stride = (int64_t)gridDim.x * SH_WPB;
    int64_t idx = (int64_t)blockIdx.x * SH_WPB + w;
    if (idx >= a.count) return;
    LDS &L = lds[w];
    for (int i = lane; i < LDS::S; i += WAVE) L.keys[i] = SH_EMPTY;
    RowRef ref = sh_ref(a, idx);
    ShEnt en = sh_load<false>(a, ref, true);
    RowRef nref = sh_ref(a, idx + stride);
    while (idx < a.count) {
        const bool nv = idx + stride < a.count;
        const ShEnt nen = sh_load<false>(a, nref, nv);
        const RowRef nnref = sh_ref(a, idx + 2 * stride);
        int32_t c[K];
        double pv[K];
        const int32_t P = short_gather<K, false>(a, L, en, c, pv);
        uint32_t slot[K];
        const int made = sh_insert<LDS::S, K>(L.keys, c, slot);
        const int nnz = __builtin_amdgcn_readlane(wave_incl_sum(made), WAVE - 1);
        if (lane == 0) {
            a.nnz_row[ref.row] = nnz;
            a.dupn[ref.row] = P - nnz > SH_DUP_MAX ? -1 : -5;
        }
        sh_wave_sync();   // every insert has landed
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (c[k] != SH_EMPTY) L.keys[slot[k]] = SH_EMPTY;   // the table empty for the next row
        sh_wave_sync();
        ref = nref;
        en = nen;
        nref = nnref;
        idx += stride;
    }
}

// R rows per wave (symbolic): the rows' staging, gathers and first probes are
// issued together, so one wave keeps R rows' dependent chains (list -> A
// entries -> B columns -> LDS CAS) in flight instead of one.
template <int K, int R, bool NUM>
__device__ __forceinline__ void short_gather_r(const ShortArgs &a, ShortLds<K, NUM> (&L)[R], const ShEnt (&en)[R],
                                               int32_t (&c)[R][K], double (&pv)[R][K], int32_t (&P)[R]) {
    const int lane = (int)(threadIdx.x & (WAVE - 1));
    int rel[R];
    uint64_t ne[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (lane < K) L[r].wmask[lane] = 0ull;
        const int incl = wave_incl_sum(en[r].bl);
        rel[r] = incl - en[r].bl;
        P[r] = __builtin_amdgcn_readlane(incl, WAVE - 1);
        ne[r] = __ballot(en[r].bl > 0);
    }
    sh_wave_sync();   // wmask cleared
#pragma unroll
    for (int r = 0; r < R; ++r)
        if (en[r].bl > 0) {
            const int o = __popcll(ne[r] & ((1ull << lane) - 1ull));
            L[r].ebs[o] = en[r].bs - rel[r];
            if (NUM) L[r].eav[o] = en[r].av;
            atomicOr(&L[r].wmask[rel[r] >> 6], 1ull << (rel[r] & 63));
        }
    sh_wave_sync();
    const uint64_t upto = (2ull << lane) - 1ull;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        int before = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const unsigned long long m = L[r].wmask[k];
            const int32_t p = 64 * k + lane;
            const int e = max(before + __popcll(m & upto) - 1, 0);
            const bool in = p < P[r];
            const int64_t kb = in ? L[r].ebs[e] + p : 0;
            c[r][k] = in ? a.bcol[kb] : SH_EMPTY;
            pv[r][k] = 0.0;
            if (NUM) pv[r][k] = in ? L[r].eav[e] * a.bval[kb] : 0.0;
            before += __popcll(m);
        }
    }
}

// sh_insert over R tables: every item's first probe is issued before any
// collision is chased.
template <int S, int K, int R, typename T>
__device__ __forceinline__ void sh_insert_r(T (&L)[R], const int32_t (&c)[R][K], uint32_t (&slot)[R][K],
                                            int (&made)[R]) {
    constexpr int LG = __builtin_ctz(S);
    int32_t g[R][K];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int k = 0; k < K; ++k) {
            slot[r][k] = sh_hash(c[r][k], LG);
            int32_t o = SH_EMPTY;   // items beyond P issue nothing (see sh_insert)
            if (c[r][k] != SH_EMPTY) o = atomicCAS(&L[r].keys[slot[r][k]], SH_EMPTY, c[r][k]);
            g[r][k] = o;
        }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        made[r] = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (c[r][k] == SH_EMPTY) continue;
            if (g[r][k] == SH_EMPTY) {
                ++made[r];
                continue;
            }
            uint32_t s = slot[r][k];
            for (int probe = 1; probe < S && g[r][k] != c[r][k]; ++probe) {
                s = (s + 1) & (S - 1);
                g[r][k] = atomicCAS(&L[r].keys[s], SH_EMPTY, c[r][k]);
                if (g[r][k] == SH_EMPTY) {
                    ++made[r];
                    break;
                }
            }
            slot[r][k] = s;
        }
    }
}

template <int K, int R>
__global__ __launch_bounds__(64 * SH_WPB) void k_short_sym_r(ShortArgs a) {
    using LDS = ShortLds<K, false>;
    __shared__ LDS lds[SH_WPB][R];
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / WAVE));
    const int lane = (int)(threadIdx.x & (WAVE - 1));
    const int64_t idx = ((int64_t)blockIdx.x * SH_WPB + w) * R;
    if (idx >= a.count) return;
    LDS(&L)[R] = lds[w];
    RowRef ref[R];
    ShEnt en[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        for (int i = lane; i < LDS::S; i += WAVE) L[r].keys[i] = SH_EMPTY;
        ref[r] = sh_ref(a, idx + r);
        en[r] = sh_load<false>(a, ref[r], idx + r < a.count);
    }
    int32_t c[R][K], P[R];
    double pv[R][K];
    short_gather_r<K, R, false>(a, L, en, c, pv, P);
    uint32_t slot[R][K];
    int made[R];
    sh_insert_r<LDS::S, K, R>(L, c, slot, made);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int nnz = __builtin_amdgcn_readlane(wave_incl_sum(made[r]), WAVE - 1);
        if (lane == 0 && idx + r < a.count) {
            a.nnz_row[ref[r].row] = nnz;
            a.dupn[ref[r].row] = P[r] - nnz > SH_DUP_MAX ? -1 : -5;
        }
    }
}

__device__ __forceinline__ double sh_readlane(double v, int l) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
constexpr int SH_NUM_WPE = 1; // minimum waves per SIMD the register allocation must allow (A/B knob)
template <int K>
__global__ __launch_bounds__(64 * SH_WPB) __attribute__((amdgpu_waves_per_eu(SH_NUM_WPE))) void k_short_num(ShortArgs a, Out out) {
    using LDS = ShortLds<K, true>;
    __shared__ LDS lds[SH_WPB];
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / WAVE));
    const int lane = (int)(threadIdx.x & (WAVE - 1));
    const int64_t stride = (int64_t)gridDim.x * SH_WPB;
    int64_t idx = (int64_t)blockIdx.x * SH_WPB + w;
    if (idx >= a.count) return;
    LDS &L = lds[w];
    for (int i = lane; i < LDS::S / 4; i += WAVE) {
        ((int4 *)L.keys)[i] = make_int4(SH_EMPTY, SH_EMPTY, SH_EMPTY, SH_EMPTY);
        ((int4 *)L.minp)[i] = make_int4(0x7FFFFFFF, 0x7FFFFFFF, 0x7FFFFFFF, 0x7FFFFFFF);
    }
    const uint64_t lt = (1ull << lane) - 1ull;
    RowRef ref = sh_ref(a, idx);
    ShEnt en = sh_load<true>(a, ref, true);
    // C's row start is loaded with the row's A entries (not after the table
    // work: one dependent global load less per row)
    int64_t st = out.start(ref.row);
    int32_t rn = out.len[ref.row];   // the row's nnz (symbolic pass)
    RowRef nref = sh_ref(a, idx + stride);
    while (idx < a.count) {
        const bool nvalid = idx + stride < a.count;
        const ShEnt nen = sh_load<true>(a, nref, nvalid);
        const int32_t nrn = nvalid ? out.len[nref.row] : 0;
        const int64_t nst = nvalid ? out.start(nref.row) : 0;
        const RowRef nnref = sh_ref(a, idx + 2 * stride);
        int32_t c[K];
        double pv[K];
        const int32_t P = short_gather<K, true>(a, L, en, c, pv);
        if (rn == P) {
            // no duplicates (nnz = products): every product is its column's
            // first touch, rank = product index — C is the products in reverse
            // (forward for COO) order, each 0.0 + a*b (a*b); no table
#pragma unroll
            for (int k = 0; k < K; ++k)
                if (c[k] != SH_EMPTY) {
                    const int32_t p = 64 * k + lane;
                    const int64_t pos = st + (out.order == 0 ? P - 1 - p : p);
                    __builtin_nontemporal_store(c[k], &out.col[pos]);
                    __builtin_nontemporal_store(out.first_assign ? pv[k] : 0.0 + pv[k], &out.val[pos]);
                }
            ref = nref;
            en = nen;
            rn = nrn;
            st = nst;
            nref = nnref;
            idx += stride;
            continue;
        }
        uint32_t slot[K];
        sh_insert<LDS::S, K>(L.keys, c, slot);
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (c[k] != SH_EMPTY) atomicMin(&L.minp[slot[k]], 64 * k + lane);
        sh_wave_sync();
        // first touches, their ranks in product order; values 0.0 + a*b (or a*b)
        bool ft[K];
        int32_t rk[K], pf[K];
        int nft = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            pf[k] = c[k] != SH_EMPTY ? L.minp[slot[k]] : -1;
            ft[k] = pf[k] == 64 * k + lane;
            const uint64_t b = __ballot(ft[k]);
            rk[k] = nft + __popcll(b & lt);
            nft += __popcll(b);
            if (ft[k] && !out.first_assign) pv[k] = 0.0 + pv[k];
        }
        sh_wave_sync();   // every lane has read the table
        // duplicates (at most SH_DUP_MAX): added to their first touch's
        // register, one at a time in product order
#pragma unroll
        for (int k = 0; k < K; ++k) {
            uint64_t dm = __ballot(c[k] != SH_EMPTY && !ft[k]);
            while (dm) {
                const int l = __builtin_ctzll(dm);
                dm &= dm - 1;
                const int f = __builtin_amdgcn_readlane(pf[k], l);
                const double add = sh_readlane(pv[k], l);
                const int kf = f >> 6, lf = f & 63;
#pragma unroll
                for (int j = 0; j <= k; ++j)
                    if (j == kf) {
                        const double v = sh_readlane(pv[j], lf) + add;
                        if (lane == lf) pv[j] = v;
                    }
            }
        }
        // The row's C entries staged by position in the table's LDS (no longer
        // needed: the next row re-initialises it) and written as ascending
        // 16-byte pieces aligned to the destination (4 columns / 2 values per
        // lane; scalar stores for the partial pieces at the ends): whole lines
        // leave instead of descending 4- / 8-byte runs (K2: 20 % write
        // amplification measured with the runs).
        int32_t *scol = L.keys;
        double *sval = (double *)L.minp;
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (ft[k]) {
                const int x = out.order == 0 ? nft - 1 - rk[k] : rk[k];
                scol[x] = c[k];
                sval[x] = pv[k];
            }
        sh_wave_sync();
        {
            const int64_t cph = (int64_t)(((uintptr_t)(out.col + st) >> 2) & 3u);
            const int64_t vph = (int64_t)(((uintptr_t)(out.val + st) >> 3) & 1u);
            const int a4 = (int)((4 - cph) & 3), a2 = (int)((2 - vph) & 1);   // first aligned index
            const int e4 = a4 + ((nft - a4) > 0 ? ((nft - a4) & ~3) : 0);
            const int e2 = a2 + ((nft - a2) > 0 ? ((nft - a2) & ~1) : 0);
            for (int x = a4 + 4 * lane; x + 4 <= e4; x += 4 * WAVE) {
                const int4 v = make_int4(scol[x], scol[x + 1], scol[x + 2], scol[x + 3]);
                __builtin_nontemporal_store(*(const sh_i32x4 *)&v, (sh_i32x4 *)(out.col + st + x));
            }
            for (int x = a2 + 2 * lane; x + 2 <= e2; x += 2 * WAVE) {
                const sh_f64x2 v = {sval[x], sval[x + 1]};
                __builtin_nontemporal_store(v, (sh_f64x2 *)(out.val + st + x));
            }
            // ends: columns [0, min(a4, nft)) and [max(e4, a4), nft); values likewise
            int xc = -1, xv = -1;
            if (lane < 3) xc = lane < min(a4, nft) ? lane : -1;
            else if (lane < 6) xc = max(e4, a4) + (lane - 3) < nft ? max(e4, a4) + (lane - 3) : -1;
            else if (lane == 6) xv = 0 < min(a2, nft) ? 0 : -1;
            else if (lane == 7) xv = max(e2, a2) < nft ? max(e2, a2) : -1;
            if (xc >= 0) __builtin_nontemporal_store(scol[xc], &out.col[st + xc]);
            if (xv >= 0) __builtin_nontemporal_store(sval[xv], &out.val[st + xv]);
        }
        sh_wave_sync();
        // the table for the next row (persistent waves only)
        if (idx + stride < a.count) {
            for (int i = lane; i < LDS::S / 4; i += WAVE) {
                ((int4 *)L.keys)[i] = make_int4(SH_EMPTY, SH_EMPTY, SH_EMPTY, SH_EMPTY);
                ((int4 *)L.minp)[i] = make_int4(0x7FFFFFFF, 0x7FFFFFFF, 0x7FFFFFFF, 0x7FFFFFFF);
            }
            sh_wave_sync();
        }
        ref = nref;
        en = nen;
        rn = nrn;
        st = nst;
        nref = nnref;
        idx += stride;
    }
}

}  // namespace dev
}  // namespace ias
