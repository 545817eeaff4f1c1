// num2_kernels.hpp — numeric pass of the streaming rows (rows whose
// duplicates fit their list, dupn >= 0) with C written through LDS in whole,
// ascending, 16-byte-aligned pieces.
//
// Restates CSR_MUL_CSR's second loop (IA-SPGEMM-CPU_release/detail/csr/
// common_csr.h:133-189) for rows the symbolic pass has already resolved: bit p
// of a row's first-touch bitmap says whether product p is its column's first
// touch, its rank (set bits before it) is the column's discovery index, and
// the entry lands at row_start + nnz-1-rank (reverse first-touch, the
// reference's linked-list order) or row_start + rank (COO_MUL_COO's order);
// the value is 0.0 + a*b (or a*b for COO).  A duplicate's product is parked at
// dupval[dup_off + p - rank] for the fix-up kernels, which add it to its
// column's entry in product order.
//
// Unit of work: one wave takes 64 consecutive A entries of one row (a unit);
// their products are one contiguous product range of the row, so the C
// entries they produce are one contiguous range of C.  Lanes walk the range
// in 64-aligned windows of the row's product space (bitmap words and their
// prefix counts are then two scalar loads per window), the window's entries
// from per-window start masks (the flat pass's mapping), and the first
// touches are staged in LDS by rank, PASS of them at a time, then leave as
// ascending 16-byte stores (4 columns / 2 values per lane) — measured: the
// flat pass's reverse-order 4- and 8-byte scatter stores took ~3 of its 5 ms.
#pragma once

#include <type_traits>

#include "spgemm_kernels.hpp"
#include "spgemm_engine.hpp"   // Counters

namespace ias {
namespace dev {

constexpr int N2_ENT = 64;     // A entries per unit (one per lane)
constexpr int N2_WPB = 4;      // waves (units) per workgroup

struct Num2Unit {
    int32_t row;
    int32_t e0;   // first A entry of the unit within the row
};

struct Num2Args {
    Rows A;                  // A's rows (entry ranges)
    AxView ax;               // expanded A: B-row start / length, A value per entry
    const int64_t *axp;      // product offset of every A entry
    const int64_t *poff;     // product offset of every row
    const int32_t *bcol;
    const double *bval;
    const Num2Unit *units;
    int64_t nunits;
    Bitmap bm;
    const int64_t *dup_off;
    double *dupval;
};

// Units: every streaming row with products gets ceil(entries / 64) of them,
// counted in three lists — rows with more than N2_BIGDUP duplicates (the
// sorted fix-ups of long lists), rows with fewer, rows without — at
// cnt[cls*rows + r], so one scan over 3*rows orders the units by class: each
// class's fix-ups can start once its units are done.
constexpr int32_t N2_BIGDUP = 1024;   // = FIXMID_CAP
__global__ void k_num2_count(Rows A, int64_t rows, const int32_t *dupn, const int32_t *prod, int32_t *cnt) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    int64_t s;
    int32_t n;
    A.row(r, s, n);
    const int32_t d = dupn[r];
    const int32_t u = (d >= 0 && prod[r] > 0) ? (n + N2_ENT - 1) / N2_ENT : 0;
    const int cls = d > N2_BIGDUP ? 0 : (d > 0 ? 1 : 2);
#pragma unroll
    for (int c = 0; c < 3; ++c) cnt[c * rows + r] = c == cls ? u : 0;
}
// uoff: exclusive scan of cnt[0 .. 3*rows] (uoff[3*rows] = all units); thread 0
// also stores the unit count and the class boundaries in the counters
__global__ void k_num2_fill(int64_t rows, const int32_t *cnt, const int64_t *uoff, Num2Unit *units,
                            Counters *tot) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) {
        tot->n2_units = (unsigned long long)uoff[3 * rows];
        tot->n2_bunits = (unsigned long long)uoff[rows];
        tot->n2_dunits = (unsigned long long)uoff[2 * rows];
    }
    if (i >= 3 * rows) return;
    const int32_t c = cnt[i];
    const int64_t o = uoff[i];
    const int32_t r = (int32_t)(i % rows);
    for (int32_t j = 0; j < c; ++j) units[o + j] = Num2Unit{r, j * N2_ENT};
}

// 16-byte non-temporal store (C is not read back by this pass)
typedef uint32_t n2_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st16(void *p, uint4 v) {
    const n2_u32x4 x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, (n2_u32x4 *)p);
}

// N2_K windows per step: their gathers are in flight together, and the next
// step's gathers are issued before this step's stores (vmcnt retires loads and
// stores in issue order, so a load behind a store would wait for the store).
constexpr int N2_K = 4;

constexpr int N2_WPE = 1;   // minimum waves per SIMD the register allocation must allow (1: no cap)
// W64: B's entries beyond 2^29 (byte offsets of its values beyond 32 bits):
// 64-bit gather addresses.  Otherwise (round 5) every gather is a 32-bit
// byte offset from the array's SGPR base, the entries' bases are 32-bit, and
// C's positions within a step are 32-bit offsets from a uniform base: the
// 64-bit address arithmetic was ~a fifth of the kernel's VALU instructions.
// ORD: C's order (0: reverse first touch, 1: forward), a template argument
// so the staging index needs no select.
template <bool W64, int ORD>
__global__ __launch_bounds__(64 * N2_WPB) __attribute__((amdgpu_waves_per_eu(N2_WPE))) void k_num2(Num2Args a,
                                                                                                 Out out) {
    constexpr int K = N2_K;
    constexpr int PASS = 64 * K;   // staged C entries per step (at most one per product)
    using BsT = typename std::conditional<W64, int64_t, int32_t>::type;
    struct Ent {
        BsT bs;       // B-row start - row-relative first product of the entry
        double av;
    };
    __shared__ Ent ent[N2_WPB][N2_ENT];
    __shared__ unsigned long long wmask[N2_WPB][K];
    // staged in C's order, aligned as C is: slot = C position - a base
    // congruent to C's 16-byte pieces, so each piece is one 16-byte LDS read
    __shared__ __attribute__((aligned(16))) int32_t scol[N2_WPB][PASS + 4];   // rows of 1,040 B
    __shared__ __attribute__((aligned(16))) double sval[N2_WPB][PASS + 2];    // rows of 2,064 B
    static_assert((PASS + 4) * 4 % 16 == 0 && (PASS + 2) * 8 % 16 == 0, "16-byte aligned staging rows");
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / WAVE));
    const int lane = (int)(threadIdx.x & (WAVE - 1));
    const int64_t u = (int64_t)blockIdx.x * N2_WPB + w;
    if (u >= a.nunits) return;
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    const Num2Unit un = a.units[u];
    const int64_t row = un.row;
    int64_t as;
    int32_t an;
    a.A.row(row, as, an);
    const int64_t q0 = as - a.A.base() + un.e0;
    const int32_t n = min(N2_ENT, an - un.e0);
    const int64_t prow = a.poff[row];
    // this lane's entry
    int32_t bl = 0, rel = 0;
    int64_t bs = 0;
    double av = 0.0;
    if (lane < n) {
        bl = a.ax.blen[q0 + lane];
        bs = a.ax.bstart[q0 + lane];
        av = a.ax.aval[q0 + lane];
        rel = (int32_t)(a.axp[q0 + lane] - prow);
    }
    // the unit's products [pa, pb) of the row
    const int32_t pa = __builtin_amdgcn_readfirstlane(rel);
    const int32_t pb = __builtin_amdgcn_readlane(rel + bl, n - 1);
    if (pb <= pa) return;
    // non-empty entries, compacted in order
    const uint64_t ne = __ballot(bl > 0);
    if (bl > 0) ent[w][__popcll(ne & ((1ull << lane) - 1ull))] = Ent{(BsT)(bs - rel), av};
    const int64_t cst = out.start(row);
    const int32_t nnz = out.len[row];
    const int64_t bmo = a.bm.off[row];
    const int64_t dbase = a.dup_off[row];
    const int64_t cbase = ORD == 0 ? cst + nnz - 1 : cst;   // C position of rank 0
    const uint64_t upto = (2ull << lane) - 1ull;           // bits 0..lane
    const uint32_t below = (1u << (lane & 31)) - 1u;
    // 16-byte pieces start where the destination address is 16-byte aligned
    const int64_t cph = (int64_t)(((uintptr_t)out.col >> 2) & 3u);
    const int64_t vph = (int64_t)(((uintptr_t)out.val >> 3) & 1u);
    // rank of the unit's first product = the row's first touches before pa
    int32_t r0;
    {
        const uint32_t wd = a.bm.bits[bmo + (pa >> 5)];
        r0 = (int32_t)a.bm.pref[bmo + (pa >> 5)] + __popc(wd & ((1u << (pa & 31)) - 1u));
    }
    struct Step {
        int32_t c[K];
        double bv[K];
        int32_t e[K];
        // the step's 2K bitmap words (lanes 0 .. 2K-1) and their prefix counts
        // (lanes 2K .. 4K-1): one load of 4K lanes instead of two 64-lane
        // loads per window — the texture addresser, not HBM, bounds this pass
        // (TA busy 90 % of its cycles, round 5), and every lane of those
        // loads read one of two addresses
        uint32_t wp;
    };
    const char *bcol = (const char *)a.bcol;
    const char *bval = (const char *)a.bval;
    // gathers of the step at window pw0.  Branch-free (clamped addresses for
    // the lanes and words outside the unit), so that the wait for a step's
    // loads counts exactly the loads issued after them.
    const int64_t lastw = bmo + ((pb - 1) >> 5);
    auto load = [&](int32_t pw0, Step &S) {
        if (lane < K) wmask[w][lane] = 0ull;
        wave_sync();
        if (bl > 0 && rel >= pw0 && rel < pw0 + PASS)
            atomicOr(&wmask[w][(rel - pw0) >> 6], 1ull << ((rel - pw0) & 63));
        wave_sync();
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int32_t pw = pw0 + 64 * k;
            const int32_t p = pw + lane;
            const int ecur = (int)__popcll(__ballot(bl > 0 && rel < pw));
            const int ei = ecur + (int)__popcll(wmask[w][k] & upto) - 1;
            S.e[k] = ei > 0 ? ei : 0;
            if constexpr (W64) {
                const int64_t kb = (p >= pa && p < pb) ? ent[w][S.e[k]].bs + p : 0;
                S.c[k] = a.bcol[kb];
                S.bv[k] = a.bval[kb];
            } else {
                const uint32_t kb = (p >= pa && p < pb) ? (uint32_t)(ent[w][S.e[k]].bs + p) : 0u;
                S.c[k] = *(const int32_t *)(bcol + (kb << 2));
                S.bv[k] = *(const double *)(bval + (kb << 3));
            }
        }
        {
            const int j = lane & (2 * K - 1);
            const int64_t wi = min(bmo + (pw0 >> 5) + j, lastw);
            const uint32_t *src = lane < 2 * K ? a.bm.bits : a.bm.pref;
            S.wp = src[wi];
        }
    };
    // window k's bitmap word and prefix for this lane (lanes 0-31: the
    // window's first word, 32-63: its second)
    auto words_of = [&](const Step &S, int k, uint32_t &word, uint32_t &pre) {
        const uint32_t w0 = (uint32_t)__builtin_amdgcn_readlane((int)S.wp, 2 * k);
        const uint32_t w1 = (uint32_t)__builtin_amdgcn_readlane((int)S.wp, 2 * k + 1);
        const uint32_t q0 = (uint32_t)__builtin_amdgcn_readlane((int)S.wp, 2 * K + 2 * k);
        const uint32_t q1 = (uint32_t)__builtin_amdgcn_readlane((int)S.wp, 2 * K + 2 * k + 1);
        word = lane < 32 ? w0 : w1;
        pre = lane < 32 ? q0 : q1;
    };
    // stage the step's first touches by rank, park its duplicates, flush
    auto store = [&](int32_t pw0, const Step &S) {
        // the step's C positions: ranks r0 .. r0 + nft - 1; ORD 0 puts rank r
        // at cbase - r (xhi = cbase - r0 + 1 known before the step), ORD 1 at
        // cbase + r (xlo = cbase + r0).  Staging bases: the step's lowest
        // possible position rounded down to a 16-byte piece of C.
        const int64_t lo = ORD == 0 ? cbase - r0 + 1 - PASS : cbase + r0;
        const int64_t xbc = ((lo + cph) & ~3ll) - cph, xbv = ((lo + vph) & ~1ll) - vph;
        // slot of rank rk: ORD 0: (cbase - xb) - rk, ORD 1: (cbase - xb) + rk
        const int32_t oc = (int32_t)(cbase - xbc), ov = (int32_t)(cbase - xbv);
        int nft = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int32_t p = pw0 + 64 * k + lane;
            uint32_t word, pre;
            words_of(S, k, word, pre);
            const bool in = p >= pa && p < pb;
            const bool ft = in && ((word >> (lane & 31)) & 1u);
            const int32_t rk = (int32_t)(pre + (uint32_t)__popc(word & below));
            const double prod = ent[w][S.e[k]].av * S.bv[k];
            if (ft) {
                scol[w][ORD == 0 ? oc - rk : oc + rk] = S.c[k];
                sval[w][ORD == 0 ? ov - rk : ov + rk] = out.first_assign ? prod : 0.0 + prod;
            } else if (in) {
                a.dupval[dbase + (p - rk)] = prod;
            }
            nft += __popcll(__ballot(ft));
        }
        wave_sync();
        // C positions of the staged ranks: [xlo, xhi)
        const int64_t xlo = ORD == 0 ? cbase - (r0 + nft - 1) : cbase + r0;
        const int64_t xhi = xlo + nft;
        // whole 16-byte pieces: [a4, e4) of the columns, [a2, e2) of the values
        const int64_t a4 = ((xlo + cph + 3) & ~3ll) - cph, e4 = ((xhi + cph) & ~3ll) - cph;
        const int64_t a2 = ((xlo + vph + 1) & ~1ll) - vph, e2 = ((xhi + vph) & ~1ll) - vph;
        {
            const int32_t sb = (int32_t)(a4 - xbc), span = (int32_t)(e4 - a4);
            int32_t *cb = out.col + a4;   // uniform base, 32-bit lane offsets
#pragma unroll
            for (int it = 0; it < (PASS / 4 + WAVE) / WAVE; ++it) {
                const int32_t d = 4 * (lane + WAVE * it);
                if (d + 4 <= span) st16(cb + d, ((const uint4 *)scol[w])[(sb + d) >> 2]);   // sb + d: a multiple of 4
            }
        }
        {
            const int32_t sb = (int32_t)(a2 - xbv), span = (int32_t)(e2 - a2);
            double *vb = out.val + a2;
#pragma unroll
            for (int it = 0; it < (PASS / 2 + WAVE) / WAVE; ++it) {
                const int32_t d = 2 * (lane + WAVE * it);
                if (d + 2 <= span) st16(vb + d, ((const uint4 *)sval[w])[(sb + d) >> 1]);   // sb + d: even
            }
        }
        // the partial pieces at both ends: lanes 0-2 / 3-5 columns, 6 / 7 values
        {
            int32_t dc = -1, dv = -1;   // offsets from xlo
            const int32_t ha4 = (int32_t)(min(a4, xhi) - xlo), he4 = (int32_t)(max(e4, a4) - xlo);
            const int32_t ha2 = (int32_t)(min(a2, xhi) - xlo), he2 = (int32_t)(max(e2, a2) - xlo);
            const int32_t n32 = nft;
            if (lane < 3) dc = lane < ha4 ? lane : -1;
            else if (lane < 6) dc = he4 + (lane - 3) < n32 ? he4 + (lane - 3) : -1;
            else if (lane == 6) dv = 0 < ha2 ? 0 : -1;
            else if (lane == 7) dv = he2 < n32 ? he2 : -1;
            const int32_t sc0 = (int32_t)(xlo - xbc), sv0 = (int32_t)(xlo - xbv);
            if (dc >= 0) __builtin_nontemporal_store(scol[w][sc0 + dc], out.col + xlo + dc);
            if (dv >= 0) __builtin_nontemporal_store(sval[w][sv0 + dv], out.val + xlo + dv);
        }
        r0 += nft;
        wave_sync();
    };
    // two step buffers, alternating (no register copies between steps)
    Step s0, s1;
    int32_t pw0 = (pa >> 6) << 6;
    load(pw0, s0);
    for (;;) {
        load(pw0 + PASS, s1);   // past the unit: clamped, harmless
        store(pw0, s0);
        pw0 += PASS;
        if (pw0 >= pb) break;
        load(pw0 + PASS, s0);
        store(pw0, s1);
        pw0 += PASS;
        if (pw0 >= pb) break;
    }
}

}  // namespace dev
}  // namespace ias
