// sym4_kernels.hpp — symbolic pass of the long rows (2,049 .. U products),
// one wave per row, the row's products in chunks of 64*KC.
//
// Restates CSR_MUL_CSR's first loop (IA-SPGEMM-CPU_release/detail/csr/
// common_csr.h:95-125: distinct columns per row) and the discovery order of
// its second loop (:133-189), producing what sym2 / sym3 produce for the
// table-free numeric pass: nnz, the row's first-touch bitmap + word prefixes,
// and each duplicate's first-touch product.
//
// sym3 (sym3_kernels.hpp) keeps a row's columns in registers (K per lane) and
// its entries one per lane, so it stops at 2,048 products (K = 32: 168 VGPRs,
// 3 waves per SIMD).  Here the columns never stay in registers beyond a chunk:
//   * the row's entries (up to U/32) are staged in groups of 64 — per entry
//     its B-row base in LDS and its start bit in the per-window start masks —
//     and each window's count of entries starting before it (one per lane);
//   * filter (per chunk of KC windows, double-buffered gathers: f1 ORs with
//     return, candidates mark f2).  Each product's f2 index (16 bits, an
//     independent hash) stays in the lanes, two per register, with its
//     candidate bit: the row's columns are gathered once;
//   * classify (registers + f2 reads): one ballot per window gives the
//     certain first touches, the possible duplicates' product indices are
//     listed over the dead f1;
//   * exact pass: the listed products' columns gathered again (only those),
//     then as in sym3, with the bitmap words and their prefixes in LDS.
// Rows beyond the kernel's bounds, or whose list overflows, go to the retry
// list that sym2's teams finish.  Measured against sym2's 512 / 1024-lane
// teams on K3': see DESIGN.md §4.
#pragma once

#include "sym3_kernels.hpp"

namespace ias {
namespace dev {

template <int U, int F1BPP>
struct Sym4Lds {
    static constexpr int NWIN = U / 64;            // 64-product windows
    static constexpr int F1B = F1BPP * U;          // f1 bits (a power of two: 16 bits of hash)
    static constexpr int F1W = F1B / 32;
    static constexpr int F2B = 2 * U;              // f2 bits
    static constexpr int F2W = F2B / 32;
    static constexpr int BW = U / 32;              // bitmap words
    static constexpr int NE = U / 32;              // A entries per row at most
    // possible-duplicate list (a product index, 4 B each) + exact table (8 B
    // per slot) over f1: 12 B per entry, whole waves (U / 6.4 at F1BPP = 16;
    // U / 8 with 8-byte entries left 17 % of K3''s 4,097 - 8,192-product rows
    // to sym2)
    static constexpr int LC = F1W / 3 / WAVE * WAVE;
    static constexpr int ES = LC;
    static constexpr int LT = LC / WAVE;           // list entries per lane
    static constexpr int WPL = BW / WAVE;          // bitmap words per lane in the finish scan
    static_assert(4 * LC + 8 * ES <= 4 * F1W, "list and exact table overlay f1");
    static_assert(BW % WAVE == 0 && LC % WAVE == 0 && NE % WAVE == 0, "whole waves");
    static_assert(NWIN <= WAVE, "one window base per lane");
    static_assert(F1B == 65536 && F2B <= 65536, "f1 and f2 indexed by at most 16 hash bits");
    __attribute__((aligned(16))) uint32_t f1[F1W];
    __attribute__((aligned(16))) uint32_t f2[F2W];
    unsigned long long smask[NWIN];                // entry start bits per window
    int32_t wbase[NWIN];                           // non-empty entries starting before each window
    uint32_t pref[BW];                             // exclusive prefixes of the bitmap words (finish)
    int32_t ebase[NE];                             // B-row start - first product, per non-empty entry
    uint32_t words[BW];                            // first-touch bitmap
    __device__ int32_t *list() { return (int32_t *)f1; }
    __device__ int32_t *keys() { return (int32_t *)(f1 + LC); }
    __device__ uint32_t *own() { return (uint32_t *)(f1 + LC + ES); }
};

// f1's and f2's bit indices: the top bits of two independent multiplicative
// hashes (f2 a coarsening of f1 made both halves of every false f1 pair
// possible duplicates: 640 vs 523 listed per 6,900-product row on K3')
template <int NB>
__device__ __forceinline__ uint32_t s4_h1(int32_t c) { return ((uint32_t)c * 0x9E3779B1u) >> (32 - ilog2(NB)); }
template <int NB>
__device__ __forceinline__ uint32_t s4_h2(int32_t c) { return ((uint32_t)c * 0x85EBCA77u) >> (32 - ilog2(NB)); }

constexpr int S4_DEPTH = 2;   // chunk buffers in flight in the filter (sym4, sym5); 3 / 4 within noise
constexpr int SYM4_WPE = 3;   // waves per SIMD the registers must allow (LDS allows 3.5 at U = 4096)
template <int U, int F1BPP, int KC, int WPB>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(SYM4_WPE))) void k_sym4(Sym3Args) {
    using LDS = Sym4Lds<U, F1BPP>;
    constexpr int NWIN = LDS::NWIN;
    constexpr int NCH = NWIN / KC;                 // chunks of KC windows
    static_assert(NWIN % KC == 0 && NWIN % 2 == 0, "whole chunks");
    __shared__ LDS lds[WPB];
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / WAVE));
    const int lane = (int)__lane_id();
    LDS &L = lds[w];
    const int64_t stride = (int64_t)gridDim.x * WPB;
    int64_t idx = (int64_t)blockIdx.x * WPB + w;
    if (idx >= s3_args()->count) return;
    for (int i = lane; i < LDS::F1W / 4; i += WAVE) ((uint4 *)L.f1)[i] = make_uint4(0u, 0u, 0u, 0u);
    for (int i = lane; i < LDS::F2W; i += WAVE) L.f2[i] = 0u;
    s3_sync();

    // a row's details: its list entry, products, and the B-row extents of its
    // first 64 entries (prefetched a row ahead)
    struct Det {
        RowRef ref;
        int32_t P, bl;
        int64_t bs;
    };
    auto details = [&](const RowRef &r) {
        Det d{r, 0, 0, 0};
        if (r.row >= 0) {
            d.P = s3_args()->prod[r.row];
            if (lane < r.n) {
                d.bl = s3_args()->ax.blen[r.q0 + lane];
                d.bs = s3_args()->ax.bstart[r.q0 + lane];
            }
        }
        return d;
    };
    Det cur = details(s3_ref(idx));
    Timer tm;   // timing builds only (phases: 0 staging, 1 filter, 2 classify, 3 exact, 4 finish, 5 clear)
    tm.start();
    for (; idx < s3_args()->count; idx += stride) {
        const RowRef ref = cur.ref;
        const int32_t row = __builtin_amdgcn_readfirstlane(ref.row);
        const int32_t E = __builtin_amdgcn_readfirstlane(ref.n);
        const int32_t P = __builtin_amdgcn_readfirstlane(cur.P);
        const RowRef nref = s3_ref(idx + stride);
        if (P > U || E > LDS::NE) {   // outside this kernel's bounds: sym2's teams finish it
            if (lane == 0) {
                const int32_t j = atomicAdd(s3_args()->retry_count, 1);
                s3_args()->retry[j] = ref;
            }
            cur = details(nref);
            continue;
        }
        const int64_t q0 = ref.q0;
        const int nwin = (P + 63) >> 6;
        if (lane < NWIN) L.smask[lane] = 0ull;
        s3_sync();
        // ---- stage the entries, 64 at a time
        {
            int carry = 0, nec = 0;
            for (int g = 0; g < E; g += WAVE) {
                const int e = g + lane;
                int32_t bl = cur.bl;
                int64_t bs = cur.bs;
                if (g > 0) {
                    bl = 0;
                    bs = 0;
                    if (e < E) {
                        bl = s3_args()->ax.blen[q0 + e];
                        bs = s3_args()->ax.bstart[q0 + e];
                    }
                }
                const int incl = wave_incl_sum(bl);
                const int rel = carry + incl - bl;
                const uint64_t nem = __ballot(bl > 0);
                if (bl > 0 && rel < P) {
                    L.ebase[nec + s3_below(nem)] = (int32_t)(bs - rel);
                    atomicOr(&L.smask[(uint32_t)rel >> 6], 1ull << (rel & 63));
                }
                carry += __builtin_amdgcn_readlane(incl, WAVE - 1);
                nec += (int)__popcll(nem);
            }
        }
        s3_sync();
        // window bases: lane k holds window k's
        {
            const int cnt = lane < nwin ? (int)__popcll(L.smask[lane]) : 0;
            if (lane < NWIN) L.wbase[lane] = wave_incl_sum(cnt) - cnt;
        }
        s3_sync();
        // product p = 64k + lane: its entry and B column (beyond P: B.col[0],
        // callers mask it)
        const char *base = (const char *)s3_args()->bcol;
        auto col_addr = [&](int k, int l) -> uint32_t {
            const int kk = min(k, NWIN - 1);
            const uint64_t m = L.smask[kk];
            const int e = min(max(L.wbase[kk] + (int)__popcll(m & ((2ull << l) - 1ull)) - 1, 0), LDS::NE - 1);
            return l < P - 64 * k ? (uint32_t)(L.ebase[e] + 64 * k + l) << 2 : 0u;
        };
        auto gather = [&](int k0, int32_t(&c)[KC]) {
            uint32_t off[KC];
#pragma unroll
            for (int t = 0; t < KC; ++t) off[t] = col_addr(k0 + t, lane);
#pragma unroll
            for (int t = 0; t < KC; ++t) c[t] = *(const int32_t *)(base + off[t]);
        };
        tm.mark(0);
        // ---- filter: one sweep; each product's 16 hash bits stay in the
        // lanes (two per register) with its candidate bit, so the classify
        // pass needs no second gather of the row's columns
        uint32_t hh2[NWIN / 2];
        uint64_t candm = 0ull;
        {
            // a ring of S4_DEPTH chunk buffers: chunks j+1 .. j+S4_DEPTH-1
            // in flight while chunk j is filtered.  The gathers are
            // unconditional (chunks past the row read B.col[0]): a gather
            // under a branch makes the compiler's wait for chunk j assume
            // the later chunks were not issued, i.e. wait for them too
            int32_t cbuf[S4_DEPTH][KC];
#pragma unroll
            for (int j = 0; j + 1 < S4_DEPTH && j < NCH; ++j) gather(KC * j, cbuf[j]);
#pragma unroll
            for (int j = 0; j < NCH; ++j) {
                if (KC * j >= nwin) break;   // beyond the row: nothing to filter
                const int jn = j + S4_DEPTH - 1;
                if (jn < NCH) gather(KC * jn, cbuf[jn % S4_DEPTH]);
                const int32_t(&c)[KC] = cbuf[j % S4_DEPTH];
                uint32_t hv[KC], old[KC], bit[KC];
#pragma unroll
                for (int t = 0; t < KC; ++t) {
                    const int k = KC * j + t;
                    const bool in = lane < P - 64 * k;
                    const uint32_t h1 = s4_h1<LDS::F1B>(c[t]);
                    hv[t] = s4_h2<LDS::F2B>(c[t]);
                    bit[t] = in ? 1u << (h1 & 31) : 0u;
                    uint32_t o = 0u;   // lanes / windows past the row issue nothing
                    if (in) o = atomicOr(&L.f1[h1 >> 5], bit[t]);
                    old[t] = o;
                }
#pragma unroll
                for (int t = 0; t < KC; ++t) {
                    const int k = KC * j + t;
                    const bool cand = (old[t] & bit[t]) != 0u;
                    candm |= (cand ? 1ull : 0ull) << k;
                    if (cand) {
                        atomicOr(&L.f2[hv[t] >> 5], 1u << (hv[t] & 31));
                    }
                    if (t & 1) hh2[k >> 1] = (hv[t] << 16) | hv[t - 1];
                }
            }
        }
        tm.mark(1);
        s3_sync();   // f1 dead from here: the list overlays it
        // ---- classify: certain first touches -> bitmap words, possible
        // duplicates -> list (product order; their columns gathered after)
        int nl = 0;
        int32_t *list = L.list();
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
            if (KC * j >= nwin) break;
            // the chunk's f2 words first (their reads in flight together)
            uint32_t f2w[KC];
#pragma unroll
            for (int t = 0; t < KC; ++t) {
                const int k = KC * j + t;
                const uint32_t h2 = (hh2[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
                f2w[t] = L.f2[lane < P - 64 * k ? h2 >> 5 : 0u];
            }
#pragma unroll
            for (int t = 0; t < KC; ++t) {
                const int k = KC * j + t;
                if (k < nwin) {
                    const int p = 64 * k + lane;
                    const bool in = lane < P - 64 * k;
                    const uint32_t h2 = (hh2[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
                    // bitwise, not short-circuit: the compiler otherwise sank the
                    // chunk's f2 reads into a branch per window, each waited on
                    const uint32_t pv = ((uint32_t)(candm >> k) | (f2w[t] >> (h2 & 31))) & (in ? 1u : 0u);
                    const bool poss = pv != 0u;
                    const uint64_t b = __ballot(in && !poss);
                    if (lane == 0) *(uint64_t *)&L.words[2 * k] = b;
                    const uint64_t pb = __ballot(poss);
                    if (poss) {
                        const int i = nl + s3_below(pb);
                        if (i < LDS::LC) list[i] = p;
                    }
                    nl += (int)__popcll(pb);
                }
            }
        }
        s3_sync();
        tm.mark(2);
        const bool retry = 4 * nl > 3 * LDS::LC;
        // the next row's details fly during the rest of this one, issued
        // after the listed products' gathers (issued before classify, the
        // first reuse of a register they load waited for them there)
        Det nxt;
        if (retry) {
            nxt = details(nref);
            if (lane == 0) {
                const int32_t j = atomicAdd(s3_args()->retry_count, 1);
                s3_args()->retry[j] = ref;
            }
        } else {
            // ---- exact: the listed products' columns (gathered again, only
            // these), then claim the column (CAS, linear probing); its
            // smallest product is the first touch
            int2 e[LDS::LT];
            uint32_t slot[LDS::LT], f[LDS::LT];
            uint32_t off[LDS::LT];
#pragma unroll
            for (int t = 0; t < LDS::LT; ++t) {
                e[t] = make_int2(0, -1);
                slot[t] = 0;
                f[t] = 0;
                off[t] = 0u;
                const int i = t * WAVE + lane;
                if (i < nl) {
                    e[t].y = list[i];
                    off[t] = col_addr(e[t].y >> 6, e[t].y & 63);
                }
            }
#pragma unroll
            for (int t = 0; t < LDS::LT; ++t)
                if (t * WAVE + lane < nl) e[t].x = *(const int32_t *)(base + off[t]);
            nxt = details(nref);
            if (nl > 0) {
                int32_t *keys = L.keys();
                uint32_t *own = L.own();
                for (int i = lane; i < LDS::ES; i += WAVE) keys[i] = EMPTY_KEY;
                s3_sync();
                uint32_t wonm = 0u;
#pragma unroll
                for (int t = 0; t < LDS::LT; ++t) {
                    const int i = t * WAVE + lane;
                    if (i < nl) {
                        uint32_t s = s3_h3(e[t].x, LDS::ES);
                        bool won = false;
                        for (int probe = 0; probe < LDS::ES; ++probe) {
                            const int32_t g = atomicCAS(&keys[s], EMPTY_KEY, e[t].x);
                            if (g == EMPTY_KEY) {
                                won = true;
                                break;
                            }
                            if (g == e[t].x) break;
                            s = s + 1u == (uint32_t)LDS::ES ? 0u : s + 1u;
                        }
                        slot[t] = s;
                        if (won) own[s] = (uint32_t)e[t].y;
                        wonm |= (won ? 1u : 0u) << t;
                    }
                }
                s3_sync();
#pragma unroll
                for (int t = 0; t < LDS::LT; ++t)
                    if (t * WAVE + lane < nl && !((wonm >> t) & 1u)) atomicMin(&own[slot[t]], (uint32_t)e[t].y);
                s3_sync();
#pragma unroll
                for (int t = 0; t < LDS::LT; ++t) {
                    if (t * WAVE + lane < nl) {
                        f[t] = own[slot[t]];
                        const uint32_t p = (uint32_t)e[t].y;
                        if (f[t] == p) atomicOr(&L.words[p >> 5], 1u << (p & 31));
                    }
                }
                s3_sync();
            }
            tm.mark(3);
            // ---- finish: nnz, word prefixes (lane-contiguous words), bitmap
            const int W = (P + 31) >> 5;
            uint32_t cnt = 0u;
#pragma unroll
            for (int j = 0; j < LDS::WPL; ++j) {
                const int wi = lane * LDS::WPL + j;
                cnt += wi < W ? (uint32_t)__popc(L.words[wi]) : 0u;
            }
            const int incl = wave_incl_sum((int)cnt);
            const int nnz = __builtin_amdgcn_readlane(incl, WAVE - 1);
            {
                uint32_t run = (uint32_t)(incl - (int)cnt);
#pragma unroll
                for (int j = 0; j < LDS::WPL; ++j) {
                    const int wi = lane * LDS::WPL + j;
                    if (wi < W) {
                        L.pref[wi] = run;
                        run += (uint32_t)__popc(L.words[wi]);
                    }
                }
            }
            s3_sync();
            const bool heavy = P - nnz > s3_args()->dcap;
            if (!heavy) {
                const int64_t bmoff = s3_args()->bm.off[row];
                for (int wi = lane; wi < W; wi += WAVE) {
                    s3_args()->bm.bits[bmoff + wi] = L.words[wi];
                    s3_args()->bm.pref[bmoff + wi] = L.pref[wi];
                }
                if (nl > 0) {
                    const int64_t dupoff = s3_args()->dup_off[row];
#pragma unroll
                    for (int t = 0; t < LDS::LT; ++t) {
                        const uint32_t p = (uint32_t)e[t].y;
                        if (t * WAVE + lane < nl && f[t] != p) {
                            const uint32_t rk =
                                L.pref[p >> 5] + (uint32_t)__popc(L.words[p >> 5] & ((1u << (p & 31)) - 1u));
                            s3_args()->gdupt[dupoff + (p - rk)] = (int32_t)f[t];
                        }
                    }
                }
            }
            if (lane == 0) {
                s3_args()->nnz_row[row] = nnz;
                s3_args()->dupn[row] = heavy ? (nnz > s3_args()->bm_need ? -3 : -1) : P - nnz;
            }
        }
        // ---- the filters empty for the next row
        tm.mark(4);
        s3_sync();
        for (int i = lane; i < LDS::F1W / 4; i += WAVE) ((uint4 *)L.f1)[i] = make_uint4(0u, 0u, 0u, 0u);
        for (int i = lane; i < LDS::F2W; i += WAVE) L.f2[i] = 0u;
        s3_sync();
        tm.mark(5);
        tm.done();
        cur = nxt;
    }
    tm.flush(27, lane == 0);
}

}  // namespace dev
}  // namespace ias
