// sym5_kernels.hpp — symbolic pass of the long rows (4,097 .. U products):
// sym4's algorithm (sym4_kernels.hpp) with NW waves per row.
//
// Restates CSR_MUL_CSR's first loop (IA-SPGEMM-CPU_release/detail/csr/
// common_csr.h:95-125) and the discovery order of its second loop (:133-189),
// producing what sym2 / sym3 / sym4 produce for the table-free numeric pass:
// nnz, the first-touch bitmap + word prefixes, each duplicate's first touch.
//
// One workgroup of NW waves per row, the row's filters shared in LDS.  Wave 0
// stages the entries (B-row bases, per-window start masks) and the per-window
// count of entries starting before it, so every window's product -> entry map
// is self-contained and the waves take the windows in chunks of KC, round
// robin, each double-buffering its gathers.  Filter and classify are sym4's;
// the possible duplicates are listed through an LDS counter (any order: the
// exact pass keeps the smallest product per column), the word prefixes are a
// workgroup scan.  A row of 8,192 products is resolved by two waves in about
// the time one wave takes for 4,096 (sym4), with the filters' LDS shared.
// Rows beyond the bounds or whose list overflows go to the retry list (sym2).
#pragma once

#include "sym4_kernels.hpp"

namespace ias {
namespace dev {

template <int U, int NW>
struct Sym5Lds {
    static constexpr int T = WAVE * NW;
    static constexpr int NWIN = U / 64;
    static constexpr int F1B = 16 * U;             // f1 bits (16 per product)
    static constexpr int F1W = F1B / 32;
    static constexpr int F2B = 2 * U;
    static constexpr int F2W = F2B / 32;
    static constexpr int BW = U / 32;
    static constexpr int NE = U / 32;              // A entries per row at most
    // list (a product index, 4 B per entry) + exact table (8 B per slot) over
    // f1, whole workgroups: U / 6.4 (U / 8 with 8-byte entries left 17 % / 69 %
    // of K3''s rows near 8,192 / 16,384 products to sym2)
    static constexpr int LC = F1W / 3 / T * T;
    static constexpr int ES = LC;
    static constexpr int LT = LC / T;              // list entries per thread
    static constexpr int WPL = BW / T;             // bitmap words per thread in the finish scan
    static constexpr int WIN_PL = NWIN / WAVE;     // windows per lane in wave 0's window scan
    static_assert(4 * LC + 8 * ES <= 4 * F1W, "list and exact table overlay f1");
    static_assert(LC % T == 0 && BW % T == 0 && NWIN % WAVE == 0, "whole workgroups");
    static_assert(F2B <= 65536, "f2 index in 16 bits");
    __attribute__((aligned(16))) uint32_t f1[F1W];
    __attribute__((aligned(16))) uint32_t f2[F2W];
    unsigned long long smask[NWIN];                // entry start bits per window
    uint32_t pref[BW];                             // word prefixes (finish)
    int32_t cbase[NWIN];                           // non-empty entries starting before each window
    int32_t ebase[NE];
    uint32_t words[BW];
    int32_t nl;                                    // list counter
    int32_t scratch[NW];
    __device__ int32_t *list() { return (int32_t *)f1; }
    __device__ int32_t *keys() { return (int32_t *)(f1 + LC); }
    __device__ uint32_t *own() { return (uint32_t *)(f1 + LC + ES); }
};

template <int U, int NW, int KC>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(3))) void k_sym5(Sym3Args) {
    using LDS = Sym5Lds<U, NW>;
    using TM = Team<LDS::T>;
    constexpr int T = LDS::T;
    constexpr int WWIN = LDS::NWIN / NW;           // windows per wave
    constexpr int NCH = WWIN / KC;                 // its chunks of KC windows
    static_assert(WWIN <= WAVE && WWIN % KC == 0 && KC % 2 == 0, "a wave's windows: one candidate mask");
    extern __shared__ __attribute__((aligned(16))) unsigned char s5_smem[];   // sizeof(LDS): 90 KB at U = 32,768
    LDS &L = *reinterpret_cast<LDS *>(s5_smem);
    const int tid = (int)threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid / WAVE);
    const int lane = (int)__lane_id();
    for (int i = tid; i < LDS::F1W / 4; i += T) ((uint4 *)L.f1)[i] = make_uint4(0u, 0u, 0u, 0u);
    for (int i = tid; i < LDS::F2W; i += T) L.f2[i] = 0u;

    // a row's details: its list entry, products, and (wave 0) the B-row
    // extents of its first 64 entries — the next row's are loaded during a
    // row (without, each row began with three dependent global loads: 3 - 4
    // us of its ~33)
    struct Det {
        RowRef ref;
        int32_t P, bl;
        int64_t bs;
    };
    auto details = [&](const RowRef &r) {
        Det d{r, 0, 0, 0};
        if (r.row >= 0) {
            d.P = s3_args()->prod[r.row];
            if (w == 0 && lane < r.n) {
                d.bl = s3_args()->ax.blen[r.q0 + lane];
                d.bs = s3_args()->ax.bstart[r.q0 + lane];
            }
        }
        return d;
    };
    int64_t idx = blockIdx.x;
    if (idx >= s3_args()->count) return;
    Det cur = details(s3_ref(idx));
    Timer tm;   // timing builds only (phases: 0 staging, 1 filter, 2 classify, 3 exact, 4 finish, 5 clear)
    tm.start();
    for (; idx < s3_args()->count; idx += gridDim.x) {
        const RowRef ref = cur.ref;
        const int32_t row = __builtin_amdgcn_readfirstlane(ref.row);
        const int32_t E = __builtin_amdgcn_readfirstlane(ref.n);
        const int32_t P = __builtin_amdgcn_readfirstlane(cur.P);
        const RowRef nref = s3_ref(idx + gridDim.x);
        if (P > U || E > LDS::NE) {
            if (tid == 0) {
                const int32_t j = atomicAdd(s3_args()->retry_count, 1);
                s3_args()->retry[j] = ref;
            }
            cur = details(nref);
            continue;
        }
        const int nwin = (P + 63) >> 6;
        const int64_t q0 = ref.q0;
        if (tid == 0) L.nl = 0;
        // ---- wave 0: entries -> ebase + start masks, then the window bases
        if (w == 0) {
            for (int k = lane; k < nwin; k += WAVE) L.smask[k] = 0ull;
            s3_sync();
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
            s3_sync();
            // window bases: lane j takes windows j*WIN_PL .. +WIN_PL
            int cnt = 0;
#pragma unroll
            for (int i = 0; i < LDS::WIN_PL; ++i) {
                const int k = lane * LDS::WIN_PL + i;
                cnt += k < nwin ? (int)__popcll(L.smask[k]) : 0;
            }
            int run = wave_incl_sum(cnt) - cnt;
#pragma unroll
            for (int i = 0; i < LDS::WIN_PL; ++i) {
                const int k = lane * LDS::WIN_PL + i;
                if (k < nwin) {
                    L.cbase[k] = run;
                    run += (int)__popcll(L.smask[k]);
                }
            }
        }
        __syncthreads();
        tm.mark(0);
        // product p = 64k + l: the byte offset of its B column (beyond P:
        // B.col[0], callers mask it)
        const char *base = (const char *)s3_args()->bcol;
        auto col_addr = [&](int k, int l) -> uint32_t {
            const int kk = min(k, LDS::NWIN - 1);
            const uint64_t m = L.smask[kk];
            const int e = min(max(L.cbase[kk] + (int)__popcll(m & ((2ull << l) - 1ull)) - 1, 0), LDS::NE - 1);
            return l < P - 64 * k ? (uint32_t)(L.ebase[e] + 64 * k + l) << 2 : 0u;
        };
        // this wave's chunk j: windows w*KC + j*NW*KC .. +KC (wr: w, opaque
        // per row, so the per-window bounds are not all hoisted out of the row
        // loop into registers that then spill)
        int wr = w;
        asm volatile("" : "+s"(wr));
        auto gather = [&](int j, int32_t(&c)[KC]) {
            const int k0 = (wr + j * NW) * KC;
            uint32_t off[KC];
#pragma unroll
            for (int t = 0; t < KC; ++t) off[t] = col_addr(k0 + t, lane);
#pragma unroll
            for (int t = 0; t < KC; ++t) c[t] = *(const int32_t *)(base + off[t]);
        };
        // ---- filter: one sweep; each product's f2 index stays in the lanes
        // (two per register) with its candidate bit, so classify gathers nothing
        uint32_t hh2[WWIN / 2];
        uint64_t candm = 0ull;
        {
            int32_t cbuf[S4_DEPTH][KC];   // sym4's ring (unconditional gathers: see there)
#pragma unroll
            for (int j = 0; j + 1 < S4_DEPTH && j < NCH; ++j) gather(j, cbuf[j]);
#pragma unroll
            for (int j = 0; j < NCH; ++j) {
                const int k0 = (wr + j * NW) * KC;
                if (k0 >= nwin) break;   // beyond the row: nothing to filter
                const int jn = j + S4_DEPTH - 1;
                if (jn < NCH) gather(jn, cbuf[jn % S4_DEPTH]);
                const int32_t(&c)[KC] = cbuf[j % S4_DEPTH];
                uint32_t hv[KC], old[KC], bit[KC];
#pragma unroll
                for (int t = 0; t < KC; ++t) {
                    const bool in = lane < P - 64 * (k0 + t);
                    const uint32_t h1 = s4_h1<LDS::F1B>(c[t]);
                    hv[t] = s4_h2<LDS::F2B>(c[t]);
                    bit[t] = in ? 1u << (h1 & 31) : 0u;
                    uint32_t o = 0u;   // lanes / windows past the row issue nothing
                    if (in) o = atomicOr(&L.f1[h1 >> 5], bit[t]);
                    old[t] = o;
                }
#pragma unroll
                for (int t = 0; t < KC; ++t) {
                    const int lk = KC * j + t;
                    const bool cand = (old[t] & bit[t]) != 0u;
                    candm |= (cand ? 1ull : 0ull) << lk;
                    if (cand) atomicOr(&L.f2[hv[t] >> 5], 1u << (hv[t] & 31));
                    if (t & 1) hh2[lk >> 1] = (hv[t] << 16) | hv[t - 1];
                }
            }
        }
        __syncthreads();   // f1 dead: the list overlays it
        tm.mark(1);
        // ---- classify: certain first touches -> bitmap words, possible
        // duplicates -> list (any order; their columns gathered after)
        int32_t *list = L.list();
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
            const int k0 = (wr + j * NW) * KC;
            if (k0 >= nwin) break;
            // the chunk's f2 words first (reads in flight together), one list
            // counter atomic per chunk
            uint32_t f2w[KC];
            bool poss[KC];
            uint64_t pb[KC];
            int cnt = 0;
#pragma unroll
            for (int t = 0; t < KC; ++t) {
                const int lk = KC * j + t;
                const uint32_t h2 = (hh2[lk >> 1] >> (16 * (lk & 1))) & 0xFFFFu;
                f2w[t] = L.f2[lane < P - 64 * (k0 + t) ? h2 >> 5 : 0u];
            }
#pragma unroll
            for (int t = 0; t < KC; ++t) {
                const int lk = KC * j + t;
                const int k = k0 + t;
                const bool in = lane < P - 64 * k;   // false for windows beyond the row
                const uint32_t h2 = (hh2[lk >> 1] >> (16 * (lk & 1))) & 0xFFFFu;
                poss[t] = (((uint32_t)(candm >> lk) | (f2w[t] >> (h2 & 31))) & (in ? 1u : 0u)) != 0u;   // bitwise (sym4)
                const uint64_t b = __ballot(in && !poss[t]);
                if (lane == 0 && k < nwin) *(uint64_t *)&L.words[2 * k] = b;
                pb[t] = __ballot(poss[t]);
                cnt += (int)__popcll(pb[t]);
            }
            if (cnt > 0) {
                int at = 0;
                if (lane == 0) at = atomicAdd(&L.nl, cnt);
                at = __shfl(at, 0);
#pragma unroll
                for (int t = 0; t < KC; ++t) {
                    const int i = at + s3_below(pb[t]);
                    if (poss[t] && i < LDS::LC) list[i] = 64 * (k0 + t) + lane;
                    at += (int)__popcll(pb[t]);
                }
            }
        }
        __syncthreads();
        tm.mark(2);
        const int32_t nl = L.nl;
        Det nxt;   // issued after the listed products' gathers (sym4)
        if (4 * nl > 3 * LDS::LC) {
            nxt = details(nref);
            if (tid == 0) {
                const int32_t j = atomicAdd(s3_args()->retry_count, 1);
                s3_args()->retry[j] = ref;
            }
        } else {
            // ---- exact: the listed products' columns (gathered again, only
            // these), then claim the column (CAS, linear probing); its
            // smallest product is the first touch
            int2 e[LDS::LT];
            uint32_t slot[LDS::LT], f[LDS::LT], off[LDS::LT];
#pragma unroll
            for (int t = 0; t < LDS::LT; ++t) {
                e[t] = make_int2(0, -1);
                slot[t] = 0;
                f[t] = 0;
                off[t] = 0u;
                const int i = t * T + tid;
                if (i < nl) {
                    e[t].y = list[i];
                    off[t] = col_addr(e[t].y >> 6, e[t].y & 63);
                }
            }
#pragma unroll
            for (int t = 0; t < LDS::LT; ++t)
                if (t * T + tid < nl) e[t].x = *(const int32_t *)(base + off[t]);
            nxt = details(nref);
            if (nl > 0) {
                int32_t *keys = L.keys();
                uint32_t *own = L.own();
                for (int i = tid; i < LDS::ES; i += T) keys[i] = EMPTY_KEY;
                __syncthreads();
                uint32_t wonm = 0u;
#pragma unroll
                for (int t = 0; t < LDS::LT; ++t) {
                    const int i = t * T + tid;
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
                __syncthreads();
#pragma unroll
                for (int t = 0; t < LDS::LT; ++t)
                    if (t * T + tid < nl && !((wonm >> t) & 1u)) atomicMin(&own[slot[t]], (uint32_t)e[t].y);
                __syncthreads();
#pragma unroll
                for (int t = 0; t < LDS::LT; ++t) {
                    if (t * T + tid < nl) {
                        f[t] = own[slot[t]];
                        const uint32_t p = (uint32_t)e[t].y;
                        if (f[t] == p) atomicOr(&L.words[p >> 5], 1u << (p & 31));
                    }
                }
                __syncthreads();
            }
            tm.mark(3);
            // ---- finish: nnz and word prefixes (thread-contiguous words)
            const int W = (P + 31) >> 5;
            int cnt = 0;
#pragma unroll
            for (int j = 0; j < LDS::WPL; ++j) {
                const int wi = tid * LDS::WPL + j;
                cnt += wi < W ? __popc(L.words[wi]) : 0;
            }
            int nnz;
            const int ex = TM::excl_sum(cnt, nnz, L.scratch);
            {
                uint32_t run = (uint32_t)ex;
#pragma unroll
                for (int j = 0; j < LDS::WPL; ++j) {
                    const int wi = tid * LDS::WPL + j;
                    if (wi < W) {
                        L.pref[wi] = run;
                        run += (uint32_t)__popc(L.words[wi]);
                    }
                }
            }
            __syncthreads();
            const bool heavy = P - nnz > s3_args()->dcap;
            if (!heavy) {
                const int64_t bmoff = s3_args()->bm.off[row];
                for (int wi = tid; wi < W; wi += T) {
                    s3_args()->bm.bits[bmoff + wi] = L.words[wi];
                    s3_args()->bm.pref[bmoff + wi] = L.pref[wi];
                }
                if (nl > 0) {
                    const int64_t dupoff = s3_args()->dup_off[row];
#pragma unroll
                    for (int t = 0; t < LDS::LT; ++t) {
                        const uint32_t p = (uint32_t)e[t].y;
                        if (t * T + tid < nl && f[t] != p) {
                            const uint32_t rk =
                                L.pref[p >> 5] + (uint32_t)__popc(L.words[p >> 5] & ((1u << (p & 31)) - 1u));
                            s3_args()->gdupt[dupoff + (p - rk)] = (int32_t)f[t];
                        }
                    }
                }
            }
            if (tid == 0) {
                s3_args()->nnz_row[row] = nnz;
                s3_args()->dupn[row] = heavy ? (nnz > s3_args()->bm_need ? -3 : -1) : P - nnz;
            }
        }
        // ---- the filters empty for the next row
        tm.mark(4);
        __syncthreads();
        for (int i = tid; i < LDS::F1W / 4; i += T) ((uint4 *)L.f1)[i] = make_uint4(0u, 0u, 0u, 0u);
        for (int i = tid; i < LDS::F2W; i += T) L.f2[i] = 0u;
        __syncthreads();
        tm.mark(5);
        tm.done();
        cur = nxt;
    }
    tm.flush(U <= 8192 ? 30 : 31, tid == 0);
}

// Rows of 16,385 .. GT_U products when B's columns do not fit the column
// bitmap (k_sym_cbm) go to k_sym5<GT_U, 8> (same algorithm, 8 waves, 90 KB
// of LDS); the rows it hands back (list overflow, more than 1,024 entries),
// and all of those rows when B's entries exceed 32-bit offsets, come here:
// one 1024-lane workgroup per row, persistent over its list (count read on
// the device), the exact table in global memory (the workgroup's 2 * GT_U
// slots of the plan's workspace).  Every product claims its column (CAS,
// linear probing) and keeps the smallest product index (atomicMin); a
// product owning its column is its first touch.  Outputs as sym5.  L2
// atomics: slow, for rare rows.  Table contents changed by atomics are read
// past the L1 (agent-scope atomic loads), as in k_sym_cbm.
constexpr int GT_BLOCK = 1024;
constexpr int GT_U = 32768;          // products per row at most
constexpr int GT_NE = GT_U / 8;      // A entries per row at most (the bins' 8 x entries <= products)
constexpr int GT_SLOTS = 2 * GT_U;   // table slots per workgroup
__global__ __launch_bounds__(GT_BLOCK) void k_sym_gtab(Sym3Args a, int32_t *gkeys, uint32_t *gown) {
    __shared__ int64_t ebase[GT_NE];         // B-row start - first product, per non-empty entry
    __shared__ int32_t erel[GT_NE];          // first product of each non-empty entry
    __shared__ uint32_t words[GT_U / 32];    // first-touch bitmap
    __shared__ uint32_t pref[GT_U / 32];
    __shared__ int scratch[GT_BLOCK / WAVE];
    using TM = Team<GT_BLOCK>;
    const int tid = (int)threadIdx.x;
    const int32_t count = *a.retry_count;    // the list's rows (device count)
    int32_t *keys = gkeys + (size_t)blockIdx.x * GT_SLOTS;
    uint32_t *own = gown + (size_t)blockIdx.x * GT_SLOTS;
    auto ld_keys = [](const int32_t *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    auto ld_own = [](const uint32_t *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    for (int64_t idx = blockIdx.x; idx < count; idx += gridDim.x) {
        const RowRef ref = a.retry[idx];
        const int32_t row = ref.row, E = ref.n;
        const int32_t P = a.prod[row];
        if (P > GT_U || E > GT_NE) {   // outside the bins' bounds: never listed here
            if (tid == 0) a.nnz_row[row] = -1;
            continue;
        }
        // ---- stage the non-empty entries: first product and B-row base
        int carry = 0, nec = 0;
        for (int g = 0; g < E; g += GT_BLOCK) {
            const int e = g + tid;
            int32_t bl = 0;
            int64_t bs = 0;
            if (e < E) {
                bl = a.ax.blen[ref.q0 + e];
                bs = a.ax.bstart[ref.q0 + e];
            }
            int tot, totn;
            const int ex = TM::excl_sum(bl, tot, scratch);
            const int exn = TM::excl_sum(bl > 0 ? 1 : 0, totn, scratch);
            if (bl > 0) {
                erel[nec + exn] = carry + ex;
                ebase[nec + exn] = bs - (carry + ex);
            }
            carry += tot;
            nec += totn;
        }
        // ---- the table: a power of two >= 2P slots; the bitmap words
        int S = 64;
        while (S < 2 * P) S <<= 1;
        const uint32_t mask = (uint32_t)S - 1u, sh = 32u - (uint32_t)(31 - __builtin_clz((unsigned)S));
        for (int i = tid; i < S; i += GT_BLOCK) {
            (void)atomicExch(&keys[i], EMPTY_KEY);   // performed in L2 before the barrier
            (void)atomicExch(&own[i], 0xFFFFFFFFu);
        }
        const int W = (P + 31) >> 5;
        for (int i = tid; i < W; i += GT_BLOCK) words[i] = 0u;
        __syncthreads();
        // product p's column (entry by binary search over the staged starts)
        auto column = [&](int32_t p) -> int32_t {
            int lo = 0, hi = nec - 1;   // the last entry starting at or before p
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (erel[mid] <= p) lo = mid;
                else hi = mid - 1;
            }
            return a.bcol[ebase[lo] + p];
        };
        auto slot_of = [&](int32_t c) -> uint32_t {   // the column's slot (it is in the table)
            uint32_t s = ((uint32_t)c * 0x9E3779B1u) >> sh;
            while (ld_keys(&keys[s]) != c) s = (s + 1u) & mask;
            return s;
        };
        // ---- claim: every product's column, its smallest product
        for (int32_t p = tid; p < P; p += GT_BLOCK) {
            const int32_t c = column(p);
            uint32_t s = ((uint32_t)c * 0x9E3779B1u) >> sh;
            for (;;) {
                const int32_t g = atomicCAS(&keys[s], EMPTY_KEY, c);
                if (g == EMPTY_KEY || g == c) break;
                s = (s + 1u) & mask;
            }
            atomicMin(&own[s], (uint32_t)p);
        }
        __syncthreads();
        // ---- first touches
        for (int32_t p = tid; p < P; p += GT_BLOCK) {
            const uint32_t f = ld_own(&own[slot_of(column(p))]);
            if (f == (uint32_t)p) atomicOr(&words[p >> 5], 1u << (p & 31));
        }
        __syncthreads();
        // ---- finish: nnz, word prefixes, bitmap, duplicates' first touches
        int nnz = 0, run = 0;
        for (int w0 = 0; w0 < W; w0 += GT_BLOCK) {
            const int wi = w0 + tid;
            const int cnt = wi < W ? __popc(words[wi]) : 0;
            int tot;
            const int ex = TM::excl_sum(cnt, tot, scratch);
            if (wi < W) pref[wi] = (uint32_t)(run + ex);
            run += tot;
        }
        nnz = run;
        __syncthreads();
        const bool heavy = P - nnz > a.dcap;
        if (!heavy) {
            const int64_t bmoff = a.bm.off[row];
            for (int wi = tid; wi < W; wi += GT_BLOCK) {
                a.bm.bits[bmoff + wi] = words[wi];
                a.bm.pref[bmoff + wi] = pref[wi];
            }
            const int64_t dupoff = a.dup_off[row];
            for (int32_t p = tid; p < P; p += GT_BLOCK) {
                const uint32_t f = ld_own(&own[slot_of(column(p))]);
                if (f != (uint32_t)p) {
                    const uint32_t rk = pref[p >> 5] + (uint32_t)__popc(words[p >> 5] & ((1u << (p & 31)) - 1u));
                    a.gdupt[dupoff + ((uint32_t)p - rk)] = (int32_t)f;
                }
            }
        }
        if (tid == 0) {
            a.nnz_row[row] = nnz;
            a.dupn[row] = heavy ? (nnz > a.bm_need ? -3 : -1) : P - nnz;
        }
        __syncthreads();   // the table and LDS arrays are the next row's
    }
}

}  // namespace dev
}  // namespace ias
