// sym3_kernels.hpp — symbolic pass of the mid-size rows (257 .. 64*K
// products, at most 64*K/8 A entries), one wave per row, no workgroup barrier.
//
// Restates CSR_MUL_CSR's first loop (IA-SPGEMM-CPU_release/detail/csr/
// common_csr.h:95-125: distinct columns per row) and the discovery order of
// its second loop (:133-189: every column's first touch, whose reverse is the
// output order), producing what sym2 (sym2_kernels.hpp) produces for the
// table-free numeric pass: nnz, the row's first-touch bitmap + word prefixes,
// and each duplicate's first-touch product.
//
// Why a second kernel for these rows: sym2's one-wave and 128-lane teams spend
// ~25 dependent LDS round trips and several team barriers per row (staging
// scans, list counters, table clears), so a CU with 20 rows in flight idles on
// latency (0.3 products / clock / CU measured on K3').  Here a row is a short
// chain — stage (one LDS atomic + two reads), gather, one filter atomic per
// product, one filter read per product, ballots — everything else lives in
// registers:
//   * the row's A entries (at most 64) sit in the lanes, entry e in lane e;
//     their product starts are a DPP scan; per 64-product
//     window k the start bits are one LDS word (atomicOr by each entry) and the
//     entries before the window a scalar running popcount, so product
//     p = 64k + lane finds its entry e = C0_k + popcount(M_k & bits<=lane) - 1
//     and its column B.col[ebase[e] + p];
//   * f1, 16 bits per product bound: each product ORs its column's hash bit
//     with return; a product that finds it set is a candidate and marks its
//     column in f2 (2 bits per product, a second hash) — a wave's LDS
//     operations complete in issue order, so no barrier is needed;
//   * a product is "possibly a duplicate" if it is a candidate or its column's
//     f2 bit is set; every other product is certainly its column's only
//     product: its first-touch bit comes from one ballot per window, kept in
//     the lanes (lane j holds bitmap word j);
//   * the possible duplicates (a few % of the products) are listed in product
//     order and resolved exactly in a small LDS table (CAS claims the column,
//     atomicMin keeps its smallest product = the first touch);
//   * nnz and the word prefixes are a DPP scan of the lanes' popcounts; a
//     duplicate's rank comes from its word's lane by ds_bpermute.
// Rows whose list overflows go to a retry list that sym2's 128-lane teams
// (with their keys-only heavy-row fallback) finish; rows with more duplicates
// than their allocated targets take the numeric table path (dupn -1 / -3),
// as in sym2.  Persistent waves; the next row's columns are gathered (DB) and
// the row after next's entries loaded while a row is resolved.
#pragma once

#include "spgemm_kernels.hpp"

namespace ias {
namespace dev {

struct Sym3Args {
    AxView ax;                 // expanded A: bstart / blen per A entry
    const int32_t *bcol;       // B's columns
    const RowRef *list;        // rows of the bin
    int32_t count;
    const int32_t *prod;       // products per row
    int32_t *nnz_row;
    Bitmap bm;
    const int64_t *dup_off;
    int32_t *dupn;
    int32_t *gdupt;
    int32_t dcap;              // duplicate targets allocated per row: more -> table path
    int32_t bm_need;           // heavy rows above this nnz get dupn -3 (global table)
    RowRef *retry;             // rows whose possible-duplicate list overflows
    int32_t *retry_count;
};

constexpr int S3_F1BPP = 32;   // f1 bits per product bound (false candidates ~ P / (2 * F1B)); 16: K3' symbolic 4.03-4.07 vs 3.98-4.02 ms
template <int K>
struct Sym3Lds {
    static constexpr int U = 64 * K;       // product bound
    // filter sizes rounded up to powers of two: the hashes' range reduction
    // is then a shift, not a 64-bit multiply per product (K = 12, 24)
    static constexpr int pow2(int x) { return x <= 1 ? 1 : 2 * pow2((x + 1) / 2); }
    static constexpr int F1B = pow2(S3_F1BPP * U);   // f1 bits
    static constexpr int F1W = F1B / 32;
    static constexpr int F2B = pow2(2 * U);      // f2 bits
    static constexpr int F2W = F2B / 32;   // >= 2K: its first words also hold the bitmap words (exact phase)
    static constexpr int NE = WAVE;        // A entries per row at most (one per lane)
    static constexpr int LC = U / 8;       // possible-duplicate list capacity
    static constexpr int ES = LC;          // exact-table slots (the list is at most 3/4 full)
    static constexpr int LT = (LC + WAVE - 1) / WAVE;   // list entries per lane
    // after classification f1 is free: the list (8 B per entry) and the exact
    // table (column + first product, 8 B per slot) live there
    static_assert(8 * LC + 8 * ES <= 4 * F1W, "list and exact table overlay f1");
    static_assert(F2W >= 2 * K && 2 * K <= WAVE, "bitmap words: one per lane");
    __attribute__((aligned(16))) uint32_t f1[F1W];
    __attribute__((aligned(16))) uint32_t f2[F2W];
    int32_t ebase[NE];              // B-row start - first product (B has < 2^30 entries)
    __attribute__((aligned(8))) uint32_t words[2 * K];   // the classified first-touch words
    unsigned long long mask[K];
    __device__ int2 *list() { return (int2 *)f1; }
    __device__ int32_t *keys() { return (int32_t *)(f1 + 2 * LC); }
    __device__ uint32_t *own() { return (uint32_t *)(f1 + 2 * LC + ES); }
};

// A row as a wave holds it before resolving it.
struct Sym3Row {
    RowRef ref;       // row < 0: none
    int32_t P;
    int64_t bmoff, dupoff;
    int32_t bl;       // B-row length of entry `lane`
    int64_t bs;       //   and start
};

__device__ __forceinline__ uint32_t s3_h1(int32_t c, uint32_t n) {
    return (uint32_t)(((uint64_t)((uint32_t)c * 0x9E3779B1u) * n) >> 32);
}
__device__ __forceinline__ uint32_t s3_h2(int32_t c, uint32_t n) {
    return (uint32_t)(((uint64_t)((uint32_t)c * 0x85EBCA77u) * n) >> 32);
}
__device__ __forceinline__ uint32_t s3_h3(int32_t c, uint32_t n) {
    return (uint32_t)(((uint64_t)((uint32_t)c * 0xC2B2AE3Du) * n) >> 32);
}
// set bits of m below this lane (v_mbcnt: no 64-bit lane mask held in
// registers, which the unrolled loops spilled)
__device__ __forceinline__ int s3_below(uint64_t m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ void s3_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ int32_t s3_opaque_zero() {
    int32_t z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    return z;
}

// The kernel's arguments, read through the kernarg segment where they are
// used (a scalar-cache load each time) rather than held in SGPRs across the
// row loop: the loop needs every SGPR it has (measured: 105-274 SGPRs spilled
// to VGPR lanes, a quarter of sym3's VALU instructions in readlane /
// writelane).  The empty asm hides the pointer's value, so the loads are not
// hoisted out of the loop.
typedef const __attribute__((address_space(4))) Sym3Args *S3A;
__device__ __forceinline__ S3A s3_args() {
    S3A p = (S3A)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return p;
}

// The list entry of row idx (loaded a row ahead of its details, so that no
// wait for it stalls the loads issued after it).
__device__ __forceinline__ RowRef s3_ref(int64_t idx) {
    const S3A a = s3_args();
    return idx < a->count ? a->list[idx + s3_opaque_zero()] : RowRef{0, -1, 0};
}
__device__ __forceinline__ Sym3Row s3_load(const RowRef &ref) {
    const S3A a = s3_args();
    Sym3Row r;
    r.ref = ref;
    r.P = 0;
    r.bmoff = r.dupoff = 0;
    r.bl = 0;
    r.bs = 0;
    if (ref.row >= 0) {
        const int64_t row = (int64_t)ref.row;
        r.P = a->prod[row];
        r.bmoff = a->bm.off[row];
        r.dupoff = a->dup_off[row];
        const int lane = (int)__lane_id();
        if (lane < ref.n) {
            r.bl = a->ax.blen[ref.q0 + lane];
            r.bs = a->ax.bstart[ref.q0 + lane];
        }
    }
    return r;
}

// Stage a row's entries and gather its columns (c[k] of product 64k + lane;
// undefined beyond P: callers test 64k + lane < P, so no select waits on the
// load right after it is issued).  Branch-free loads: windows beyond P read B.col[0].  A row
// outside the kernel's bounds (P > U, more than 64 entries) is not staged:
// the caller sends it to the retry list.
template <int K>
__device__ __forceinline__ void s3_gather(Sym3Lds<K> &L, const Sym3Row &r, int32_t (&c)[K]) {
    const int lane = (int)__lane_id();
    const bool fits = r.P <= 64 * K && r.ref.n <= WAVE;
    const int32_t P = fits ? __builtin_amdgcn_readfirstlane(r.P) : 0;
    const int incl = wave_incl_sum(r.bl);
    const int rel = incl - r.bl;
    const uint64_t ne = __ballot(r.bl > 0);
    if (lane < K) L.mask[lane] = 0ull;
    s3_sync();
    if (r.bl > 0 && rel < P) {
        L.ebase[s3_below(ne)] = (int32_t)(r.bs - rel);
        atomicOr(&L.mask[(uint32_t)rel >> 6], 1ull << (rel & 63));
    }
    s3_sync();
    const uint64_t upto = (2ull << lane) - 1ull;
    // every window's entry base first (branch-free LDS reads, one wait), then
    // every window's column load (all in flight together).  The window masks
    // are LDS broadcast reads into VGPRs, not readlanes into SGPRs (those
    // stayed live together and spilled).
    int c0 = 0;   // non-empty entries starting before window k
    int32_t eb[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t m = L.mask[k];
        const int e = min(max(c0 + (int)__popcll(m & upto) - 1, 0), WAVE - 1);   // int: __popcll is unsigned
        eb[k] = L.ebase[e];
        c0 += (int)__popcll(m);
    }
    // 32-bit byte offsets from the uniform base (the caller guarantees
    // B.nnz < 2^30): one VGPR per address, the SGPR-base form of the load
    const char *base = (const char *)s3_args()->bcol;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int p = 64 * k + lane;
        const uint32_t off = p < P ? (uint32_t)(eb[k] + p) << 2 : 0u;   // beyond P: B.col[0], masked by the caller
        c[k] = *(const int32_t *)(base + off);
    }
}

// waves per SIMD the register allocation must allow (K columns per lane)
template <int K>
constexpr int sym3_wpe() { return K <= 8 ? 6 : (K <= 12 ? 5 : (K <= 16 ? 4 : 3)); }   // K3': K = 8 289 vs 296 us, K = 12 248 vs 258 us (K = 16 at 5: 211 vs 205)
template <int K, int WPB, bool DB>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(sym3_wpe<K>()))) void k_sym3(Sym3Args) {
    using LDS = Sym3Lds<K>;
    constexpr int CH = K < 8 ? K : (K % 8 == 0 ? 8 : (K % 6 == 0 ? 6 : 4));   // filter chunk: products per lane whose LDS atomics fly together
    static_assert(K % CH == 0, "K in whole chunks");
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

    // Pipeline, row i = cur.  DB: list entries two rows ahead, details and
    // columns one row ahead (row i+1's gathers fly while row i is resolved;
    // twice the column registers).  Otherwise row i+1's columns are gathered
    // into the same registers as soon as row i's classification no longer
    // needs them, so they fly during row i's exact phase and finish, and row
    // i+2's details with them.
    Sym3Row cur = s3_load(s3_ref(idx));
    int32_t c[K];
    s3_gather<K>(L, cur, c);
    Sym3Row nxt = s3_load(s3_ref(idx + stride));
    RowRef nref = s3_ref(idx + 2 * stride);
    Timer tm;   // timing builds only (phases: 0 top wait, 1 next row's gather / details issue (DB),
                // 2 filter, 3 classify + list, 4 exact, 5 finish, 6 filter clear, 7 next row's gather)
    tm.start();
    while (true) {
        if constexpr (DB) __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): row i's columns, row i+1's details
        tm.mark(0);
        const int32_t row = __builtin_amdgcn_readfirstlane(cur.ref.row);
        if (row < 0) break;
        const int32_t P = __builtin_amdgcn_readfirstlane(cur.P);
        const int32_t nent = __builtin_amdgcn_readfirstlane(cur.ref.n);
        const int64_t bmoff = __builtin_amdgcn_readfirstlane(0) + cur.bmoff;
        const int64_t dupoff = cur.dupoff;
        const RowRef cref = cur.ref;
        int32_t cn[DB ? K : 1];
        Sym3Row nn;
        if constexpr (DB) {
            s3_gather<K>(L, nxt, cn);   // nxt.row < 0: dummy loads of B.col[0]
            nn = s3_load(nref);
            nref = s3_ref(idx + 3 * stride);
        }
        tm.mark(1);

        // windows holding a product of this lane (64k + lane < P <=> k < nwin),
        // a VGPR re-derived per phase: one compare per window there, instead of
        // K window masks the compiler would keep in SGPRs across phases
        int nwin = (P - lane + 63) >> 6;
        // ---- filter: f1 with return, candidates mark f2 (CH items at a time)
        asm volatile("" : "+v"(nwin));
        uint32_t candm = 0u;
#pragma unroll
        for (int k0 = 0; k0 < K; k0 += CH) {
            uint32_t old[CH], bit[CH];
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                const int32_t cc = c[k0 + t];
                const bool in = k0 + t < nwin;
                const uint32_t h = s3_h1(cc, LDS::F1B);
                bit[t] = in ? 1u << (h & 31) : 0u;
                // lanes past the row issue nothing (a same-address atomic of
                // every idle lane serialises in one bank)
                uint32_t o = 0u;
                if (in) o = atomicOr(&L.f1[h >> 5], bit[t]);
                old[t] = o;
            }
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                const bool cand = (old[t] & bit[t]) != 0u;
                candm |= (cand ? 1u : 0u) << (k0 + t);
                if (cand) {
                    const uint32_t h = s3_h2(c[k0 + t], LDS::F2B);
                    atomicOr(&L.f2[h >> 5], 1u << (h & 31));
                }
            }
        }
        s3_sync();
        tm.mark(2);
        // ---- classify: certain first touches -> bitmap words in the lanes,
        // possible duplicates -> list (product order) over f1 (its reads, the
        // filter's atomics, are complete: a wave's LDS operations complete in
        // order)
        uint32_t wd = 0u;   // lane j: bitmap word j
        int32_t nl = 0;
        int2 *list = L.list();
        int32_t *keys = L.keys();
        uint32_t *own = L.own();
        asm volatile("" : "+v"(nwin));
#pragma unroll
        for (int k0 = 0; k0 < K; k0 += CH) {
            uint32_t f2w[CH];
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                const int32_t cc = c[k0 + t];
                f2w[t] = L.f2[k0 + t < nwin ? s3_h2(cc, LDS::F2B) >> 5 : 0u];
            }
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                const int k = k0 + t;
                const int32_t cc = c[k];
                const bool in = k < nwin;
                // bitwise, not short-circuit: the compiler otherwise branched
                // per window around the f2 test
                const uint32_t pv = ((candm >> k) | (f2w[t] >> (s3_h2(cc, LDS::F2B) & 31))) & (in ? 1u : 0u);
                const bool poss = pv != 0u;
                const uint64_t b = __ballot(in && !poss);
                // words 2k, 2k+1 via LDS into lanes 2k, 2k+1 after the loop (a
                // select on lane == 2k kept 2K lane masks live in SGPRs: spills)
                if (lane == 0) *(uint64_t *)&L.words[2 * k] = b;
                const uint64_t pb = __ballot(poss);
                if (poss) {
                    const int i = nl + s3_below(pb);
                    if (i < LDS::LC) list[i] = make_int2(cc, 64 * k + lane);
                }
                nl += (int)__popcll(pb);
            }
        }
        s3_sync();
        wd = lane < 2 * K ? L.words[lane] : 0u;
        const int32_t row_nw = (P + 31) >> 5;
        tm.mark(3);
        if constexpr (!DB) {
            // row i's columns are dead: row i+1's gathers fly from here on
            s3_gather<K>(L, nxt, c);
            nn = s3_load(nref);
            nref = s3_ref(idx + 3 * stride);
            tm.mark(7);
        }
        const bool retry = 4 * nl > 3 * LDS::LC || P > LDS::U || nent > WAVE;
        if (nl > 0 && !retry) {
            // ---- exact: claim the column (CAS, linear probing); its smallest
            // product is the first touch
            for (int i = lane; i < LDS::ES; i += WAVE) keys[i] = EMPTY_KEY;
            for (int i = lane; i < LDS::F2W; i += WAVE) L.f2[i] = i < 2 * K ? wd : 0u;   // bitmap words -> LDS (f2 is done)
            s3_sync();
            int2 e[LDS::LT];
            uint32_t slot[LDS::LT];
            uint32_t wonm = 0u;
#pragma unroll
            for (int t = 0; t < LDS::LT; ++t) {
                const int i = t * WAVE + lane;
                slot[t] = 0;
                e[t] = make_int2(0, 0);
                if (i < nl) {
                    e[t] = list[i];
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
            uint32_t f[LDS::LT];
#pragma unroll
            for (int t = 0; t < LDS::LT; ++t) {
                f[t] = 0;
                if (t * WAVE + lane < nl) {
                    f[t] = own[slot[t]];
                    const uint32_t p = (uint32_t)e[t].y;
                    if (f[t] == p) atomicOr(&L.f2[p >> 5], 1u << (p & 31));
                }
            }
            s3_sync();
            wd = lane < 2 * K ? L.f2[lane] : 0u;
            tm.mark(4);
            // ---- finish with duplicates
            const uint32_t cnt = lane < row_nw ? (uint32_t)__popc(wd) : 0u;
            const int incl = wave_incl_sum((int)cnt);
            const int nnz = __builtin_amdgcn_readlane(incl, WAVE - 1);
            const uint32_t pre = (uint32_t)(incl - (int)cnt);
            const bool heavy = P - nnz > s3_args()->dcap;
            if (!heavy) {
                if (lane < row_nw) {
                    s3_args()->bm.bits[bmoff + lane] = wd;
                    s3_args()->bm.pref[bmoff + lane] = pre;
                }
#pragma unroll
                for (int t = 0; t < LDS::LT; ++t) {
                    const uint32_t p = (uint32_t)e[t].y;
                    // the word and prefix of p's lane
                    const uint32_t pw = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((p >> 5) << 2), (int)wd);
                    const uint32_t pp = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((p >> 5) << 2), (int)pre);
                    if (t * WAVE + lane < nl && f[t] != p) {
                        const uint32_t rk = pp + (uint32_t)__popc(pw & ((1u << (p & 31)) - 1u));
                        s3_args()->gdupt[dupoff + (p - rk)] = (int32_t)f[t];
                    }
                }
            }
            if (lane == 0) {
                s3_args()->nnz_row[row] = nnz;
                s3_args()->dupn[row] = heavy ? (nnz > s3_args()->bm_need ? -3 : -1) : P - nnz;
            }
        } else if (!retry) {
            // ---- finish, no possible duplicate: every product is a first touch
            const uint32_t cnt = lane < row_nw ? (uint32_t)__popc(wd) : 0u;
            const int incl = wave_incl_sum((int)cnt);
            const int nnz = __builtin_amdgcn_readlane(incl, WAVE - 1);
            if (lane < row_nw) {
                s3_args()->bm.bits[bmoff + lane] = wd;
                s3_args()->bm.pref[bmoff + lane] = (uint32_t)(incl - (int)cnt);
            }
            if (lane == 0) {
                s3_args()->nnz_row[row] = nnz;
                s3_args()->dupn[row] = P - nnz;
            }
        } else if (lane == 0) {
            // outside this kernel's bounds: sym2's teams finish this row
            const int32_t j = atomicAdd(s3_args()->retry_count, 1);
            s3_args()->retry[j] = cref;
        }
        // ---- the filters empty for the next row
        tm.mark(5);
        s3_sync();
        for (int i = lane; i < LDS::F1W / 4; i += WAVE) ((uint4 *)L.f1)[i] = make_uint4(0u, 0u, 0u, 0u);
        for (int i = lane; i < LDS::F2W; i += WAVE) L.f2[i] = 0u;
        s3_sync();
        tm.mark(6);
        if constexpr (DB) {
#pragma unroll
            for (int k = 0; k < K; ++k) c[k] = cn[DB ? k : 0];
        }
        cur = nxt;
        nxt = nn;
        tm.done();
        idx += stride;
    }
    tm.flush(24 + (K >= 16 ? 2 : (K >= 12 ? 1 : 0)), lane == 0);
}

}  // namespace dev
}  // namespace ias
