// sym2_kernels.hpp — symbolic pass of the LDS-bin rows, gathering each
// product's column straight from B (no materialised expansion).
//
// Restates CSR_MUL_CSR's first loop (IA-SPGEMM-CPU_release/detail/csr/
// common_csr.h:95-125: distinct columns per row) and, for the table-free
// numeric pass, the discovery order of its second loop (:133-189: the first
// touch of every column, whose reverse is the output order).  Per row, one
// team (64..1024 lanes) does:
//   1. stage: the row's A entries (expanded A: B-row start and length) are
//      compacted to the non-empty ones; their product prefix gives each a base
//      (B-row start - first product) and a start bit in a P-bit mask, whose
//      64-bit words carry prefix popcounts — product p's entry is then
//      wpre[p/64] + popcount(mask word below p) - 1, two LDS reads per 64
//      products (broadcast), no per-product search;
//   2. gather: K products per lane (p = k*TEAM + lane), all K column loads in
//      flight at once, B.col[base(e) + p];
//   3. filter: duplicates are rare (nnz(C) / flops = 0.99 on R-MAT), so no
//      product pays for an exact hash insert unless it may be one.  Each
//      product sets the bit of its column's hash in a 16-bits-per-product
//      bitmap f1 with one returning LDS atomicOr; a product that finds its bit
//      already set is a candidate and marks the bit in f2.  After a barrier a
//      product is "possibly a duplicate" when it is a candidate or its f2 bit
//      is set; every other product is certainly its column's only product, so
//      its first-touch bit is set from a ballot.  ~20 VALU + 3 LDS operations
//      per 64 products instead of a hash insert's ~200 (measured: the bucketed
//      CAS insert made the pass instruction-bound, SQ_INSTS_VALU);
//   4. exact: the possible duplicates (all products of every duplicated
//      column, plus hash-collision false positives, ~5-10 %) are compacted
//      into a list and inserted into a small LDS table (linear probing, one
//      CAS to claim); the CAS winner writes its product into own[slot], the
//      losers then atomicMin theirs in, and the column's first touch is the
//      minimum — its bit is set; every other product gets (p, first touch).
//      A row whose list overflows (more than a quarter of its products) only
//      counts its distinct columns (keys-only table over the whole region)
//      and, like a row with more duplicates than its allocated targets,
//      takes the numeric pass's table path (dupn = -1);
//   5. finish: bitmap words + per-word prefix popcounts to HBM, nnz, and each
//      duplicate's target at its product-order index d = p - rank(p).
// A team works on two rows at once: the next row is staged and its column
// loads fly while the current row is filtered and resolved.
#pragma once

#include "spgemm_kernels.hpp"

namespace ias {
namespace dev {

// LDS layout of one sym2 team for rows of at most U products:
// [f1 4FW | f2 4FW | list 8LC | keys 4ES | own 4ES | ebase 8EC | mask 8W | wpre 4W | lbits 8W | lpref 8W | scratch]
// FW = filter words (8 or 16 bits per product), LC = list capacity (U/8 or U/4), ES =
// exact-table slots (2 LC), EC = non-empty entries (U/8), W = 64-bit mask words.
struct Sym2Layout {
    uint32_t U, FW, LC, ES, EC, W;
    __host__ __device__ static constexpr size_t r16(size_t b) { return (b + 15) & ~size_t(15); }
    __host__ __device__ size_t f1() const { return 0; }
    __host__ __device__ size_t f2() const { return f1() + r16(4ull * FW); }
    __host__ __device__ size_t list() const { return f2() + r16(4ull * FW); }
    __host__ __device__ size_t keys() const { return list() + r16(8ull * LC); }
    __host__ __device__ size_t own() const { return keys() + r16(4ull * ES); }
    __host__ __device__ size_t ebase() const { return own() + r16(4ull * ES); }
    __host__ __device__ size_t mask() const { return ebase() + r16(8ull * EC); }
    __host__ __device__ size_t wpre() const { return mask() + r16(8ull * W); }
    __host__ __device__ size_t lbits() const { return wpre() + r16(4ull * W); }
    __host__ __device__ size_t lpref() const { return lbits() + r16(8ull * W); }
    __host__ __device__ size_t scratch() const { return lpref() + r16(8ull * W); }
    __host__ __device__ size_t bytes() const { return scratch() + 256; }
    // the heavy-row fallback's keys-only table spans f1 .. own
    __host__ __device__ uint32_t heavy_slots() const { return (uint32_t)((ebase() - f1()) / 4); }
    // one-wave teams (wide rows on one wave: LDS per wave is the limit) keep
    // 8 filter bits and an eighth of the products for the exact list; the
    // workgroup teams 16 bits and a quarter; the widest bin (16384 products,
    // one team per CU) 8 bits and a quarter
    enum Mode { TEAM_LAYOUT = 0, ONE_WAVE = 1, WIDE = 2 };
    __host__ static Sym2Layout for_bound(uint32_t upper, Mode m) {
        Sym2Layout L;
        L.U = upper;
        L.FW = m == TEAM_LAYOUT ? upper / 2 : upper / 4;
        L.LC = m == ONE_WAVE ? upper / 8 : upper / 4;
        L.ES = 2 * L.LC;
        L.EC = upper / 8;
        L.W = (upper + 63) / 64;
        return L;
    }
};

struct Sym2Args {
    AxView ax;                 // expanded A: bstart / blen per A entry
    const int32_t *bcol;       // B's columns
    const RowRef *list;        // rows of the bin: q0 = first A entry, n = A entries
    int32_t count;
    const int32_t *prod;       // products per row
    Sym2Layout lay;
    int32_t *nnz_row;
    Bitmap bm;
    const int64_t *dup_off;
    int32_t *dupn;
    int32_t *gdupt;
    int32_t dcap;              // duplicate targets allocated per row (dup_off spacing): more -> table path
    int32_t bm_need;           // heavy rows above this nnz get dupn -3: the numeric pass's
                               // partitioned path needs a bitmap they do not have
    const int32_t *count_dev;  // non-null: the row count is read here (sym3's retry list)
};

// What a team prefetches of a row before it works on it.
struct Sym2Row {
    RowRef ref;      // row < 0: none
    int32_t P;       // products
    int64_t bmoff;   // bitmap word offset
    int64_t dupoff;  // duplicate-list offset
    int32_t bl;      // this lane's A entry of the row's first 64 entries (first wave): B-row length
    int64_t bs;      //   and start
};

// A zero the compiler cannot see through: row-uniform prefetches indexed
// with it load into VGPRs, so the compiler does not move them into SGPRs
// (v_readfirstlane) — and wait for them — right where they are issued; they
// become scalars (uni / uni64) only where they are used, a row later.
__device__ __forceinline__ int32_t opaque_zero() {
    int32_t z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    return z;
}
__device__ __forceinline__ int32_t uni(int32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ int64_t uni64(int64_t x) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)x);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)((uint64_t)x >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// The kernel's arguments, read through the kernarg segment where they are
// used (scalar-cache loads) instead of held in SGPRs across the row loop (as
// in sym3_kernels.hpp: the loop's hoisted pointer arithmetic spilled).
typedef const __attribute__((address_space(4))) Sym2Args *S2A;
__device__ __forceinline__ S2A s2_args() {
    S2A p = (S2A)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return p;
}

template <int TEAM>
__device__ __forceinline__ RowRef sym2_ref(int32_t count, int64_t idx) {
    return idx < count ? s2_args()->list[idx + opaque_zero()] : RowRef{0, -1, 0};
}

template <int TEAM>
__device__ __forceinline__ Sym2Row sym2_detail(const RowRef &ref) {
    const S2A a = s2_args();
    Sym2Row r;
    r.ref = ref;
    r.P = 0;
    r.bmoff = r.dupoff = 0;
    r.bl = 0;
    r.bs = 0;
    if (ref.row >= 0) {
        const int64_t row = (int64_t)ref.row + opaque_zero();
        r.P = a->prod[row];
        r.bmoff = a->bm.off[row];
        r.dupoff = a->dup_off[row];
        const int lane = Team<TEAM>::lane();
        if (lane < WAVE && lane < ref.n) {
            r.bl = a->ax.blen[ref.q0 + lane];
            r.bs = a->ax.bstart[ref.q0 + lane];
        }
    }
    return r;
}

constexpr int SYM2_DB_MAX = 8; // K up to which a team double-buffers the next row's columns in registers

// range reduction of a 32-bit hash onto [0, n)
__device__ __forceinline__ uint32_t reduce32(uint32_t h, uint32_t n) {
    return (uint32_t)(((uint64_t)h * n) >> 32);
}
__device__ __forceinline__ uint32_t fib(int32_t c) { return (uint32_t)c * 0x9E3779B1u; }

// WPE: minimum waves per SIMD the register allocation must allow (one-wave
// teams with K >= 16 would otherwise take 160-256 VGPRs, 2 waves per SIMD).
template <int TEAM, int K, int TPW, int WPE>
__global__ __launch_bounds__(TEAM *TPW) __attribute__((amdgpu_waves_per_eu(WPE))) void k_sym2(Sym2Args a0) {
    const int32_t count = a0.count_dev ? *a0.count_dev : a0.count;
    static_assert(TEAM >= WAVE && (TEAM <= WAVE || TPW == 1), "teams are whole waves; multi-wave teams own the WG");
    static_assert(TEAM == WAVE ? K <= 32 : K <= 16, "finish() covers the bitmap words in one pass");
    using TM = Team<TEAM>;
    constexpr int LPASS = K > 4 ? K / 4 : 1;   // list capacity <= U/4 <= LPASS * TEAM
    constexpr int CH = K < 8 ? K : (TEAM > WAVE && K > 8 ? 4 : 8);   // items per register chunk (1024-lane teams: 128 VGPRs)
    constexpr bool DB = K <= SYM2_DB_MAX;      // next row's columns gathered during this row's work
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const Sym2Layout L = a0.lay;
    const int team = (TPW == 1) ? 0 : (int)(threadIdx.x / TEAM);
    unsigned char *base = smem + (size_t)team * L.bytes();
    uint32_t *f1 = (uint32_t *)(base + L.f1());
    uint32_t *f2 = (uint32_t *)(base + L.f2());
    int2 *list = (int2 *)(base + L.list());
    int32_t *keys = (int32_t *)(base + L.keys());
    uint32_t *own = (uint32_t *)(base + L.own());
    int64_t *ebase = (int64_t *)(base + L.ebase());
    unsigned long long *mask = (unsigned long long *)(base + L.mask());
    uint32_t *wpre = (uint32_t *)(base + L.wpre());
    uint32_t *lbits = (uint32_t *)(base + L.lbits());
    uint32_t *lpref = (uint32_t *)(base + L.lpref());
    int *scratch = (int *)(base + L.scratch());
    int *lcount = scratch + 60;   // possible duplicates listed (scratch[0..16) serves the team scans)
    int *hcount = scratch + 61;   // heavy rows: distinct columns
    int lane = TM::lane();   // re-hidden every row (below): no lane compares hoisted out of the row loop
    const uint32_t FB = 32u * L.FW;   // filter bits
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    Timer tm;   // timing builds only (phases: 0 wait for row i's columns, 1 stage row i+1, 2 gather
                // row i+1 + prefetch issue, 7 filter pass 3a, 4 classify 3b, 3 exact, 5 finish,
                // 6 final barrier)
    // f1, f2 zero and the exact table empty, for the next row
    auto clear_tables = [&]() __attribute__((always_inline)) {
        for (uint32_t i = lane; i < L.FW / 2; i += TEAM) ((uint4 *)f1)[i] = make_uint4(0u, 0u, 0u, 0u);
        for (uint32_t i = lane; i < L.ES / 4; i += TEAM) ((int4 *)keys)[i] = make_int4(-1, -1, -1, -1);
    };

    // ---- stage a row, by the team's first wave alone (one team barrier at
    // the end): compact its non-empty entries into bases + start bits, then
    // the start-bit word prefixes.  The first 64 entries were prefetched into
    // the first wave's lanes (bl0/bs0); longer entry lists load the rest here.
    auto stage = [&](int64_t q0, int32_t n, int32_t P, int32_t bl0, int64_t bs0) __attribute__((always_inline)) {
        if (lane < WAVE) {
            const uint32_t W = (uint32_t)((P + 63) / 64);
            for (uint32_t w = lane; w < W; w += WAVE) mask[w] = 0ull;
            wave_sync();
            int carry = 0;   // products before the chunk | non-empty entries before it << 16
            for (int32_t e0 = 0; e0 < n; e0 += WAVE) {
                int32_t bl = bl0;
                int64_t bs = bs0;
                if (e0 > 0) {
                    bl = 0;
                    if (e0 + lane < n) {
                        bl = s2_args()->ax.blen[q0 + e0 + lane];
                        bs = s2_args()->ax.bstart[q0 + e0 + lane];
                    }
                }
                const int v = bl + (bl > 0 ? (1 << 16) : 0);
                int tot;
                const int ex = carry + Team<WAVE>::excl_sum(v, tot, scratch);
                if (bl > 0) {
                    const int s = ex & 0xFFFF;
                    ebase[ex >> 16] = bs - s;
                    atomicOr(&mask[s >> 6], 1ull << (s & 63));
                }
                carry += tot;
            }
            wave_sync();
            int carry2 = 0;
            for (uint32_t w0 = 0; w0 < W; w0 += WAVE) {
                const uint32_t w = w0 + lane;
                const int c = w < W ? __popcll(mask[w]) : 0;
                int tot;
                const int ex = Team<WAVE>::excl_sum(c, tot, scratch);
                if (w < W) wpre[w] = (uint32_t)(carry2 + ex);
                carry2 += tot;
            }
        }
        TM::sync();
    };
    // ---- gather the staged row's columns: K loads in flight per lane, not waited here
    auto gather = [&](int32_t P, int32_t (&c)[K]) __attribute__((always_inline)) {
        // branch-free (clamped indices, a safe dummy address for items beyond
        // P): the compiler then issues a chunk's LDS reads together and its
        // loads back to back instead of one exec-masked block per item
#pragma unroll
        for (int k0 = 0; k0 < K; k0 += CH) {
            int64_t at[CH];
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                const int p = (k0 + t) * TEAM + lane;
                const int pc = p < P ? p : 0;
                const unsigned long long m = mask[pc >> 6];
                const int e = (int)wpre[pc >> 6] + __popcll(m & ((2ull << (pc & 63)) - 1ull)) - 1;
                at[t] = ebase[e] + pc;
            }
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                const int p = (k0 + t) * TEAM + lane;
                c[k0 + t] = s2_args()->bcol[p < P ? at[t] : 0];
            }
        }
    };
    // ---- filter + exact resolution (steps 3-4); returns the listed count L,
    // or -1 for a heavy row (then *hcount = its distinct columns)
    auto resolve = [&](int32_t P, const int32_t (&c)[K]) __attribute__((always_inline)) -> int32_t {
        // 3a. f1 with return; candidates mark f2 (branch-free: items beyond P
        // OR nothing into word 0, so a chunk's atomics issue back to back)
        uint32_t candm = 0u;
#pragma unroll
        for (int k0 = 0; k0 < K; k0 += CH) {
            uint32_t word[CH], bitm[CH], old[CH];
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                const bool in = (k0 + t) * TEAM + lane < P;
                const uint32_t bit = reduce32(fib(c[k0 + t]), FB);
                word[t] = in ? bit >> 5 : 0u;
                bitm[t] = in ? 1u << (bit & 31) : 0u;
            }
#pragma unroll
            for (int t = 0; t < CH; ++t) old[t] = atomicOr(&f1[word[t]], bitm[t]);
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                const bool cand = (old[t] & bitm[t]) != 0u;
                candm |= (cand ? 1u : 0u) << (k0 + t);
                // candidates only (a few %): an all-lane atomic at random words
                // doubled the LDS bank conflicts of the pass
                if (cand) atomicOr(&f2[word[t]], bitm[t]);
            }
        }
        TM::sync();
        tm.mark(7);
        // 3b. classify: certain first touches -> bitmap words; possible
        // duplicates -> list (one list atomic per wave and chunk)
#pragma unroll
        for (int k0 = 0; k0 < K; k0 += CH) {
            uint32_t f2w[CH], bitm[CH];
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                const bool in = (k0 + t) * TEAM + lane < P;
                const uint32_t bit = reduce32(fib(c[k0 + t]), FB);
                bitm[t] = in ? 1u << (bit & 31) : 0u;
                f2w[t] = f2[in ? bit >> 5 : 0u];
            }
            uint64_t pb[CH];
            uint32_t possm = 0u;
            int ptot = 0;
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                const int k = k0 + t;
                const int p = k * TEAM + lane;
                const bool poss = ((candm >> k) & 1u) || (f2w[t] & bitm[t]) != 0u;
                possm |= (poss ? 1u : 0u) << t;
                const uint64_t wb = __ballot(p < P && !poss);
                const uint32_t p0 = (uint32_t)(k * TEAM) + (uint32_t)(lane & ~(WAVE - 1));   // 64-aligned
                if ((lane & (WAVE - 1)) == 0 && p0 < (uint32_t)P) {
                    lbits[p0 >> 5] = (uint32_t)wb;
                    lbits[(p0 >> 5) + 1] = (uint32_t)(wb >> 32);
                }
                pb[t] = __ballot(poss);
                ptot += __popcll(pb[t]);
            }
            if (ptot) {
                int at = 0;
                if (__lane_id() == 0) at = atomicAdd(lcount, ptot);
                at = __builtin_amdgcn_readfirstlane(at);
                const uint64_t lt = (1ull << __lane_id()) - 1ull;
#pragma unroll
                for (int t = 0; t < CH; ++t) {
                    if ((possm >> t) & 1u) {
                        const int i = at + __popcll(pb[t] & lt);
                        if ((uint32_t)i < L.LC) list[i] = make_int2(c[k0 + t], (k0 + t) * TEAM + lane);
                    }
                    at += __popcll(pb[t]);
                }
            }
        }
        TM::sync();
        tm.mark(4);
        const int32_t nl = *lcount;
        if ((uint32_t)nl > L.LC) {
            // heavy row: count distinct columns in a keys-only table over f1 .. own
            int32_t *hk = (int32_t *)f1;
            const uint32_t HS = L.heavy_slots();
            for (uint32_t i = lane; i < HS; i += TEAM) hk[i] = EMPTY_KEY;
            TM::sync();
            int made = 0;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int p = k * TEAM + lane;
                if (p >= P) continue;
                uint32_t s = reduce32(fib(c[k]), HS);
                for (uint32_t probe = 0; probe < HS; ++probe) {
                    const int32_t g = atomicCAS(&hk[s], EMPTY_KEY, c[k]);
                    if (g == EMPTY_KEY) { ++made; break; }
                    if (g == c[k]) break;
                    s = (s + 1u == HS) ? 0u : s + 1u;
                }
            }
            const int tot = TM::sum(made, scratch);
            if (lane == 0) *hcount = tot;
            return -1;
        }
        if (TM::MULTI && nl > 0 && nl <= WAVE) {
            // 4'. a short list (the common case: a few % of the products): the
            // team's first wave resolves it alone with wave-level syncs, one
            // team barrier instead of three
            if (lane < WAVE) {
                uint32_t s = 0;
                bool won = false;
                int2 e = make_int2(0, 0);
                if (lane < nl) {
                    e = list[lane];
                    s = reduce32(fib(e.x), L.ES);
                    for (uint32_t probe = 0; probe < L.ES; ++probe) {
                        const int32_t g = atomicCAS(&keys[s], EMPTY_KEY, e.x);
                        if (g == EMPTY_KEY) { won = true; break; }
                        if (g == e.x) break;
                        s = (s + 1u == L.ES) ? 0u : s + 1u;
                    }
                    if (won) own[s] = (uint32_t)e.y;
                }
                wave_sync();
                if (lane < nl && !won) atomicMin(&own[s], (uint32_t)e.y);
                wave_sync();
                if (lane < nl) {
                    const uint32_t p = (uint32_t)e.y;
                    const uint32_t f = own[s];
                    if (f == p) atomicOr(&lbits[p >> 5], 1u << (p & 31));
                    list[lane] = make_int2((int32_t)p, (int32_t)f);
                }
            }
            TM::sync();
        } else if (nl > 0) {
            // 4. exact: claim a slot per column (linear probing), winners own it
            for (int32_t i = lane; i < nl; i += TEAM) {
                const int2 e = list[i];
                uint32_t s = reduce32(fib(e.x), L.ES);
                bool won = false;
                for (uint32_t probe = 0; probe < L.ES; ++probe) {
                    const int32_t g = atomicCAS(&keys[s], EMPTY_KEY, e.x);
                    if (g == EMPTY_KEY) { won = true; break; }
                    if (g == e.x) break;
                    s = (s + 1u == L.ES) ? 0u : s + 1u;
                }
                if (won) own[s] = (uint32_t)e.y;
                list[i].x = (int32_t)((won ? 0x80000000u : 0u) | (s << 16) | (uint32_t)e.y);
            }
            TM::sync();
            for (int32_t i = lane; i < nl; i += TEAM) {
                const uint32_t v = (uint32_t)list[i].x;
                if (!(v >> 31)) atomicMin(&own[(v >> 16) & 0x7FFFu], v & 0xFFFFu);
            }
            TM::sync();
            // first touch = the column's smallest product; the others point at it
            for (int32_t i = lane; i < nl; i += TEAM) {
                const uint32_t v = (uint32_t)list[i].x;
                const uint32_t p = v & 0xFFFFu;
                const uint32_t f = own[(v >> 16) & 0x7FFFu];
                if (f == p) atomicOr(&lbits[p >> 5], 1u << (p & 31));
                list[i] = make_int2((int32_t)p, (int32_t)f);
            }
            TM::sync();
        }
        return nl;
    };
    // ---- finish a row (LDS and global stores only: the next row's gathers
    // stay in flight): bitmap words + prefixes, nnz, duplicate targets
    auto finish = [&](int32_t row, int32_t P, int64_t bmoff, int64_t dupoff, int32_t nl) __attribute__((always_inline)) {
        // One pass (no loop: a loop holding global stores makes the compiler
        // flush the wait count at its entry, i.e. wait for the next row's
        // gathers): nw = ceil(P/32) <= TEAM*K/32 <= TEAM for K <= 32.
        const uint32_t nw = (uint32_t)((P + 31) / 32);
        const uint32_t word = (uint32_t)lane < nw ? lbits[lane] : 0u;
        int nnz;
        const int ex = TM::excl_sum(__popc(word), nnz, scratch);
        if (nl < 0) nnz = *hcount;
        // more duplicates than the row's allocated targets: the numeric pass's table path
        const bool heavy = nl < 0 || P - nnz > s2_args()->dcap;
        if ((uint32_t)lane < nw && !heavy) {
            lpref[lane] = (uint32_t)ex;
            s2_args()->bm.bits[bmoff + lane] = word;
            s2_args()->bm.pref[bmoff + lane] = (uint32_t)ex;
        }
        if (nl > 0 && !heavy) {
            TM::sync();   // lpref complete
            // each duplicate's target at its duplicate index d = p - rank(p)
#pragma unroll
            for (int t = 0; t < LPASS; ++t) {
                const int32_t i = t * TEAM + lane;
                if (i < nl) {
                    const int2 e = list[i];
                    const uint32_t x = (uint32_t)e.x;
                    if (x != (uint32_t)e.y) {
                        const uint32_t rk = lpref[x >> 5] + (uint32_t)__popc(lbits[x >> 5] & ((1u << (x & 31)) - 1u));
                        s2_args()->gdupt[dupoff + (x - rk)] = e.y;
                    }
                }
            }
        }
        if (lane == 0) {
            s2_args()->nnz_row[row] = nnz;
            s2_args()->dupn[row] = heavy ? (nnz > s2_args()->bm_need ? -3 : -1) : P - nnz;
            *lcount = 0;   // every lane read it before this pass's barriers
        }
        clear_tables();   // the caller's barrier follows
    };

    clear_tables();
    if (lane == 0) *lcount = 0;
    const int64_t nteams = (int64_t)gridDim.x * TPW;
    int64_t idx = (int64_t)blockIdx.x * TPW + team;
    // the current row (scalars, so nothing of it lives in scratch memory)
    Sym2Row cur = sym2_detail<TEAM>(sym2_ref<TEAM>(count, idx));
    int32_t row = uni(cur.ref.row), P = uni(cur.P);
    int64_t bmoff = uni64(cur.bmoff), dupoff = uni64(cur.dupoff);
    int32_t c[K];
    if (row >= 0) {
        stage(uni64(cur.ref.q0), uni(cur.ref.n), P, cur.bl, cur.bs);
        gather(P, c);
        TM::sync();   // every wave has read the staging arrays before the loop's stage() rewrites them
    }
    Sym2Row nxt = sym2_detail<TEAM>(sym2_ref<TEAM>(count, idx + nteams));
    RowRef nref = sym2_ref<TEAM>(count, idx + 2 * nteams);
    tm.start();
    // Software pipeline, per iteration (row i): stage + gather row i+1, its
    // column loads then fly during row i's resolution; prefetch row i+2's
    // details and row i+3's list entry; resolve row i; finish row i.
    while (row >= 0) {
        // the compiler would otherwise hoist every lane-vs-constant compare of
        // the loop body out of it and keep the masks in SGPRs (spilled)
        asm volatile("" : "+v"(lane));
        // row i's columns and row i+1's details have landed (an explicit
        // vmcnt(0) the compiler's wait-count pass sees: the loads issued next
        // are then the only ones in flight)
        __builtin_amdgcn_s_waitcnt(0x0F70);
        tm.mark(0);
        const int32_t nrow = uni(nxt.ref.row), nP = uni(nxt.P);
        int32_t cn[DB ? K : 1];
        if (nrow >= 0) {
            stage(uni64(nxt.ref.q0), uni(nxt.ref.n), nP, nxt.bl, nxt.bs);
            tm.mark(1);
            if constexpr (DB) gather(nP, cn);
        }
        const Sym2Row nn = sym2_detail<TEAM>(nref);
        nref = sym2_ref<TEAM>(count, idx + 3 * nteams);
        tm.mark(2);
        const int32_t nl = resolve(P, c);
        tm.mark(3);
        finish(row, P, bmoff, dupoff, nl);
        tm.mark(5);
        TM::sync();   // tables / lbits / list are the next row's
        tm.mark(6);
        tm.done();
        if constexpr (DB) {
#pragma unroll
            for (int k = 0; k < K; ++k) c[k] = cn[(DB ? k : 0)];
        } else if (nrow >= 0) {
            gather(nP, c);   // one register set: other waves cover the load latency
            TM::sync();      // every wave has read the staging arrays before the next stage()
        }
        row = nrow;
        P = nP;
        bmoff = uni64(nxt.bmoff);
        dupoff = uni64(nxt.dupoff);
        nxt = nn;
        idx += nteams;
    }
    tm.flush(ilog2(TEAM), lane == 0);
}

}  // namespace dev
}  // namespace ias
