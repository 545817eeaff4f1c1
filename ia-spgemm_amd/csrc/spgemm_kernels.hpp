// spgemm_kernels.hpp — gfx950 device code of the row-wise SpGEMM hot path.
//
// Algorithm (Gustavson row-wise, C(i,:) = sum_j A(i,j) * B(j,:)), restating
// CSR_MUL_CSR (IA-SPGEMM-CPU_release/detail/csr/common_csr.h:85-193) so that
// the output is value-for-value identical to it:
//   * symbolic: distinct output columns per row, counted in a per-row
//     open-addressing hash table (keys only) held in LDS;
//   * numeric: the same hash, now carrying a value and the first-touch
//     ("discovery") rank of every column.  The products of a row are taken in
//     the reference's order p = 0..P-1 (A entries in row order, then B entries
//     in row order), TEAM*K of them per step, K per lane.  Items of a step that
//     hit the same column are serialised in product order (owner =
//     atomicMin of the item id), so every sum is formed as the reference forms
//     it: s = 0.0 + p0, s = s + p1, ... (no FMA: -ffp-contract=off).  A column's
//     rank is the number of distinct columns discovered before it; the entry
//     lands at nnz-1-rank (reverse first-touch, the reference's linked-list
//     order) or at rank (forward first-touch, COO_MUL_COO's order).
// Rows are binned by work (products for symbolic, nnz for numeric); each bin
// has a team size (16..1024 lanes) and an LDS table.  Rows too large for one
// LDS table are split by a hash of the column into `nparts` partitions, one
// workgroup each; the symbolic pass then also records, per row, a bitmap of
// first-touch product positions (and its word prefix counts) from which a
// partition computes the global discovery rank of its columns.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace ias {
namespace dev {

constexpr int WAVE = 64;
constexpr int32_t EMPTY_KEY = -1;

// a read of the expansion (tcol): streamed once per pass
__device__ __forceinline__ int32_t ld_stream(const int32_t *p) {
    return __builtin_nontemporal_load(p);
}

// Timing-only builds (-DIAS_TIMING=1, tools/timing.sh; never shipped): per-
// phase wall-clock cycles of the row kernels, summed per (kind, log2 TEAM)
// slot into g_timing and read back by ias_debug_timing().
#ifndef IAS_TIMING
#define IAS_TIMING 0
#endif
constexpr int TIMING_SLOTS = 32, TIMING_PHASES = 8, TIMING_REPS = 32;
#if IAS_TIMING
// replicated per workgroup group so the flush atomics do not contend
__device__ unsigned long long g_timing[TIMING_REPS * TIMING_SLOTS * (TIMING_PHASES + 1)];
#endif
struct Timer {
#if IAS_TIMING
    unsigned long long acc[TIMING_PHASES] = {};
    unsigned long long last = 0;
    unsigned long long cnt = 0;   // units timed (0: one per flush)
    __device__ __forceinline__ void start() { last = wall_clock64(); }
    __device__ __forceinline__ void done() { ++cnt; }
    __device__ __forceinline__ void mark(int i) {
        const unsigned long long t = wall_clock64();
        acc[i] += t - last;
        last = t;
    }
    // sampled: one workgroup in 8 reports
    __device__ __forceinline__ void flush(int slot, bool leader) {
        if (!leader || (blockIdx.x & 7) != 0) return;
        unsigned long long *g =
            g_timing + ((blockIdx.x >> 3) % TIMING_REPS) * (TIMING_SLOTS * (TIMING_PHASES + 1)) +
            slot * (TIMING_PHASES + 1);
        for (int i = 0; i < TIMING_PHASES; ++i) atomicAdd(&g[i], acc[i]);
        atomicAdd(&g[TIMING_PHASES], cnt ? cnt : 1ull);
    }
#else
    __device__ __forceinline__ void start() {}
    __device__ __forceinline__ void done() {}
    __device__ __forceinline__ void mark(int) {}
    __device__ __forceinline__ void flush(int, bool) {}
#endif
};
__host__ __device__ constexpr int ilog2(int x) { return x <= 1 ? 0 : 1 + ilog2(x / 2); }

// ---------------------------------------------------------------- row views
// An operand's rows: CSR (ptr != nullptr) or ELL (start = i*stride, len[i]).
struct Rows {
    const int64_t *ptr;
    const int32_t *len;
    int64_t stride;
    const int32_t *col;
    const double *val;
    __device__ __forceinline__ void row(int64_t i, int64_t &s, int32_t &n) const {
        if (ptr) {
            s = ptr[i];
            n = (int32_t)(ptr[i + 1] - s);
        } else {
            s = i * stride;
            n = len[i];
        }
    }
    __device__ __forceinline__ int64_t base() const { return ptr ? ptr[0] : 0; }
};

// Expanded A, written once by the analysis pass: for every stored A entry
// q (relative to the first entry of A), the extent of the B row it selects
// and its value.  The row kernels read only these arrays and B, so a row
// costs one dependent gather (B) after its work item instead of three
// (A row pointer, A column, B row pointer).
struct AxView {
    const int64_t *bstart;
    const int32_t *blen;
    const double *aval;
};
struct AxOut {
    int64_t *bstart;
    int32_t *blen;
    double *aval;
    int32_t *wide_b;   // nullable: set to 1 when a selected B row ends beyond 2^30 entries
    int32_t *wide_v;   // nullable: set to 1 when one ends beyond 2^29 (k_num2's 32-bit value offsets)
};

// A row of a bin list: its first expanded-A entry and entry count.
struct RowRef {
    int64_t q0;
    int32_t row;
    int32_t n;
};
// One hash partition of a partitioned row.
struct PartItem {
    RowRef ref;
    uint32_t part;
    uint32_t nparts;
};
// The products of one partition, bucketed: pairs (column, product index) at
// bucket[start .. start + len); len < 0: not bucketed (the partition rescans
// the row's expansion).
struct PartSpan {
    int64_t start;
    int32_t len;
    int32_t pad;
};

// Where row i of C goes: CSR/COO (start = ptr[i]) or ELL (start = i*stride);
// len[i] = nnz of row i (from the symbolic pass).
struct Out {
    const int64_t *ptr;   // C row pointer (CSR/COO); nullptr for ELL
    int64_t stride;       // ELL width
    int32_t *col;
    double *val;
    int32_t *row_idx;     // COO: row index of every entry (nullable; filled by k_fill_rows)
    int32_t order;        // 0: reverse first-touch, 1: forward first-touch
    int32_t first_assign; // 1: first product assigned (COO); 0: 0.0 + product
    const int32_t *len;   // nnz per row (set by the engine)
    __device__ __forceinline__ int64_t start(int64_t i) const { return ptr ? ptr[i] : i * stride; }
};

// First-touch bitmap of the partitioned rows (written by the symbolic pass):
// row r owns words [off[r], off[r] + ceil(P/32)) of `bits`, and `pref` holds
// the exclusive prefix popcount of those words.
struct Bitmap {
    uint32_t *bits;
    uint32_t *pref;
    const int64_t *off;   // per row, in words
};

// ---------------------------------------------------------------- wave scan
// Inclusive prefix sum over the 64 lanes of a wave with DPP moves (no LDS
// round trip per step, unlike __shfl_up = ds_bpermute): row_shr 1/2/4/8 scan
// each 16-lane row, row_bcast:15 / row_bcast:31 carry across rows (GFX9 DPP,
// gfx950).  Inactive source lanes read as 0 (old = 0).
__device__ __forceinline__ int wave_incl_sum(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false);   // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false);   // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);   // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);   // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);   // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);   // row_bcast:31 -> rows 2, 3
    return x;
}

// ---------------------------------------------------------------- team ops
// A team is TEAM consecutive lanes.  TEAM <= 64: several teams per wave,
// synchronised at wave level.  TEAM > 64: exactly one team per workgroup.
template <int TEAM>
struct Team {
    static constexpr bool MULTI = TEAM > WAVE;
    static constexpr int NWAVES = MULTI ? TEAM / WAVE : 1;

    __device__ __forceinline__ static int lane() {
        return MULTI ? (int)threadIdx.x : (int)(threadIdx.x & (TEAM - 1));
    }
    __device__ __forceinline__ static uint64_t mask() {
        if constexpr (TEAM >= WAVE) {
            return ~0ull;
        } else {
            const int base = (int)(__lane_id() & ~(TEAM - 1));
            return ((1ull << TEAM) - 1ull) << base;
        }
    }
    __device__ __forceinline__ static void sync() {
        if constexpr (MULTI) {
            __syncthreads();
        } else {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
    // Exclusive prefix sum of v over the team; `total` = team sum.
    __device__ __forceinline__ static int excl_sum(int v, int &total, int *scratch) {
        constexpr int W = MULTI ? WAVE : TEAM;
        const int l = (int)(threadIdx.x & (W - 1));
        int x = v;
        if constexpr (W == WAVE) {
            x = wave_incl_sum(v);
        } else {
#pragma unroll
            for (int d = 1; d < W; d <<= 1) {
                const int t = __shfl_up(x, d, W);
                if (l >= d) x += t;
            }
        }
        if constexpr (!MULTI) {
            total = W == WAVE ? __builtin_amdgcn_readlane(x, WAVE - 1) : __shfl(x, W - 1, W);
            return x - v;
        } else {
            const int w = threadIdx.x / WAVE;
            if (l == WAVE - 1) scratch[w] = x;
            __syncthreads();
            int before = 0, tot = 0;
#pragma unroll
            for (int i = 0; i < NWAVES; ++i) {
                const int c = scratch[i];
                before += (i < w) ? c : 0;
                tot += c;
            }
            __syncthreads();
            total = tot;
            return before + x - v;
        }
    }
    // Exclusive count of K flags per lane in item order (item id = k*TEAM +
    // lane, k-major); rank[k] gets each item's count, returns the team total.
    template <int K>
    __device__ __forceinline__ static int excl_count_items(const bool (&f)[K], int (&rank)[K],
                                                           int *scratch) {
        const uint64_t lt = (1ull << __lane_id()) - 1ull;
        uint64_t b[K];
#pragma unroll
        for (int k = 0; k < K; ++k) b[k] = __ballot(f[k]);
        if constexpr (!MULTI) {
            const uint64_t m = mask();
            int run = 0;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                rank[k] = run + __popcll(b[k] & m & lt);
                run += __popcll(b[k] & m);
            }
            return run;
        } else {
            const int w = threadIdx.x / WAVE;
            if ((threadIdx.x & (WAVE - 1)) == 0) {
#pragma unroll
                for (int k = 0; k < K; ++k) scratch[w * K + k] = __popcll(b[k]);
            }
            __syncthreads();
            int run = 0;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                int before = 0, tot = 0;
#pragma unroll
                for (int i = 0; i < NWAVES; ++i) {
                    const int c = scratch[i * K + k];
                    before += (i < w) ? c : 0;
                    tot += c;
                }
                rank[k] = run + before + __popcll(b[k] & lt);
                run += tot;
            }
            __syncthreads();
            return run;
        }
    }
    __device__ __forceinline__ static bool any(bool p) {
        if constexpr (MULTI) return __syncthreads_or(p) != 0;
        else return (__ballot(p) & mask()) != 0ull;
    }
    __device__ __forceinline__ static int sum(int v, int *scratch) {
        int total;
        excl_sum(v, total, scratch);
        return total;
    }
};

// first-touch bits of a partitioned row staged in LDS by each partition's
// workgroup (positions < 32 * LBITS_WORDS; later ones go to global atomics)
constexpr int LBITS_WORDS = 2048;

// table slot hash (multiply-shift onto [0, size), any size) and an
// independent partition hash
__device__ __forceinline__ uint32_t slot_hash(int32_t c, uint32_t size) {
    return (uint32_t)(((uint64_t)((uint32_t)c * 0x9E3779B1u) * size) >> 32);
}
__device__ __forceinline__ uint32_t part_of(int32_t c, uint32_t nparts) {
    const uint32_t h = ((uint32_t)c * 0x85EBCA6Bu) ^ ((uint32_t)c >> 16);
    return (uint32_t)(((uint64_t)(h * 0xC2B2AE35u) * nparts) >> 32);
}

// ---------------------------------------------------------------- tables
// Keys (+ optional first-touch position) table of the symbolic pass.
// insert returns 1 when it created the key, 0 when present, -1 when the
// table is full (only possible for hash partitions; the caller flags it).
template <bool FT>
struct SymTable {
    int32_t *key;
    uint32_t *minp;   // FT only
    uint32_t size;
    __device__ __forceinline__ int insert(int32_t c, uint32_t p) const {
        uint32_t s = slot_hash(c, size);
        for (uint32_t probe = 0; probe < size; ++probe) {
            const int32_t prev = atomicCAS(&key[s], EMPTY_KEY, c);
            if (prev == EMPTY_KEY || prev == c) {
                if constexpr (FT) atomicMin(&minp[s], p);
                return prev == EMPTY_KEY ? 1 : 0;
            }
            s = (s + 1u == size) ? 0u : s + 1u;
        }
        return -1;
    }
    // FT tables: slot of c (created when absent), first-touch position kept
    // as the min product index; -1 when full.
    __device__ __forceinline__ int insert_slot(int32_t c, uint32_t p, bool &made) const {
        uint32_t s = slot_hash(c, size);
        for (uint32_t probe = 0; probe < size; ++probe) {
            const int32_t prev = atomicCAS(&key[s], EMPTY_KEY, c);
            if (prev == EMPTY_KEY || prev == c) {
                atomicMin(&minp[s], p);
                made = prev == EMPTY_KEY;
                return (int)s;
            }
            s = (s + 1u == size) ? 0u : s + 1u;
        }
        made = false;
        return -1;
    }
};

// Numeric table, LDS flavour: meta = rank << 13 | owner (owner 0x1FFF = none,
// rank 0x7FFFF = not yet discovered).  Global flavour (rows beyond 2^19 nnz):
// 64-bit meta, rank << 32 | owner.
template <bool WIDE>
struct MetaTraits;
template <>
struct MetaTraits<false> {
    using T = uint32_t;
    static constexpr int SHIFT = 13;
    static constexpr T OWN = 0x1FFFu;
    static constexpr T RANK_NONE = 0x7FFFFu;
    static constexpr T INIT = 0xFFFFFFFFu;
};
template <>
struct MetaTraits<true> {
    using T = unsigned long long;
    static constexpr int SHIFT = 32;
    static constexpr T OWN = 0xFFFFFFFFull;
    static constexpr T RANK_NONE = 0xFFFFFFFFull;
    static constexpr T INIT = ~0ull;
};

template <bool WIDE>
struct NumTable {
    using MT = MetaTraits<WIDE>;
    using M = typename MT::T;
    int32_t *key;
    M *meta;
    double *val;
    uint32_t size;

    __device__ __forceinline__ int find_or_insert(int32_t c) const {
        uint32_t s = slot_hash(c, size);
        for (uint32_t probe = 0; probe < size; ++probe) {
            const int32_t prev = atomicCAS(&key[s], EMPTY_KEY, c);
            if (prev == EMPTY_KEY || prev == c) return (int)s;
            s = (s + 1u == size) ? 0u : s + 1u;
        }
        return -1;
    }
    __device__ __forceinline__ void claim(uint32_t s, uint32_t id) const {
        const M cur = __hip_atomic_load(&meta[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        atomicMin(&meta[s], (cur & ~MT::OWN) | (M)id);
    }
    __device__ __forceinline__ M load(uint32_t s) const {
        return __hip_atomic_load(&meta[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
};

// ---------------------------------------------------------------- segment
// Up to SEG A entries of the row being expanded, staged in LDS: bstart =
// start of the B row, aval = A value, pref = exclusive prefix of B row lengths.
template <int SEG, bool NUMERIC>
struct Seg {
    int64_t bstart[SEG];
    int32_t pref[SEG];
    double aval[NUMERIC ? SEG : 1];
};

// Largest jj in [0, n) with pref[jj] <= p (pref[0] == 0 <= p).
__device__ __forceinline__ int seg_find(const int32_t *pref, int n, int p) {
    int lo = 0, hi = n;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (pref[mid] <= p) lo = mid;
        else hi = mid;
    }
    return lo;
}

// Stage entries [seg0, seg0 + SEG) of the row's expanded A; returns the
// products of the segment (team-uniform).  Requires SEG <= TEAM.
template <int TEAM, int SEG, bool NUMERIC>
__device__ __forceinline__ int load_segment(const AxView &ax, int64_t q0, int32_t an, int32_t seg0,
                                            Seg<SEG, NUMERIC> &sg, int *scratch, int &nseg) {
    static_assert(SEG <= TEAM, "segment loads one entry per lane");
    using TM = Team<TEAM>;
    const int lane = TM::lane();
    nseg = min(SEG, an - seg0);
    int blen = 0;
    if (lane < nseg) {
        const int64_t q = q0 + seg0 + lane;
        sg.bstart[lane] = ax.bstart[q];
        if constexpr (NUMERIC) sg.aval[lane] = ax.aval[q];
        blen = ax.blen[q];
    }
    int total;
    const int ex = TM::excl_sum(blen, total, scratch);
    if (lane < nseg) sg.pref[lane] = ex;
    TM::sync();
    return total;
}

// ---------------------------------------------------------------- expansion
// The product columns of every row, materialised once in product order:
// tcol[P_off[row] + p] = column of product p of the row (P_off = exclusive
// prefix of products per row = axp at the row's first A entry).  The row
// kernels of the symbolic pass then read a row's products as one contiguous
// run instead of re-deriving and gathering them.

// ---------------------------------------------------------------- symbolic
// K inserts per lane into a keys + first-touch table, one CAS round trip at a
// time (measured: issuing the K first-probe CASes back to back was slower,
// K3' symbolic 8.7 vs 7.6 ms — several returning LDS atomics in flight per
// wave cost more than they hide).  minp
// keeps the smallest product per column (atomicMin without return).
// slot[k] = the column's slot or -1 (none, or table full: *full set).
template <int K>
__device__ __forceinline__ void insert_k(int32_t *key, uint32_t *minp, uint32_t S, const int32_t (&c)[K],
                                         const uint32_t (&p)[K], bool (&use)[K], int (&slot)[K],
                                         int &created, bool &full) {
    // Bucketed probing: the home position is a 16-byte bucket of 4 slots,
    // read with one LDS load; the column is found in it, or CASed into its
    // first empty slot, or the probe moves to the next bucket.  Linear
    // probing over single slots left long probe tails at load 1/2..2/3, and
    // a wave waits for its slowest lane (S is a multiple of 4).
    const uint32_t nb = S >> 2;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        slot[k] = -1;
        if (!use[k]) continue;
        uint32_t b = slot_hash(c[k], nb);
        for (uint32_t probe = 0; probe < S; ++probe) {
            const int4 q = ((const int4 *)key)[b];
            int hit = -1, empty = -1;
            if (q.w == c[k]) hit = 3;
            if (q.z == c[k]) hit = 2;
            if (q.y == c[k]) hit = 1;
            if (q.x == c[k]) hit = 0;
            if (q.w == EMPTY_KEY) empty = 3;
            if (q.z == EMPTY_KEY) empty = 2;
            if (q.y == EMPTY_KEY) empty = 1;
            if (q.x == EMPTY_KEY) empty = 0;
            if (hit >= 0) {
                slot[k] = (int)(4 * b + hit);
                break;
            }
            if (empty < 0) {
                b = (b + 1u == nb) ? 0u : b + 1u;
                continue;
            }
            const int32_t v = atomicCAS(&key[4 * b + empty], EMPTY_KEY, c[k]);
            if (v == EMPTY_KEY || v == c[k]) {
                created += v == EMPTY_KEY ? 1 : 0;
                slot[k] = (int)(4 * b + empty);
                break;
            }
            // another column took that slot: re-read the same bucket
        }
        if (slot[k] >= 0) atomicMin(&minp[slot[k]], p[k]);
        else full = true;
    }
}

// One team counts the distinct columns of one hash partition of a row whose
// products are tcol[ref.q0 .. ref.q0 + ref.n), with the first-touch position
// of every column published as bits of the row's bitmap.  Duplicates (a
// product whose column was touched first by an earlier product — all of a
// column's products fall in one partition) are appended unordered as
// (product, first touch) pairs to the row's list `pairs` through the row's
// counter *dcnt (one atomic per wave and step); entries beyond `cap` are
// counted but not stored.  Returns the team's count; *overflow is set when
// the table filled up.
template <int TEAM, int K>
__device__ __forceinline__ int32_t symbolic_part_row(const int32_t *tcol, const RowRef &ref,
                                                     const SymTable<true> &table, uint32_t part,
                                                     uint32_t nparts, int *scratch, uint32_t *lbits,
                                                     uint32_t *gbits, uint2 *pairs, int32_t *dcnt,
                                                     uint32_t cap, int *overflow) {
    using TM = Team<TEAM>;
    const int lane = TM::lane();
    const uint32_t S = table.size;
    for (uint32_t s = lane; s < S; s += TEAM) {
        table.key[s] = EMPTY_KEY;
        table.minp[s] = 0xFFFFFFFFu;
    }
    TM::sync();
    const int32_t P = ref.n;
    const int32_t *pc = tcol + ref.q0;
    int created = 0;
    bool full = false;
    for (int p0 = 0; p0 < P; p0 += TEAM * K) {
        int32_t c[K];
        uint32_t pp[K];
        bool use[K];
        int slot[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int p = p0 + k * TEAM + lane;
            c[k] = p < P ? ld_stream(pc + p) : EMPTY_KEY;
            pp[k] = (uint32_t)p;
        }
#pragma unroll
        for (int k = 0; k < K; ++k) use[k] = c[k] != EMPTY_KEY && part_of(c[k], nparts) == part;
        insert_k<K>(table.key, table.minp, S, c, pp, use, slot, created, full);
        if (pairs) {
            TM::sync();   // first touches of this step's columns are final
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const uint32_t m = slot[k] >= 0 ? table.minp[slot[k]] : 0u;
                const bool dup = slot[k] >= 0 && m != pp[k];
                const uint64_t b = __ballot(dup);
                if (b == 0ull) continue;
                int base = 0;
                if ((__lane_id()) == (uint32_t)__builtin_ctzll(b)) base = atomicAdd(dcnt, __popcll(b));
                base = __shfl(base, __builtin_ctzll(b));
                const uint32_t i = (uint32_t)base + (uint32_t)__popcll(b & ((1ull << __lane_id()) - 1ull));
                if (dup && i < cap) pairs[i] = make_uint2(pp[k], m);
            }
        }
    }
    TM::sync();
    for (uint32_t s = lane; s < S; s += TEAM)
        if (table.key[s] != EMPTY_KEY) {
            const uint32_t p = table.minp[s];
            if ((p >> 5) < (uint32_t)LBITS_WORDS) atomicOr(&lbits[p >> 5], 1u << (p & 31));   // LDS staging
            else atomicOr(&gbits[p >> 5], 1u << (p & 31));
        }
    TM::sync();
    if (full) atomicOr(overflow, 1);
    return TM::sum(created, scratch);
}

// Slot of a column known to be in a table filled by insert_k's bucketed
// probing (the column sits in its home bucket or in one of the full buckets
// after it).
__device__ __forceinline__ int table_find(const int32_t *key, uint32_t S, int32_t c) {
    const uint32_t nb = S >> 2;
    uint32_t b = slot_hash(c, nb);
    for (uint32_t probe = 0; probe < nb; ++probe) {
        const int4 q = ((const int4 *)key)[b];
        if (q.x == c) return (int)(4 * b);
        if (q.y == c) return (int)(4 * b + 1);
        if (q.z == c) return (int)(4 * b + 2);
        if (q.w == c) return (int)(4 * b + 3);
        b = (b + 1u == nb) ? 0u : b + 1u;
    }
    return -1;
}

// symbolic_part_row over a bucketed partition: the pairs (column, product)
// of this partition only, in no particular order — so first touches are final
// only after every insert, and the duplicates are listed in a second pass.
template <int TEAM, int K>
__device__ __forceinline__ int32_t symbolic_bucket_row(const uint2 *bk, int32_t bn, const SymTable<true> &table,
                                                       int *scratch, uint32_t *lbits, uint32_t *gbits,
                                                       uint2 *pairs, int32_t *dcnt, uint32_t cap, int *overflow,
                                                       Timer &tm) {
    using TM = Team<TEAM>;
    const int lane = TM::lane();
    const uint32_t S = table.size;
    {
        const uint4 ek = make_uint4((uint32_t)EMPTY_KEY, (uint32_t)EMPTY_KEY, (uint32_t)EMPTY_KEY,
                                    (uint32_t)EMPTY_KEY);
        const uint4 em = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
        for (uint32_t s = lane; s < S / 4; s += TEAM) {
            ((uint4 *)table.key)[s] = ek;
            ((uint4 *)table.minp)[s] = em;
        }
    }
    if (lane == 0) scratch[60] = 0;   // duplicate counter of the one-step path
    TM::sync();
    tm.mark(1);
    int created = 0;
    bool full = false;
    auto first_touch = [&](uint32_t p) {
        if ((p >> 5) < (uint32_t)LBITS_WORDS) atomicOr(&lbits[p >> 5], 1u << (p & 31));   // LDS staging
        else atomicOr(&gbits[p >> 5], 1u << (p & 31));
    };
    // list the duplicates of one wave's items (dup: minp of the column != p)
    auto list_dups = [&](bool dup, uint32_t p, uint32_t m) {
        const uint64_t b = __ballot(dup);
        if (b == 0ull) return;
        int base = 0;
        if ((__lane_id()) == (uint32_t)__builtin_ctzll(b)) base = atomicAdd(dcnt, __popcll(b));
        base = __shfl(base, __builtin_ctzll(b));
        const uint32_t j = (uint32_t)base + (uint32_t)__popcll(b & ((1ull << __lane_id()) - 1ull));
        if (dup && j < cap) pairs[j] = make_uint2(p, m);
    };
    if (bn <= TEAM * K) {
        // one step: the items stay in registers with their slots, so the
        // first-touch bits and the duplicates come from minp[slot] directly
        // (no second read of the bucket, no table search, no slot scan)
        int32_t c[K];
        uint32_t pp[K];
        bool use[K];
        int slot[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int i = k * TEAM + lane;
            use[k] = i < bn;
            const uint2 e = use[k] ? bk[i] : make_uint2((uint32_t)EMPTY_KEY, 0u);
            c[k] = (int32_t)e.x;
            pp[k] = e.y;
        }
        insert_k<K>(table.key, table.minp, S, c, pp, use, slot, created, full);
        tm.mark(2);
        TM::sync();
        tm.mark(3);
        uint32_t m[K];   // all K reads in flight before the atomics
#pragma unroll
        for (int k = 0; k < K; ++k) m[k] = slot[k] >= 0 ? table.minp[slot[k]] : 0u;
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (slot[k] >= 0 && m[k] == pp[k]) first_touch(pp[k]);
        // duplicates: ranks from an LDS counter, then one global atomic per
        // workgroup for the row-wide base (a returning global atomic per wave
        // and item serialised this pass)
        int jl[K];
        const bool listing = pairs && !full;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const bool dup = listing && slot[k] >= 0 && m[k] != pp[k];
            const uint64_t b = __ballot(dup);
            jl[k] = -1;
            if (b == 0ull) continue;
            int base = 0;
            if ((__lane_id()) == (uint32_t)__builtin_ctzll(b)) base = atomicAdd(&scratch[60], __popcll(b));
            base = __shfl(base, __builtin_ctzll(b));
            if (dup) jl[k] = base + __popcll(b & ((1ull << __lane_id()) - 1ull));
        }
        tm.mark(4);
        TM::sync();
        if (lane == 0) scratch[61] = scratch[60] > 0 ? atomicAdd(dcnt, scratch[60]) : 0;
        TM::sync();
        const int gb = scratch[61];
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (jl[k] >= 0 && (uint32_t)(gb + jl[k]) < cap) pairs[gb + jl[k]] = make_uint2(pp[k], m[k]);
        tm.mark(5);
    } else {
        for (int i0 = 0; i0 < bn; i0 += TEAM * K) {
            int32_t c[K];
            uint32_t pp[K];
            bool use[K];
            int slot[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int i = i0 + k * TEAM + lane;
                use[k] = i < bn;
                const uint2 e = use[k] ? bk[i] : make_uint2((uint32_t)EMPTY_KEY, 0u);
                c[k] = (int32_t)e.x;
                pp[k] = e.y;
            }
            insert_k<K>(table.key, table.minp, S, c, pp, use, slot, created, full);
        }
        tm.mark(2);
        TM::sync();
        tm.mark(3);
        if (pairs && !full) {
            for (int i0 = 0; i0 < bn; i0 += TEAM) {
                const int i = i0 + lane;
                bool dup = false;
                uint32_t p = 0, m = 0;
                if (i < bn) {
                    const uint2 e = bk[i];
                    p = e.y;
                    const int s = table_find(table.key, S, (int32_t)e.x);
                    m = table.minp[s];
                    dup = m != p;
                }
                list_dups(dup, p, m);
            }
        }
        tm.mark(4);
        for (uint32_t s = lane; s < S; s += TEAM)
            if (table.key[s] != EMPTY_KEY) first_touch(table.minp[s]);
        TM::sync();
        tm.mark(5);
    }
    if (full) atomicOr(overflow, 1);
    return TM::sum(created, scratch);
}

// ---------------------------------------------------------------- numeric, streaming rows
// The streaming rows' numeric pass is k_num2 (num2_kernels.hpp); a duplicate's
// product is parked at dupval[dup_off[row] + d] (d = duplicates before it in
// the row) for the fix-up kernels below.

// Bitonic sort (ascending) of key[0, n2), n2 a power of two <= CAP, by a team
// of TEAM lanes.  Each stage's compare-exchange pairs are numbered q = 0 ..
// n2/2 - 1 (lower index: q with a zero bit inserted at the stride's
// position), so every lane is busy, and a lane's PP pairs are all read before
// any is compared: one LDS round trip per stage rather than one per pair (the
// per-pair form waits on each read, ~60 us per 4096-key list).
template <int TEAM, int CAP, typename K>
__device__ __forceinline__ void bitonic_lds(K *key, uint32_t n2) {
    using TM = Team<TEAM>;
    constexpr int PP = (CAP / 2 + TEAM - 1) / TEAM;
    const uint32_t lane = (uint32_t)TM::lane(), np = n2 >> 1;
    for (uint32_t k = 2; k <= n2; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            K a[PP], b[PP];
            uint32_t lo[PP];
#pragma unroll
            for (int r = 0; r < PP; ++r) {
                const uint32_t q = (uint32_t)r * TEAM + lane;
                lo[r] = ((q & ~(j - 1)) << 1) | (q & (j - 1));
                if (q < np) {
                    a[r] = key[lo[r]];
                    b[r] = key[lo[r] | j];
                }
            }
#pragma unroll
            for (int r = 0; r < PP; ++r) {
                const uint32_t q = (uint32_t)r * TEAM + lane;
                if (q < np && (a[r] > b[r]) == ((lo[r] & k) == 0)) {
                    key[lo[r]] = b[r];
                    key[lo[r] | j] = a[r];
                }
            }
            TM::sync();
        }
    }
}

// Fix-up of a streaming row with many duplicates (more than one wave's
// list): (first touch, index) keys sorted in LDS (bitonic, nd <= cap2 = a
// power of two), then each run of equal first touches adds its products to
// its entry in product order (sorted by index within the run).  After the
// sort every lane gathers its entries' values (independent loads, one round
// of latency) into the key array's slots, run heads go to a bit mask, and the
// runs are walked in LDS.
template <int TEAM, int CAP>
__device__ __forceinline__ void numeric_fixup_big(int64_t row, const uint32_t *bits, const uint32_t *bpref,
                                                  const int32_t *gdupt, const double *gdupval,
                                                  int32_t ndup, unsigned long long *key, const Out &out) {
    using TM = Team<TEAM>;
    constexpr int PER = CAP / TEAM;
    static_assert(PER * TEAM == CAP && TEAM % WAVE == 0, "whole waves over the key array");
    const int lane = TM::lane();
    uint64_t *head = (uint64_t *)(key + CAP);   // CAP / 64 words
    uint32_t n2 = 1;
    while (n2 < (uint32_t)ndup) n2 <<= 1;
    for (uint32_t i = lane; i < n2; i += TEAM)
        key[i] = i < (uint32_t)ndup ? (((unsigned long long)(uint32_t)gdupt[i] << 32) | i) : ~0ull;
    TM::sync();
    bitonic_lds<TEAM, CAP>(key, n2);
    uint32_t tt[PER];
    double vv[PER];
    bool hd[PER];
#pragma unroll
    for (int r = 0; r < PER; ++r) {
        const uint32_t i = (uint32_t)(r * TEAM + lane);
        const bool in = i < (uint32_t)ndup;
        const unsigned long long kk = in ? key[i] : 0ull;
        tt[r] = (uint32_t)(kk >> 32);
        hd[r] = in && (i == 0 || (uint32_t)(key[i - 1] >> 32) != tt[r]);
        vv[r] = in ? gdupval[(uint32_t)kk] : 0.0;
    }
    TM::sync();   // every key read before the values overwrite them
#pragma unroll
    for (int r = 0; r < PER; ++r) {
        const uint32_t i = (uint32_t)(r * TEAM + lane);
        const uint64_t hb = __ballot(hd[r]);
        if (i < (uint32_t)ndup) key[i] = __builtin_bit_cast(unsigned long long, vv[r]);
        if ((lane & (WAVE - 1)) == 0 && i < n2) head[i >> 6] = hb;
    }
    TM::sync();
    const double *val = (const double *)key;
    const int64_t st = out.start(row);
    const uint32_t nnz = (uint32_t)out.len[row];
#pragma unroll
    for (int r = 0; r < PER; ++r) {
        if (!hd[r]) continue;
        const uint32_t i = (uint32_t)(r * TEAM + lane), t = tt[r];
        const uint32_t rk = bpref[t >> 5] + (uint32_t)__popc(bits[t >> 5] & ((1u << (t & 31)) - 1u));
        const int64_t pos = st + (out.order == 0 ? (int64_t)(nnz - 1u - rk) : (int64_t)rk);
        double v = out.val[pos] + val[i];
        for (uint32_t j = i + 1; j < (uint32_t)ndup && !((head[j >> 6] >> (j & 63)) & 1ull); ++j) v = v + val[j];
        out.val[pos] = v;
    }
}

// The same with the values staged in a second LDS array (16 B per list entry
// in all, few registers): the 256-lane kernels that sit beside the streaming
// pass's waves on a CU.  key: CAP keys, then CAP values, then CAP/64 head words.
template <int TEAM, int CAP>
__device__ __forceinline__ void numeric_fixup_lds(int64_t row, const uint32_t *bits, const uint32_t *bpref,
                                                  const int32_t *gdupt, const double *gdupval,
                                                  int32_t ndup, unsigned long long *key, const Out &out) {
    using TM = Team<TEAM>;
    static_assert(CAP % TEAM == 0 && TEAM % WAVE == 0, "whole waves over the key array");
    const int lane = TM::lane();
    double *val = (double *)(key + CAP);
    uint64_t *head = (uint64_t *)(key + 2 * CAP);
    uint32_t n2 = 1;
    while (n2 < (uint32_t)ndup) n2 <<= 1;
    for (uint32_t i = lane; i < n2; i += TEAM)
        key[i] = i < (uint32_t)ndup ? (((unsigned long long)(uint32_t)gdupt[i] << 32) | i) : ~0ull;
    TM::sync();
    bitonic_lds<TEAM, CAP>(key, n2);
    // run heads and the values in sorted order (the loads of a group of
    // entries issued together)
    constexpr int G = 4;
    for (uint32_t i0 = 0; i0 < n2; i0 += G * TEAM) {
        double v[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const uint32_t i = i0 + g * TEAM + lane;
            const bool in = i < (uint32_t)ndup;
            const unsigned long long kk = in ? key[i] : 0ull;
            const bool hd = in && (i == 0 || (uint32_t)(key[i - 1] >> 32) != (uint32_t)(kk >> 32));
            const uint64_t hb = __ballot(hd);
            if ((lane & (WAVE - 1)) == 0 && i < n2) head[i >> 6] = hb;
            v[g] = in ? gdupval[(uint32_t)kk] : 0.0;
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const uint32_t i = i0 + g * TEAM + lane;
            if (i < (uint32_t)ndup) val[i] = v[g];
        }
    }
    TM::sync();
    const int64_t st = out.start(row);
    const uint32_t nnz = (uint32_t)out.len[row];
    for (uint32_t i = lane; i < (uint32_t)ndup; i += TEAM) {
        if (!((head[i >> 6] >> (i & 63)) & 1ull)) continue;
        const uint32_t t = (uint32_t)(key[i] >> 32);
        const uint32_t rk = bpref[t >> 5] + (uint32_t)__popc(bits[t >> 5] & ((1u << (t & 31)) - 1u));
        const int64_t pos = st + (out.order == 0 ? (int64_t)(nnz - 1u - rk) : (int64_t)rk);
        double v = out.val[pos] + val[i];
        for (uint32_t j = i + 1; j < (uint32_t)ndup && !((head[j >> 6] >> (j & 63)) & 1ull); ++j) v = v + val[j];
        out.val[pos] = v;
    }
}

// ---------------------------------------------------------------- numeric
// Modes of a numeric row:
//   M_VAL   : whole row in one LDS table with values; ranks from team scans;
//             emission staged through LDS so C is written with coalesced
//             stores (rows with many duplicate products: values stay in LDS).
//   M_WIDE  : as M_VAL with the table in global memory (64-bit meta) and
//             entries stored straight to their final positions.
//   M_DW    : direct write.  The LDS table holds keys and ranks only (8 B per
//             slot); a column's first touch writes (col, 0.0 + p) to its final
//             position in C at once and later products of it accumulate there
//             in product order.  No emission pass.  For rows whose products
//             are mostly distinct columns.
//   M_DWPART: M_DW over hash partition `part` of the row, ranks from the
//             symbolic first-touch bitmap.
enum { M_VAL = 0, M_WIDE = 1, M_DW = 2, M_DWPART = 3 };

template <int TEAM, int K, int SEG, int MODE, int PER>
__device__ __forceinline__ void numeric_row(const AxView &ax, const Rows &B, const RowRef &ref,
                                            const NumTable<MODE == M_WIDE> &t, uint32_t part,
                                            uint32_t nparts, const uint32_t *bits,
                                            const uint32_t *bpref, Seg<SEG, true> &sg,
                                            int *scratch, const Out &out, int *overflow) {
    constexpr bool WIDE = MODE == M_WIDE;
    constexpr bool DW = MODE == M_DW || MODE == M_DWPART;
    constexpr bool PART = MODE == M_DWPART;
    using TM = Team<TEAM>;
    using MT = MetaTraits<WIDE>;
    using M = typename MT::T;
    static_assert((unsigned long long)TEAM * K < (unsigned long long)MT::OWN,
                  "item ids must fit the owner field");
    const int lane = TM::lane();
    const uint32_t S = t.size;
    const int64_t row = ref.row;
    for (uint32_t s = lane; s < S; s += TEAM) {
        t.key[s] = EMPTY_KEY;
        t.meta[s] = MT::INIT;
    }
    // direct-write modes need the row's place in C up front (loads overlap the gathers)
    int64_t o = 0;
    uint32_t nnz = 0;
    if constexpr (DW) {
        if (row >= 0) {
            o = out.start(row);
            nnz = (uint32_t)out.len[row];
        }
    }
    TM::sync();
    const int32_t an = ref.n;
    uint32_t base_rank = 0;
    uint32_t pbase = 0;
    bool full = false;
    for (int32_t seg0 = 0; seg0 < an; seg0 += SEG) {
        int nseg;
        const int P = load_segment<TEAM, SEG, true>(ax, ref.q0, an, seg0, sg, scratch, nseg);
        for (int p0 = 0; p0 < P; p0 += TEAM * K) {
            int slot[K];
            double prod[K];
            bool pend[K];
            int32_t c[K];
            int jj[K];
            int64_t kk[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int p = p0 + k * TEAM + lane;
                pend[k] = p < P;
                if (pend[k]) {
                    jj[k] = seg_find(sg.pref, nseg, p);
                    kk[k] = sg.bstart[jj[k]] + (p - sg.pref[jj[k]]);
                    c[k] = B.col[kk[k]];
                }
            }
            if constexpr (PART) {
#pragma unroll
                for (int k = 0; k < K; ++k) pend[k] = pend[k] && part_of(c[k], nparts) == part;
            }
#pragma unroll
            for (int k = 0; k < K; ++k)
                if (pend[k]) prod[k] = sg.aval[jj[k]] * B.val[kk[k]];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                slot[k] = 0;
                if (pend[k]) {
                    const int s = t.find_or_insert(c[k]);
                    if (s < 0) {
                        full = true;
                        pend[k] = false;
                    } else {
                        slot[k] = s;
                    }
                }
            }
            bool first_round = true;
            while (true) {
#pragma unroll
                for (int k = 0; k < K; ++k)
                    if (pend[k]) t.claim((uint32_t)slot[k], (uint32_t)(k * TEAM + lane));
                TM::sync();
                bool win[K];
                M rank[K];
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const M m = pend[k] ? t.load((uint32_t)slot[k]) : (M)0;
                    win[k] = pend[k] && (m & MT::OWN) == (M)(k * TEAM + lane);
                    rank[k] = m >> MT::SHIFT;
                }
                bool ft[K];
#pragma unroll
                for (int k = 0; k < K; ++k) ft[k] = first_round && win[k] && rank[k] == MT::RANK_NONE;
                if (first_round) {
                    if constexpr (!PART) {
                        int r[K] = {};
                        const int total = TM::template excl_count_items<K>(ft, r, scratch);
#pragma unroll
                        for (int k = 0; k < K; ++k)
                            if (ft[k]) rank[k] = (M)(base_rank + (uint32_t)r[k]);
                        base_rank += (uint32_t)total;
                    } else {
#pragma unroll
                        for (int k = 0; k < K; ++k)
                            if (ft[k]) {
                                const uint32_t p = pbase + (uint32_t)(p0 + k * TEAM + lane);
                                rank[k] = (M)(bpref[p >> 5] + __popc(bits[p >> 5] & ((1u << (p & 31)) - 1u)));
                            }
                    }
                }
#pragma unroll
                for (int k = 0; k < K; ++k)
                    if (win[k]) {
                        if constexpr (DW) {
                            const uint32_t r = (uint32_t)rank[k];
                            const int64_t pos = o + (out.order == 0 ? (int64_t)(nnz - 1u - r) : (int64_t)r);
                            if (ft[k]) {
                                out.col[pos] = c[k];
                                out.val[pos] = out.first_assign ? prod[k] : 0.0 + prod[k];
                            } else {
                                out.val[pos] = out.val[pos] + prod[k];
                            }
                        } else {
                            const double v = ft[k] ? (out.first_assign ? prod[k] : 0.0 + prod[k])
                                                   : t.val[slot[k]] + prod[k];
                            t.val[slot[k]] = v;
                        }
                        t.meta[slot[k]] = (rank[k] << MT::SHIFT) | MT::OWN;
                        pend[k] = false;
                    }
                first_round = false;
                bool any_pend = false;
#pragma unroll
                for (int k = 0; k < K; ++k) any_pend |= pend[k];
                if constexpr (!TM::MULTI) TM::sync();
                if (!TM::any(any_pend)) break;
            }
        }
        pbase += (uint32_t)P;
        TM::sync();
    }
    if (full) atomicOr(overflow, 1);
    if constexpr (DW) return;
    if (row < 0) return;
    if constexpr (WIDE) {
        const int64_t ow = out.start(row);
        const uint32_t n = base_rank;
        for (uint32_t s = lane; s < S; s += TEAM) {
            const int32_t cc = t.key[s];
            if (cc != EMPTY_KEY) {
                const uint32_t r = (uint32_t)(t.meta[s] >> MT::SHIFT);
                const int64_t pos = ow + (out.order == 0 ? (int64_t)(n - 1u - r) : (int64_t)r);
                out.col[pos] = cc;
                out.val[pos] = t.val[s];
            }
        }
    } else {
        // LDS-staged emission: slots -> registers -> (col, val) at their final
        // position in the key/val arrays -> coalesced stores of the row.
        // PER >= ceil(S / TEAM) slots per lane (compile-time, from the kernel).
        const int64_t ow = out.start(row);
        const uint32_t n = base_rank;
        int32_t kc[PER];
        uint32_t kr[PER];
        double kv[PER];
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const uint32_t s = (uint32_t)i * TEAM + lane;
            kc[i] = EMPTY_KEY;
            if (s < S) {
                kc[i] = t.key[s];
                kr[i] = (uint32_t)(t.meta[s] >> MT::SHIFT);
                kv[i] = t.val[s];
            }
        }
        TM::sync();
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            if (kc[i] != EMPTY_KEY) {
                const uint32_t pos = out.order == 0 ? n - 1u - kr[i] : kr[i];
                t.key[pos] = kc[i];
                t.val[pos] = kv[i];
            }
        }
        TM::sync();
        for (uint32_t e = lane; e < n; e += TEAM) {
            __builtin_nontemporal_store(t.key[e], &out.col[ow + e]);
            __builtin_nontemporal_store(t.val[e], &out.val[ow + e]);
        }
    }
}

}  // namespace dev
}  // namespace ias
