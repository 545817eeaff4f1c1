// spgemm_kernels.hpp — gfx950 device code of the row-wise SpGEMM hot path.
//
// Algorithm (Gustavson row-wise, C(i,:) = sum_j A(i,j) * B(j,:)), restating
// CSR_MUL_CSR (IA-SPGEMM-CPU_release/detail/csr/common_csr.h:85-193) so that
// the output is value-for-value identical to it:
//   * pass 1 (symbolic): distinct output columns per row, counted in a
//     per-row open-addressing hash table (keys only) held in LDS;
//   * pass 2 (numeric): the same hash, now carrying a value and the
//     first-touch ("discovery") rank of every column.  Products of a row are
//     processed in the reference's order p = 0..P-1 (A entries in row order,
//     then B entries in row order), P consecutive products per step, one per
//     lane.  Lanes whose products hit the same column inside a step are
//     serialised in lane order (owner = atomicMin), so every sum is formed as
//     the reference forms it: s = 0.0 + p0, s = s + p1, ... (no FMA: the file
//     is compiled with -ffp-contract=off).  A column's rank is the number of
//     distinct columns discovered before it; it is placed at nnz-1-rank
//     (reverse first-touch, the reference's linked-list order) or at rank
//     (forward first-touch, COO_MUL_COO's order).
// Rows are binned by work (products for pass 1, nnz for pass 2); each bin has
// a team size (32..1024 lanes) and an LDS table size; rows beyond the LDS
// capacity use the same code on a per-row table in global memory.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace ias {
namespace dev {

constexpr int WAVE = 64;
constexpr int32_t EMPTY_KEY = -1;

// ---------------------------------------------------------------- row views
// A "rows" operand: CSR (ptr != nullptr) or ELL (start = i*stride, len[i]).
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
};

// Where row i of C goes: CSR/COO (start = ptr[i]) or ELL (start = i*stride).
struct Out {
    const int64_t *ptr;   // C row pointer (CSR/COO); nullptr for ELL
    int64_t stride;       // ELL width
    int32_t *col;
    double *val;
    int32_t *row_idx;     // COO: row index of every entry (nullable)
    int32_t order;        // 0: reverse first-touch, 1: forward first-touch
    int32_t first_assign; // 1: first product assigned (COO); 0: 0.0 + product
    __device__ __forceinline__ int64_t start(int64_t i) const { return ptr ? ptr[i] : i * stride; }
};

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
    // Exclusive count of `flag` over the team in lane order; `total` = team count.
    __device__ __forceinline__ static int excl_count(bool flag, int &total, int *scratch) {
        const uint64_t b = __ballot(flag);
        const uint64_t lt = (1ull << __lane_id()) - 1ull;
        if constexpr (!MULTI) {
            const uint64_t m = b & mask();
            total = __popcll(m);
            return __popcll(m & lt);
        } else {
            const int w = threadIdx.x / WAVE;
            if ((threadIdx.x & (WAVE - 1)) == 0) scratch[w] = __popcll(b);
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
            return before + __popcll(b & lt);
        }
    }
    // Exclusive prefix sum of v over the team; `total` = team sum.
    __device__ __forceinline__ static int excl_sum(int v, int &total, int *scratch) {
        constexpr int W = MULTI ? WAVE : TEAM;
        const int l = (int)(threadIdx.x & (W - 1));
        int x = v;
#pragma unroll
        for (int d = 1; d < W; d <<= 1) {
            const int t = __shfl_up(x, d, W);
            if (l >= d) x += t;
        }
        if constexpr (!MULTI) {
            total = __shfl(x, W - 1, W);
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

__device__ __forceinline__ uint32_t hash_col(int32_t c) { return (uint32_t)c * 0x9E3779B1u; }

// ---------------------------------------------------------------- tables
// Keys-only table (symbolic).  `log2s` is the table's log2 size.
struct KeyTable {
    int32_t *key;
    uint32_t log2s;
    __device__ __forceinline__ uint32_t first(int32_t c) const {
        return log2s ? (hash_col(c) >> (32u - log2s)) : 0u;
    }
    // Returns true when this call inserted the key.
    __device__ __forceinline__ bool insert(int32_t c) const {
        const uint32_t m = (1u << log2s) - 1u;
        uint32_t s = first(c);
        while (true) {
            const int32_t prev = atomicCAS(&key[s], EMPTY_KEY, c);
            if (prev == EMPTY_KEY) return true;
            if (prev == c) return false;
            s = (s + 1u) & m;
        }
    }
};

// Numeric table, LDS flavour: meta = rank << 12 | owner (owner 0xFFF = none,
// rank 0xFFFFF = not yet discovered).  Global flavour: 64-bit meta, rank << 32 | owner.
template <bool WIDE>
struct MetaTraits;
template <>
struct MetaTraits<false> {
    using T = uint32_t;
    static constexpr int SHIFT = 12;
    static constexpr T OWN = 0xFFFu;
    static constexpr T RANK_NONE = 0xFFFFFu;
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
    uint32_t log2s;

    __device__ __forceinline__ uint32_t find_or_insert(int32_t c) const {
        const uint32_t m = (1u << log2s) - 1u;
        uint32_t s = log2s ? (hash_col(c) >> (32u - log2s)) : 0u;
        while (true) {
            const int32_t prev = atomicCAS(&key[s], EMPTY_KEY, c);
            if (prev == EMPTY_KEY || prev == c) return s;
            s = (s + 1u) & m;
        }
    }
    __device__ __forceinline__ void claim(uint32_t s, int lane) const {
        const M cur = __hip_atomic_load(&meta[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        atomicMin(&meta[s], (cur & ~MT::OWN) | (M)lane);
    }
    __device__ __forceinline__ M load(uint32_t s) const {
        return __hip_atomic_load(&meta[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
};

// ---------------------------------------------------------------- segment
// The A entries of the row currently being expanded, staged in LDS:
// bstart = start of B row, aval = A value, pref = exclusive prefix of B row lengths.
template <int TEAM, bool NUMERIC>
struct Seg {
    int64_t bstart[TEAM];
    int32_t pref[TEAM];
    double aval[NUMERIC ? TEAM : 1];
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

// Load segment [seg0, seg0+TEAM) of A row (as, an) into LDS; returns the
// number of products of the segment (team-uniform).
template <int TEAM, bool NUMERIC>
__device__ __forceinline__ int load_segment(const Rows &A, const Rows &B, int64_t as, int32_t an,
                                            int32_t seg0, Seg<TEAM, NUMERIC> &sg, int *scratch,
                                            int &nseg) {
    using TM = Team<TEAM>;
    const int lane = TM::lane();
    nseg = min(TEAM, an - seg0);
    int blen = 0;
    if (lane < nseg) {
        const int64_t e = as + seg0 + lane;
        const int32_t j = A.col[e];
        int64_t bs;
        int32_t bn;
        B.row(j, bs, bn);
        sg.bstart[lane] = bs;
        if constexpr (NUMERIC) sg.aval[lane] = A.val[e];
        blen = bn;
    }
    int total;
    const int ex = TM::excl_sum(blen, total, scratch);
    if (lane < nseg) sg.pref[lane] = ex;
    TM::sync();
    return total;
}

// ---------------------------------------------------------------- symbolic
// One team counts the distinct columns of one row into `table`.
template <int TEAM>
__device__ __forceinline__ int32_t symbolic_row(const Rows &A, const Rows &B, int64_t row,
                                                const KeyTable &table, Seg<TEAM, false> &sg,
                                                int *scratch) {
    using TM = Team<TEAM>;
    const int lane = TM::lane();
    const uint32_t S = 1u << table.log2s;
    for (uint32_t s = lane; s < S; s += TEAM) table.key[s] = EMPTY_KEY;
    TM::sync();
    int64_t as = 0;
    int32_t an = 0;
    if (row >= 0) A.row(row, as, an);
    int created = 0;
    for (int32_t seg0 = 0; seg0 < an; seg0 += TEAM) {
        int nseg;
        const int P = load_segment<TEAM, false>(A, B, as, an, seg0, sg, scratch, nseg);
        for (int p0 = 0; p0 < P; p0 += TEAM) {
            const int p = p0 + lane;
            if (p < P) {
                const int jj = seg_find(sg.pref, nseg, p);
                const int64_t kk = sg.bstart[jj] + (p - sg.pref[jj]);
                created += table.insert(B.col[kk]) ? 1 : 0;
            }
        }
        TM::sync();
    }
    return TM::sum(created, scratch);
}

// ---------------------------------------------------------------- numeric
template <int TEAM, bool WIDE>
__device__ __forceinline__ void numeric_row(const Rows &A, const Rows &B, int64_t row,
                                            const NumTable<WIDE> &t, Seg<TEAM, true> &sg,
                                            int *scratch, const Out &out) {
    using TM = Team<TEAM>;
    using MT = MetaTraits<WIDE>;
    using M = typename MT::T;
    const int lane = TM::lane();
    const uint32_t S = 1u << t.log2s;
    for (uint32_t s = lane; s < S; s += TEAM) {
        t.key[s] = EMPTY_KEY;
        t.meta[s] = MT::INIT;
    }
    TM::sync();
    int64_t as = 0;
    int32_t an = 0;
    if (row >= 0) A.row(row, as, an);
    uint32_t base_rank = 0;
    for (int32_t seg0 = 0; seg0 < an; seg0 += TEAM) {
        int nseg;
        const int P = load_segment<TEAM, true>(A, B, as, an, seg0, sg, scratch, nseg);
        for (int p0 = 0; p0 < P; p0 += TEAM) {
            const int p = p0 + lane;
            bool pending = p < P;
            uint32_t slot = 0;
            double prod = 0.0;
            if (pending) {
                const int jj = seg_find(sg.pref, nseg, p);
                const int64_t kk = sg.bstart[jj] + (p - sg.pref[jj]);
                const int32_t c = B.col[kk];
                prod = sg.aval[jj] * B.val[kk];
                slot = t.find_or_insert(c);
            }
            bool first_round = true;
            while (true) {
                if (pending) t.claim(slot, lane);
                TM::sync();
                M m = pending ? t.load(slot) : (M)0;
                const bool win = pending && ((m & MT::OWN) == (M)lane);
                M rank = m >> MT::SHIFT;
                if (first_round) {
                    const bool ft = win && rank == MT::RANK_NONE;
                    int total;
                    const int r = TM::excl_count(ft, total, scratch);
                    if (ft) rank = (M)(base_rank + (uint32_t)r);
                    base_rank += (uint32_t)total;
                    if (win) {
                        const double v = ft ? (out.first_assign ? prod : 0.0 + prod)
                                            : t.val[slot] + prod;
                        t.val[slot] = v;
                    }
                } else if (win) {
                    t.val[slot] = t.val[slot] + prod;
                }
                if (win) {
                    t.meta[slot] = (rank << MT::SHIFT) | MT::OWN;
                    pending = false;
                }
                first_round = false;
                if constexpr (!TM::MULTI) TM::sync();
                if (!TM::any(pending)) break;
            }
        }
        TM::sync();
    }
    if (row < 0) return;
    // emit
    const int64_t o = out.start(row);
    const uint32_t nnz = base_rank;
    for (uint32_t s = lane; s < S; s += TEAM) {
        const int32_t c = t.key[s];
        if (c != EMPTY_KEY) {
            const uint32_t r = (uint32_t)(t.meta[s] >> MT::SHIFT);
            const int64_t pos = o + (out.order == 0 ? (int64_t)(nnz - 1u - r) : (int64_t)r);
            out.col[pos] = c;
            out.val[pos] = t.val[s];
            if (out.row_idx) out.row_idx[pos] = (int32_t)row;
        }
    }
}

}  // namespace dev
}  // namespace ias
