// onepass_kernels.hpp — single-pass SpGEMM over row chunks (gfx950).
//
// One launch does, per chunk of consecutive rows, what the two-phase engine
// does in a symbolic pass, a scan and a numeric pass:
//   1. gather the chunk's products (B column + A·B value) into registers,
//      product p of the chunk = p-th product of its rows in the reference's
//      order (A entries in row order, then B entries in row order);
//   2. insert every product into its row's region of one LDS hash table of
//      64-bit slots (column << 32 | first product index): CAS on an empty
//      slot, atomicMin on a slot already holding the column, so each slot
//      ends with the column's first touch (CSR_MUL_CSR's discovery order,
//      IA-SPGEMM-CPU_release/detail/csr/common_csr.h:156-170);
//   3. a ballot per wave and step gives the chunk's first-touch bitmap; its
//      prefix counts give nnz per row and every column's discovery rank;
//   4. the chunk's nnz is published at once (decoupled look-back over chunks
//      taken in row order from a ticket counter), so C's row pointer and the
//      chunk's offset in C come out of the same launch;
//   5. first touches park (column, 0.0 + a·b) in LDS at their output slot
//      (reverse first-touch = the reference's linked-list order, or forward
//      for COO_MUL_COO), duplicates park (target slot, a·b) in product order;
//      one wave adds the duplicates in product order (s = s + p, exactly the
//      reference's summation, no FMA), and the chunk's C entries leave LDS as
//      one coalesced, contiguous store stream.
// Rows with more than OP_BIG products are excluded from chunks: they are
// singleton chunks whose nnz comes from the two-phase engine run on them
// beforehand, and whose values that engine writes afterwards.
#pragma once

#include "spgemm_kernels.hpp"

namespace ias {
namespace dev {

constexpr int OP_BLOCK = 512;                // threads of a chunk workgroup
constexpr int OP_NPM = 4096;                 // products per chunk (capacity)
constexpr int OP_BIG = 2048;                 // rows with more products: big-row path
constexpr int OP_WIN = OP_NPM - OP_BIG;      // chunk window in the row product prefix
constexpr int OP_RMAX = 1024;                // rows per chunk
constexpr unsigned long long OP_EMPTY = ~0ull;
constexpr unsigned long long OP_FA = 1ull << 62;   // look-back: aggregate published
constexpr unsigned long long OP_FI = 2ull << 62;   // look-back: inclusive prefix published
constexpr unsigned long long OP_VM = (1ull << 62) - 1ull;

struct OnepassArgs {
    Rows A;                      // CSR view (row starts give each chunk's entry range)
    Rows B;
    AxView ax;                   // expanded A: B-row start and A value per entry
    const int32_t *axr;          // row of every A entry (view-relative)
    const int64_t *axp;          // product offset of every A entry
    const int64_t *poff;         // product offset of every row
    const int32_t *prod;         // products per row (big rows: > OP_BIG)
    const int64_t *chunk_row0;   // first row of every chunk, + rows at [nchunks]
    const int32_t *nchunks;      // device scalar
    const int32_t *big_nnz;      // nnz of every big row (two-phase engine, compact order)
    const int64_t *bigpos;       // compact index of every big row
    unsigned long long *status;  // look-back words, zeroed per call
    int32_t *ticket;             // zeroed per call
    int64_t *cptr;               // C row pointer (written here)
    int32_t *ccol;
    double *cval;
    int64_t rows;
    int64_t cap;                 // capacity of ccol/ccval: nothing is written beyond
    int32_t order;               // 0: reverse first-touch, 1: forward
    int32_t first_assign;        // 1: first product assigned (COO), 0: 0.0 + product
};

// Chunk boundaries: a new chunk starts at row 0, at every big row and the row
// after it, every OP_RMAX rows, and where the row product prefix enters a new
// OP_WIN window — so a chunk of small rows holds < OP_WIN + OP_BIG products.
__global__ void k_op_flags(const int64_t *poff, const int32_t *prod, int64_t rows, int32_t *cflag,
                           int32_t *bflag) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    const bool big = prod[r] > OP_BIG;
    bool f = r == 0 || big || (r % OP_RMAX) == 0;
    if (!f) f = prod[r - 1] > OP_BIG || (poff[r] / OP_WIN) != (poff[r - 1] / OP_WIN);
    cflag[r] = f ? 1 : 0;
    bflag[r] = big ? 1 : 0;
}

// Chunk list and big-row list from the exclusive scans of the flags.
__global__ void k_op_lists(const int32_t *cflag, const int64_t *cid, const int32_t *bflag,
                           const int64_t *bigpos, int64_t rows, int64_t *chunk_row0, int32_t *nchunks,
                           int64_t *bigrow) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    if (cflag[r]) chunk_row0[cid[r]] = r;
    if (bflag[r]) bigrow[bigpos[r]] = r;
    if (r == rows - 1) {
        const int64_t n = cid[r] + cflag[r];
        chunk_row0[n] = rows;
        *nchunks = (int32_t)n;
    }
}

// Entry counts of the big rows (zero beyond the big-row count, so a scan over
// `rows` slots sizes the compact copy without a host round trip).
__global__ void k_op_biglen(Rows A, const int64_t *bigpos, const int64_t *bigrow, int64_t rows, int32_t *len) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= rows) return;
    int32_t n = 0;
    if (k < bigpos[rows]) {
        int64_t s;
        A.row(bigrow[k], s, n);
    }
    len[k] = n;
}

// Compact copy of the big rows' entries (one workgroup per big row).
__global__ void k_op_bigcopy(Rows A, const int64_t *bigrow, const int64_t *bptr, int32_t *bcol, double *bval) {
    const int64_t k = blockIdx.x;
    int64_t s;
    int32_t n;
    A.row(bigrow[k], s, n);
    const int64_t d = bptr[k];
    for (int32_t i = threadIdx.x; i < n; i += blockDim.x) {
        bcol[d + i] = A.col[s + i];
        bval[d + i] = A.val[s + i];
    }
}

// C row starts of the big rows, for the two-phase engine's Out.
__global__ void k_op_bigptr(const int64_t *cptr, const int64_t *bigrow, int64_t nbig, int64_t *bcptr) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < nbig) bcptr[k] = cptr[bigrow[k]];
}

// max nnz per row of C (report only)
__global__ void k_op_maxlen(const int64_t *cptr, int64_t rows, int32_t *mx) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int v = r < rows ? (int)(cptr[r + 1] - cptr[r]) : 0;
#pragma unroll
    for (int d = WAVE / 2; d > 0; d >>= 1) v = max(v, __shfl_xor(v, d));
    if ((threadIdx.x & (WAVE - 1)) == 0 && v > 0) atomicMax(mx, v);
}

__device__ __forceinline__ void op_store(unsigned long long *p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Decoupled look-back, one whole wave: publishes the chunk's aggregate, sums
// the predecessors' words (64 per poll) back to the first inclusive one, then
// publishes the inclusive prefix.  Returns the chunk's exclusive offset.
__device__ __forceinline__ int64_t op_lookback(unsigned long long *status, int64_t c, int64_t agg, int lane) {
    if (c == 0) {
        if (lane == 0) op_store(&status[0], OP_FI | (unsigned long long)agg);
        return 0;
    }
    if (lane == 0) op_store(&status[c], OP_FA | (unsigned long long)agg);
    int64_t acc = 0;
    int64_t i = c - 1;
    for (;;) {
        const int64_t idx = i - lane;
        const unsigned long long st =
            idx >= 0 ? __hip_atomic_load(&status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : OP_FI;
        const unsigned long long fl = st >> 62;
        const uint64_t inc = __ballot(fl == 2ull);
        const uint64_t zer = __ballot(fl == 0ull);
        const int fi = inc ? __ffsll((long long)inc) - 1 : 64;
        const uint64_t lim = fi >= 63 ? ~0ull : ((2ull << fi) - 1ull);
        if (zer & lim) {
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        int64_t v = lane <= fi ? (int64_t)(st & OP_VM) : 0;
#pragma unroll
        for (int d = WAVE / 2; d > 0; d >>= 1) v += __shfl_xor(v, d);
        acc += v;
        if (fi < 64) break;
        i -= WAVE;
    }
    if (lane == 0) op_store(&status[c], OP_FI | (unsigned long long)(acc + agg));
    return acc;
}

// exclusive rank of position pos in a bitmap with per-word exclusive prefix
__device__ __forceinline__ int op_rank(const uint32_t *bits, const int32_t *pref, int pos) {
    const int w = pos >> 5;
    return pref[w] + __popc(bits[w] & ((1u << (pos & 31)) - 1u));
}

// Persistent workgroups; each takes chunks in row order from the ticket.
template <int T, int NPM>
__global__ __launch_bounds__(T) void k_onepass(OnepassArgs a) {
    constexpr int K = NPM / T;
    constexpr int NW = NPM / 32;          // bitmap words
    constexpr int TS = NPM * 3 / 2;       // table slots
    constexpr int NWV = T / WAVE;
    static_assert(NPM % T == 0 && T % WAVE == 0 && NW % WAVE == 0, "shape");
    __shared__ unsigned long long tab[TS + 2];   // hash table, then the staging area of C
    __shared__ uint32_t ebits[NW + 1];           // entry starts (non-empty entries)
    __shared__ int32_t epref[NW + 1];
    __shared__ uint32_t fbits[NW + 1];           // first touches
    __shared__ int32_t fpref[NW + 1];
    __shared__ int32_t ne[NPM];                  // k-th non-empty entry of the chunk (local index)
    __shared__ int32_t roff[OP_RMAX + 1];        // row product offsets, then row ranks
    __shared__ int64_t sh_c, sh_off;

    const int tid = threadIdx.x;
    const int lane = tid & (WAVE - 1);
    const int w = tid / WAVE;
    const int32_t nch = *a.nchunks;
    const bool rev = a.order == 0;
    Timer tmr, tmb;   // timing builds only: small chunks (slot 31), big-row chunks (slot 30)

    // wave-0 scan of a bitmap's word popcounts into its exclusive prefix
    auto scan_words = [&](const uint32_t *bits, int32_t *pref) {
        constexpr int PER = NW / WAVE;
        int cnt[PER];
        int s = 0;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            cnt[i] = __popc(bits[lane * PER + i]);
            s += cnt[i];
        }
        int x = s;
#pragma unroll
        for (int d = 1; d < WAVE; d <<= 1) {
            const int t = __shfl_up(x, d);
            if (lane >= d) x += t;
        }
        int run = x - s;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            pref[lane * PER + i] = run;
            run += cnt[i];
        }
        if (lane == WAVE - 1) pref[NW] = x;
    };

    for (;;) {
        tmr.start();
        tmb.start();
        if (tid == 0) sh_c = atomicAdd(a.ticket, 1);
        __syncthreads();
        const int64_t c = sh_c;
        if (c >= nch) break;
        const int64_t r0 = a.chunk_row0[c], r1 = a.chunk_row0[c + 1];
        if (r1 - r0 == 1 && a.prod[r0] > OP_BIG) {
            // big row: nnz known from the two-phase engine
            if (w == 0) {
                const int64_t nz = a.big_nnz[a.bigpos[r0]];
                const int64_t off = op_lookback(a.status, c, nz, lane);
                if (lane == 0) {
                    a.cptr[r0] = off;
                    if (c == nch - 1) a.cptr[a.rows] = off + nz;
                }
            }
            __syncthreads();
            tmb.mark(0);
            tmb.done();
            continue;
        }
        const int nr = (int)(r1 - r0);
        const int64_t P0 = a.poff[r0];
        const int np = (int)(a.poff[r1] - P0);
        int64_t e0, e1;
        {
            int64_t s;
            int32_t n;
            a.A.row(r0, s, n);
            e0 = s - a.A.base();
            a.A.row(r1 - 1, s, n);
            e1 = s + n - a.A.base();
        }
        // ---- setup: row offsets, empty table, entry-start bitmap
        for (int i = tid; i <= nr; i += T) roff[i] = (int)(a.poff[r0 + i] - P0);
        {
            const int nslots = (3 * np) / 2;
            for (int i = tid; i < nslots; i += T) tab[i] = OP_EMPTY;
        }
        for (int i = tid; i <= NW; i += T) {
            ebits[i] = 0u;
            fbits[i] = 0u;
        }
        __syncthreads();
        for (int64_t e = e0 + tid; e < e1; e += T) {
            if (a.ax.blen[e] > 0) {
                const int o = (int)(a.axp[e] - P0);
                atomicOr(&ebits[o >> 5], 1u << (o & 31));
            }
        }
        __syncthreads();
        if (w == 0) scan_words(ebits, epref);
        __syncthreads();
        for (int64_t e = e0 + tid; e < e1; e += T) {
            if (a.ax.blen[e] > 0) {
                const int o = (int)(a.axp[e] - P0);
                ne[op_rank(ebits, epref, o)] = (int)(e - e0);
            }
        }
        __syncthreads();
        tmr.mark(0);

        // ---- products: gather, then insert
        int32_t col[K], rl[K];
        double v[K];
        uint32_t slot[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int p = k * T + tid;
            rl[k] = -1;
            col[k] = 0;
            v[k] = 0.0;
            if (p < np) {
                const int kk = op_rank(ebits, epref, p + 1) - 1;   // last entry starting at or before p
                const int64_t e = e0 + ne[kk];
                const int64_t bi = a.ax.bstart[e] + ((P0 + p) - a.axp[e]);
                col[k] = a.B.col[bi];
                v[k] = a.ax.aval[e] * a.B.val[bi];
                rl[k] = a.axr[e] - (int32_t)r0;
            }
        }
#if IAS_TIMING
        {
            int32_t z = 0;
#pragma unroll
            for (int k = 0; k < K; ++k) z |= col[k];
            if (z == -12345) a.ccol[0] = 0;   // force the loads to complete here
        }
#endif
        tmr.mark(1);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            slot[k] = 0;
            if (rl[k] >= 0) {
                const uint32_t p = (uint32_t)(k * T + tid);
                const int lo = roff[rl[k]], hi = roff[rl[k] + 1];
                const uint32_t base = (uint32_t)((3 * lo) / 2);
                const uint32_t end = (uint32_t)((3 * hi) / 2);
                const unsigned long long key = ((unsigned long long)(uint32_t)col[k] << 32) | p;
                uint32_t s = base + slot_hash(col[k], end - base);
                for (;;) {
                    const unsigned long long prev = atomicCAS(&tab[s], OP_EMPTY, key);
                    if (prev == OP_EMPTY) break;
                    if ((uint32_t)(prev >> 32) == (uint32_t)col[k]) {
                        if ((uint32_t)prev > p) atomicMin(&tab[s], key);
                        break;
                    }
                    s = (s + 1u == end) ? base : s + 1u;
                }
                slot[k] = s;
            }
        }
        tmr.mark(2);
        __syncthreads();
        tmr.mark(3);
        // ---- first touches -> bitmap (one ballot per wave and step)
        uint32_t own[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t p = (uint32_t)(k * T + tid);
            own[k] = rl[k] >= 0 ? (uint32_t)tab[slot[k]] : 0u;
            const uint64_t b = __ballot(rl[k] >= 0 && own[k] == p);
            if (lane == 0) {
                const int wi = (k * T + w * WAVE) >> 5;
                fbits[wi] = (uint32_t)b;
                fbits[wi + 1] = (uint32_t)(b >> 32);
            }
        }
        __syncthreads();
        if (w == 0) {
            scan_words(fbits, fpref);
            // publish the aggregate at once (successors' look-back)
            const int64_t agg = __shfl(fpref[NW], WAVE - 1);
            if (c > 0 && lane == 0) op_store(&a.status[c], OP_FA | (unsigned long long)agg);
        }
        __syncthreads();
        const int nnzc = fpref[NW];
        const int D = np - nnzc;
        // row offsets -> row ranks (in place)
        for (int i = tid; i <= nr; i += T) roff[i] = op_rank(fbits, fpref, roff[i]);
        __syncthreads();
        tmr.mark(4);
        // ---- stage C entries (first touches) and duplicates (product order)
        char *stage = (char *)tab;
        double *oval = (double *)stage;
        int32_t *ocol = (int32_t *)(stage + 8 * (size_t)nnzc);
        const size_t dvo = ((size_t)12 * nnzc + 7) & ~(size_t)7;
        double *dv = (double *)(stage + dvo);
        int32_t *dq = (int32_t *)(stage + dvo + 8 * (size_t)D);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (rl[k] >= 0) {
                const int p = k * T + tid;
                const int r = op_rank(fbits, fpref, p);
                const int lo = roff[rl[k]], hi = roff[rl[k] + 1];
                if (own[k] == (uint32_t)p) {
                    const int q = rev ? lo + hi - 1 - r : r;
                    ocol[q] = col[k];
                    oval[q] = a.first_assign ? v[k] : 0.0 + v[k];
                } else {
                    const int ro = op_rank(fbits, fpref, (int)own[k]);
                    const int d = p - r;
                    dq[d] = rev ? lo + hi - 1 - ro : ro;
                    dv[d] = v[k];
                }
            }
        }
        tmr.mark(5);
        if (w == 0) {
            int64_t off;
            if (c == 0) {
                off = 0;
                if (lane == 0) op_store(&a.status[0], OP_FI | (unsigned long long)nnzc);
            } else {
                // aggregate already published: look back only
                int64_t acc = 0;
                int64_t i = c - 1;
                for (;;) {
                    const int64_t idx = i - lane;
                    const unsigned long long st =
                        idx >= 0 ? __hip_atomic_load(&a.status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                 : OP_FI;
                    const unsigned long long fl = st >> 62;
                    const uint64_t inc = __ballot(fl == 2ull);
                    const uint64_t zer = __ballot(fl == 0ull);
                    const int fi = inc ? __ffsll((long long)inc) - 1 : 64;
                    const uint64_t lim = fi >= 63 ? ~0ull : ((2ull << fi) - 1ull);
                    if (zer & lim) {
                        __builtin_amdgcn_s_sleep(2);
                        continue;
                    }
                    int64_t x = lane <= fi ? (int64_t)(st & OP_VM) : 0;
#pragma unroll
                    for (int d = WAVE / 2; d > 0; d >>= 1) x += __shfl_xor(x, d);
                    acc += x;
                    if (fi < 64) break;
                    i -= WAVE;
                }
                off = acc;
                if (lane == 0) op_store(&a.status[c], OP_FI | (unsigned long long)(acc + nnzc));
            }
            if (lane == 0) sh_off = off;
        }
        __syncthreads();
        tmr.mark(6);
        const int64_t off = sh_off;
        // ---- duplicates, in product order (last wave); row pointer (others)
        if (w == NWV - 1) {
            for (int g = 0; g < D; g += WAVE) {
                const int d = g + lane;
                const bool ok = d < D;
                const int q = ok ? dq[d] : -1 - lane;
                const double x = ok ? dv[d] : 0.0;
                int depth = 0;
                for (int i = 1; i < WAVE; ++i) {
                    const int qq = __shfl(q, lane - i);
                    if (lane >= i && qq == q) ++depth;
                }
                int md = depth;
#pragma unroll
                for (int s = WAVE / 2; s > 0; s >>= 1) md = max(md, __shfl_xor(md, s));
                for (int r = 0; r <= md; ++r) {
                    if (ok && depth == r) oval[q] = oval[q] + x;
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                }
            }
        } else {
            for (int i = tid; i < nr; i += T - WAVE) a.cptr[r0 + i] = off + roff[i];
            if (tid == 0 && c == nch - 1) a.cptr[a.rows] = off + nnzc;
        }
        __syncthreads();
        // ---- emission: contiguous, coalesced
        const int nemit = off + nnzc <= a.cap ? nnzc : 0;
        for (int q = tid; q < nemit; q += T) {
            __builtin_nontemporal_store(ocol[q], &a.ccol[off + q]);
            __builtin_nontemporal_store(oval[q], &a.cval[off + q]);
        }
        __syncthreads();
        tmr.mark(7);
        tmr.done();
    }
    tmr.flush(31, tid == 0);
    tmb.flush(30, tid == 0);
}

}  // namespace dev
}  // namespace ias
