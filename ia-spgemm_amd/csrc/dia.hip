// dia.hip — DIA x DIA for banded inputs (replaces DIA_mul_DIA,
// IA-SPGEMM-CPU_release/detail/dia/common_dia.h:101-195, and the unused
// DIA_MUL_DIA_DEV, GPU/detail/dia_dev/common_dia_dev.h:138-182).
//
// C's diagonal set is computed on the host from the offsets alone, exactly as
// the reference's triple loop decides it (dia:107-140: offset a+b exists when
// some row i has i+a in [0, A.cols) and i+a+b in [0, B.cols)).  For every C
// slot the contributing (A diagonal, B diagonal) pairs are listed in the
// reference's loop order (ja ascending), so one lane per C element
//     C[i][slot] = ((0.0 + A[i][ja0]*B[i+a0][kb0]) + A[i][ja1]*B[i+a1][kb1]) ...
// reproduces the reference's sums bit for bit (-ffp-contract=off).  One lane
// per element makes the C store fully coalesced (row-major rows x nd_C); A
// and B rows are re-read from L2 by the nd_C lanes of a row (k_dia_mul; the
// tiled form k_dia_tile stages them in LDS).  Narrow bands are HBM-bound
// (~0.4 flop/byte at 7 diagonals) and stay on the VALU; wide dense bands take
// the f64 MFMA form k_dia_mfma (DIA).
#include "ias.h"
#include "ias_internal.hpp"
#include "spgemm_engine.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

namespace ias {
namespace dev {

struct DiaPairs {
    const int32_t *start;  // nd_C + 1
    const int32_t *ja;     // A diagonal slot of each pair
    const int32_t *kb;     // B diagonal slot of each pair
};

__global__ __launch_bounds__(256) void k_dia_mul(int64_t rows, int64_t a_cols, int64_t b_cols,
                                                 int32_t nda, const int32_t *__restrict__ offa,
                                                 const double *__restrict__ va, int32_t ndb,
                                                 const int32_t *__restrict__ offb,
                                                 const double *__restrict__ vb, int32_t ndc,
                                                 DiaPairs pairs, double *__restrict__ vc) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= rows * ndc) return;
    const int64_t i = e / ndc;
    const int32_t slot = (int32_t)(e - i * ndc);
    double acc = 0.0;
    for (int32_t p = pairs.start[slot]; p < pairs.start[slot + 1]; ++p) {
        const int32_t ja = pairs.ja[p], kb = pairs.kb[p];
        const int64_t acol = i + offa[ja];
        if (acol < 0 || acol >= a_cols) continue;
        const int64_t bcol = acol + offb[kb];
        if (bcol < 0 || bcol >= b_cols) continue;
        const double prod = va[i * nda + ja] * vb[acol * ndb + kb];
        acc = acc + prod;
    }
    vc[e] = acc;
}

// LDS-tiled form: one workgroup per tile of TR consecutive rows.  The tile's A
// rows (TR x nda) and the B rows they reach (TR + span(offa) rows x ndb) are
// two contiguous ranges of the row-major DIA arrays: staged in LDS with
// coalesced loads, so every A / B value is read from HBM once per tile (the
// per-element kernel above re-reads them from L2 for each of the nd_C lanes
// of a row).  The C tile (TR x nd_C) is one contiguous range: lanes over its
// elements, non-temporal stores.  32-bit indexing inside the tile; e / nd_C
// by a multiply-high.  Same per-element pair order as k_dia_mul (bitwise).
struct DiaTileArgs {
    int32_t rows, a_cols, b_cols;
    int32_t nda, ndb, ndc, np;
    int32_t lo_a, span_a;       // min A offset, max - min
    int32_t tr;                 // rows per tile
    uint64_t ndc_magic;         // ceil(2^32 / ndc)
    const int32_t *offa, *offb;
    const double *va, *vb;
    const int32_t *tab;         // start[ndc + 1], ja[np], kb[np]
    double *vc;
};

__global__ __launch_bounds__(256) void k_dia_tile(DiaTileArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int r0 = (int)blockIdx.x * a.tr;
    const int tr = min(a.tr, a.rows - r0);
    const int b0 = max(r0 + a.lo_a, 0);
    const int b1 = min(r0 + tr - 1 + a.lo_a + a.span_a, a.a_cols - 1);   // inclusive
    const int nbr = max(b1 - b0 + 1, 0);
    double *sA = (double *)smem;
    double *sB = sA + a.tr * a.nda;
    int32_t *soa = (int32_t *)(sB + (a.tr + a.span_a) * a.ndb);
    int32_t *sob = soa + a.nda;
    int32_t *st = sob + a.ndb;
    const int t = (int)threadIdx.x;
    {
        const double *ga = a.va + (int64_t)r0 * a.nda;
        for (int i = t; i < tr * a.nda; i += 256) sA[i] = __builtin_nontemporal_load(ga + i);
        const double *gb = a.vb + (int64_t)b0 * a.ndb;
        for (int i = t; i < nbr * a.ndb; i += 256) sB[i] = gb[i];
        for (int i = t; i < a.nda; i += 256) soa[i] = a.offa[i];
        for (int i = t; i < a.ndb; i += 256) sob[i] = a.offb[i];
        for (int i = t; i < a.ndc + 1 + 2 * a.np; i += 256) st[i] = a.tab[i];
    }
    __syncthreads();
    const int32_t *sja = st + a.ndc + 1, *skb = sja + a.np;
    const int n = tr * a.ndc;
    double *gc = a.vc + (int64_t)r0 * a.ndc;
    for (int e = t; e < n; e += 256) {
        const int i = (int)(((uint64_t)(uint32_t)e * a.ndc_magic) >> 32);   // e / ndc (e < 2^20)
        const int slot = e - i * a.ndc;
        const int gi = r0 + i;
        double acc = 0.0;
        for (int p = st[slot]; p < st[slot + 1]; ++p) {
            const int ja = sja[p], kb = skb[p];
            const int acol = gi + soa[ja];
            if (acol < 0 || acol >= a.a_cols) continue;
            const int bcol = acol + sob[kb];
            if (bcol < 0 || bcol >= a.b_cols) continue;
            acc = acc + sA[i * a.nda + ja] * sB[(acol - b0) * a.ndb + kb];
        }
        __builtin_nontemporal_store(acc, gc + e);
    }
}

// MFMA form (IAS_DIA_MFMA=1, A/B against k_dia_tile): the band of a tile of
// 16 rows as dense blocks — A_t (16 x W_A, W_A = 16 + span(offa) columns from
// i0 + min offa) times B_t (W_A x W_C, W_C = W_A + span(offb)) with
// v_mfma_f64_16x16x4f64, operands built on the fly from the staged DIA rows
// through offset -> diagonal maps (zeros off the band); the C block's band
// elements go to their C diagonals.  The MFMA sums in its own order (fused,
// not the reference's (0.0 + a*b) + a*b sequence), so this form matches the
// reference within the north-star tolerance, not bitwise.  Waves of the
// workgroup take the 16-column C blocks round-robin; C is zeroed first (the
// DIA layout's off-matrix slots).
typedef double dia_f64x4 __attribute__((ext_vector_type(4)));
struct DiaMfmaArgs {
    int32_t rows, a_cols, b_cols;
    int32_t nda, ndb, ndc;
    int32_t lo_a, span_a, lo_b, span_b, lo_c, span_c;
    const int32_t *amap, *bmap, *cmap;   // offset - lo -> diagonal slot or -1
    const double *va, *vb;
    double *vc;
    const int32_t *offa, *offb;          // diagonal offsets (the VALU fallback)
    const int32_t *tab;                  // pair table: start[ndc + 1], ja[np], kb[np]
    int32_t np;
};

__global__ __launch_bounds__(256) void k_dia_mfma(DiaMfmaArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int i0 = (int)blockIdx.x * 16;
    const int WA = 16 + a.span_a, WC = WA + a.span_b;
    const int cA0 = i0 + a.lo_a;           // global column of A_t column 0 (= B row of B_t row 0)
    const int cC0 = cA0 + a.lo_b;          // global column of C_t column 0
    double *sA = (double *)smem;                         // 16 x nda
    double *sB = sA + 16 * a.nda;                        // WA x ndb (B rows cA0 ..)
    int32_t *am = (int32_t *)(sB + WA * a.ndb);
    int32_t *bm = am + a.span_a + 1;
    int32_t *cm = bm + a.span_b + 1;
    const int t = (int)threadIdx.x;
    int bad = 0;   // a non-finite operand: 0 * Inf in the dense block would be NaN
    for (int i = t; i < 16 * a.nda; i += 256) {
        const int r = i / a.nda;
        const double v = i0 + r < a.rows ? a.va[(int64_t)(i0 + r) * a.nda + (i - r * a.nda)] : 0.0;
        bad |= !__builtin_isfinite(v);
        sA[i] = v;
    }
    for (int i = t; i < WA * a.ndb; i += 256) {
        const int r = i / a.ndb, br = cA0 + r;
        const double v = (br >= 0 && br < a.a_cols) ? a.vb[(int64_t)br * a.ndb + (i - r * a.ndb)] : 0.0;
        bad |= !__builtin_isfinite(v);
        sB[i] = v;
    }
    for (int i = t; i <= a.span_a; i += 256) am[i] = a.amap[i];
    for (int i = t; i <= a.span_b; i += 256) bm[i] = a.bmap[i];
    for (int i = t; i <= a.span_c; i += 256) cm[i] = a.cmap[i];
    if (__syncthreads_or(bad)) {
        // this tile holds an Inf / NaN: the reference's pair sums on the VALU
        // (k_dia_tile's loop over the staged rows; bitwise the reference)
        const int32_t *sja = a.tab + a.ndc + 1, *skb = sja + a.np;
        for (int e = t; e < 16 * a.ndc; e += 256) {
            const int i = e / a.ndc, slot = e - i * a.ndc, gi = i0 + i;
            if (gi >= a.rows) break;
            double acc = 0.0;
            for (int p = a.tab[slot]; p < a.tab[slot + 1]; ++p) {
                const int ja = sja[p], kb = skb[p];
                const int acol = gi + a.offa[ja];
                if (acol < 0 || acol >= a.a_cols) continue;
                const int bcol = acol + a.offb[kb];
                if (bcol < 0 || bcol >= a.b_cols) continue;
                acc = acc + sA[i * a.nda + ja] * sB[(acol - cA0) * a.ndb + kb];
            }
            a.vc[(int64_t)gi * a.ndc + slot] = acc;
        }
        return;
    }
    const int w = t >> 6, l = t & 63;
    const int nblk = (WC + 15) / 16;
    for (int cb = w; cb < nblk; cb += 4) {
        dia_f64x4 acc = {0.0, 0.0, 0.0, 0.0};
        // A_t columns that reach this C block: c'' - c' in [0, span_b]
        const int k_lo = max(0, cb * 16 - a.span_b), k_hi = min(WA, cb * 16 + 16);
        for (int k0 = k_lo & ~3; k0 < k_hi; k0 += 4) {
            const int kk = l >> 4, rr = l & 15;
            const int ca = k0 + kk;                          // A_t column / B_t row
            // A operand: A_t[rr][ca]; diagonal offset (cA0 + ca) - (i0 + rr)
            const int oa = ca - rr;                          // minus lo_a
            double av = 0.0;
            if (oa >= 0 && oa <= a.span_a && ca < WA) {
                const int ja = am[oa];
                const int acol = cA0 + ca;
                if (ja >= 0 && acol >= 0 && acol < a.a_cols) av = sA[rr * a.nda + ja];
            }
            // B operand: B_t[ca][cc], global column cC0 + cb*16 + cc
            const int cc = l & 15;
            const int ob = cb * 16 + cc - ca;                // (col - brow) - lo_b
            double bv = 0.0;
            if (ob >= 0 && ob <= a.span_b && ca < WA) {
                const int kb = bm[ob];
                const int col = cC0 + cb * 16 + cc;
                if (kb >= 0 && col >= 0 && col < a.b_cols) bv = sB[ca * a.ndb + kb];
            }
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
        }
        // C_t[row][col]: row = (l >> 4) + 4j, col = l & 15
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = (l >> 4) + 4 * j, col = l & 15;
            const int gi = i0 + row, gc = cC0 + cb * 16 + col;
            const int oc = (gc - gi) - a.lo_c;
            if (gi < a.rows && cb * 16 + col < WC && gc >= 0 && gc < a.b_cols && oc >= 0 && oc <= a.span_c) {
                const int d = cm[oc];
                if (d >= 0) a.vc[(int64_t)gi * a.ndc + d] = acc[j];
            }
        }
    }
}

// C's offsets (a copy of the plan's) and diagonal_ind in one pass:
// ind[o + rows - 1] = the C diagonal of offset o, 0 elsewhere (offc ascending,
// binary search) — one launch instead of a copy, a memset and a scatter.
// A reused plan's check (flag non-null): the operands' current offsets against
// the ones the plan was made from; any difference sets *flag (host-mapped), and
// the call redoes the product with a plan of the current offsets.
struct DiaCheck {
    const int32_t *ca, *pa;
    int32_t nda;
    const int32_t *cb, *pb;
    int32_t ndb;
    int32_t *flag;
};
__global__ void k_dia_meta(int32_t ndc, const int32_t *offc, int64_t rows, int64_t span, int32_t *offs,
                           int32_t *ind, DiaCheck chk) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (chk.flag && ((i < chk.nda && chk.ca[i] != chk.pa[i]) || (i < chk.ndb && chk.cb[i] != chk.pb[i])))
        *chk.flag = 1;
    if (i < ndc) offs[i] = offc[i];
    if (i >= span) return;
    const int64_t o = i - (rows - 1);
    int32_t lo = 0, hi = ndc;   // first d with offc[d] >= o
    while (lo < hi) {
        const int32_t m = (lo + hi) >> 1;
        if (offc[m] < o) lo = m + 1;
        else hi = m;
    }
    ind[i] = (lo < ndc && offc[lo] == o) ? lo : 0;
}

}  // namespace dev
}  // namespace ias

using namespace ias;

// Host: C diagonal set and per-slot pair lists (reference loop order).
static void dia_plan(const int32_t *offa, int32_t nda, const int32_t *offb, int32_t ndb,
                     int64_t rows, int64_t a_cols, int64_t b_cols, std::vector<int32_t> &offc,
                     std::vector<int32_t> &start, std::vector<int32_t> &ja,
                     std::vector<int32_t> &kb) {
    std::vector<int64_t> reach;
    for (int32_t x = 0; x < nda; ++x)
        for (int32_t y = 0; y < ndb; ++y) {
            const int64_t oa = offa[x], ob = offb[y];
            int64_t lo = 0, hi = rows;
            lo = std::max(lo, -oa);
            hi = std::min(hi, a_cols - oa);
            lo = std::max(lo, -oa - ob);
            hi = std::min(hi, b_cols - oa - ob);
            if (lo < hi) reach.push_back(oa + ob);
        }
    std::sort(reach.begin(), reach.end());
    reach.erase(std::unique(reach.begin(), reach.end()), reach.end());
    offc.assign(reach.begin(), reach.end());
    const int32_t ndc = (int32_t)offc.size();
    start.assign(ndc + 1, 0);
    std::vector<std::vector<std::pair<int32_t, int32_t>>> lists(ndc);
    for (int32_t x = 0; x < nda; ++x)
        for (int32_t y = 0; y < ndb; ++y) {
            const int64_t o = (int64_t)offa[x] + offb[y];
            auto it = std::lower_bound(reach.begin(), reach.end(), o);
            if (it != reach.end() && *it == o) lists[it - reach.begin()].push_back({x, y});
        }
    ja.clear();
    kb.clear();
    for (int32_t d = 0; d < ndc; ++d) {
        for (auto &pr : lists[d]) {
            ja.push_back(pr.first);
            kb.push_back(pr.second);
        }
        start[d + 1] = (int32_t)ja.size();
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

// Per offset set (A's and B's diagonal offsets and the shapes), everything
// the call derives from the offsets alone: C's offsets, the pair table, the
// MFMA offset maps, and their device copies — computed once and reused by
// later calls (the K1 step is a 31 µs kernel: the host plan, three small
// synchronous uploads and two event creations cost more than the kernel).
namespace {
struct DiaPlan {
    std::vector<int32_t> offc, pst, pja, pkb, maps;
    int32_t lo_a = 0, span_a = 0, lo_b = 0, span_b = 0, lo_c = 0, span_c = 0;
    int64_t flops = 0;                // multiply pairs formed (in range)
    int device = 0;
    int32_t *d_offc = nullptr, *d_tab = nullptr, *d_maps = nullptr;
    int32_t *d_offa = nullptr, *d_offb = nullptr;
    // the device tables go back to the block cache, which hands a block out
    // again only after a device sync (queued kernels of the last call first)
    ~DiaPlan() {
        int cur = 0;
        const bool had = hipGetDevice(&cur) == hipSuccess;
        for (int32_t *q : {d_offc, d_tab, d_maps, d_offa, d_offb}) dev_free(q, device);
        if (had) hipSetDevice(cur);   // dev_free selects the plan's device
    }
};
// Plans by key, at most CAP of them: a new key beyond that evicts the least
// recently used plan (a caller still holding it keeps it alive).
struct DiaCache {
    static constexpr size_t CAP = 256;
    std::mutex mu;
    uint64_t tick = 0;
    std::map<std::vector<int64_t>, std::pair<std::shared_ptr<const DiaPlan>, uint64_t>> plans;
};
DiaCache &dia_cache() {
    static DiaCache *c = new DiaCache;
    return *c;
}
ias_status upload_i32(int32_t **d, const std::vector<int32_t> &h, int device) {
    IAS_TRY(dev_alloc((void **)d, 4 * std::max<size_t>(h.size(), 1), device));
    if (!h.empty()) IAS_TRY(dev_copy_h2d(*d, h.data(), 4 * h.size(), device));
    return IAS_SUCCESS;
}
ias_status dia_plan_get(const std::vector<int32_t> &offa, const std::vector<int32_t> &offb, int64_t rows,
                        int64_t a_cols, int64_t b_cols, int device, std::shared_ptr<const DiaPlan> *out) {
    std::vector<int64_t> key{device, rows, a_cols, b_cols, (int64_t)offa.size()};
    key.insert(key.end(), offa.begin(), offa.end());
    key.insert(key.end(), offb.begin(), offb.end());
    DiaCache &c = dia_cache();
    std::lock_guard<std::mutex> g(c.mu);
    auto it = c.plans.find(key);
    if (it != c.plans.end()) {
        it->second.second = ++c.tick;
        *out = it->second.first;
        return IAS_SUCCESS;
    }
    std::shared_ptr<DiaPlan> P = std::make_shared<DiaPlan>();
    P->device = device;
    const int32_t nda = (int32_t)offa.size(), ndb = (int32_t)offb.size();
    dia_plan(offa.data(), nda, offb.data(), ndb, rows, a_cols, b_cols, P->offc, P->pst, P->pja, P->pkb);
    const int32_t ndc = (int32_t)P->offc.size();
    if (nda && ndb && ndc) {
        P->lo_a = *std::min_element(offa.begin(), offa.end());
        P->span_a = *std::max_element(offa.begin(), offa.end()) - P->lo_a;
        P->lo_b = *std::min_element(offb.begin(), offb.end());
        P->span_b = *std::max_element(offb.begin(), offb.end()) - P->lo_b;
        P->lo_c = P->offc.front();
        P->span_c = P->offc.back() - P->lo_c;
        // offset -> slot maps of the MFMA operands, only for bands narrow
        // enough for its LDS (a wide-offset band never takes that kernel)
        const int64_t mlen = (int64_t)P->span_a + P->span_b + P->span_c + 3;
        if (mlen <= (1 << 16)) {
            P->maps.assign((size_t)mlen, -1);
            for (int32_t j = 0; j < nda; ++j) P->maps[offa[j] - P->lo_a] = j;
            for (int32_t j = 0; j < ndb; ++j) P->maps[(size_t)P->span_a + 1 + (offb[j] - P->lo_b)] = j;
            for (int32_t j = 0; j < ndc; ++j)
                P->maps[(size_t)P->span_a + P->span_b + 2 + (P->offc[j] - P->lo_c)] = j;
        }
    }
    for (int32_t d = 0; d < ndc; ++d)
        for (int32_t q = P->pst[d]; q < P->pst[d + 1]; ++q) {
            const int64_t oa = offa[P->pja[q]], ob = offb[P->pkb[q]];
            const int64_t lo = std::max<int64_t>(0, std::max<int64_t>(-oa, -oa - ob));
            const int64_t hi = std::min<int64_t>(rows, std::min<int64_t>(a_cols - oa, b_cols - oa - ob));
            if (hi > lo) P->flops += hi - lo;
        }
    std::vector<int32_t> tab;
    tab.insert(tab.end(), P->pst.begin(), P->pst.end());
    tab.insert(tab.end(), P->pja.begin(), P->pja.end());
    tab.insert(tab.end(), P->pkb.begin(), P->pkb.end());
    ias_status st;
    if ((st = upload_i32(&P->d_offc, P->offc, device)) || (st = upload_i32(&P->d_tab, tab, device)) ||
        (st = upload_i32(&P->d_maps, P->maps, device)) || (st = upload_i32(&P->d_offa, offa, device)) ||
        (st = upload_i32(&P->d_offb, offb, device))) {
        return st;   // P's destructor frees what was uploaded
    }
    if (c.plans.size() >= DiaCache::CAP) {
        auto lru = c.plans.begin();
        for (auto j = c.plans.begin(); j != c.plans.end(); ++j)
            if (j->second.second < lru->second.second) lru = j;
        c.plans.erase(lru);
    }
    c.plans[key] = {P, ++c.tick};
    *out = P;
    return IAS_SUCCESS;
}
// two timing events per (thread, device), created once
void dia_events(int device, hipEvent_t *e0, hipEvent_t *e1) {
    thread_local std::map<int, std::pair<hipEvent_t, hipEvent_t>> evs;
    auto it = evs.find(device);
    if (it == evs.end()) {
        hipEvent_t a = nullptr, b = nullptr;
        if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) {
            *e0 = *e1 = nullptr;
            return;
        }
        it = evs.emplace(device, std::make_pair(a, b)).first;
    }
    *e0 = it->second.first;
    *e1 = it->second.second;
}
// Device-resident offsets of an `into` call: the plan of the last call with the
// same offset arrays (pointers, counts, shapes) is reused without reading the
// offsets back (a synchronous copy, ~a third of K1's 60 µs call); k_dia_meta
// checks them against the plan's on the device (DiaCheck) and the call is
// redone with the current offsets when they changed.  Per thread, as the
// host-mapped flag word the check writes.
struct DiaFast {
    std::map<std::vector<int64_t>, std::shared_ptr<const DiaPlan>> plans;
    std::map<int, std::pair<int32_t *, int32_t *>> flags;   // host and device address of the word
};
DiaFast &dia_fast() {
    thread_local DiaFast f;
    return f;
}
bool dia_flag(int device, int32_t **host, int32_t **dev) {
    auto &m = dia_fast().flags;
    auto it = m.find(device);
    if (it == m.end()) {
        void *p = nullptr, *d = nullptr;
        if (hipHostMalloc(&p, 64, hipHostMallocMapped) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
            (void)hipGetLastError();
            hipHostFree(p);
            return false;
        }
        it = m.emplace(device, std::make_pair((int32_t *)p, (int32_t *)d)).first;
    }
    *host = it->second.first;
    *dev = it->second.second;
    return true;
}
}  // namespace

// into: C is the caller's device DIA (capacity C->num_diagonals diagonals:
// diagonal_offsets of that many entries, diagonal_ind of rows + cols - 1, val
// of rows x capacity); C is written in place with num_diagonals = nd_C.
static ias_status dia_mul(const ias_dia *A, const ias_dia *B, ias_dia *C, const ias_opts *opts,
                          ias_report *rep, bool into) {
    if (!A || !B || !C) return IAS_ERROR_INVALID_ARGUMENT;
    if (!A->choice || !B->choice) return IAS_ERROR_INFEASIBLE;
    if (A->cols != B->rows) return IAS_ERROR_DIMENSION_MISMATCH;
    ias_opts o;
    ias_opts_default(&o);
    if (opts) o = *opts;
    if (rep) memset(rep, 0, sizeof *rep);
    const int device = o.device >= 0 ? o.device : (A->memory == IAS_MEMORY_DEVICE ? A->device : 0);
    const int out_mem = o.output_memory >= 0 ? o.output_memory : A->memory;
    HIPC(hipSetDevice(device));

    // offsets on the host (tiny)
    std::vector<int32_t> offa(A->num_diagonals), offb(B->num_diagonals);
    auto read_offsets = [&](const ias_dia *X, std::vector<int32_t> &h) -> ias_status {
        if (h.empty()) return IAS_SUCCESS;
        if (X->memory == IAS_MEMORY_DEVICE) return dev_copy_d2h(h.data(), X->diagonal_offsets, 4 * h.size(), X->device);
        memcpy(h.data(), X->diagonal_offsets, 4 * h.size());
        return IAS_SUCCESS;
    };
    std::shared_ptr<const DiaPlan> P;
    // into with device-resident offsets: the last such call's plan, checked on the device
    const bool fast = into && A->memory == IAS_MEMORY_DEVICE && B->memory == IAS_MEMORY_DEVICE &&
                      A->device == device && B->device == device && A->num_diagonals > 0 && B->num_diagonals > 0;
    const std::vector<int64_t> fkey{device, A->rows, A->cols, B->cols, A->num_diagonals, B->num_diagonals,
                                    (int64_t)(intptr_t)A->diagonal_offsets, (int64_t)(intptr_t)B->diagonal_offsets};
    int32_t *flag = nullptr, *dflag = nullptr;   // host / device address of the check's word
    if (fast) {
        auto it = dia_fast().plans.find(fkey);
        if (it != dia_fast().plans.end() && dia_flag(device, &flag, &dflag)) P = it->second;
    }
    auto plan_now = [&]() -> ias_status {   // from the offsets as they are now
        IAS_TRY(read_offsets(A, offa));
        if (B == A) offb = offa;
        else IAS_TRY(read_offsets(B, offb));
        IAS_TRY(dia_plan_get(offa, offb, A->rows, A->cols, B->cols, device, &P));
        if (fast) {
            auto &m = dia_fast().plans;
            if (m.size() >= 16) m.clear();
            m[fkey] = P;
        }
        return IAS_SUCCESS;
    };
    if (!P) IAS_TRY(plan_now());
  for (int attempt = 0;; ++attempt) {
    const int32_t ndc = (int32_t)P->offc.size();

    hipStream_t s = (hipStream_t)o.stream;
    bool own = false;
    if (!s && o.plan) s = (hipStream_t)((ias_plan *)o.plan)->stream;
    if (!s) {
        HIPC(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        own = true;
    }
    // Everything this call allocates is released on every exit path (after
    // its stream has drained): staging copies, and D unless handed to C.
    struct Cleanup {
        std::vector<void *> p;
        int dev;
        hipStream_t s;
        bool own;
        ias_dia *D = nullptr;
        ~Cleanup() {
            hipStreamSynchronize(s);
            for (void *x : p) dev_free(x, dev);
            if (D) ias_dia_free(D);
            if (own) hipStreamDestroy(s);
        }
    } cl{{}, device, s, own};
    auto stage = [&](const void *src, size_t bytes, int mem, int sdev, const void **out) -> ias_status {
        if (mem == IAS_MEMORY_DEVICE && sdev == device) {
            *out = src;
            return IAS_SUCCESS;
        }
        void *d = nullptr;
        IAS_TRY(dev_alloc(&d, bytes, device));
        cl.p.push_back(d);
        if (bytes) {
            if (mem == IAS_MEMORY_DEVICE) HIPC(hipMemcpy(d, src, bytes, hipMemcpyDeviceToDevice));
            else HIPC(hipMemcpy(d, src, bytes, hipMemcpyHostToDevice));
        }
        *out = d;
        return IAS_SUCCESS;
    };
    const void *da_val, *db_val;
    const size_t na = (size_t)A->rows * A->num_diagonals, nb = (size_t)B->rows * B->num_diagonals;
    IAS_TRY(stage(A->val, 8 * na, A->memory, A->device, &da_val));
    if (B == A) db_val = da_val;
    else IAS_TRY(stage(B->val, 8 * nb, B->memory, B->device, &db_val));

    ias_dia D{};
    D.rows = A->rows;
    D.cols = B->cols;
    D.num_diagonals = ndc;
    D.choice = 1;
    D.memory = IAS_MEMORY_DEVICE;
    D.device = device;
    const int64_t span = std::max<int64_t>(A->rows + B->cols - 1, 0);
    if (into) {
        if (C->num_diagonals < ndc && flag) {   // a reused plan: decide on the current offsets
            flag = nullptr;
            IAS_TRY(plan_now());
            continue;
        }
        if (C->num_diagonals < ndc) {
            set_last_error("C needs %d diagonals, capacity %d", ndc, C->num_diagonals);
            C->num_diagonals = ndc;
            return IAS_ERROR_INSUFFICIENT_CAPACITY;
        }
        D.diagonal_offsets = C->diagonal_offsets;
        D.diagonal_ind = C->diagonal_ind;
        D.val = C->val;
    } else {
        cl.D = &D;
        IAS_TRY(dev_alloc((void **)&D.diagonal_offsets, 4 * (size_t)ndc, device));
        IAS_TRY(dev_alloc((void **)&D.diagonal_ind, 4 * (size_t)span, device));
        IAS_TRY(dev_alloc((void **)&D.val, 8 * (size_t)A->rows * ndc, device));
    }

    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (rep) dia_events(device, &e0, &e1);
    if (e0) HIPC(hipEventRecord(e0, s));
    const int64_t n = A->rows * (int64_t)ndc;
    const int32_t nda = A->num_diagonals, ndb = B->num_diagonals, np = (int32_t)P->pja.size();
    if (span > 0 || ndc > 0) {
        const int64_t m = std::max<int64_t>(span, ndc);
        if (flag) *(volatile int32_t *)flag = 0;
        const dev::DiaCheck chk{A->diagonal_offsets, P->d_offa, nda, B->diagonal_offsets, P->d_offb, ndb,
                                flag ? dflag : nullptr};
        dev::k_dia_meta<<<(unsigned)((m + 255) / 256), 256, 0, s>>>(ndc, P->d_offc, A->rows, span,
                                                                    D.diagonal_offsets, D.diagonal_ind, chk);
    }
    if (ndc > 0) {
        if (n > 0) {
            const int32_t *t = P->d_tab;
            const int32_t lo_a = P->lo_a, span_a = P->span_a, lo_b = P->lo_b, span_b = P->span_b;
            const bool small = A->rows < (1ll << 30) && A->cols < (1ll << 30) && B->cols < (1ll << 30);
            int32_t tr = 64;
            auto tile_lds = [&](int32_t r) {
                return 8ull * ((uint64_t)r * nda + (uint64_t)(r + span_a) * ndb) + 4ull * (nda + ndb + ndc + 1 + 2 * np);
            };
            while (tile_lds(tr) > 65536 && tr > 16) tr /= 2;
            // MFMA for wide DENSE bands (measured: 65 contiguous diagonals, K1w,
            // 0.57 ms vs 5.5 ms for the tiled VALU kernel; 7 diagonals, K1, 54
            // vs 32 us): at least 256 diagonal pairs, and the 16-row tile's
            // dense blocks (16 x W_A x W_C products) at most 4x the band's
            // products (16 x nd_A x nd_B) — a band of widely spaced diagonals
            // (a 27-point stencil at offsets of +-n^2) would be almost all
            // padding — and its operands within one CU's LDS.  IAS_DIA_MFMA=0/1
            // forces either where the MFMA form is possible at all.
            const int64_t WA = 16 + (int64_t)span_a, WC = WA + span_b;
            const size_t mfma_lds = 8ull * (16ull * nda + (uint64_t)WA * ndb) + 4ull * P->maps.size();
            const bool mfma_ok = small && !P->maps.empty() && mfma_lds <= 160 * 1024;
            const char *mf = getenv("IAS_DIA_MFMA");
            const bool dense = (int64_t)nda * ndb >= 256 && WA * WC <= 4ll * nda * ndb;
            const bool use_mfma = mfma_ok && (mf ? *mf == '1' : dense);
            if (rep) rep->kernel = use_mfma ? IAS_DIA_KERNEL_MFMA
                                            : (small && tile_lds(tr) <= 65536 ? IAS_DIA_KERNEL_TILE : IAS_DIA_KERNEL_PAIRS);
            if (use_mfma) {
                const int32_t *m = P->d_maps;
                if (mfma_lds > 65536)
                    HIPC(hipFuncSetAttribute((const void *)dev::k_dia_mfma,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
                HIPC(hipMemsetAsync(D.val, 0, 8 * (size_t)n, s));
                dev::DiaMfmaArgs ma{(int32_t)A->rows, (int32_t)A->cols, (int32_t)B->cols, nda, ndb, ndc,
                                    lo_a, span_a, lo_b, span_b, P->lo_c, P->span_c,
                                    m, m + span_a + 1, m + span_a + span_b + 2,
                                    (const double *)da_val, (const double *)db_val, D.val,
                                    P->d_offa, P->d_offb, t, np};
                dev::k_dia_mfma<<<(unsigned)((A->rows + 15) / 16), 256, mfma_lds, s>>>(ma);
            } else if (small && tile_lds(tr) <= 65536) {
                const uint64_t magic = ((1ull << 32) + (uint64_t)ndc - 1) / (uint64_t)ndc;
                dev::DiaTileArgs ta{(int32_t)A->rows, (int32_t)A->cols, (int32_t)B->cols, nda, ndb, ndc, np,
                                    lo_a, span_a, tr, magic, P->d_offa, P->d_offb,
                                    (const double *)da_val, (const double *)db_val, t, D.val};
                dev::k_dia_tile<<<(unsigned)((A->rows + tr - 1) / tr), 256, tile_lds(tr), s>>>(ta);
            } else {
                dev::DiaPairs pr{t, t + P->pst.size(), t + P->pst.size() + P->pja.size()};
                dev::k_dia_mul<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(
                    A->rows, A->cols, B->cols, nda, P->d_offa, (const double *)da_val, ndb, P->d_offb,
                    (const double *)db_val, ndc, pr, D.val);
            }
        }
    }
    HIPC(hipGetLastError());
    if (e1) HIPC(hipEventRecord(e1, s));
    HIPC((hipError_t)host_wait(s));
    if (flag && *(volatile int32_t *)flag != 0 && attempt == 0) {   // the offsets changed: redo with theirs
        flag = nullptr;
        IAS_TRY(plan_now());
        continue;
    }
    if (rep) {
        float t = 0;
        if (e0 && e1) hipEventElapsedTime(&t, e0, e1);
        rep->ms_total = t;
        rep->ms_numeric = t;
        rep->flops = P->flops;
        rep->nnz_c = n;
    }
    if (into) {
        C->rows = D.rows;
        C->cols = D.cols;
        C->num_diagonals = ndc;
        C->choice = 1;
    } else if (out_mem == IAS_MEMORY_HOST) {
        ias_dia H{};
        IAS_TRY(ias_dia_copy(&D, &H, IAS_MEMORY_HOST, 0));
        *C = H;   // D is freed by the cleanup
    } else {
        *C = D;
        cl.D = nullptr;
    }
    return IAS_SUCCESS;
  }
}

extern "C" ias_status ias_dia_mul_dia(const ias_dia *A, const ias_dia *B, ias_dia *C,
                                      const ias_opts *opts, ias_report *rep) {
    return dia_mul(A, B, C, opts, rep, false);
}

// [p, p + a) and [q, q + b) share a byte
static bool overlaps(const void *p, size_t a, const void *q, size_t b) {
    if (!p || !q || a == 0 || b == 0) return false;
    const uintptr_t x = (uintptr_t)p, y = (uintptr_t)q;
    return x < y + b && y < x + a;
}

extern "C" ias_status ias_dia_mul_dia_into(const ias_dia *A, const ias_dia *B, ias_dia *C,
                                           const ias_opts *opts, ias_report *rep) {
    if (!A || !B || !C || C->memory != IAS_MEMORY_DEVICE || C->num_diagonals < 0 || !C->diagonal_ind ||
        (C->num_diagonals > 0 && (!C->diagonal_offsets || !C->val)) || A->num_diagonals < 0 ||
        B->num_diagonals < 0 || A->rows < 0 || A->cols < 0 || B->cols < 0)
        return IAS_ERROR_INVALID_ARGUMENT;
    // C is written in place while A and B are read: no array of C may share
    // memory with one of theirs (C = A would race the kernel's reads)
    const size_t cr = (size_t)A->rows, ccols = (size_t)B->cols;
    const size_t c_bytes[3] = {8 * cr * (size_t)C->num_diagonals, 4 * (size_t)C->num_diagonals,
                               4 * (cr + ccols > 0 ? cr + ccols - 1 : 0)};
    const void *c_arr[3] = {C->val, C->diagonal_offsets, C->diagonal_ind};
    for (const ias_dia *X : {A, B}) {
        const size_t xr = (size_t)X->rows, xc = (size_t)X->cols;
        const size_t x_bytes[3] = {8 * xr * (size_t)X->num_diagonals, 4 * (size_t)X->num_diagonals,
                                   4 * (xr + xc > 0 ? xr + xc - 1 : 0)};
        const void *x_arr[3] = {X->val, X->diagonal_offsets, X->diagonal_ind};
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                if (overlaps(c_arr[i], c_bytes[i], x_arr[j], x_bytes[j])) {
                    set_last_error("ias_dia_mul_dia_into: C's arrays overlap an operand's");
                    return IAS_ERROR_INVALID_ARGUMENT;
                }
    }
    ias_opts o;
    ias_opts_default(&o);
    if (opts) o = *opts;
    o.device = C->device;
    return dia_mul(A, B, C, &o, rep, true);
}

extern "C" ias_status ias_dia_mul_dia_ndiag(const ias_dia *A, const ias_dia *B, int32_t *nd_c) {
    if (!A || !B || !nd_c || A->num_diagonals < 0 || B->num_diagonals < 0 ||
        (A->num_diagonals > 0 && !A->diagonal_offsets) || (B->num_diagonals > 0 && !B->diagonal_offsets))
        return IAS_ERROR_INVALID_ARGUMENT;
    if (!A->choice || !B->choice) return IAS_ERROR_INFEASIBLE;   // as dia_mul
    if (A->cols != B->rows) return IAS_ERROR_DIMENSION_MISMATCH;
    std::vector<int32_t> offa(A->num_diagonals), offb(B->num_diagonals);
    for (auto xo : {std::make_pair(A, &offa), std::make_pair(B, &offb)}) {
        std::vector<int32_t> &h = *xo.second;
        if (h.empty()) continue;
        if (xo.first->memory == IAS_MEMORY_DEVICE)
            IAS_TRY(dev_copy_d2h(h.data(), xo.first->diagonal_offsets, 4 * h.size(), xo.first->device));
        else
            memcpy(h.data(), xo.first->diagonal_offsets, 4 * h.size());
    }
    std::vector<int32_t> offc, pst, pja, pkb;
    dia_plan(offa.data(), (int32_t)offa.size(), offb.data(), (int32_t)offb.size(), A->rows, A->cols, B->cols,
             offc, pst, pja, pkb);
    *nd_c = (int32_t)offc.size();
    return IAS_SUCCESS;
}
