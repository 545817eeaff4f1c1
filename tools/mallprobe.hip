// mallprobe.hip — does a streamed output evict a gathered table from the
// Infinity Cache, and does any store policy or output allocation avoid it?
// The shape of k_num2: lanes gather B-row-shaped runs (20
// consecutive entries of a 4-byte column array and an 8-byte value array,
// a 250 MB table like K3''s B) and write every gathered item once, in order,
// as 16-byte stores (C).  Per variant: the gather+store launch, then a
// gather-only launch of the same table — its time says whether the table
// stayed resident behind the stores.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mallprobe.hip -o build_tim/mallprobe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#pragma clang diagnostic ignored "-Wunused-result"

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e = (x);                                                   \
        if (e != hipSuccess) {                                                \
            printf("%s: %s\n", #x, hipGetErrorString(e));                     \
            return 1;                                                         \
        }                                                                     \
    } while (0)

constexpr int RUN = 20;
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint64_t item_addr(uint64_t g, uint64_t n) {
    const uint64_t run = g / RUN;
    const uint32_t h = (uint32_t)(run * 0x9E3779B97F4A7C15ull >> 32);
    const uint64_t base = ((uint64_t)h * (uint64_t)(n - RUN)) >> 32;
    return base + (uint32_t)(g - run * RUN);
}

// POL: 0 no store (sink), 1 plain, 2 nontemporal builtin, 3 buffer store
// with cache-policy bits AUX (sc0 = 1, nt = 2, sc1 = 16); GATHER = false:
// the stores alone (values from the item index).  A wave takes tiles of 256
// items; every store instruction writes 1 KB contiguous (lane l: 16 bytes at
// 16 l): the columns of items 4l..4l+3, the values of items 2l, 2l+1 and of
// 128+2l, 128+2l+1 — whole lines, as k_num2 stages them.
template <int POL, int AUX, bool GATHER>
__global__ __launch_bounds__(256) void probe(const int32_t *col, const double *val, uint64_t n, uint64_t tiles,
                                              int32_t *oc, double *ov, unsigned long long *sink) {
    const int lane = threadIdx.x & 63;
    const uint64_t wv = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    constexpr int K = 2;   // tiles per wave in flight
    __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(oc, 0, 0x7fffffff, 0x00020000);
    __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(ov, 0, 0x7fffffff, 0x00020000);
    int64_t acc = 0;
    for (uint64_t t0 = wv; t0 < tiles; t0 += nw * K) {
        int32_t c[K][4];
        double v[K][4];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t t = t0 + (uint64_t)k * nw;
            const uint64_t b = (t < tiles ? t : 0) * 256;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint64_t gc = b + 4 * lane + e;
                const uint64_t gv = b + (e < 2 ? 2 * lane + e : 128 + 2 * lane + e - 2);
                if (GATHER) {
                    c[k][e] = col[item_addr(gc, n)];
                    v[k][e] = val[item_addr(gv, n)];
                } else {
                    c[k][e] = (int32_t)gc;
                    v[k][e] = (double)gv;
                }
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t t = t0 + (uint64_t)k * nw;
            if (t >= tiles) continue;
            const i32x4 xc = {c[k][0], c[k][1], c[k][2], c[k][3]};
            const f64x2 xv0 = {v[k][0], v[k][1]}, xv1 = {v[k][2], v[k][3]};
            int32_t *pc = oc + t * 256 + 4 * lane;
            double *pv0 = ov + t * 256 + 2 * lane, *pv1 = pv0 + 128;
            if (POL == 0) {
                acc += c[k][0] + c[k][1] + c[k][2] + c[k][3] + (int64_t)(v[k][0] + v[k][1] + v[k][2] + v[k][3]);
            } else if (POL == 1) {
                *(i32x4 *)pc = xc;
                *(f64x2 *)pv0 = xv0;
                *(f64x2 *)pv1 = xv1;
            } else if (POL == 2) {
                __builtin_nontemporal_store(xc, (i32x4 *)pc);
                __builtin_nontemporal_store(xv0, (f64x2 *)pv0);
                __builtin_nontemporal_store(xv1, (f64x2 *)pv1);
            } else {
                // byte offsets within 2 GB: the output region wraps (the bytes
                // still stream past the caches)
                const uint32_t oc_b = (uint32_t)((t * 1024 + 16 * lane) & 0x7fffffffull);
                const uint32_t ov_b = (uint32_t)((t * 2048 + 16 * lane) & 0x7fffffffull);
                typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
                __builtin_amdgcn_raw_buffer_store_b128(*(const u32x4 *)&xc, rc, oc_b, 0, AUX);
                __builtin_amdgcn_raw_buffer_store_b128(*(const u32x4 *)&xv0, rv, ov_b, 0, AUX);
                __builtin_amdgcn_raw_buffer_store_b128(*(const u32x4 *)&xv1, rv, ov_b + 1024, 0, AUX);
            }
        }
    }
    if (acc == 0x7fffffffffffll) sink[0] = (unsigned long long)acc;
}

struct Env {
    const int32_t *col;
    const double *val;
    uint64_t n, tiles;
    int32_t *oc;
    double *ov;
    unsigned long long *sink;
    hipEvent_t a, b;
};

template <int POL, int AUX, bool GATHER>
float run(const Env &e, int32_t *oc, double *ov) {
    const int grid = 256 * 8 / 4;   // 8 waves per CU
    hipEventRecord(e.a);
    probe<POL, AUX, GATHER><<<grid, 256>>>(e.col, e.val, e.n, e.tiles, oc, ov, e.sink);
    hipEventRecord(e.b);
    hipEventSynchronize(e.b);
    float ms;
    hipEventElapsedTime(&ms, e.a, e.b);
    return ms;
}

template <int POL, int AUX>
void variant(const Env &e, const char *name, int32_t *oc, double *ov) {
    // warm: the table into the caches by a gather-only pass
    run<0, 0, true>(e, oc, ov);
    const float g0 = run<0, 0, true>(e, oc, ov);
    const float t1 = run<POL, AUX, true>(e, oc, ov);
    const float after = run<0, 0, true>(e, oc, ov);
    const float t2 = run<POL, AUX, true>(e, oc, ov);
    const float so = run<POL, AUX, false>(e, oc, ov);
    const double items = 256.0 * e.tiles;
    printf("%-34s gather-only %.3f ms | gather+store %.3f / %.3f ms (%.0f GB/s stored) | gather-only after %.3f ms | "
           "store-only %.3f ms (%.0f GB/s)\n",
           name, g0, t1, t2, items * 12 / t2 / 1e6, after, so, items * 12 / so / 1e6);
}

int main() {
    const uint64_t n = 21000000;   // B of K3': 84 MB columns + 168 MB values
    const uint64_t groups = 1ull << 26;   // 2^28 items: 3.2 GB of output, one k_num2 launch's C
    int32_t *col, *oc, *ocu, *ocf;
    double *val, *ov, *ovu, *ovf;
    unsigned long long *sink;
    CK(hipMalloc(&col, n * 4));
    CK(hipMalloc(&val, n * 8));
    CK(hipMemset(col, 1, n * 4));
    CK(hipMemset(val, 0, n * 8));
    CK(hipMalloc(&oc, groups * 16));
    CK(hipMalloc(&ov, groups * 32));
    CK(hipMalloc(&sink, 16));
    CK(hipExtMallocWithFlags((void **)&ocu, groups * 16, hipDeviceMallocUncached));
    CK(hipExtMallocWithFlags((void **)&ovu, groups * 32, hipDeviceMallocUncached));
    CK(hipExtMallocWithFlags((void **)&ocf, groups * 16, hipDeviceMallocFinegrained));
    CK(hipExtMallocWithFlags((void **)&ovf, groups * 32, hipDeviceMallocFinegrained));
    Env e{col, val, n, groups / 64, oc, ov, sink, {}, {}};
    hipEventCreate(&e.a);
    hipEventCreate(&e.b);
    printf("# table %.0f MB (RUN %d), output %.2f GB per launch, 8 waves/CU\n", n * 12 / 1e6, RUN,
           groups * 48 / 1e9);
    {
        // gather-only by table size: where a 252 MB table is served from
        const uint64_t nb = 170000000;   // 2 GB
        int32_t *bc;
        double *bv;
        CK(hipMalloc(&bc, nb * 4));
        CK(hipMalloc(&bv, nb * 8));
        CK(hipMemset(bc, 1, nb * 4));
        CK(hipMemset(bv, 0, nb * 8));
        for (uint64_t m : {300000ull, 2600000ull, 10000000ull, 21000000ull, 40000000ull, 170000000ull}) {
            Env f = e;
            f.col = bc;
            f.val = bv;
            f.n = m;
            run<0, 0, true>(f, oc, ov);
            const float t = run<0, 0, true>(f, oc, ov);
            printf("gather-only, table %6.0f MB: %.3f ms (%.0f GB/s of items)\n", m * 12 / 1e6, t,
                   256.0 * f.tiles * 12 / t / 1e6);
        }
        CK(hipFree(bc));
        CK(hipFree(bv));
    }
    variant<1, 0>(e, "plain", oc, ov);
    variant<2, 0>(e, "nontemporal builtin", oc, ov);
    variant<3, 0>(e, "buffer aux 0", oc, ov);
    variant<3, 2>(e, "buffer nt", oc, ov);
    variant<3, 1>(e, "buffer sc0", oc, ov);
    variant<3, 16>(e, "buffer sc1", oc, ov);
    variant<3, 17>(e, "buffer sc0 sc1", oc, ov);
    variant<3, 3>(e, "buffer sc0 nt", oc, ov);
    variant<3, 18>(e, "buffer sc1 nt", oc, ov);
    variant<3, 19>(e, "buffer sc0 sc1 nt", oc, ov);
    variant<1, 0>(e, "plain, uncached output", ocu, ovu);
    variant<2, 0>(e, "nontemporal, uncached output", ocu, ovu);
    variant<1, 0>(e, "plain, fine-grained output", ocf, ovf);
    variant<2, 0>(e, "nontemporal, fine-grained output", ocf, ovf);
    return 0;
}
