// membench.hip — memory-system probes that shape the SpGEMM kernels
// (DESIGN.md §4): dependent-load latency vs footprint (L2 / Infinity Cache /
// HBM / translation reach), and the rate of B-row-shaped gathers (runs of
// ~20 consecutive 4-byte columns at random row starts) under full occupancy.
// Build: hipcc --offload-arch=gfx950 -O3 tools/membench.hip -o build_tim/membench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>
#pragma clang diagnostic ignored "-Wunused-result"

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e = (x);                                                   \
        if (e != hipSuccess) {                                                \
            printf("%s: %s\n", #x, hipGetErrorString(e));                     \
            return 1;                                                         \
        }                                                                     \
    } while (0)

// one lane chases a random cycle: average latency per dependent load
__global__ void chase(const uint32_t *next, int steps, uint32_t start, unsigned long long *out) {
    uint32_t i = start;
    const unsigned long long t0 = wall_clock64();
    for (int s = 0; s < steps; ++s) i = next[i];
    const unsigned long long t1 = wall_clock64();
    out[0] = t1 - t0;
    out[1] = i;
}

// every lane gathers runs: item g -> run r = hash(g / RUN), element g % RUN
template <int RUN, int K>
__global__ void gather(const int32_t *col, uint64_t n, uint64_t items, unsigned long long *sink) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    int32_t acc = 0;
    for (uint64_t g0 = tid; g0 < items; g0 += stride * K) {
        int32_t v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t g = g0 + (uint64_t)k * stride;
            const uint64_t run = g / RUN;
            const uint32_t h = (uint32_t)(run * 0x9E3779B97F4A7C15ull >> 32);
            const uint64_t base = ((uint64_t)h * (uint64_t)(n - RUN)) >> 32;   // multiply-shift range
            v[k] = col[base + (uint32_t)(g - run * RUN)];
        }
#pragma unroll
        for (int k = 0; k < K; ++k) acc += v[k];
    }
    if (acc == 0x7fffffff) sink[0] = acc;
}

// gather runs and store each item contiguously (the expansion pattern);
// PIPE: the loads of the next step are issued before this step's stores
template <int RUN, int K, bool PIPE>
__global__ void gather_store(const int32_t *col, uint64_t n, uint64_t items, int32_t *out) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    auto addr = [&](uint64_t g) {
        const uint64_t run = g / RUN;
        const uint32_t h = (uint32_t)(run * 0x9E3779B97F4A7C15ull >> 32);
        const uint64_t base = ((uint64_t)h * (uint64_t)(n - RUN)) >> 32;
        return base + (uint32_t)(g - run * RUN);
    };
    int32_t v[K], w[K];
    uint64_t g0 = tid;
    if (PIPE) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t g = g0 + (uint64_t)k * stride;
            v[k] = g < items ? col[addr(g)] : 0;
        }
    }
    for (; g0 < items; g0 += stride * K) {
        if (PIPE) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const uint64_t g = g0 + stride * K + (uint64_t)k * stride;
                w[k] = g < items ? col[addr(g)] : 0;
            }
        } else {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const uint64_t g = g0 + (uint64_t)k * stride;
                v[k] = col[addr(g)];
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t g = g0 + (uint64_t)k * stride;
            if (g < items) out[g] = v[k];
        }
        if (PIPE) {
#pragma unroll
            for (int k = 0; k < K; ++k) v[k] = w[k];
        }
    }
}

int main() {
    unsigned long long *d_out;
    CK(hipMalloc(&d_out, 16));
    printf("# dependent-load latency (one lane, random cycle over the footprint)\n");
    for (size_t mb : {1, 4, 16, 64, 128, 256, 512, 1024, 4096}) {
        const size_t n = mb * (1u << 20) / 4;
        std::vector<uint32_t> perm(n), next(n);
        // random cycle with a 256-byte stride granularity (distinct lines)
        const size_t step = 64;
        const size_t m = n / step;
        std::vector<uint32_t> ord(m);
        for (size_t i = 0; i < m; ++i) ord[i] = (uint32_t)(i * step);
        std::mt19937_64 rng(1);
        for (size_t i = m - 1; i > 0; --i) std::swap(ord[i], ord[rng() % (i + 1)]);
        for (size_t i = 0; i < m; ++i) next[ord[i]] = ord[(i + 1) % m];
        uint32_t *d;
        CK(hipMalloc(&d, n * 4));
        CK(hipMemcpy(d, next.data(), n * 4, hipMemcpyHostToDevice));
        const int steps = 20000;
        chase<<<1, 1>>>(d, 2000, ord[0], d_out);   // warm
        chase<<<1, 1>>>(d, steps, ord[0], d_out);
        unsigned long long h[2];
        CK(hipMemcpy(h, d_out, 16, hipMemcpyDeviceToHost));
        printf("footprint %5zu MB: %.0f ns per load\n", mb, h[0] * 10.0 / steps);
        CK(hipFree(d));
    }
    printf("# B-row gathers (runs of 20 x 4 B at random starts), 4 B per item\n");
    for (size_t mb : {4, 84, 336, 2048}) {
        const uint64_t n = mb * (1ull << 20) / 4;
        int32_t *d;
        CK(hipMalloc(&d, n * 4));
        CK(hipMemset(d, 1, n * 4));
        const uint64_t items = 1ull << 30;
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        for (int occ : {2, 8, 32}) {
            const int grid = 256 * occ / 4;   // 256-thread blocks = 4 waves
            gather<20, 8><<<grid, 256>>>(d, n, items, d_out);
            hipEventRecord(a);
            gather<20, 8><<<grid, 256>>>(d, n, items, d_out);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            printf("table %5zu MB, %2d waves/CU: %.1f G items/s (%.0f GB/s useful)\n", mb, occ,
                   items / ms / 1e6, items * 4.0 / ms / 1e6);
        }
        CK(hipFree(d));
    }
    printf("# gather + contiguous store (expansion pattern), 84 MB table\n");
    {
        const uint64_t n = 84ull * (1ull << 20) / 4;
        const uint64_t items = 1ull << 28;
        int32_t *d, *o;
        CK(hipMalloc(&d, n * 4));
        CK(hipMalloc(&o, items * 4));
        CK(hipMemset(d, 1, n * 4));
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        for (int occ : {8, 16, 32}) {
            const int grid = 256 * occ / 4;
            for (int pipe = 0; pipe < 2; ++pipe) {
                for (int rep = 0; rep < 2; ++rep) {
                    hipEventRecord(a);
                    if (pipe) gather_store<20, 8, true><<<grid, 256>>>(d, n, items, o);
                    else gather_store<20, 8, false><<<grid, 256>>>(d, n, items, o);
                    hipEventRecord(b);
                    hipEventSynchronize(b);
                }
                float ms;
                hipEventElapsedTime(&ms, a, b);
                printf("%2d waves/CU pipe %d: %.1f G items/s\n", occ, pipe, items / ms / 1e6);
            }
        }
    }
    return 0;
}
