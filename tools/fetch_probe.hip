// fetch_probe.hip — calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE for the
// access shapes of k_num2 (MI355X_MICROARCH.md: FETCH_SIZE reads half the
// bytes of a 16-B-per-lane stream; other widths are uncalibrated).  Each
// kernel touches a known number of distinct bytes of a 4 GiB buffer (16x the
// Infinity Cache, so nothing is served on-die from an earlier kernel):
//   stream16 / stream8 / stream4: every byte once, 16 / 8 / 4 B per lane, coalesced;
//   runs4 / runs8: runs of R consecutive 4-B (8-B) elements at random
//     run starts (R = 32: a gathered B row of 32 entries, as k_num2's window);
//   write16 / write4: stores, 16 / 4 B per lane, coalesced.
// Printed: kernel, distinct bytes touched; rocprofv3 --pmc gives the counters.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/fetch_probe tools/fetch_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <typename T>
__global__ void k_stream(const T *__restrict__ a, size_t n, unsigned long long *sink) {
    T acc{};
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const T v = a[i];
        acc = acc + v;
    }
    if (*(volatile int *)&acc == 0x7fffffff) atomicAdd(sink, 1ull);
}
__global__ void k_stream16(const uint4 *__restrict__ a, size_t n, unsigned long long *sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x7fffffffu) atomicAdd(sink, 1ull);
}
// one wave per run: lanes read R consecutive elements at a random start
template <typename T, int R>
__global__ void k_runs(const T *__restrict__ a, const uint32_t *__restrict__ starts, size_t nruns,
                       unsigned long long *sink) {
    const size_t w = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) / 64;
    const int lane = threadIdx.x & 63;
    T acc{};
    for (size_t r = w; r < nruns; r += (size_t)gridDim.x * blockDim.x / 64)
        if (lane < R) acc = acc + a[(size_t)starts[r] * R + lane];
    if (*(volatile int *)&acc == 0x7fffffff) atomicAdd(sink, 1ull);
}
template <typename T>
__global__ void k_write(T *__restrict__ a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        __builtin_nontemporal_store(T{}, &a[i]);
}

int main() {
    const size_t bytes = 4ull << 30;
    char *buf;
    unsigned long long *sink;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&sink, 8));
    CK(hipMemset(buf, 1, bytes));
    const int grid = 256 * 16, block = 256;
    CK(hipDeviceSynchronize());
    k_stream16<<<grid, block>>>((const uint4 *)buf, bytes / 16, sink);
    CK(hipDeviceSynchronize());
    printf("stream16 %zu\n", bytes);
    k_stream<uint64_t><<<grid, block>>>((const uint64_t *)buf, bytes / 8, sink);
    CK(hipDeviceSynchronize());
    printf("stream8 %zu\n", bytes);
    k_stream<uint32_t><<<grid, block>>>((const uint32_t *)buf, bytes / 4, sink);
    CK(hipDeviceSynchronize());
    printf("stream4 %zu\n", bytes);
    // runs: distinct random runs (a permutation prefix), 1/4 of the buffer
    for (int es : {4, 8}) {
        const size_t run_bytes = 32ull * es, nall = bytes / run_bytes, nruns = nall / 4;
        std::vector<uint32_t> st(nall);
        for (size_t i = 0; i < nall; ++i) st[i] = (uint32_t)i;
        uint64_t x = 88172645463325252ull;
        for (size_t i = nall - 1; i > 0; --i) {   // Fisher-Yates, xorshift
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            std::swap(st[i], st[x % (i + 1)]);
        }
        uint32_t *dst;
        CK(hipMalloc(&dst, 4 * nruns));
        CK(hipMemcpy(dst, st.data(), 4 * nruns, hipMemcpyHostToDevice));
        if (es == 4) k_runs<uint32_t, 32><<<grid, block>>>((const uint32_t *)buf, dst, nruns, sink);
        else k_runs<uint64_t, 32><<<grid, block>>>((const uint64_t *)buf, dst, nruns, sink);
        CK(hipDeviceSynchronize());
        printf("runs%d %zu\n", es, nruns * run_bytes);
        CK(hipFree(dst));
    }
    k_write<u32x4><<<grid, block>>>((u32x4 *)buf, bytes / 16);
    CK(hipDeviceSynchronize());
    printf("write16 %zu\n", bytes);
    k_write<uint32_t><<<grid, block>>>((uint32_t *)buf, bytes / 4);
    CK(hipDeviceSynchronize());
    printf("write4 %zu\n", bytes);
    return 0;
}
