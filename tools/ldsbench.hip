// ldsbench.hip — LDS operation throughput probes (hash-table inserts of the
// symbolic pass): random-address 32/64-bit atomics vs plain reads/writes,
// 16 waves per CU, per CU lane-operations per clock (clock from wall time).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#pragma clang diagnostic ignored "-Wunused-result"

constexpr int SLOTS = 8192;   // 32 KB of u32 / 64 KB of u64

template <int OP>
__global__ __launch_bounds__(1024) void lds_op(int iters, unsigned long long *sink) {
    __shared__ unsigned long long t64[SLOTS];
    uint32_t *t32 = (uint32_t *)t64;
    for (int i = threadIdx.x; i < SLOTS; i += blockDim.x) t64[i] = 0;
    __syncthreads();
    uint32_t h = threadIdx.x * 0x9E3779B1u + blockIdx.x * 0x85EBCA6Bu;
    unsigned long long acc = 0;
    for (int it = 0; it < iters; ++it) {
        h = h * 1664525u + 1013904223u;
        const uint32_t s = h >> 19;   // 0..8191
        if (OP == 0) acc += atomicCAS(&t32[s], 0u, h);
        if (OP == 1) atomicMin(&t32[s], h);
        if (OP == 2) acc += atomicAdd(&t32[s], 1u);
        if (OP == 3) acc += atomicCAS(&t64[s], 0ull, (unsigned long long)h);
        if (OP == 4) acc += t32[s];
        if (OP == 5) t32[s] = h;
        if (OP == 6) atomicOr(&t32[s], h);
    }
    __syncthreads();
    if (acc == 12345) sink[0] = acc + t32[threadIdx.x];
}

int main() {
    unsigned long long *sink;
    hipMalloc(&sink, 8);
    int dev = 0, cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const char *names[] = {"atomicCAS u32 (rtn)", "atomicMin u32 (no rtn)", "atomicAdd u32 (rtn)",
                           "atomicCAS u64 (rtn)", "read u32", "write u32", "atomicOr u32 (no rtn)"};
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int iters = 4096;
    for (int op = 0; op < 7; ++op) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a);
            const int grid = cus * 2;   // 2 x 1024 threads = 32 waves per CU
            switch (op) {
                case 0: lds_op<0><<<grid, 1024>>>(iters, sink); break;
                case 1: lds_op<1><<<grid, 1024>>>(iters, sink); break;
                case 2: lds_op<2><<<grid, 1024>>>(iters, sink); break;
                case 3: lds_op<3><<<grid, 1024>>>(iters, sink); break;
                case 4: lds_op<4><<<grid, 1024>>>(iters, sink); break;
                case 5: lds_op<5><<<grid, 1024>>>(iters, sink); break;
                case 6: lds_op<6><<<grid, 1024>>>(iters, sink); break;
            }
            hipEventRecord(b);
            hipEventSynchronize(b);
        }
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double ops = (double)cus * 2 * 1024 * iters;
        printf("%-24s %.2f lane-ops/clk/CU (at 2.4 GHz), %.1f G lane-ops/s\n", names[op],
               ops / (ms * 1e-3) / cus / 2.4e9, ops / (ms * 1e-3) / 1e9);
    }
    return 0;
}
