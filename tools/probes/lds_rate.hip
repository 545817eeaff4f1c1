// LDS op-rate probe: random-address ds ops (32 KiB table per workgroup),
// 1024 workgroups x 256 threads, ITER ops per lane.  Prints lane-ops per clock
// per CU for: plain read, plain write, CAS with return, min without return,
// add with return.  Build: hipcc --offload-arch=gfx950 -O3 lds_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int N = 8192;   // table words
constexpr int ITER = 4096;

template <int OP>
__global__ __launch_bounds__(256) void k(unsigned *out, unsigned seed) {
    __shared__ unsigned tab[N];
    for (int i = threadIdx.x; i < N; i += 256) tab[i] = 0xFFFFFFFFu;
    __syncthreads();
    unsigned x = seed ^ (blockIdx.x * 256 + threadIdx.x) * 0x9E3779B1u, acc = 0;
    for (int it = 0; it < ITER; ++it) {
        x = x * 1664525u + 1013904223u;
        const unsigned a = (x >> 8) & (N - 1);
        if constexpr (OP == 0) acc += tab[a];
        else if constexpr (OP == 1) tab[a] = x;
        else if constexpr (OP == 2) acc += atomicCAS(&tab[a], 0xFFFFFFFFu, x);
        else if constexpr (OP == 3) atomicMin(&tab[a], x);
        else if constexpr (OP == 4) acc += atomicAdd(&tab[a], 1u);
        else if constexpr (OP == 5) { acc += tab[a]; tab[(a * 7) & (N - 1)] = acc; }   // read then write
        else if constexpr (OP == 6) acc += atomicCAS(&tab[a & ~3u], 0xFFFFFFFFu, x);   // 16 banks only
        else if constexpr (OP == 7) atomicMin(&tab[a & ~3u], x);
        else if constexpr (OP == 8) { const uint4 q = ((const uint4 *)tab)[a >> 2]; acc += q.x ^ q.y ^ q.z ^ q.w; }
        else if constexpr (OP == 9) { const uint2 q = ((const uint2 *)tab)[a >> 1]; acc += q.x ^ q.y; }
        else if constexpr (OP == 10) {   // bucket insert chain: b128 read, CAS, min
            const uint4 q = ((const uint4 *)tab)[a >> 2];
            const unsigned v = atomicCAS(&tab[a & ~3u], q.x == 0xFFFFFFFFu ? 0xFFFFFFFFu : q.x, x);
            atomicMin(&tab[(a & ~3u) ^ 1u], v);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = acc + tab[x & (N - 1)];
}

template <int OP>
void run(const char *name, unsigned *d) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    const int blocks = 256 * 8;
    k<OP><<<blocks, 256>>>(d, 1);
    hipEventRecord(a);
    k<OP><<<blocks, 256>>>(d, 2);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    int clk = 0, cus = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);   // kHz
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const double ops = (double)blocks * 256 * ITER;
    const double clocks = ms * 1e-3 * clk * 1e3;
    printf("%-22s %8.3f ms  %8.2f lane-ops/clk/CU  (%.1f Gops/s)\n", name, ms, ops / clocks / cus, ops / ms / 1e6);
}

int main() {
    unsigned *d;
    hipMalloc(&d, 1 << 20);
    run<0>("read", d);
    run<1>("write", d);
    run<2>("cas_rtn", d);
    run<3>("min_noret", d);
    run<4>("add_rtn", d);
    run<5>("read+write", d);
    run<6>("cas_rtn slot0-of-4", d);
    run<7>("min slot0-of-4", d);
    run<8>("read_b128", d);
    run<9>("read_b64", d);
    run<10>("b128+cas+min chain", d);
    return 0;
}
