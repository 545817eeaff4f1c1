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
        if (OP == 7) h ^= atomicCAS(&t32[s], 0u, h);   // result feeds the next address
        if (OP == 8) h ^= t32[s];                        // dependent read chain
    }
    __syncthreads();
    if (acc == 12345) sink[0] = acc + t32[threadIdx.x];
}

// hash-insert probe: each 64-lane team (one wave) inserts N random keys into
// its own table of S = 2N slots (load 0.5), K keys per lane per step, the way
// the symbolic pass does; MODE 0: one key at a time (CAS loop then min),
// MODE 1: K CASes in flight then resolve.  Reports inserts per clock per CU.
template <int K, int MODE, int F>
__global__ __launch_bounds__(256) void hash_ins(int rows, int n, unsigned long long *sink) {
    extern __shared__ uint32_t sm[];
    const int w = threadIdx.x / 64, lane = threadIdx.x & 63;
    const uint32_t S = F * n;
    uint32_t *key = sm + w * 2 * S, *minp = key + S;
    int created = 0;
    for (int r = blockIdx.x; r < rows; r += gridDim.x) {
        for (uint32_t s = lane; s < S; s += 64) { key[s] = 0xFFFFFFFFu; minp[s] = 0xFFFFFFFFu; }
        __builtin_amdgcn_wave_barrier();
        for (int p0 = 0; p0 < n; p0 += 64 * K) {
            uint32_t c[K], pos[K];
            bool pend[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const uint32_t p = p0 + k * 64 + lane;
                pend[k] = p < (uint32_t)n;
                c[k] = (p * 0x9E3779B1u + r * 0x85EBCA6Bu) & 0x7FFFFFF;
                pos[k] = (uint32_t)(((uint64_t)(c[k] * 0x9E3779B1u) * S) >> 32);
            }
            if (MODE == 0 || MODE == 2) {
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    if (!pend[k]) continue;
                    uint32_t s = pos[k];
                    while (true) {
                        if (MODE == 2) {   // read first: CAS only an empty slot
                            const uint32_t r0 = key[s];
                            if (r0 == c[k]) { atomicMin(&minp[s], p0 + k * 64 + lane); break; }
                            if (r0 != 0xFFFFFFFFu) { s = s + 1 == S ? 0 : s + 1; continue; }
                        }
                        const uint32_t v = atomicCAS(&key[s], 0xFFFFFFFFu, c[k]);
                        if (v == 0xFFFFFFFFu || v == c[k]) { created += v == 0xFFFFFFFFu; atomicMin(&minp[s], p0 + k * 64 + lane); break; }
                        s = s + 1 == S ? 0 : s + 1;
                    }
                }
            } else {
                while (true) {
                    uint32_t v[K];
#pragma unroll
                    for (int k = 0; k < K; ++k) if (pend[k]) v[k] = atomicCAS(&key[pos[k]], 0xFFFFFFFFu, c[k]);
                    bool again = false;
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        if (!pend[k]) continue;
                        if (v[k] == 0xFFFFFFFFu || v[k] == c[k]) { created += v[k] == 0xFFFFFFFFu; atomicMin(&minp[pos[k]], p0 + k * 64 + lane); pend[k] = false; }
                        else { pos[k] = pos[k] + 1 == S ? 0 : pos[k] + 1; again = true; }
                    }
                    if (!again) break;
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (created == -1) sink[0] = created;
}

// dependent LDS CAS chain latency vs waves per CU (one block of `threads` per CU)
__global__ void cas_chain(int iters, unsigned long long *sink, unsigned long long *cyc) {
    __shared__ uint32_t t[8192];
    for (int i = threadIdx.x; i < 8192; i += blockDim.x) t[i] = 0;
    __syncthreads();
    uint32_t h = threadIdx.x * 0x9E3779B1u + 12345u;
    const unsigned long long t0 = wall_clock64();
    for (int it = 0; it < iters; ++it) {
        const uint32_t s = (h >> 7) & 8191u;
        const uint32_t v = atomicCAS(&t[s], 0u, h | 1u);
        h = h * 1664525u + 1013904223u + v;
    }
    const unsigned long long t1 = wall_clock64();
    if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
    if (h == 7) sink[0] = h;
}

int main() {
    unsigned long long *sink;
    hipMalloc(&sink, 8);
    int dev = 0, cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const char *names[] = {"atomicCAS u32 (rtn)", "atomicMin u32 (no rtn)", "atomicAdd u32 (rtn)",
                           "atomicCAS u64 (rtn)", "read u32", "write u32", "atomicOr u32 (no rtn)",
                           "atomicCAS dependent", "read dependent"};
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int iters = 4096;
    for (int op = 0; op < 9; ++op) {
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
                case 7: lds_op<7><<<grid, 1024>>>(iters, sink); break;
                case 8: lds_op<8><<<grid, 1024>>>(iters, sink); break;
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
    {
        unsigned long long *cyc;
        hipMalloc(&cyc, 8);
        for (int thr : {64, 256, 512, 1024}) {
            const int iters = 2000;
            cas_chain<<<cus, thr>>>(iters, sink, cyc);
            cas_chain<<<cus, thr>>>(iters, sink, cyc);
            unsigned long long h;
            hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
            printf("dependent CAS chain, %2d waves/CU: %.0f ns per CAS (%.0f clocks at 2.4 GHz)\n", thr / 64,
                   h * 10.0 / iters, h * 10.0 / iters * 2.4);
        }
    }
    for (int n : {64, 512, 2048}) {
        for (int mode = 0; mode < 3; ++mode) {
            for (int F : {2, 4}) {
                const int rows = 256 * 64;
                const size_t lds = 4 * 2 * F * n * 4;   // 4 waves x (key + minp) x S
                if (lds > 160 * 1024) continue;
                for (int rep = 0; rep < 2; ++rep) {
                    hipEventRecord(a);
                    if (mode == 0 && F == 2) hash_ins<4, 0, 2><<<cus * 4, 256, lds>>>(rows, n, sink);
                    if (mode == 1 && F == 2) hash_ins<4, 1, 2><<<cus * 4, 256, lds>>>(rows, n, sink);
                    if (mode == 2 && F == 2) hash_ins<4, 2, 2><<<cus * 4, 256, lds>>>(rows, n, sink);
                    if (mode == 0 && F == 4) hash_ins<4, 0, 4><<<cus * 4, 256, lds>>>(rows, n, sink);
                    if (mode == 1 && F == 4) hash_ins<4, 1, 4><<<cus * 4, 256, lds>>>(rows, n, sink);
                    if (mode == 2 && F == 4) hash_ins<4, 2, 4><<<cus * 4, 256, lds>>>(rows, n, sink);
                    hipEventRecord(b);
                    hipEventSynchronize(b);
                }
                float ms;
                hipEventElapsedTime(&ms, a, b);
                const double ins = (double)rows * 4 * n;   // 4 waves per block each a row
                printf("hash insert n=%4d S=%dn mode %d: %.2f inserts/clk/CU\n", n, F, mode,
                       ins / (ms * 1e-3) / cus / 2.4e9);
            }
        }
    }
    return 0;
}
