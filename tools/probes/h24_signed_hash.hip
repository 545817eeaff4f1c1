// Compile-only reproducer of round 5's h24 ISA (profiles/r05/h24_sym3_filter_isa.txt):
//   v_lshrrev_b32_sdwa vX, vS, sext(vH) ... src1_sel:WORD_1
//   v_and_b32 vX, 0x1ffffffc, vX
//   v_lshlrev_b32_sdwa vB, sext(vH), v1 ... src0_sel:WORD_1
//   ds_or_rtn_b32 ...
// k_signed keeps a 24-bit hash product in an int: a product >= 2^31 (the hash's
// top 16 bits times a filter range above 2^15 bits) is negative, its high half
// is taken by an arithmetic shift, and the word index (uint32_t)b >> 5 lands far
// beyond the LDS allocation — exactly what C's semantics ask for, so the ISA is
// a correct compilation of a source bug, not a miscompile.  k_unsigned, the
// same hash in uint32_t, compiles to a logical shift (no sext).  Checked by
// tests/test_h24_repro.py (hipcc --cuda-device-only -S; no GPU).
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void k_signed(const int32_t *in, uint32_t *out, int32_t n) {
    __shared__ uint32_t f1[4096];
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) f1[i] = 0;
    __syncthreads();
    const int32_t c = in[blockIdx.x * blockDim.x + threadIdx.x];
    const int32_t h = __mul24((int32_t)(((uint32_t)c * 0x9E3779B1u) >> 16), n);
    const int32_t b = h >> 16;
    out[blockIdx.x * blockDim.x + threadIdx.x] = atomicOr(&f1[(uint32_t)b >> 5], 1u << (b & 31));
}

__global__ void k_unsigned(const int32_t *in, uint32_t *out, uint32_t n) {
    __shared__ uint32_t f1[4096];
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) f1[i] = 0;
    __syncthreads();
    const int32_t c = in[blockIdx.x * blockDim.x + threadIdx.x];
    const uint32_t h = __umul24(((uint32_t)c * 0x9E3779B1u) >> 16, n);
    const uint32_t b = h >> 16;
    out[blockIdx.x * blockDim.x + threadIdx.x] = atomicOr(&f1[b >> 5], 1u << (b & 31));
}
