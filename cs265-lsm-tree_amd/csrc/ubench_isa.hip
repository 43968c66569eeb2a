// ubench_isa.hip — throughput of single VALU instructions on gfx950, to
// price rewrites of the hash / modulo arithmetic (tools/ubench.py isa).
// Each lane runs 8 independent dependency chains of the instruction.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CHAINS 8

#define DEF64(NAME, ASM)                                                               \
    __global__ void NAME(int iters, uint64_t *sink) {                                  \
        uint64_t x[CHAINS];                                                            \
        uint32_t y = threadIdx.x | 1;                                                  \
        for (int c = 0; c < CHAINS; c++) x[c] = threadIdx.x * 0x9E3779B97F4A7C15ull + c;\
        for (int i = 0; i < iters; i++) {                                              \
            _Pragma("unroll") for (int c = 0; c < CHAINS; c++) {                       \
                asm volatile(ASM : "+v"(x[c]) : "v"(y));                               \
            }                                                                          \
        }                                                                              \
        uint64_t a = 0;                                                                \
        for (int c = 0; c < CHAINS; c++) a ^= x[c];                                    \
        if (a == 0x12345) sink[0] = a;                                                 \
    }
#define DEF32(NAME, ASM)                                                               \
    __global__ void NAME(int iters, uint64_t *sink) {                                  \
        uint32_t x[CHAINS];                                                            \
        const uint32_t k = 0x27d4eb2du ^ (uint32_t)iters;                              \
        for (int c = 0; c < CHAINS; c++) x[c] = threadIdx.x * 0x9E3779B9u + c;         \
        for (int i = 0; i < iters; i++) {                                              \
            _Pragma("unroll") for (int c = 0; c < CHAINS; c++) {                       \
                asm volatile(ASM : "+v"(x[c]) : "s"(k));                               \
            }                                                                          \
        }                                                                              \
        uint32_t a = 0;                                                                \
        for (int c = 0; c < CHAINS; c++) a ^= x[c];                                    \
        if (a == 0x12345) sink[0] = a;                                                 \
    }

DEF64(k_mad_u64_u32, "v_mad_u64_u32 %0, vcc, %1, 5, %0")
DEF64(k_lshl_add_u64, "v_lshl_add_u64 %0, %0, 2, %0")
DEF64(k_lshlrev_b64, "v_lshlrev_b64 %0, 15, %0")
DEF64(k_lshrrev_b64, "v_lshrrev_b64 %0, 12, %0")
DEF64(k_add_u64, "v_lshl_add_u64 %0, %0, 0, %0")
DEF32(k_xor_b32, "v_xor_b32 %0, %1, %0")
DEF32(k_mul_lo_u32, "v_mul_lo_u32 %0, %0, %1")
DEF32(k_mul_hi_u32, "v_mul_hi_u32 %0, %0, %1")
DEF32(k_alignbit, "v_alignbit_b32 %0, %0, %1, 12")
DEF32(k_mad_u32_u24, "v_mad_u32_u24 %0, %0, %1, %0")
DEF32(k_add_u32, "v_add_u32 %0, %1, %0")
DEF32(k_lshl_add_u32, "v_lshl_add_u32 %0, %0, 3, %0")
DEF32(k_bitop3_xor3, "v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96")
DEF32(k_alignbit16, "v_alignbit_b32 %0, %0, %0, 16")

extern "C" int ubench_isa(int which, uint64_t *sink, int grid, int block, int iters, void *stream) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    switch (which) {
        case 0: k_mad_u64_u32<<<grid, block, 0, s>>>(iters, sink); break;
        case 1: k_lshl_add_u64<<<grid, block, 0, s>>>(iters, sink); break;
        case 2: k_lshlrev_b64<<<grid, block, 0, s>>>(iters, sink); break;
        case 3: k_lshrrev_b64<<<grid, block, 0, s>>>(iters, sink); break;
        case 4: k_add_u64<<<grid, block, 0, s>>>(iters, sink); break;
        case 5: k_xor_b32<<<grid, block, 0, s>>>(iters, sink); break;
        case 6: k_mul_lo_u32<<<grid, block, 0, s>>>(iters, sink); break;
        case 7: k_mul_hi_u32<<<grid, block, 0, s>>>(iters, sink); break;
        case 8: k_alignbit<<<grid, block, 0, s>>>(iters, sink); break;
        case 9: k_mad_u32_u24<<<grid, block, 0, s>>>(iters, sink); break;
        case 10: k_add_u32<<<grid, block, 0, s>>>(iters, sink); break;
        case 11: k_lshl_add_u32<<<grid, block, 0, s>>>(iters, sink); break;
        case 12: k_bitop3_xor3<<<grid, block, 0, s>>>(iters, sink); break;
        case 13: k_alignbit16<<<grid, block, 0, s>>>(iters, sink); break;
        default: return -22;
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// Semantics probe: v_lshl_add_u64 with immediate shifts 0..7 on n inputs
// (the CDNA3 ISA guide limits the shift to 0..4); out[8 * i + s].
template <int S>
__device__ uint64_t lshl_add_imm(uint64_t a, uint64_t b) {
    uint64_t r;
    asm volatile("v_lshl_add_u64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "i"(S), "v"(b));
    return r;
}
__global__ void k_lshl_add_check(const uint64_t *in, uint64_t *out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t a = in[2 * i], b = in[2 * i + 1];
    out[8 * i + 0] = lshl_add_imm<0>(a, b);
    out[8 * i + 1] = lshl_add_imm<1>(a, b);
    out[8 * i + 2] = lshl_add_imm<2>(a, b);
    out[8 * i + 3] = lshl_add_imm<3>(a, b);
    out[8 * i + 4] = lshl_add_imm<4>(a, b);
    out[8 * i + 5] = lshl_add_imm<5>(a, b);
    out[8 * i + 6] = lshl_add_imm<6>(a, b);
    out[8 * i + 7] = lshl_add_imm<7>(a, b);
}
extern "C" int ubench_lshl_add_check(const uint64_t *in, uint64_t *out, int n, void *stream) {
    k_lshl_add_check<<<(n + 255) / 256, 256, 0, reinterpret_cast<hipStream_t>(stream)>>>(in, out, n);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
