// mul_probe.hip — issue-rate probe of the integer multiplies the PCG64
// jump-ahead uses (diagnostic, not product code).  Each kernel runs ITER
// iterations of 8 independent instances of one instruction per lane (inline
// asm, so the compiler cannot fold them), over enough waves to fill every
// SIMD; the result is SIMD cycles per wave64 instruction at the given clock.
//   hipcc --offload-arch=gfx950 -O2 -o tools/mul_probe tools/mul_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITER 4096

#define K8(stmt) stmt(0) stmt(1) stmt(2) stmt(3) stmt(4) stmt(5) stmt(6) stmt(7)

__global__ void k_add(uint32_t *out, uint32_t seed) {
    uint32_t v[8];
    for (int i = 0; i < 8; i++) v[i] = threadIdx.x * 7 + i + seed;
    const uint32_t m = seed | 1;
    for (int it = 0; it < ITER; it++) {
#define S(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[i]) : "v"(m));
        K8(S)
#undef S
    }
    uint32_t r = 0;
    for (int i = 0; i < 8; i++) r ^= v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mul_lo(uint32_t *out, uint32_t seed) {
    uint32_t v[8];
    for (int i = 0; i < 8; i++) v[i] = threadIdx.x * 7 + i + seed;
    const uint32_t m = seed | 1;
    for (int it = 0; it < ITER; it++) {
#define S(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(v[i]) : "v"(m));
        K8(S)
#undef S
    }
    uint32_t r = 0;
    for (int i = 0; i < 8; i++) r ^= v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mul_hi(uint32_t *out, uint32_t seed) {
    uint32_t v[8];
    for (int i = 0; i < 8; i++) v[i] = threadIdx.x * 7 + i + seed;
    const uint32_t m = seed | 1;
    for (int it = 0; it < ITER; it++) {
#define S(i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(v[i]) : "v"(m));
        K8(S)
#undef S
    }
    uint32_t r = 0;
    for (int i = 0; i < 8; i++) r ^= v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mul_u24(uint32_t *out, uint32_t seed) {
    uint32_t v[8];
    for (int i = 0; i < 8; i++) v[i] = threadIdx.x * 7 + i + seed;
    const uint32_t m = seed | 1;
    for (int it = 0; it < ITER; it++) {
#define S(i) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(v[i]) : "v"(m));
        K8(S)
#undef S
    }
    uint32_t r = 0;
    for (int i = 0; i < 8; i++) r ^= v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mad64(uint32_t *out, uint32_t seed) {
    uint64_t v[8];
    for (int i = 0; i < 8; i++) v[i] = threadIdx.x * 7 + i + seed;
    const uint32_t m = seed | 1;
    for (int it = 0; it < ITER; it++) {
#define S(i) asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %1, %0" : "+v"(v[i]) : "v"(m) : "s0", "s1");
        K8(S)
#undef S
    }
    uint64_t r = 0;
    for (int i = 0; i < 8; i++) r ^= v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(r ^ (r >> 32));
}

__global__ void k_lshl_add64(uint32_t *out, uint32_t seed) {
    uint64_t v[8];
    for (int i = 0; i < 8; i++) v[i] = threadIdx.x * 7 + i + seed;
    const uint64_t m = seed | 1;
    for (int it = 0; it < ITER; it++) {
#define S(i) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(v[i]) : "v"(m));
        K8(S)
#undef S
    }
    uint64_t r = 0;
    for (int i = 0; i < 8; i++) r ^= v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(r ^ (r >> 32));
}


// one-operand-pair 32-bit forms: v = op(v, m)
#define K32(NAME, ASM)                                                                  \
    __global__ void NAME(uint32_t *out, uint32_t seed) {                                \
        uint32_t v[8];                                                                  \
        for (int i = 0; i < 8; i++) v[i] = threadIdx.x * 7 + i + seed;                  \
        const uint32_t m = seed | 1;                                                    \
        for (int it = 0; it < ITER; it++) {                                             \
            _Pragma("unroll") for (int i = 0; i < 8; i++) asm volatile(ASM : "+v"(v[i]) : "v"(m)); \
        }                                                                               \
        uint32_t r = 0;                                                                 \
        for (int i = 0; i < 8; i++) r ^= v[i];                                          \
        out[blockIdx.x * blockDim.x + threadIdx.x] = r;                                 \
    }
K32(k_alignbit, "v_alignbit_b32 %0, %0, %1, %1")
K32(k_bfe, "v_bfe_u32 %0, %0, %1, 1")
K32(k_dpp, "v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
K32(k_cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
K32(k_xor, "v_xor_b32 %0, %0, %1")
K32(k_add_e64, "v_add_u32_e64 %0, %0, %1")               // the same add in the 8-byte VOP3 encoding
K32(k_or3, "v_or3_b32 %0, %0, %1, %1")

#define K64(NAME, ASM)                                                                  \
    __global__ void NAME(uint32_t *out, uint32_t seed) {                                \
        uint64_t v[8];                                                                  \
        for (int i = 0; i < 8; i++) v[i] = threadIdx.x * 7 + i + seed;                  \
        const uint32_t m = (seed | 1) & 31;                                             \
        for (int it = 0; it < ITER; it++) {                                             \
            _Pragma("unroll") for (int i = 0; i < 8; i++) asm volatile(ASM : "+v"(v[i]) : "v"(m)); \
        }                                                                               \
        uint64_t r = 0;                                                                 \
        for (int i = 0; i < 8; i++) r ^= v[i];                                          \
        out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(r ^ (r >> 32));         \
    }
K64(k_lshl64, "v_lshlrev_b64 %0, %1, %0")
K64(k_mov64, "v_mov_b64 %0, %0")

int main() {
    int dev = 0;
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, dev);
    const int cus = p.multiProcessorCount;
    const double clk_ghz = p.clockRate / 1e6;
    const int waves_per_simd = 8, blocks = cus * 4 * waves_per_simd;    // one-wave workgroups
    uint32_t *out;
    hipMalloc(&out, (size_t)blocks * 64 * 4);
    struct K { const char *name; void (*f)(uint32_t *, uint32_t); };
    K ks[] = {{"v_add_u32", k_add}, {"v_mul_lo_u32", k_mul_lo}, {"v_mul_hi_u32", k_mul_hi},
              {"v_mul_u32_u24", k_mul_u24}, {"v_mad_u64_u32", k_mad64}, {"v_lshl_add_u64", k_lshl_add64},
              {"v_alignbit_b32", k_alignbit}, {"v_bfe_u32", k_bfe}, {"v_mov_b32_dpp", k_dpp},
              {"v_cndmask_b32", k_cndmask}, {"v_xor_b32", k_xor}, {"v_add_u32_e64", k_add_e64}, {"v_or3_b32", k_or3}, {"v_lshlrev_b64", k_lshl64},
              {"v_mov_b64", k_mov64}};
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    printf("CUs %d, clock %.2f GHz, %d one-wave blocks\n", cus, clk_ghz, blocks);
    for (auto &k : ks) {
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(64), 0, 0, out, 3u);   // warm
        hipEventRecord(a);
        for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(64), 0, 0, out, 3u + r);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        const double insts_per_simd = 5.0 * waves_per_simd * ITER * 8;
        const double cycles = ms * 1e-3 * clk_ghz * 1e9;
        printf("%-16s %8.3f ms  %.2f SIMD cycles per wave64 instruction\n", k.name, ms, cycles / insts_per_simd);
    }
    hipFree(out);
    return 0;
}
