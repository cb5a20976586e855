// pcg64.h — numpy Generator(PCG64) stream on gfx950, bit-exact.
//
// The reference draws every random number from ONE np.random.default_rng(seed)
// per env (tile_match_env.py:49): Generator.integers(1, k+1, n) for the
// initial board / remove_colour_lines / refill (board.py:97,129,239) and
// Generator.shuffle(arange(RC)) for shuffle (board.py:116).  numpy's PCG64 is
// the 128-bit LCG  s' = s * A + inc  with XSL-RR output, plus a persistent
// 32-bit half-word buffer used by next_uint32.
//
// On the device a batch of M 32-bit draws is produced lane-parallel by
// jump-ahead: lane j computes s_{j+1} = A^{j+1} s + G_{j+1} inc
// (G_j = sum_{i<j} A^i) from a 64-entry table built on the host, so one
// wave64 round yields 64 outputs = 128 uint32 draws.
#pragma once
#include <stdint.h>

namespace tmg {

struct U128 {
    uint64_t lo, hi;
};

__host__ __device__ __forceinline__ U128 mul128(U128 a, U128 b) {   // low 128 bits of a*b
#if defined(__HIP_DEVICE_COMPILE__)
    // The ten 32x32 partial products below 2^128 (the compiler's 64-bit
    // lowering of lo*lo, umulhi and the two cross terms issues thirteen): six
    // 32x32+64 multiply-adds (v_mad_u64_u32) for the terms whose high halves
    // matter, four 32-bit products for the ones that land at bits 96..127.
    // Integer multiplies issue at ~1/1.7 the rate of a 32-bit add on gfx950
    // (tools/mul_probe.hip), and the PCG64 jump-ahead is most of a redraw's VALU
    // (A/B against the compiler's 64-bit lowering: c2 7.30 vs 7.26, c5 1.24 vs
    // 1.20 x 10^8).
    const uint32_t a0 = (uint32_t)a.lo, a1 = (uint32_t)(a.lo >> 32), a2 = (uint32_t)a.hi, a3 = (uint32_t)(a.hi >> 32);
    const uint32_t b0 = (uint32_t)b.lo, b1 = (uint32_t)(b.lo >> 32), b2 = (uint32_t)b.hi, b3 = (uint32_t)(b.hi >> 32);
    const uint64_t p00 = (uint64_t)a0 * b0;
    const uint64_t p01 = (uint64_t)a0 * b1 + (p00 >> 32);
    const uint64_t p10 = (uint64_t)a1 * b0 + (uint32_t)p01;
    uint64_t hi = (uint64_t)a1 * b1 + (p01 >> 32);
    hi = (uint64_t)a0 * b2 + hi;
    hi = (uint64_t)a2 * b0 + hi;
    hi += (p10 >> 32) + ((uint64_t)(a0 * b3 + a1 * b2 + a2 * b1 + a3 * b0) << 32);
    return U128{(p10 << 32) | (uint32_t)p00, hi};
#else
    uint64_t hi = (uint64_t)(((unsigned __int128)a.lo * b.lo) >> 64) + a.lo * b.hi + a.hi * b.lo;
    return U128{a.lo * b.lo, hi};
#endif
}

__host__ __device__ __forceinline__ U128 add128(U128 a, U128 b) {
    U128 r;
    r.lo = a.lo + b.lo;
    r.hi = a.hi + b.hi + (r.lo < a.lo ? 1 : 0);
    return r;
}

__host__ __device__ __forceinline__ uint64_t xsl_rr(U128 s) {
    uint64_t x = s.hi ^ s.lo;
    unsigned rot = (unsigned)(s.hi >> 58);                 // state >> 122
    return (x >> rot) | (x << ((64u - rot) & 63u));
}

// PCG_DEFAULT_MULTIPLIER_128
static constexpr uint64_t PCG_A_LO = 0x4385DF649FCCF645ULL;
static constexpr uint64_t PCG_A_HI = 0x2360ED051FC65DA4ULL;

// Host: jump table [64][4] = {A^j lo, A^j hi, G_j lo, G_j hi} for j = 1..64.
inline void build_jump_table(uint64_t *tab) {
    U128 A{PCG_A_LO, PCG_A_HI};
    U128 Aj{1, 0}, Gj{0, 0};
    for (int j = 1; j <= 64; j++) {
        Gj = add128(Gj, Aj);          // G_j = G_{j-1} + A^{j-1}
        Aj = mul128(Aj, A);           // A^j
        tab[(j - 1) * 4 + 0] = Aj.lo;
        tab[(j - 1) * 4 + 1] = Aj.hi;
        tab[(j - 1) * 4 + 2] = Gj.lo;
        tab[(j - 1) * 4 + 3] = Gj.hi;
    }
}

}  // namespace tmg
