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
// wave64 round yields 64 outputs = 128 uint32 draws.  The row-plane generate
// (tmg_board.hip, bp_*) then advances each lane by 64 outputs at a time
// (A^64, G_64) and recovers an exact position by a backward jump (rows 64..71).
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

// s = A * f + g (mod 2^128): the jump-ahead s_j = A^j s + G_j inc of a lane
// (A, g per lane, f = the wave-uniform stream state, in SGPRs; or X, A^64,
// G_64 inc of the row-plane generate's lane-local batches).  f MUST be
// wave-uniform: its limbs are "s" operands, and for a value the compiler
// holds in VGPRs it inserts a v_readfirstlane, i.e. every lane would get lane
// 0's f.  Device: ten v_mad_u64_u32 / v_mul_lo_u32 in three short chains
// (below), whose carry-outs (SGPR masks) are added back with v_addc.  Round 4
// chained all ten through their 64-bit addends (P = a0 f0 + g.lo, Q = a0 f1 +
// (g2:P.hi), R = a1 f0 + Q, S = a0 f2 + (g3:R.hi), ... ten deep); the same
// multiplies three deep measured c2 +2 %, its 20-step window +3.5 %, c5 +2 %
// (profiles/r05/s15).  The compiler's lowering of mul128 + add128 issues 16
// multiplies and a dozen moves for the same value.
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ uint64_t mad64c(uint32_t a, uint32_t b, uint64_t c, uint64_t &carry) {   // a*b + c, carry out
    uint64_t d;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=&v"(d), "=s"(carry) : "v"(a), "s"(b), "v"(c));
    return d;
}
__device__ __forceinline__ uint32_t addc32(uint32_t x, uint64_t cin, uint64_t &cout) {                 // x + carry-in bit
    uint32_t r;
    asm("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(r), "=s"(cout) : "v"(x), "s"(cin));
    return r;
}
__device__ __forceinline__ uint32_t addc32v(uint32_t x, uint32_t y, uint64_t cin, uint64_t &cout) {   // x + y + carry-in bit
    uint32_t r;
    asm("v_addc_co_u32_e64 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cout) : "v"(x), "v"(y), "s"(cin));
    return r;
}
#endif
__host__ __device__ __forceinline__ U128 add128(U128 a, U128 b);
__host__ __device__ __forceinline__ U128 jump128(const U128 &A, const U128 &f, const U128 &g) {
#if defined(__HIP_DEVICE_COMPILE__)
    // The same sum as three short chains: bits 0..95 (a0 f0 + g.lo, + a0 f1,
    // + a1 f0: carries c1 at 2^64, c3 at 2^96), the 2^64 column (g.hi + a0 f2
    // + a1 f1 + a2 f0) and the 2^96 column's low words (four v_mul_lo), then
    // two add-with-carry steps.  Ten quarter-rate multiplies as before, but
    // three deep instead of ten: a fill's state update no longer waits on one
    // carry chain through every product.
    const uint32_t a0 = (uint32_t)A.lo, a1 = (uint32_t)(A.lo >> 32), a2 = (uint32_t)A.hi, a3 = (uint32_t)(A.hi >> 32);
    const uint32_t f0 = (uint32_t)f.lo, f1 = (uint32_t)(f.lo >> 32), f2 = (uint32_t)f.hi, f3 = (uint32_t)(f.hi >> 32);
    uint64_t c1, c3, k, cx;
    const uint64_t P = mad64c(a0, f0, g.lo, c1);
    const uint64_t Q = mad64c(a0, f1, P >> 32, cx);                  // < 2^64: no carry
    const uint64_t R = mad64c(a1, f0, Q, c3);
    uint64_t S = mad64c(a0, f2, g.hi, cx);                           // carries out of the 2^64 column are >= 2^128
    S = mad64c(a1, f1, S, cx);
    const uint64_t U = mad64c(a2, f0, S, cx);
    const uint32_t w = a0 * f3 + a1 * f2 + a2 * f1 + a3 * f0;
    const uint32_t r2 = addc32v((uint32_t)U, (uint32_t)(R >> 32), c1, k);
    const uint32_t r3 = addc32(addc32v((uint32_t)(U >> 32), w, c3, cx), k, cx);
    return U128{(R << 32) | (uint32_t)P, ((uint64_t)r3 << 32) | r2};
#else
    const unsigned __int128 a = ((unsigned __int128)A.hi << 64) | A.lo, b = ((unsigned __int128)f.hi << 64) | f.lo;
    const unsigned __int128 s = a * b + (((unsigned __int128)g.hi << 64) | g.lo);
    return U128{(uint64_t)s, (uint64_t)(s >> 64)};
#endif
}

__host__ __device__ __forceinline__ uint64_t xsl_rr(U128 s) {
    uint64_t x = s.hi ^ s.lo;
    unsigned rot = (unsigned)(s.hi >> 58);                 // state >> 122
    return (x >> rot) | (x << ((64u - rot) & 63u));
}

// PCG_DEFAULT_MULTIPLIER_128
static constexpr uint64_t PCG_A_LO = 0x4385DF649FCCF645ULL;
static constexpr uint64_t PCG_A_HI = 0x2360ED051FC65DA4ULL;

// Host: jump table [kJumpRows][4]:
//   rows 0..63:  {A^j lo, A^j hi, G_j lo, G_j hi} for j = 1..64 (s_j = A^j s + G_j inc);
//   rows 64..71: {B lo, B hi, D lo, D hi} with B = A^{-64m}, D = -A^{-64m} G_{64m}
//                for m = 1..8, so s = B s_{64m} + D inc (64m outputs back).
constexpr int kJumpRows = 72;
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
    // A^{-1} mod 2^128 (A odd) by Newton's iteration x <- x (2 - A x): A x = 1
    // mod 2^3 for x = A, each step doubles the exact low bits
    U128 inv = A;
    for (int it = 0; it < 6; it++) {
        const U128 ax = mul128(A, inv);
        inv = mul128(inv, add128(U128{2, 0}, U128{~ax.lo + 1, ~ax.hi + (ax.lo == 0 ? 1ULL : 0ULL)}));
    }
    const U128 A64{tab[63 * 4], tab[63 * 4 + 1]}, G64{tab[63 * 4 + 2], tab[63 * 4 + 3]};
    U128 Gm{0, 0}, Binv{1, 0};                      // G_{64m}, A^{-64m}
    U128 inv64{1, 0};
    for (int j = 0; j < 64; j++) inv64 = mul128(inv64, inv);
    for (int m = 1; m <= 8; m++) {
        Gm = add128(mul128(A64, Gm), G64);          // G_{64m} = A^64 G_{64(m-1)} + G_64
        Binv = mul128(Binv, inv64);
        const U128 d = mul128(Binv, Gm);
        tab[(63 + m) * 4 + 0] = Binv.lo;
        tab[(63 + m) * 4 + 1] = Binv.hi;
        tab[(63 + m) * 4 + 2] = ~d.lo + 1;          // -d mod 2^128
        tab[(63 + m) * 4 + 3] = ~d.hi + (d.lo == 0 ? 1ULL : 0ULL);
    }
}

}  // namespace tmg
