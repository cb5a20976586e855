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
    uint64_t hi = __umul64hi(a.lo, b.lo) + a.lo * b.hi + a.hi * b.lo;
#else
    uint64_t hi = (uint64_t)(((unsigned __int128)a.lo * b.lo) >> 64) + a.lo * b.hi + a.hi * b.lo;
#endif
    return U128{a.lo * b.lo, hi};
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
