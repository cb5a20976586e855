// tmg_lane.h — the lean step with one LANE per board (boards of <= 128 cells,
// no specials enabled, cached effective-action mask trusted).
//
// The wave-per-board kernels (tmg_board.hip, tmg_sb.hip) spend one wave
// instruction on one board: a 10x10 board keeps 10..100 of 64 lanes busy and
// its cascade runs on the scalar unit.  Here lane i of a wave owns env i
// outright: the board lives in VGPRs as NB colour bit-planes of 128 bits (cell
// p = r*C + c is bit p: `lo` cells 0..63, `hi` 64..127; a colour c is the bit
// pattern c - 1 across the planes), the env's PCG64 stream is stepped by the
// lane itself, and every board operation of the lean path is a handful of
// 64-bit bitwise ops on those planes, so one VALU instruction advances 64
// boards.  Nothing here talks across lanes; the same code compiles for the
// host (tests/lane_host.cpp runs it env by env against the oracle).
//
// Reference semantics restated (src/tile_match_gym/board.py):
//   move :330-395 with every tile normal (no specials):
//     is_move_effective :735-787 (the cached mask), swap :355, the cascade
//     :367-376 = get_colour_lines :149-215 (first pass :158-193 stops after
//     the lowest row holding a line; the perpendicular pass :195-214) ->
//     every line a normal match (process_colour_lines :269-327 with no
//     special enabled) -> all its cells cleared -> gravity :217-229 ->
//     refill :231-241 (row-major, Generator.integers(1, k+1));
//     then "while not possible_move() or lines" :381-391 (shuffle :114-118,
//     remove_colour_lines :120-131).
//   The regeneration of a finished episode (generate_board :95-109) is left
//   to reset_kernel (the host launches it masked by FL_RESET after the step).
#pragma once
#include <stdint.h>

#include "pcg64.h"

namespace tmg {
namespace lane {

#define TMG_LN __host__ __device__ __forceinline__
#ifndef TMG_LANE_NOTE_ITERS
#define TMG_LANE_NOTE_ITERS(n) ((void)(n))      // host statistics hooks (tools/lane_host)
#define TMG_LANE_NOTE_PASS() ((void)0)
#define TMG_LANE_NOTE_HOLES(n) ((void)(n))
#endif

// flags / status bits (same values as tmg_board.hip's FL_* / ST_*)
enum : int { LF_DONE = 1, LF_SHUF = 4, LF_RESET = 8, LF_ERR = 0x80 };
enum : uint32_t { LS_INTERNAL = 1, LS_CALLER = 4 };
constexpr int kLaneMaxShuffles = 1 << 12;     // kMaxShuffles

// A 128-cell bitboard.  TMG_LANE_W32 (default): four 32-bit words, so a
// shift is one funnel shift (v_alignbit_b32) per word instead of 64-bit
// shifts and ORs; otherwise two 64-bit halves.
#ifndef TMG_LANE_W32
#define TMG_LANE_W32 1
#endif
TMG_LN uint32_t funnel(uint32_t hi, uint32_t lo, int s) {   // ({hi, lo} >> s) & 0xFFFFFFFF, 0 <= s < 32
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(hi, lo, (unsigned)s);
#else
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> s);
#endif
}
#if TMG_LANE_W32
struct B {
    uint32_t w[4];
};
TMG_LN constexpr B from_halves(uint64_t lo, uint64_t hi) {
    return B{{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)}};
}
TMG_LN uint64_t half(B x, int i) { return (uint64_t)x.w[2 * i] | ((uint64_t)x.w[2 * i + 1] << 32); }
TMG_LN B operator&(B x, B y) { return B{{x.w[0] & y.w[0], x.w[1] & y.w[1], x.w[2] & y.w[2], x.w[3] & y.w[3]}}; }
TMG_LN B operator|(B x, B y) { return B{{x.w[0] | y.w[0], x.w[1] | y.w[1], x.w[2] | y.w[2], x.w[3] | y.w[3]}}; }
TMG_LN B operator^(B x, B y) { return B{{x.w[0] ^ y.w[0], x.w[1] ^ y.w[1], x.w[2] ^ y.w[2], x.w[3] ^ y.w[3]}}; }
TMG_LN B andn(B x, B y) { return B{{x.w[0] & ~y.w[0], x.w[1] & ~y.w[1], x.w[2] & ~y.w[2], x.w[3] & ~y.w[3]}}; }
TMG_LN bool any(B x) { return (x.w[0] | x.w[1] | x.w[2] | x.w[3]) != 0u; }
TMG_LN int popc(B x) {
    return __builtin_popcount(x.w[0]) + __builtin_popcount(x.w[1]) + __builtin_popcount(x.w[2]) +
           __builtin_popcount(x.w[3]);
}
// content moves D cells forward (bit p -> p + D) / back (bit p -> p - D)
template <int D>
TMG_LN B fwd(B x) {
    static_assert(D > 0 && D < 128, "shift");
    constexpr int q = D >> 5, r = D & 31;
    B o;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t hi = i - q >= 0 ? x.w[i - q] : 0u, lo = i - q - 1 >= 0 ? x.w[i - q - 1] : 0u;
        o.w[i] = r ? funnel(hi, lo, 32 - r) : hi;
    }
    return o;
}
template <int D>
TMG_LN B bwd(B x) {
    static_assert(D > 0 && D < 128, "shift");
    constexpr int q = D >> 5, r = D & 31;
    B o;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t lo = i + q <= 3 ? x.w[i + q] : 0u, hi = i + q + 1 <= 3 ? x.w[i + q + 1] : 0u;
        o.w[i] = r ? funnel(hi, lo, r) : lo;
    }
    return o;
}
TMG_LN B isolate_lowest(B h) {                    // the lowest set bit of h (h != 0)
    const uint32_t m0 = h.w[0] & (~h.w[0] + 1u), m1 = h.w[1] & (~h.w[1] + 1u);
    const uint32_t m2 = h.w[2] & (~h.w[2] + 1u), m3 = h.w[3] & (~h.w[3] + 1u);
    const bool z0 = h.w[0] == 0u, z1 = z0 && h.w[1] == 0u, z2 = z1 && h.w[2] == 0u;
    return B{{m0, z0 ? m1 : 0u, z1 ? m2 : 0u, z2 ? m3 : 0u}};
}
#else
struct B {
    uint64_t lo, hi;
};
TMG_LN constexpr B from_halves(uint64_t lo, uint64_t hi) { return B{lo, hi}; }
TMG_LN uint64_t half(B x, int i) { return i ? x.hi : x.lo; }
TMG_LN B operator&(B x, B y) { return B{x.lo & y.lo, x.hi & y.hi}; }
TMG_LN B operator|(B x, B y) { return B{x.lo | y.lo, x.hi | y.hi}; }
TMG_LN B operator^(B x, B y) { return B{x.lo ^ y.lo, x.hi ^ y.hi}; }
TMG_LN B andn(B x, B y) { return B{x.lo & ~y.lo, x.hi & ~y.hi}; }     // x & ~y
TMG_LN bool any(B x) { return (x.lo | x.hi) != 0ULL; }
TMG_LN int popc(B x) { return __builtin_popcountll(x.lo) + __builtin_popcountll(x.hi); }
template <int D>
TMG_LN B fwd(B x) {
    static_assert(D > 0 && D < 128, "shift");
    if constexpr (D >= 64) return B{0, x.lo << (D - 64)};
    else return B{x.lo << D, (x.hi << D) | (x.lo >> (64 - D))};
}
template <int D>
TMG_LN B bwd(B x) {
    static_assert(D > 0 && D < 128, "shift");
    if constexpr (D >= 64) return B{x.hi >> (D - 64), 0};
    else return B{(x.lo >> D) | (x.hi << (64 - D)), x.hi >> D};
}
TMG_LN B isolate_lowest(B h) { return h.lo ? B{h.lo & (~h.lo + 1), 0} : B{0, h.hi & (~h.hi + 1)}; }
#endif
// the rarer helpers, on the two 64-bit halves
TMG_LN int bit(B x, int p) { return (int)((half(x, p >> 6) >> (p & 63)) & 1ULL); }
TMG_LN B one(int p) { return p < 64 ? from_halves(1ULL << p, 0) : from_halves(0, 1ULL << (p - 64)); }
TMG_LN int lowest(B x) {                          // x != 0
    const uint64_t lo = half(x, 0);
    return lo ? __builtin_ctzll(lo) : 64 + __builtin_ctzll(half(x, 1));
}
TMG_LN int highest(B x) {                         // x != 0
    const uint64_t hi = half(x, 1);
    return hi ? 127 - __builtin_clzll(hi) : 63 - __builtin_clzll(half(x, 0));
}
TMG_LN B drop_lowest(B x) { return x ^ isolate_lowest(x); }
TMG_LN B fwd_v(B x, int s) {                      // 0 <= s < 128
    const uint64_t lo = half(x, 0), hi = half(x, 1);
    if (s >= 64) return from_halves(0, lo << (s - 64));
    if (s == 0) return x;
    return from_halves(lo << s, (hi << s) | (lo >> (64 - s)));
}
TMG_LN B cells_below(int n) {                     // cells 0..n-1, 0 <= n <= 128
    if (n >= 128) return from_halves(~0ULL, ~0ULL);
    if (n >= 64) return from_halves(~0ULL, n == 64 ? 0ULL : (~0ULL >> (128 - n)));
    return from_halves(n == 0 ? 0ULL : (~0ULL >> (64 - n)), 0);
}

// rows r0..r1 x columns c0..c1 of a C-column board (empty when r1 < r0 or c1 < c0)
TMG_LN constexpr B rect(int C, int r0, int r1, int c0, int c1) {
    uint64_t lo = 0, hi = 0;
    for (int r = r0; r <= r1; r++)
        for (int c = c0; c <= c1; c++) {
            const int p = r * C + c;
            if (p < 64) lo |= 1ULL << p;
            else hi |= 1ULL << (p - 64);
        }
    return from_halves(lo, hi);
}

// ------------------------------------------------------------------- RNG
// numpy's PCG64 (pcg64.h's constants) with the persistent half-word buffer,
// one stream per lane
struct Rng {
    uint64_t slo, shi, ilo, ihi;
    uint32_t has, buf;
};
TMG_LN void rng_load(Rng &g, const uint64_t *w) {
    g.slo = w[0]; g.shi = w[1]; g.ilo = w[2]; g.ihi = w[3];
    g.has = (uint32_t)(w[4] >> 32) & 1u;
    g.buf = (uint32_t)w[4];
}
TMG_LN void rng_store(const Rng &g, uint64_t *w) {
    w[0] = g.slo; w[1] = g.shi; w[2] = g.ilo; w[3] = g.ihi;
    w[4] = ((uint64_t)g.has << 32) | g.buf;
}
TMG_LN uint64_t next64(Rng &g) {
    const U128 s = add128(mul128(U128{g.slo, g.shi}, U128{PCG_A_LO, PCG_A_HI}), U128{g.ilo, g.ihi});
    g.slo = s.lo;
    g.shi = s.hi;
    return xsl_rr(s);
}
TMG_LN uint32_t next32(Rng &g) {
    if (g.has) {
        g.has = 0;
        return g.buf;
    }
    const uint64_t x = next64(g);
    g.has = 1;
    g.buf = (uint32_t)(x >> 32);
    return (uint32_t)x;
}
// Generator.integers(1, K+1) - 1: numpy's buffered bounded Lemire draw
template <int K>
TMG_LN int draw_code(Rng &g) {
    if constexpr (K == 1) {
        return 0;                                  // rng == 0: numpy draws nothing
    } else {
        constexpr uint32_t thr = (0xFFFFFFFFu - (uint32_t)(K - 1)) % (uint32_t)K;
        uint64_t m = (uint64_t)next32(g) * (uint32_t)K;
        if constexpr (thr != 0u) {
            while ((uint32_t)m < thr) m = (uint64_t)next32(g) * (uint32_t)K;
        }
        return (int)(m >> 32);
    }
}
// random_interval(max) of Generator.shuffle (masked rejection)
TMG_LN uint32_t interval(Rng &g, uint32_t max) {
    uint32_t mask = max;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t v;
    while ((v = (next32(g) & mask)) > max) {
    }
    return v;
}

// --------------------------------------------------------------- the board
template <int R_, int C_, int K_>
struct Board {
    static constexpr int R = R_, C = C_, K = K_, N = R * C;
    static constexpr int NB = K <= 2 ? 1 : K <= 4 ? 2 : K <= 8 ? 3 : 4;
    static constexpr int A = 2 * R * C - R - C, AV = C * (R - 1), W = (A + 63) / 64;
    static_assert(N <= 128 && R >= 3 && C >= 3 && 3 * C < 64, "lane boards: <= 128 cells, 3C < 64");
    static_assert(W <= 4, "mask words");

    B x[NB];                                        // colour bit-planes

    TMG_LN void swap_cells(int p, int q) {
#pragma unroll
        for (int b = 0; b < NB; b++) {
            if (bit(x[b], p) != bit(x[b], q)) x[b] = x[b] ^ (one(p) | one(q));
        }
    }
    TMG_LN void set_code(int p, int code) {         // cell p (all planes 0 there) <- code
        const B m = one(p);
#pragma unroll
        for (int b = 0; b < NB; b++)
            if ((code >> b) & 1) x[b] = x[b] | m;
    }
    TMG_LN int code(int p) const {
        int v = 0;
#pragma unroll
        for (int b = 0; b < NB; b++) v |= bit(x[b], p) << b;
        return v;
    }
    // cells whose colour differs from the cell D further on (garbage where
    // that cell is off the board or in another row: callers mask)
    template <int D>
    TMG_LN B ne() const {
        B r = x[0] ^ bwd<D>(x[0]);
#pragma unroll
        for (int b = 1; b < NB; b++) r = r | (x[b] ^ bwd<D>(x[b]));
        return r;
    }
};

// get_colour_lines' first pass on the planes: eqR = same colour as the right
// neighbour, eqD = as the cell below; h3 / v3 = the first cell of a horizontal
// / the top cell of a vertical window of three equal colours
template <class BD>
struct Det {
    B eqR, eqD, h3, v3;
};
template <class BD>
TMG_LN Det<BD> detect(const BD &b) {
    constexpr int R = BD::R, C = BD::C;
    constexpr B NR1 = rect(C, 0, R - 1, 0, C - 2), ND1 = rect(C, 0, R - 2, 0, C - 1);
    Det<BD> d;
    d.eqR = andn(NR1, b.template ne<1>());
    d.eqD = andn(ND1, b.template ne<C>());
    d.h3 = d.eqR & bwd<1>(d.eqR);
    d.v3 = d.eqD & bwd<C>(d.eqD);
    return d;
}
template <class BD>
TMG_LN bool has_line(const Det<BD> &d) { return any(d.h3 | d.v3); }

// The bottom row of get_colour_lines' first pass (it scans rows bottom-up and
// stops at the first row holding a line): the largest row of a horizontal
// window or of a vertical window's bottom cell.
template <class BD>
TMG_LN int bottom_row(const Det<BD> &d) {
    constexpr int C = BD::C;
    return highest(d.h3 | fwd<2 * C>(d.v3)) / C;
}

// One cascade step (board.py:367-376, every line a normal match): the union
// of get_colour_lines' lines — the first-pass coords K of row rs (its
// horizontal runs, the vertical runs ending in it, walked up while the colour
// holds, :163-193) and the perpendicular pass's lines through K (:195-214;
// only horizontal runs through a vertical run's cells above rs can be lines
// there: a vertical run through a coord would extend a first-pass vertical or
// reach below rs).
template <class BD>
TMG_LN B clear_set(const Det<BD> &d, int rs) {
    constexpr int R = BD::R, C = BD::C;
    constexpr B IN = rect(C, 0, R - 1, 0, C - 1), NL1 = rect(C, 0, R - 1, 1, C - 1);
    constexpr B ROW0 = rect(C, 0, 0, 0, C - 1);
    const B row = fwd_v(ROW0, rs * C);
    const B h = d.h3 & row;
    B K = h | fwd<1>(h) | fwd<2>(h);
    const B v = fwd<2 * C>(d.v3) & row;             // bottoms of vertical windows in row rs
    if (any(v)) {
        const B eqU = fwd<C>(d.eqD);                // same colour as the cell above
        B t = bwd<2 * C>(v);
        K = K | v | bwd<C>(v) | t;
        for (;;) {
            t = bwd<C>(t & eqU);
            if (!any(t)) break;
            K = K | t;
        }
    }
    B clr = K;
    const B walk = andn(IN, K);
    const B r1 = fwd<1>(K & d.eqR) & walk;
    const B l1 = bwd<1>(K & NL1) & d.eqR & walk;
    if (any(r1 | l1)) {
        const B r2 = fwd<1>(r1 & d.eqR) & walk;
        const B l2 = bwd<1>(l1 & NL1) & d.eqR & walk;
        const B q = K & (bwd<2>(r2) | fwd<2>(l2) | (bwd<1>(r1) & fwd<1>(l1)));
        if (any(q)) {
            B f = fwd<1>(q & d.eqR) & walk;
            while (any(f)) { clr = clr | f; f = fwd<1>(f & d.eqR) & walk; }
            B g = bwd<1>(q & NL1) & d.eqR & walk;
            while (any(g)) { clr = clr | g; g = bwd<1>(g & NL1) & d.eqR & walk; }
        }
    }
    return clr;
}

// OR of x moved 1..R-1 rows up (bit p -> p - jC)
template <int R, int C>
TMG_LN B smear_up(B x) {
    static_assert(R <= 12, "smear_up covers 11 rows");
    const B s = bwd<C>(x);
    if constexpr (R <= 2) return s;
    else if constexpr (R <= 4) return s | bwd<C>(s) | bwd<2 * C>(s);          // rows 1..3
    else {
        const B t = s | bwd<C>(s) | bwd<2 * C>(s);                              // 1..3
        if constexpr (R <= 10) return t | bwd<3 * C>(t) | bwd<6 * C>(t);        // 1..9
        else return t | bwd<3 * C>(t) | bwd<6 * C>(t) | bwd<9 * C>(t);          // 1..12 (R <= 12 with 3C < 64, N <= 128)
    }
}

// refill (board.py:231-241): the holes h (planes 0 there) take draws in
// row-major order.  For a power-of-two k (no Lemire rejection) a PCG output
// holds the codes of two holes (its low then high half, numpy's half-word
// buffer); with rejections possible, draw by draw.
template <class BD>
TMG_LN void deposit(BD &b, B &h, int code) {      // code -> the lowest hole of h, which leaves h
    const B lb = isolate_lowest(h);
#pragma unroll
    for (int k = 0; k < BD::NB; k++)
        if ((code >> k) & 1) b.x[k] = b.x[k] | lb;
    h = h ^ lb;
}
template <class BD>
TMG_LN void refill(BD &b, B h, Rng &g) {
    constexpr uint32_t K = (uint32_t)BD::K;
    if constexpr (K > 1 && (K & (K - 1)) == 0) {
        if (g.has && any(h)) {
            g.has = 0;
            deposit(b, h, (int)(((uint64_t)g.buf * K) >> 32));
        }
        while (any(h)) {
            const uint64_t x = next64(g);
            g.buf = (uint32_t)(x >> 32);                // the buffer keeps the high half either way
            deposit(b, h, (int)(((x & 0xFFFFFFFFULL) * K) >> 32));
            if (any(h)) deposit(b, h, (int)(((x >> 32) * K) >> 32));
            else g.has = 1;
        }
    } else {
        while (any(h)) deposit(b, h, draw_code<BD::K>(g));
    }
}

// gravity + refill (board.py:217-241) of the holes E (planes already 0 there):
// each pass closes the lowest hole of every column that still has one (the
// cells above it drop a row, the column's top cell becomes a hole), then the
// holes — now the top cells of their columns — take the refill draws in
// row-major order
template <class BD>
TMG_LN void gravity_refill(BD &b, B E, Rng &g) {
    constexpr int R = BD::R, C = BD::C;
    constexpr B ROW0 = rect(C, 0, 0, 0, C - 1);
    for (;;) {
        // cells with a hole somewhere below = the cells above their column's
        // lowest hole (holes among them)
        const B AL = smear_up<R, C>(E);
        const B L = andn(E, AL);                    // the lowest hole of each column
        // settled: no hole has a cell above it that is not a hole
        if (!any(andn(AL, E))) break;
        TMG_LANE_NOTE_PASS();
        const B M = AL | L;
#pragma unroll
        for (int k = 0; k < BD::NB; k++) b.x[k] = andn(b.x[k], M) | fwd<C>(b.x[k] & AL);
        E = andn(E, M) | fwd<C>(E & AL) | (M & ROW0);
    }
    TMG_LANE_NOTE_HOLES(popc(E));
    refill(b, E, g);
}

// rows 0..row <- Generator.integers(1, k+1, (row+1)*C) (remove_colour_lines :129)
template <class BD>
TMG_LN void redraw_rows(BD &b, int row, Rng &g) {
    const int M = (row + 1) * BD::C;
    const B keep = andn(from_halves(~0ULL, ~0ULL), cells_below(M));
#pragma unroll
    for (int k = 0; k < BD::NB; k++) b.x[k] = b.x[k] & keep;
    for (int p = 0; p < M; p++) b.set_code(p, draw_code<BD::K>(g));
}

// remove_colour_lines' row (board.py:126): the first line get_colour_lines
// returns — in row rs, the leftmost anchor, a vertical one first on a tie —
// and its first coord's row (a vertical line's top, :166-172)
template <class BD>
TMG_LN int first_line_row(const Det<BD> &d, int rs) {
    constexpr int C = BD::C;
    constexpr B ROW0 = rect(C, 0, 0, 0, BD::C - 1);
    const B row = fwd_v(ROW0, rs * C);
    const B va = fwd<2 * C>(d.v3) & row, ha = d.h3 & row;
    const int pv = any(va) ? lowest(va) : 1 << 20, ph = any(ha) ? lowest(ha) : 1 << 20;
    if (ph < pv) return rs;
    const B eqU = fwd<C>(d.eqD);
    int t = pv - 2 * C;
    while (t >= C && bit(eqU, t)) t -= C;
    return t / C;
}

// Generator.shuffle of the board's cells (board.py:114-118): Fisher-Yates on
// an index array (the lane's scratch, >= N bytes), then new[p] = old[idx[p]]
template <class BD>
TMG_LN void shuffle(BD &b, Rng &g, uint8_t *ix) {
    constexpr int N = BD::N;
    for (int p = 0; p < N; p++) ix[p] = (uint8_t)p;
    for (int i = N - 1; i >= 1; i--) {
        const int j = (int)interval(g, (uint32_t)i);
        const uint8_t t = ix[i];
        ix[i] = ix[j];
        ix[j] = t;
    }
    BD nb;
#pragma unroll
    for (int k = 0; k < BD::NB; k++) nb.x[k] = from_halves(0, 0);
    for (int p = 0; p < N; p++) nb.set_code(p, b.code(ix[p]));
    b = nb;
}

// The effective-action mask of a line-free all-normal board
// (is_move_effective, board.py:735-787): a swap is effective iff it puts a
// line through one of the two cells.  eq<O> = colour(p) == colour(p + O)
// where both cells exist in the right geometric relation; the patterns below
// compare each moved tile's new neighbours with its colour.  Action order
// (board.py:77-93): vertical swaps (r,c)-(r+1,c) first, a = r*C + c, then
// horizontal (r,c)-(r,c+1), a = C(R-1) + r(C-1) + c.
template <class BD>
TMG_LN void effective_mask(const BD &b, uint64_t *m) {
    constexpr int R = BD::R, C = BD::C;
    const B E2 = andn(rect(C, 0, R - 1, 0, C - 3), b.template ne<2>());
    const B E3 = andn(rect(C, 0, R - 1, 0, C - 4), b.template ne<3>());
    const B Ec1m = andn(rect(C, 0, R - 2, 1, C - 1), b.template ne<C - 1>());
    const B Ec1p = andn(rect(C, 0, R - 2, 0, C - 2), b.template ne<C + 1>());
    const B Ec2m = andn(rect(C, 0, R - 2, 2, C - 1), b.template ne<C - 2>());
    const B Ec2p = andn(rect(C, 0, R - 2, 0, C - 3), b.template ne<C + 2>());
    const B E2c = andn(rect(C, 0, R - 3, 0, C - 1), b.template ne<2 * C>());
    const B E3c = andn(rect(C, 0, R - 4, 0, C - 1), b.template ne<3 * C>());
    const B E2c1m = andn(rect(C, 0, R - 3, 1, C - 1), b.template ne<2 * C - 1>());
    const B E2c1p = andn(rect(C, 0, R - 3, 0, C - 2), b.template ne<2 * C + 1>());
    // vertical swap at u (d = u + C): u takes d's colour, d takes u's
    const B Lm1 = fwd<1>(Ec1p), Lm2 = fwd<2>(Ec2p), Rp1 = bwd<1>(Ec1m), Rp2 = bwd<2>(Ec2m);
    const B Um1 = fwd<C>(E2c), Um2 = fwd<2 * C>(E3c);
    const B V = ((Lm2 & Lm1) | (Lm1 & Rp1) | (Rp1 & Rp2) | (Um1 & Um2) |
                 (Ec2m & Ec1m) | (Ec1m & Ec1p) | (Ec1p & Ec2p) | (E2c & E3c)) & rect(C, 0, R - 2, 0, C - 1);
    // horizontal swap at u (v = u + 1)
    const B uL1 = fwd<1>(E2), uL2 = fwd<2>(E3), uU1 = fwd<C>(Ec1p), uU2 = fwd<2 * C>(E2c1p);
    const B uD1 = bwd<1>(Ec1m), uD2 = bwd<1>(E2c1m);
    const B vU1 = fwd<C - 1>(Ec1m), vU2 = fwd<2 * C - 1>(E2c1m);
    const B H = ((uL1 & uL2) | (uU1 & uU2) | (uU1 & uD1) | (uD1 & uD2) |
                 (E2 & E3) | (vU1 & vU2) | (vU1 & Ec1p) | (Ec1p & E2c1p)) & rect(C, 0, R - 1, 0, C - 2);
    // pack: actions 0..AV-1 are V's cells 0..AV-1; action AV + r(C-1) + c is H's cell rC + c
    const uint64_t Vlo = half(V, 0), Vhi = half(V, 1), Hlo = half(H, 0), Hhi = half(H, 1);
    uint64_t w[4] = {Vlo, 0, 0, 0};
    if constexpr (BD::AV > 64) w[1] = Vhi & (~0ULL >> (128 - BD::AV));
    else w[0] &= (BD::AV == 64 ? ~0ULL : (~0ULL >> (64 - BD::AV)));
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int src = r * C, dst = BD::AV + r * (C - 1);
        const uint64_t row = (src >= 64 ? Hhi >> (src - 64) : ((Hlo >> src) | (src ? Hhi << (64 - src) : 0ULL))) &
                             ((1ULL << (C - 1)) - 1ULL);
        const int wi = dst >> 6, off = dst & 63;
        w[wi] |= row << off;
        if (off + (C - 1) > 64) w[wi + 1] |= row >> (64 - off);
    }
#pragma unroll
    for (int i = 0; i < BD::W; i++) m[i] = w[i];
}

// "while not possible_move() or lines" (board.py:102-109, 381-391): clean =
// the board is known to be line-free.  Leaves the mask in m; returns LF_SHUF
// when a shuffle ran, LF_ERR when the shuffle cap ended the loop.
template <class BD>
TMG_LN int ensure(BD &b, Rng &g, uint64_t *m, bool clean, uint8_t *scratch) {
    int fl = 0;
    for (int shuffles = 0;; shuffles++) {
        if (!clean) {
            for (;;) {
                const Det<BD> d = detect(b);
                if (!has_line(d)) break;
                const int r0 = first_line_row(d, bottom_row(d));
                redraw_rows(b, BD::R - 1 < r0 + 1 ? BD::R - 1 : r0 + 1, g);
            }
        }
        effective_mask(b, m);
        uint64_t anyb = 0;
#pragma unroll
        for (int i = 0; i < BD::W; i++) anyb |= m[i];
        if (anyb) break;
        if (shuffles >= kLaneMaxShuffles) { fl |= LF_ERR; break; }
        shuffle(b, g, scratch);
        fl |= LF_SHUF;
        clean = false;
    }
    return fl;
}

// Board.move for an effective action (the caller tested the mask): swap,
// cascade, ensure playable.  Returns the eliminations (:374-378).
template <class BD>
TMG_LN int move(BD &b, Rng &g, int p1, int p2, int &flags, uint64_t *m, uint8_t *scratch) {
    b.swap_cells(p1, p2);
    int elim = 0, iters = 0;
    for (;; iters++) {
        const Det<BD> d = detect(b);
        if (!has_line(d)) break;
        const B clr = clear_set(d, bottom_row(d));
        elim += popc(clr);
#pragma unroll
        for (int k = 0; k < BD::NB; k++) b.x[k] = andn(b.x[k], clr);
        gravity_refill(b, clr, g);
    }
    TMG_LANE_NOTE_ITERS(iters);
    flags |= ensure(b, g, m, true, scratch);
    return elim;
}

// ------------------------------------------------------- board <-> bytes
// The colour plane of the HBM board (int8 colours 1..k, row-major), read and
// written as 8-byte words (byte j of dword i is cell 4i + j).  A plane's bit
// of 4 cells is one v_dot4_u32_u8 of the masked bytes with (1, 2, 4, 8); the
// inverse spreads a nibble to the 4 bytes by one multiply.
TMG_LN uint32_t gather4(uint32_t d) {             // bit 0 of each byte of d -> bits 0..3
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_udot4(d & 0x01010101u, 0x08040201u, 0u, false);
#else
    d &= 0x01010101u;
    return (d | (d >> 7) | (d >> 14) | (d >> 21)) & 0xFu;
#endif
}
TMG_LN uint32_t spread4(uint32_t n) {             // bits 0..3 of n -> bit 0 of bytes 0..3
    return (n * 0x00204081u) & 0x01010101u;
}
template <class BD>
TMG_LN void unpack(BD &b, const uint64_t *q) {
    constexpr int ND = (BD::N + 3) / 4;
    uint64_t lo[BD::NB], hi[BD::NB];
#pragma unroll
    for (int k = 0; k < BD::NB; k++) lo[k] = hi[k] = 0;
#pragma unroll
    for (int i = 0; i < ND; i++) {
        const uint64_t qq = q[i >> 1];
        const uint32_t d = (uint32_t)(i & 1 ? qq >> 32 : qq) - 0x01010101u;   // colour codes 0..k-1 per byte
#pragma unroll
        for (int k = 0; k < BD::NB; k++) {
            uint64_t v = gather4(d >> k);
            if (4 * i + 4 > BD::N) v &= (1ULL << (BD::N - 4 * i)) - 1ULL;
            if (i < 16) lo[k] |= v << (4 * i);
            else hi[k] |= v << (4 * i - 64);
        }
    }
#pragma unroll
    for (int k = 0; k < BD::NB; k++) b.x[k] = from_halves(lo[k], hi[k]);
}
// 8-byte word i of the colour plane (cells 8i..8i+7; bytes past N are 1)
template <class BD>
TMG_LN uint64_t pack_word(const BD &b, int i) {
    uint32_t d[2];
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const int c = 8 * i + 4 * j;                // first cell of the dword
        uint32_t w = 0x01010101u;
#pragma unroll
        for (int k = 0; k < BD::NB; k++) {
            const uint32_t n = (uint32_t)(half(b.x[k], c >> 6) >> (c & 63)) & 0xFu;
            w += spread4(n) << k;
        }
        d[j] = w;
    }
    return (uint64_t)d[0] | ((uint64_t)d[1] << 32);
}

// ------------------------------------------------------------- the policy
// tmg_sample_effective's draw (tmg_board.hip policy_draw / draw_row): the
// r-th set bit of the mask, r = h * count >> 32, or h * A >> 32 when empty
TMG_LN uint64_t splitmix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}
TMG_LN int select_bit(uint64_t x, int r) {         // r < popcount(x)
    int pos = 0;
#pragma unroll
    for (int sh = 32; sh > 0; sh >>= 1) {
        const int c = __builtin_popcountll(x & ((1ULL << sh) - 1ULL));
        const bool up = r >= c;
        r -= up ? c : 0;
        x = up ? x >> sh : x;
        pos += up ? sh : 0;
    }
    return pos;
}
template <int W>
TMG_LN int policy_action(const uint64_t *m, int A, uint64_t key, uint64_t gid, int32_t t) {
    const uint64_t base = splitmix(key * 0xD1B54A32D192ED03ULL + gid);
    const uint64_t h = splitmix(base ^ ((uint64_t)t * 0x9E3779B97F4A7C15ULL)) >> 32;
    int count = 0;
#pragma unroll
    for (int j = 0; j < W; j++) count += __builtin_popcountll(m[j]);
    if (count == 0) return (int)((h * (uint64_t)A) >> 32);
    int r = (int)((h * (uint64_t)count) >> 32);
    int j = 0;
    uint64_t x = m[0];
#pragma unroll
    for (int i = 0; i < W - 1; i++) {
        const int c = __builtin_popcountll(x);
        if (r < c) break;
        r -= c;
        x = m[++j];
    }
    return j * 64 + select_bit(x, r);
}

// ------------------------------------------------------------ one env step
// The per-env arrays of a step launch (include/tmg.h tmg_step), already
// offset to the launch's first env.
struct StepIO {
    int8_t *board;
    uint64_t *rng;
    int32_t *timer;
    int32_t *actions;
    int32_t *reward, *n_new, *n_act;
    uint8_t *flags;
    uint64_t *eff;
    int num_moves;
    int autoreset;          // step_env's codes: 0 none, 2 same step (deferred), 4 next step (deferred)
    int sample;             // the in-kernel policy (Params::sample): actions[e] <- its draw
    uint64_t pol_key;
    int64_t pol_first;
    int32_t pol_t;
};

// TileMatchEnv.step for env e (tile_match_env.py:93-112), the lean path with
// a deferred autoreset; returns the LS_* status bits it raises.
template <class BD>
TMG_LN uint32_t step_env(const StepIO &io, int64_t e, uint8_t *scratch) {
    constexpr int W = BD::W, N = BD::N;
    uint64_t mw[W];
    const uint64_t *em = io.eff + e * W;
#pragma unroll
    for (int i = 0; i < W; i++) mw[i] = em[i];
    int a = io.actions[e];
    const int t0 = io.timer[e];
    if (io.sample) {
        a = policy_action<W>(mw, BD::A, io.pol_key, (uint64_t)(io.pol_first + e), io.pol_t);
        io.actions[e] = a;
    }
    const int M = io.num_moves;
    const bool pend = io.autoreset == 4 && t0 >= M;                    // next step: reset() now
    if (!pend && (t0 >= M || a < 0 || a >= BD::A)) {                 // tile_match_env.py:94-95
        io.reward[e] = 0; io.n_new[e] = 0; io.n_act[e] = 0;
        io.flags[e] = (uint8_t)LF_ERR;
        return LS_CALLER;
    }
    const int t1 = t0 + 1;
    const bool same = io.autoreset == 2;
    const bool done = !pend && t1 == M;                              // tile_match_env.py:100-101
    const bool regen = pend || (done && same);
    int flags = done ? LF_DONE : 0;
    const bool effective = !pend && ((mw[a >> 6] >> (a & 63)) & 1ULL);
    int elim = 0;
    if (effective) {
        BD b;
        unpack(b, reinterpret_cast<const uint64_t *>(io.board + e * 2 * N));
        Rng g;
        rng_load(g, io.rng + e * 5);
        int r1, c1, r2, c2;
        if (a < BD::AV) { r1 = a / BD::C; c1 = a - r1 * BD::C; r2 = r1 + 1; c2 = c1; }
        else { const int i = a - BD::AV; r1 = i / (BD::C - 1); c1 = i - r1 * (BD::C - 1); r2 = r1; c2 = c1 + 1; }
        elim = move(b, g, r1 * BD::C + c1, r2 * BD::C + c2, flags, mw, scratch);
        uint64_t *ob = reinterpret_cast<uint64_t *>(io.board + e * 2 * N);
        constexpr int NQ = N / 8;
#pragma unroll
        for (int i = 0; i < NQ; i++) ob[i] = pack_word(b, i);
        if constexpr (N % 8 != 0) {                                  // the tail cells, 4 / 2 / 1 bytes
            const uint64_t w = pack_word(b, NQ);
            uint8_t *tb = reinterpret_cast<uint8_t *>(ob + NQ);
            int j = 0;
            if constexpr ((N % 8) & 4) { *reinterpret_cast<uint32_t *>(tb) = (uint32_t)w; j = 4; }
            if constexpr ((N % 8) & 2) { *reinterpret_cast<uint16_t *>(tb + j) = (uint16_t)(w >> (8 * j)); j += 2; }
            if constexpr ((N % 8) & 1) { tb[j] = (uint8_t)(w >> (8 * j)); }
        }
        rng_store(g, io.rng + e * 5);
    }
    uint64_t *ge = io.eff + e * W;
    if (done && !same) {                                             // tile_match_env.py:119-120
#pragma unroll
        for (int i = 0; i < W; i++) ge[i] = 0ULL;
    } else if (effective && !regen) {                                // (a regenerated env's mask comes from reset_kernel)
#pragma unroll
        for (int i = 0; i < W; i++) ge[i] = mw[i];
    }
    if (regen) flags |= LF_RESET;
    io.timer[e] = regen ? 0 : t1;
    io.reward[e] = elim;
    io.n_new[e] = 0;
    io.n_act[e] = 0;
    io.flags[e] = (uint8_t)flags;
    return (flags & LF_ERR) ? LS_INTERNAL : 0u;
}

}  // namespace lane
}  // namespace tmg
