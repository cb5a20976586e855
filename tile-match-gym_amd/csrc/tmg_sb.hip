// tmg_sb.hip — scalar bitboards: the no-specials path for boards of <= 128
// cells (c2/c4: 10x10, 4 colours).  Included by tmg_board.hip.
//
// Cell p = r*C + c is bit p>>1 of word p&1 (`a` = even cells, `b` = odd
// cells), and a colour is NB bit-planes of (colour - 1).  With one wave per
// board, lane j's PCG output j carries the colours of cells 2j and 2j+1, so
// one __ballot per plane turns a lane-parallel draw straight into bitboards.
// Everything wave-uniform — line detection (get_colour_lines' first pass,
// board.py:158-193), its perpendicular pass (:195-214), the clear mask of a
// cascade step and remove_colour_lines' first line (:120-131) — then runs as
// 64-bit SALU ops on SGPRs, leaving the VALU to the RNG and the lane-parallel
// gravity/refill scatter.  The int8 LDS board stays in sync at the points the
// shared code reads it (effective-action scan, shuffle, store).


struct Pair {
    uint64_t a, b;
};
__device__ __forceinline__ Pair operator&(Pair x, Pair y) { return Pair{x.a & y.a, x.b & y.b}; }
__device__ __forceinline__ Pair operator|(Pair x, Pair y) { return Pair{x.a | y.a, x.b | y.b}; }
__device__ __forceinline__ Pair operator^(Pair x, Pair y) { return Pair{x.a ^ y.a, x.b ^ y.b}; }
__device__ __forceinline__ Pair andn(Pair x, Pair y) { return Pair{x.a & ~y.a, x.b & ~y.b}; }   // x & ~y
__device__ __forceinline__ bool nonzero(Pair x) { return (x.a | x.b) != 0ULL; }
__device__ __forceinline__ int popc(Pair x) { return __popcll(x.a) + __popcll(x.b); }
__device__ __forceinline__ uint64_t lowmask(int n) { return n >= 64 ? ~0ULL : ((1ULL << n) - 1ULL); }   // n >= 0
__device__ __forceinline__ bool test(Pair x, int p) { return (((p & 1) ? x.b : x.a) >> (p >> 1)) & 1ULL; }
__device__ __forceinline__ int ctz64(uint64_t x) { return __ffsll((unsigned long long)x) - 1; }

// per-row masks from Params::sb_rows, read through the scalar cache
#ifndef TMG_CONST_AS
#define TMG_CONST_AS __attribute__((address_space(4)))
#endif
typedef const TMG_CONST_AS uint64_t sbrow_t;

// an empty asm that reads three VGPR values: they must exist at this point
#ifndef TMG_KEEP_V3
#define TMG_KEEP_V3(x, y, z) asm volatile("" ::"v"(x), "v"(y), "v"(z))
#endif
// cells of row r.  Even C: row r is bits [rC/2, rC/2 + C/2) of both words,
// two SALU ops instead of two dependent scalar loads in the cascade loop.
template <bool CODD>
__device__ __forceinline__ Pair sb_row(const Params &P, int r) {
    if constexpr (!CODD) {
        const int h = P.C >> 1;
        const uint64_t m = lowmask(h) << (r * h);
        return Pair{m, m};
    } else {
        const sbrow_t *t = (const sbrow_t *)P.sb_rows + 4 * r;
        return Pair{t[0], t[1]};
    }
}

// fwd: result[q] = x[q - d] (content moves d cells forward); bwd: result[q] =
// x[q + d].  ODD = parity of d.  Requires d <= 127 - 1 (shifts < 64).
template <bool ODD>
__device__ __forceinline__ Pair fwd(Pair x, int d) {
    if constexpr (ODD) return Pair{x.b << ((d + 1) >> 1), x.a << ((d - 1) >> 1)};
    else return Pair{x.a << (d >> 1), x.b << (d >> 1)};
}
template <bool ODD>
__device__ __forceinline__ Pair bwd(Pair x, int d) {
    if constexpr (ODD) return Pair{x.b >> ((d - 1) >> 1), x.a >> ((d + 1) >> 1)};
    else return Pair{x.a >> (d >> 1), x.b >> (d >> 1)};
}

template <int NB>
struct SB {
    Pair p[NB];
};

// number of bit-planes for colour codes 0..k-1
__host__ __device__ constexpr int sb_planes(int k) { return k <= 2 ? 1 : k <= 4 ? 2 : k <= 8 ? 3 : 4; }

// The lane-side copy of the same board: colour codes (colour - 1) of cells
// 2*lane (a) and 2*lane+1 (b), 0 outside the board.  Draws and the gravity
// scatter update these; the bitboards are their ballots.
struct SBC {
    int a, b;
};

template <int NB>
__device__ __forceinline__ SB<NB> sb_planes_of(const SBC &c) {
    SB<NB> s;
#pragma unroll
    for (int b = 0; b < NB; b++) {
        s.p[b].a = __ballot((c.a >> b) & 1);
        s.p[b].b = __ballot((c.b >> b) & 1);
    }
    return s;
}

__device__ __forceinline__ SBC sb_codes_from_lds(const Params &P, const int8_t *brd, int lane) {
    const int q0 = 2 * lane, N = P.N;
    return SBC{q0 < N ? (int)brd[q0] - 1 : 0, q0 + 1 < N ? (int)brd[q0 + 1] - 1 : 0};
}

__device__ __forceinline__ void sb_codes_to_lds(const Params &P, int8_t *brd, int8_t *trash, int lane, const SBC &c) {
    const int q0 = 2 * lane, N = P.N;
    *(q0 < N ? brd + q0 : trash + lane) = (int8_t)(c.a + 1);
    *(q0 + 1 < N ? brd + q0 + 1 : trash + 64 + lane) = (int8_t)(c.b + 1);
}

// get_colour_lines' first pass on a full board (board.py:158-193): va = a
// vertical line has its bottom cell here (r >= 2, same colour as the two cells
// above), ha = a horizontal run of >= 3 may start here (c <= C-3).  neU / neR:
// colour differs from the cell above / to the right (garbage at the edges).
struct SBDet {
    Pair va, ha, neU, neR;
};

// z: colourless cells (cookies, colour 0), which match nothing (anchors need
// type > 0, runs extend by colour, board.py:163-188, 196).
template <int NB, bool CODD>
__device__ __forceinline__ SBDet sb_detect(const Params &P, const SB<NB> &s, Pair z = Pair{0, 0}) {
    const int C = P.C;
    SBDet d;
    d.neU = z | fwd<CODD>(z, C);
    d.neR = z | bwd<true>(z, 1);
#pragma unroll
    for (int b = 0; b < NB; b++) {
        d.neU = d.neU | (s.p[b] ^ fwd<CODD>(s.p[b], C));
        d.neR = d.neR | (s.p[b] ^ bwd<true>(s.p[b], 1));
    }
    d.va = andn(Pair{P.sb_v[0], P.sb_v[1]}, d.neU | fwd<CODD>(d.neU, C));
    d.ha = andn(Pair{P.sb_h[0], P.sb_h[1]}, d.neR | bwd<true>(d.neR, 1));
    return d;
}

// bottom-most row holding a line start (get_colour_lines scans rows bottom-up
// and stops at the first row with a line), or -1
__device__ __forceinline__ int sb_bottom_row(const Params &P, const SBDet &d) {
    const Pair m = d.va | d.ha;
    const int pa = m.a ? 2 * (63 - __clzll(m.a)) : -1;
    const int pb = m.b ? 2 * (63 - __clzll(m.b)) + 1 : -1;
    const int pm = pa > pb ? pa : pb;
    return pm < 0 ? -1 : div_c(P, pm);
}

// remove_colour_lines (board.py:120-131) needs the row of the first coord of
// the first line get_colour_lines returns: sb_first_line_key gives that line's
// key (or -1: no line), sb_line_row_of_key the row.  get_colour_lines scans rows
// bottom-up and, in the first row holding a line, columns left to right with
// the vertical check first; so the first line is the maximum over anchor
// cells of key = (row, -col, is_vertical), taken lane-parallel (keyA/keyB:
// the cells' (row << 8 | 255 - col) << 1, -1 outside the board) by one DPP
// max.  A vertical line starts at the top of its run (:166-172).
template <int NB, bool CODD>
__device__ __forceinline__ int sb_first_line_key(const Params &P, const SBDet &d, int lane, int keyA, int keyB) {
    (void)P;
    const int vA = (int)(d.va.a >> lane) & 1, hA = (int)(d.ha.a >> lane) & 1;
    const int vB = (int)(d.va.b >> lane) & 1, hB = (int)(d.ha.b >> lane) & 1;
    const int ka = (vA | hA) ? keyA | vA : -1, kb = (vB | hB) ? keyB | vB : -1;
    return wave_max(ka > kb ? ka : kb);
}
template <bool CODD>
__device__ __forceinline__ int sb_line_row_of_key(const Params &P, const SBDet &d, int key) {   // key >= 0
    const int rs = key >> 9;
    if (!(key & 1)) return rs;
    const int C = P.C;
    int t = (rs - 2) * C + 255 - ((key >> 1) & 255);
    while (t >= C && !test(d.neU, t)) t -= C;
    return div_c(P, t);
}
// the keys of sb_first_line_key for cells 2*lane, 2*lane+1
__device__ __forceinline__ void sb_line_keys(const Params &P, int lane, int &keyA, int &keyB) {
    const int q0 = 2 * lane, q1 = q0 + 1;
    const int r0 = div_c(P, q0), r1 = div_c(P, q1);
    keyA = q0 < P.N ? ((r0 << 8) | (255 - (q0 - r0 * P.C))) << 1 : -1;
    keyB = q1 < P.N ? ((r1 << 8) | (255 - (q1 - r1 * P.C))) << 1 : -1;
}

// The first-pass coords of get_colour_lines' bottom row rs (board.py:158-193):
// kh = cells of its horizontal runs, kv = cells of the vertical runs ending
// in it (from the bottom up while the colour holds, :166-172).
template <bool CODD>
__device__ __forceinline__ void sb_coords(const Params &P, const SBDet &d, int rs, Pair &kh, Pair &kv) {
    const int C = P.C;
    const Pair row = sb_row<CODD>(P, rs);
    const Pair eqU = andn(Pair{P.sb_u[0], P.sb_u[1]}, d.neU);      // same colour as the cell above
    const Pair h = d.ha & row;
    kh = h | fwd<true>(h, 1) | fwd<false>(h, 2);
    const Pair v = d.va & row;
    kv = Pair{0, 0};
    if (nonzero(v)) {
        Pair t = bwd<false>(v, 2 * C);
        kv = v | bwd<CODD>(v, C) | t;
        for (;;) {
            t = bwd<CODD>(t & eqU, C);
            if (!nonzero(t)) break;
            kv = kv | t;
        }
    }
}

// get_colour_lines' perpendicular pass (board.py:195-214): from every coord of K
// walk each axis over non-coord cells of the same colour; a run of >= 3 is a
// line.  Adds the cells of those lines to clr; returns whether there is one.
// On a board of type-1 tiles (the lean path) only the horizontal part can find
// a line: a vertical run through a coord would extend a first-pass vertical or
// be anchored below row rs (HORIZ_ONLY skips it).
template <bool CODD, bool HORIZ_ONLY = false>
__device__ __forceinline__ bool sb_perpendicular(const Params &P, const SBDet &d, const Pair K, Pair &clr) {
    const int C = P.C;
    const Pair inb{P.sb_in[0], P.sb_in[1]};
    const Pair nf{P.sb_nf[0], P.sb_nf[1]};
    const Pair eqR = andn(Pair{P.sb_nl[0], P.sb_nl[1]}, d.neR);   // same colour as the right neighbour
    const Pair eqU = andn(Pair{P.sb_u[0], P.sb_u[1]}, d.neU);      // same colour as the cell above
    const Pair walk = andn(inb, K);
    bool any = false;
    // horizontal runs through coords
    const Pair r1 = fwd<true>(K & eqR, 1) & walk;
    const Pair l1 = bwd<true>(K & nf, 1) & eqR & walk;
    if (nonzero(r1 | l1)) {
        const Pair r2 = fwd<true>(r1 & eqR, 1) & walk;
        const Pair l2 = bwd<true>(l1 & nf, 1) & eqR & walk;
        const Pair q = K & (bwd<false>(r2, 2) | fwd<false>(l2, 2) | (bwd<true>(r1, 1) & fwd<true>(l1, 1)));
        if (nonzero(q)) {
            any = true;
            Pair f = fwd<true>(q & eqR, 1) & walk;
            while (nonzero(f)) { clr = clr | f; f = fwd<true>(f & eqR, 1) & walk; }
            Pair g = bwd<true>(q & nf, 1) & eqR & walk;
            while (nonzero(g)) { clr = clr | g; g = bwd<true>(g & nf, 1) & eqR & walk; }
        }
    }
    if constexpr (HORIZ_ONLY) return any;
    // vertical runs through coords
    const Pair d1 = fwd<CODD>(K, C) & eqU & walk;
    const Pair u1 = bwd<CODD>(K & eqU, C) & walk;
    if (nonzero(d1 | u1)) {
        const Pair d2 = fwd<CODD>(d1, C) & eqU & walk;
        const Pair u2 = bwd<CODD>(u1 & eqU, C) & walk;
        const Pair q = K & (fwd<false>(u2, 2 * C) | bwd<false>(d2, 2 * C) | (fwd<CODD>(u1, C) & bwd<CODD>(d1, C)));
        if (nonzero(q)) {
            any = true;
            Pair f = fwd<CODD>(q, C) & eqU & walk;
            while (nonzero(f)) { clr = clr | f; f = fwd<CODD>(f, C) & eqU & walk; }
            Pair g = bwd<CODD>(q & eqU, C) & walk;
            while (nonzero(g)) { clr = clr | g; g = bwd<CODD>(g & eqU, C) & walk; }
        }
    }
    return any;
}

// One cascade step when no special can exist (board.py:367-376 with every
// line a normal match): the union of get_colour_lines' lines in row rs.
template <int NB, bool CODD>
__device__ __forceinline__ Pair sb_clear(const Params &P, const SBDet &d, int rs) {
    Pair kh, kv;
    sb_coords<CODD>(P, d, rs, kh, kv);
    const Pair K = kh | kv;
    Pair clr = K;
    sb_perpendicular<CODD, true>(P, d, K, clr);
    return clr;
}

// gravity + refill (board.py:217-241) of the cleared cells E (total of them),
// as one LDS scatter: each lane owns cells 2*lane and 2*lane+1; a kept cell
// drops by the empties below it in its column, the top `empties` cells of a
// column take the refill draws in row-major order.  Leaves the new board in
// LDS and in c.
// TYPES: move the type plane too (boards with specials); the refilled cells
// become normal tiles (type 1).  Without it the type plane is all 1 and stays.
template <bool CODD, bool TYPES = false, class WS>
__device__ __forceinline__ void sb_gravity_refill(const Params &P, WS &w, int lane_, const LaneJump &J, Rng &g,
                                                  const Pair E, int total, SBC &c) {
    const int N = P.N, C = P.C;
    // the refill draws first, while nothing per-lane is live beside the RNG
    // (the jump-ahead's 128-bit products need the registers)
    draw_colours<true>(P, lane_, J, g, total, w.u.draw, w.trash);
    const int lane = loop_lane(lane_);           // the per-lane column masks below are rebuilt per call
    int8_t *col = w.brd, *typ = w.brd + N;
    const int q0 = 2 * lane, q1 = q0 + 1;
    const int r0 = div_c(P, q0), c0 = q0 - r0 * C;
    const int r1 = div_c(P, q1), c1 = q1 - r1 * C;
    // the cells of a column: zcol shifted to the column's first bit in each word
    uint64_t ca0, cb0, ca1, cb1;
    if constexpr (CODD) {
        // rows with (r + c) even are even cells
        const int sa0 = ((c0 & 1) * C + c0) >> 1, sb0 = ((1 - (c0 & 1)) * C + c0) >> 1;
        const int sa1 = ((c1 & 1) * C + c1) >> 1, sb1 = ((1 - (c1 & 1)) * C + c1) >> 1;
        ca0 = P.sb_z << sa0; cb0 = P.sb_z << sb0;
        ca1 = P.sb_z << sa1; cb1 = P.sb_z << sb1;
    } else {
        // cell 2*lane has an even column (all even cells), 2*lane+1 an odd one
        ca0 = P.sb_z << (c0 >> 1); cb0 = 0;
        ca1 = 0; cb1 = P.sb_z << (c1 >> 1);
    }
    const uint64_t ea0 = E.a & ca0, eb0 = E.b & cb0, ea1 = E.a & ca1, eb1 = E.b & cb1;
    const int ec0 = __popcll(ea0) + __popcll(eb0);
    const int ec1 = __popcll(ea1) + __popcll(eb1);
    // empties strictly below: cells > q of the column
    const int below0 = __popcll(ea0 & ~lowmask((q0 >> 1) + 1)) + __popcll(eb0 & ~lowmask((q0 + 1) >> 1));
    const int below1 = __popcll(ea1 & ~lowmask((q1 >> 1) + 1)) + __popcll(eb1 & ~lowmask((q1 + 1) >> 1));
    const bool v0 = q0 < N, v1 = q1 < N;
    const bool e0 = v0 && ((E.a >> lane) & 1ULL), e1 = v1 && ((E.b >> lane) & 1ULL);
    const bool n0 = v0 && r0 < ec0, n1 = v1 && r1 < ec1;   // refilled after gravity
    const uint64_t NA = __ballot(n0), NBm = __ballot(n1);
    const int rank0 = popc_below(NA) + popc_below(NBm);
    const int rank1 = rank0 + (n0 ? 1 : 0);
    int8_t y0 = 1, y1 = 1;
    if constexpr (TYPES) {
        y0 = typ[v0 ? q0 : 0];
        y1 = typ[v1 ? q1 : 0];
    }
    WSYNC();
    const int8_t d0 = (int8_t)w.u.draw[n0 ? rank0 : 0], d1 = (int8_t)w.u.draw[n1 ? rank1 : 0];
    WFENCE();
    *(v0 && !e0 ? col + q0 + below0 * C : w.trash + lane) = (int8_t)(c.a + 1);
    *(v1 && !e1 ? col + q1 + below1 * C : w.trash + 64 + lane) = (int8_t)(c.b + 1);
    *(n0 ? col + q0 : w.trash + 128 + lane) = d0;
    *(n1 ? col + q1 : w.trash + 192 + lane) = d1;
    if constexpr (TYPES) {
        WFENCE();
        *(v0 && !e0 ? typ + q0 + below0 * C : w.trash + lane) = y0;
        *(v1 && !e1 ? typ + q1 + below1 * C : w.trash + 64 + lane) = y1;
        *(n0 ? typ + q0 : w.trash + 128 + lane) = (int8_t)1;
        *(n1 ? typ + q1 : w.trash + 192 + lane) = (int8_t)1;
    }
    WSYNC();
    c = sb_codes_from_lds(P, col, lane);
}

// rows 0..row (M = (row+1)*C cells) <- Generator.integers(1, k+1, M)
// (board.py:97 generate, :129 remove_colour_lines).  Lane j evaluates PCG
// output j by jump-ahead (as draw_colours; M <= 128 is one 64-output pass)
// and keeps the two colours of its own cells: output j holds draws 2j and
// 2j+1, or, after a buffered half-word (draw 0), draws 2j+1 and 2j+2.
// The batch's jump-ahead depends only on the stream position, not on the row:
// remove_colour_lines computes it before the line search of the board it
// replaces, so the VALU chain issues beside that search's SALU work.
struct SBDrawPre {
    U128 sj;
    uint64_t out;
};
__device__ __forceinline__ SBDrawPre sb_draw_pre(const LaneJump &J, const Rng &g) {
    const U128 sj = jump128(J.Aj, U128{g.slo, g.shi}, J.incG);
    return SBDrawPre{sj, xsl_rr(sj)};
}

template <int NB, class WS>
__device__ __forceinline__ void sb_draw_rows(const Params &P, WS &w, int lane, const LaneJump &J, Rng &g, int row,
                                             SBC &c, const SBDrawPre &pre) {
    const uint32_t k = (uint32_t)P.k;
    const int M = (row + 1) * P.C;
    const bool inA = 2 * lane < M, inB = 2 * lane + 1 < M;
    if (k == 1) {                                        // rng == 0: numpy draws nothing, every colour is 1
        c.a = inA ? 0 : c.a;
        c.b = inB ? 0 : c.b;
        return;
    }
    const int off = (int)(g.h >> 32) & 1;                // draw 0 is the buffered half-word
    const uint64_t mbuf = (uint64_t)(uint32_t)g.h * k;
    const bool rbuf = off && (uint32_t)mbuf < P.thr;
    const int need = M - off;
    const int n64 = (need + 1) >> 1;
    const U128 sj = pre.sj;
    const uint64_t out = pre.out;
    const uint64_t m0 = (uint64_t)(uint32_t)out * k, m1 = (out >> 32) * k;
    const bool ok0 = lane < n64, ok1 = 2 * lane + 1 < need;
    const bool rej = (ok0 && (uint32_t)m0 < P.thr) || (ok1 && (uint32_t)m1 < P.thr);
    if (P.thr != 0u && (rbuf || __ballot(rej) != 0ULL)) {
        // Lemire rejection somewhere: exact serial replay
        draw_colours<true>(P, lane, J, g, M, w.u.draw, w.trash);
        WSYNC();
        c.a = inA ? (int)w.u.draw[2 * lane] - 1 : c.a;
        c.b = inB ? (int)w.u.draw[2 * lane + 1] - 1 : c.b;
        WSYNC();
        return;
    }
    const int lo = (int)(m0 >> 32), hi = (int)(m1 >> 32);          // colour codes 0..k-1
    const int hprev = __builtin_amdgcn_update_dpp((int)(mbuf >> 32), hi, 0x138, 0xf, 0xf, false);   // wave_shr:1
    c.a = inA ? (off ? hprev : lo) : c.a;
    c.b = inB ? (off ? lo : hi) : c.b;
    if (n64 > 0) {
        g.slo = rdlane64(sj.lo, n64 - 1);
        g.shi = rdlane64(sj.hi, n64 - 1);
        g.h = ((uint64_t)(need & 1) << 32) | (uint32_t)rdlane64(out >> 32, n64 - 1);
    } else {
        g.h = (uint32_t)g.h;                             // only the buffered half was used
    }
}

// "while not possible_move() or lines" (board.py:102-109, 381-391) on the
// bitboards.  The LDS board is brought in sync before the effective-action
// scan (whose mask it leaves in w.effw) and the shuffle.  `dirty`: c is newer
// than the LDS board; `clean`: the board is known to hold no line.  Returns
// FL_SHUF when a shuffle ran, FL_ERR when the shuffle cap ended the loop.
// GEN: the loop of generate_board (the cover counters tell the two apart).
template <int NB, bool CODD, bool GEN = false, class WS>
__device__ __forceinline__ int sb_ensure(const Params &P, WS &w, int lane, const LaneJump &J, Rng &g,
                                         const Cells<WS::NP> &cl, SBC &c, bool dirty, bool clean) {
    int keyA, keyB;
    sb_line_keys(P, lane, keyA, keyB);
    int fl = 0;
    for (int shuffles = 0;; shuffles++) {
        if (!clean) {
            for (;;) {
                cover_uniform(P, lane, U128{g.slo, g.shi});
                const SBDrawPre pre = sb_draw_pre(J, g);
                const SBDet d = sb_detect<NB, CODD>(P, sb_planes_of<NB>(c));
                const int key = sb_first_line_key<NB, CODD>(P, d, lane, keyA, keyB);
                TMG_KEEP_V3(pre.sj.lo, pre.sj.hi, pre.out);   // keep the jump-ahead above the exit test
                if (key < 0) break;
                const int r0 = sb_line_row_of_key<CODD>(P, d, key);
                const int row = P.R - 1 < r0 + 1 ? P.R - 1 : r0 + 1;   // colour plane only, rows 0..row
                sb_draw_rows<NB>(P, w, lane, J, g, row, c, pre);
                dirty = true;
            }
        }
        if (dirty) {
            WFENCE();
            sb_codes_to_lds(P, w.brd, w.trash, lane, c);
            WSYNC();
            dirty = false;
        }
#ifndef TMG_KO
#define TMG_KO 0     // diagnostic knock-outs (instruction-count attribution only; results wrong)
#endif
        if (TMG_KO & 1) break;
        if ((TMG_RSCAN & 2) && P.C <= kRowScanMaxC ? scan_rows<false>(P, w, lane, true) != 0
                                                    : scan_effective_clean<false>(P, w, lane))
            break;                                           // types all 1, no line
        if (shuffles >= kMaxShuffles) { fl |= FL_ERR; break; }
        COVER(GEN ? CV_SHUFFLE_GEN : CV_SHUFFLE);
        WSYNC();
        shuffle(P, w, lane, g);
        c = sb_codes_from_lds(P, w.brd, lane);
        fl |= FL_SHUF;
        clean = false;
    }
    WSYNC();
    return fl;
}

// generate_board, board.py:95-109 (types all 1; colours from the env stream),
// draw by draw on the scalar bitboards: boards of C > 32 columns and the exact
// redo after a Lemire rejection (bp_generate otherwise); returns FL_ERR when
// a safety cap was hit
template <int NB, bool CODD, class WS>
__device__ __forceinline__ int sb_generate_exact(const Params &P, WS &w, int lane, const LaneJump &J, Rng &g,
                                                 const Cells<WS::NP> &cl) {
    SBC c{0, 0};
    cover_uniform(P, lane, U128{g.slo, g.shi});
    sb_draw_rows<NB>(P, w, lane, J, g, P.R - 1, c, sb_draw_pre(J, g));
    for (int p = lane; p < P.N; p += 64) w.brd[P.N + p] = 1;
    return sb_ensure<NB, CODD, true>(P, w, lane, J, g, cl, c, true, false) & FL_ERR;
}

// Board.move, board.py:330-395, for a board that can hold no special (every
// type 1, no specials enabled) — the effectiveness test (:352) is the
// caller's.  Returns eliminations; leaves the final board's effective mask in
// w.effw.
template <int NB, bool CODD, class WS>
__device__ __forceinline__ int sb_move(const Params &P, WS &w, int lane, const LaneJump &J, Rng &g,
                                       const Cells<WS::NP> &cl, int p1, int p2, int &flags, int64_t e) {
    (void)e;
    int8_t *col = w.brd;
    if (lane == 0) {                                     // swap_coords :355 (types are all 1)
        int8_t x = col[p1]; col[p1] = col[p2]; col[p2] = x;
    }
    WSYNC();
    SBC c = sb_codes_from_lds(P, col, lane);
    int elim = 0;
    for (; !(TMG_KO & 4);) {                             // :367-376
        const SBDet d = sb_detect<NB, CODD>(P, sb_planes_of<NB>(c));
        const int rs = sb_bottom_row(P, d);
        if (rs < 0) break;
        COVER(CV_SB_LEAN);
        const Pair clr = sb_clear<NB, CODD>(P, d, rs);
        const int tot = popc(clr);
        elim += tot;                                     // R*C - nnz(type) after the resolve (:374)
        sb_gravity_refill<CODD>(P, w, lane, J, g, clr, tot, c);
    }
    flags |= sb_ensure<NB, CODD>(P, w, lane, J, g, cl, c, false, true);   // :381-391
    return elim;
}

// One cascade step of the general kernel (specials enabled, board.py:367-376)
// on bitboards, when process_colour_lines (:269-327) makes every line a
// normal match, a laser or a bomb of the patterns below (no cookie created)
// and, if a matched cell holds a special, no cookie is on the board.
// Returns -1 when there is no line, 0 when the step is not of that kind (the
// caller runs the list machinery on the unchanged LDS board), otherwise the
// number of cleared cells (the board in LDS has been cleared, dropped and
// refilled).
template <int NB, bool CODD, class WS>
__device__ __forceinline__ int sb_simple_step(const Params &P, WS &w, int lane, const LaneJump &J, Rng &g) {
    const int N = P.N, C = P.C;
    const int8_t *col = w.brd, *typ = w.brd + N;
    const int q0 = 2 * lane;
    const int x0 = q0 < N ? (int)col[q0] : 1, x1 = q0 + 1 < N ? (int)col[q0 + 1] : 1;
    const int y0 = q0 < N ? (int)typ[q0] : 1, y1 = q0 + 1 < N ? (int)typ[q0 + 1] : 1;
    // the bitboards model tiles of type >= 1 with colours 1..k and colourless
    // cookies; empty cells (gravity would move them too), cookies that gained a
    // colour (remove_colour_lines, :129) and out-of-range values take the list path
    const auto odd_cell = [&](int x, int y) { return y == 0 || y > 4 || y < -1 || (y < 0 && x != 0) || x < 0 || x > P.k; };
    if (__ballot(odd_cell(x0, y0) || odd_cell(x1, y1)) != 0ULL) return 0;
    SBC c{x0 - 1, x1 - 1};
    const Pair z{__ballot(x0 == 0), __ballot(x1 == 0)};                    // colourless (cookies)
    const SBDet d = sb_detect<NB, CODD>(P, sb_planes_of<NB>(c), z);
    const int rs = sb_bottom_row(P, d);
    if (rs < 0) return -1;
    const int S = P.smask;
    const Pair row = sb_row<CODD>(P, rs);
    const Pair eqU = andn(Pair{P.sb_u[0], P.sb_u[1]}, d.neU);
    // first-pass line lengths: a horizontal run of L cells holds L-2 anchors
    const Pair h = d.ha & row;
    const Pair h2 = h & bwd<true>(h, 1);
    const bool h5 = nonzero(h2 & bwd<false>(h, 2));
    const Pair x4 = bwd<CODD>(bwd<false>(d.va & row, 2 * C) & eqU, C);    // 4th cell of a vertical run
    const bool v5 = nonzero(x4 & eqU);
    if ((h5 || v5) && (S & SP_COOKIE)) return 0;
    const bool hlas = (S & (SP_HLASER | SP_VLASER)) != 0, vlas = (S & SP_VLASER) != 0;
    Pair kh, kv;
    sb_coords<CODD>(P, d, rs, kh, kv);
    const Pair K = kh | kv;
    const Pair inb{P.sb_in[0], P.sb_in[1]};
    // get_colour_lines' perpendicular pass (:195-214).  On a plain board its
    // lines are horizontal runs through a cell of a vertical line above row rs
    // (a run through a row-rs cell, or a vertical one, would be a first-pass
    // line of a row >= rs); X = those crossing cells.
    const Pair eqR = andn(Pair{P.sb_nl[0], P.sb_nl[1]}, d.neR);          // same colour as the right neighbour
    const Pair walk = andn(inb, K);
    Pair X{0, 0};
    {
        const Pair nf{P.sb_nf[0], P.sb_nf[1]};
        const Pair r1 = fwd<true>(K & eqR, 1) & walk;
        const Pair l1 = bwd<true>(K & nf, 1) & eqR & walk;
        if (nonzero(r1 | l1)) {
            const Pair r2 = fwd<true>(r1 & eqR, 1) & walk;
            const Pair l2 = bwd<true>(l1 & nf, 1) & eqR & walk;
            X = K & (bwd<false>(r2, 2) | fwd<false>(l2, 2) | (bwd<true>(r1, 1) & fwd<true>(l1, 1)));
        }
        const Pair d1 = fwd<CODD>(K, C) & eqU & walk;
        const Pair u1 = bwd<CODD>(K & eqU, C) & walk;
        if (nonzero(d1 | u1)) {
            const Pair d2 = fwd<CODD>(d1, C) & eqU & walk;
            const Pair u2 = bwd<CODD>(u1 & eqU, C) & walk;
            if (nonzero(K & (fwd<false>(u2, 2 * C) | bwd<false>(d2, 2 * C) | (fwd<CODD>(u1, C) & bwd<CODD>(d1, C)))))
                return 0;
        }
    }
    if (nonzero(X & (row | kh))) return 0;
    // process_colour_lines (:269-327).  Lines sort by their first coord's row
    // (stable): a vertical before the runs crossing it and before row rs's
    // horizontals.  A 4-line becomes a laser (:294-302; no bomb test); a vertical
    // of 3 or >= 5 cells with bombs enabled becomes a bomb with the first line
    // sharing a cell (:304-320) — its topmost crossing run, else the row-rs run
    // it ends in — taking that line's two cells nearest the shared one (by
    // distance, then column) and, the line being < 6 cells, removing it (its
    // other cells stay).  A crossing run left in the list holds one coord, whose
    // vertical is gone, so it is a normal match (3 cells; longer ones take the
    // list path).  The bomb goes to the shared cell: get_special_creation_pos'
    // corner (:437-447), the bomb's most common row and column.
    uint64_t vcols = 0, xb = 0;                                            // vertical columns; bombs into the row-rs run
    Pair pall{0, 0}, keep{0, 0}, pbomb{0, 0};                              // crossing runs, cells that stay, bomb cells
    if (nonzero(X) || nonzero(kh & kv)) {
        vcols = __ballot(lane < C && test(kv, rs * C + lane));
        for (uint64_t m = vcols; m; m &= m - 1) {
            const int cc = ctz64(m);
            Pair colm;
            if constexpr (CODD) {
                colm = Pair{P.sb_z << ((((cc & 1) * C) + cc) >> 1), P.sb_z << ((((1 - (cc & 1)) * C) + cc) >> 1)};
            } else {
                colm = (cc & 1) ? Pair{0, P.sb_z << (cc >> 1)} : Pair{P.sb_z << (cc >> 1), 0};
            }
            colm = colm & inb;
            const int L = popc(kv & colm);
            const bool bomber = (S & SP_BOMB) && L != 4 && !(L >= 5 && (S & SP_COOKIE));
            bool first = true;
            for (Pair xc = X & colm; nonzero(xc); first = false) {
                const int qa = xc.a ? 2 * ctz64(xc.a) : 1 << 20, qb = xc.b ? 2 * ctz64(xc.b) + 1 : 1 << 20;
                const int q = qa < qb ? qa : qb;                           // topmost crossing left
                if (q & 1) xc.b &= xc.b - 1; else xc.a &= xc.a - 1;
                int lf = 0, rt = 0;
                while (cc - lf - 1 >= 0 && test(walk, q - lf - 1) && test(eqR, q - lf - 1)) lf++;
                while (cc + rt + 1 < C && test(walk, q + rt + 1) && test(eqR, q + rt)) rt++;
                Pair run{0, 0};
                for (int p = q - lf; p <= q + rt; p++) {
                    if (p & 1) run.b |= 1ULL << (p >> 1); else run.a |= 1ULL << (p >> 1);
                }
                if (nonzero(run & pall)) return 0;                         // runs sharing cells
                pall = pall | run;
                const int len = lf + rt + 1;
                if (bomber && first) {
                    if (len > 5) return 0;
                    const int t1 = lf > 0 && rt > 0 ? q - 1 : lf == 0 ? q + 1 : q - 1;
                    const int t2 = lf > 0 && rt > 0 ? q + 1 : lf == 0 ? q + 2 : q - 2;
                    Pair take{0, 0};
                    for (const int p : {q, t1, t2}) {
                        if (p & 1) take.b |= 1ULL << (p >> 1); else take.a |= 1ULL << (p >> 1);
                    }
                    keep = keep | andn(run, take);
                    if (q & 1) pbomb.b |= 1ULL << (q >> 1); else pbomb.a |= 1ULL << (q >> 1);
                } else if (len != 3) {
                    return 0;
                }
            }
            if (bomber && first && test(kh, rs * C + cc)) xb |= 1ULL << cc;
        }
    }
    uint64_t keepc = 0, gonec = 0;                                         // row-rs runs a bomb took
    if (xb) {
        const uint64_t hbc = __ballot(lane < C && test(h, rs * C + lane));
        if (!bomb_plan(hbc, xb, keepc, vcols, gonec)) return 0;
    }
    Pair clr = andn(K | pall, keep);                                       // matched cells
    const Pair sp{__ballot(y0 >= 2), __ballot(y1 >= 2)};                  // lasers / bombs
    // specials on matched cells activate (resolve_colour_match :460-471).  With
    // no cookie on the board (the only order-dependent special) the result is
    // the closure: each activated special clears its column (v-laser), row
    // (h-laser) or 3x3 (bomb) and activates the specials there (:473-525).
    const bool act = nonzero(clr & sp);
    if (act && nonzero(z)) return 0;
    // creation cells (create_special :572-597, after every activation): lasers
    // at a straight 4-line's second cell in (row, col) order, (rs, s+1) for a
    // horizontal run from s not taken by a bomb, (top+1, c) for a vertical one
    // (nothing of theirs is taken, :429-458); bombs at their shared cell
    int8_t *ty = w.brd + N;
    const int r0 = div_c(P, q0), r1 = div_c(P, q0 + 1);
    const int c0 = q0 - rs * C, c1 = q0 + 1 - rs * C;
    const bool in0 = r0 == rs, in1 = r1 == rs;                             // cells of row rs
    Pair ph = hlas ? fwd<true>(andn(andn(h2, bwd<false>(h, 2)), fwd<true>(h, 1)), 1) : Pair{0, 0};
    if (gonec) ph = andn(ph, Pair{__ballot(in0 && ((gonec >> c0) & 1)), __ballot(in1 && ((gonec >> c1) & 1))});
    const Pair pv = vlas ? fwd<CODD>(andn(x4, eqU), C) : Pair{0, 0};
    const Pair bombs = pbomb | Pair{__ballot(in0 && ((xb >> c0) & 1)), __ballot(in1 && ((xb >> c1) & 1))};
    keep = keep | Pair{__ballot(in0 && ((keepc >> c0) & 1)), __ballot(in1 && ((keepc >> c1) & 1))};
    clr = andn(clr, keep);
    {
        const int th = (S & SP_HLASER) ? 3 : 2;
        // the lane owning the cell writes its type; sb_gravity_refill reads it back on the same lane
        const int t0 = test(ph, q0) ? th : test(pv, q0) ? 2 : test(bombs, q0) ? 4 : 0;
        const int t1 = test(ph, q0 + 1) ? th : test(pv, q0 + 1) ? 2 : test(bombs, q0 + 1) ? 4 : 0;
        *(t0 ? ty + q0 : w.trash + lane) = (int8_t)t0;
        *(t1 ? ty + q0 + 1 : w.trash + 64 + lane) = (int8_t)t1;
    }
    const Pair pos = ph | pv | bombs;
    if (act) {
        const Pair vls{__ballot(y0 == 2), __ballot(y1 == 2)}, hls{__ballot(y0 == 3), __ballot(y1 == 3)};
        Pair done{0, 0}, front = clr & sp;
        while (nonzero(front)) {
            const int s = front.a ? 2 * ctz64(front.a) : 2 * ctz64(front.b) + 1;
            const Pair bit{(s & 1) ? 0ULL : 1ULL << (s >> 1), (s & 1) ? 1ULL << (s >> 1) : 0ULL};
            done = done | bit;
            const int r = div_c(P, s), cc = s - r * C;
            Pair area;
            if (nonzero(bit & vls)) {                                      // v-laser: column cc
                if constexpr (CODD) {
                    area = Pair{P.sb_z << ((((cc & 1) * C) + cc) >> 1), P.sb_z << ((((1 - (cc & 1)) * C) + cc) >> 1)};
                } else {
                    area = (cc & 1) ? Pair{0, P.sb_z << (cc >> 1)} : Pair{P.sb_z << (cc >> 1), 0};
                }
                area = area & inb;
            } else if (nonzero(bit & hls)) {                               // h-laser: row r
                area = sb_row<CODD>(P, r);
            } else {                                                       // bomb: 3x3
                area = Pair{0, 0};
                for (int i = r > 0 ? r - 1 : 0; i <= (r + 1 < P.R ? r + 1 : P.R - 1); i++)
                    for (int j = cc > 0 ? cc - 1 : 0; j <= (cc + 1 < C ? cc + 1 : C - 1); j++) {
                        const int q = i * C + j;
                        if (q & 1) area.b |= 1ULL << (q >> 1);
                        else area.a |= 1ULL << (q >> 1);
                    }
            }
            clr = clr | area;
            front = andn(clr & sp, done);
        }
        if (lane == 0) w.sc[SC_NACT] += popc(done);
    }
    if (nonzero(pos)) {
        clr = andn(clr, pos);
        if (lane == 0) w.sc[SC_NNEW] += popc(pos);
    }
    const int tot = popc(clr);
#if TMG_COVER
    if (nonzero(ph | pv)) COVER(CV_SB_LASER);
    if (nonzero(pbomb)) COVER(CV_SB_PERP_BOMB);
    if (xb) COVER(CV_SB_ROW_BOMB);
    if (act) COVER(CV_SB_CLOSURE);
    if (!nonzero(pos) && !act) COVER(CV_SB_NORMAL);
#endif
    sb_gravity_refill<CODD, true>(P, w, lane, J, g, clr, tot, c);
    return tot;
}
