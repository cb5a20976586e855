// tmg_board.hip — the batched tile-match Board on MI355X (gfx950).
//
// One wavefront (64 lanes) owns one board.  The board's int8 colour/type
// planes live in LDS for the whole call; lanes map to cells for the
// data-parallel stages (line detection by ballot, effective-action scan,
// gravity scatter, refill, colour regeneration, shuffle apply) and to 64
// consecutive PCG64 outputs for random draws (jump-ahead).  Detection results
// stay in wave-uniform ballot masks; the per-env RNG state stays in scalar
// registers for the whole call.  The order-dependent list logic of the
// reference (get_colour_lines' perpendicular pass, process_colour_lines,
// special placement, the recursive activate_special DFS, combination_match)
// runs on lane 0 against LDS with an explicit stack; it is compiled only into
// the general kernel variant.  With no specials enabled the lean variant keeps
// the whole cascade wave-parallel.
//
// Reference: akshilpatel/tile-match-gym v1.0.6, src/tile_match_gym/board.py
// and tile_match_env.py (file:line cited per function).  Bit-exact per seed.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pcg64.h"

namespace tmg {

// One wave (one board) per 64-thread workgroup: a workgroup's slot is held
// until its slowest wave ends, so 2 / 4 boards per workgroup measured slower
// (DESIGN.md §7).  The wave synchronises its LDS accesses with the workgroup
// barrier.
#define WSYNC() __syncthreads()

// Minimum waves per SIMD asked of the register allocator (launch bounds), per
// kernel; each measured on the MI355X against its neighbours.
// step_kernel<128, false>: the c2 / c4 kernel.  8 waves/SIMD (64 VGPRs, no
// scratch) since round 6 (the row-plane scan freed registers): c4 shard 12.4
// -> 12.8, c2-eff 4.9 -> 5.0 x 10^8, c2 and its 20-step window the same
// (profiles/r06/s9); round 5 measured 7 ahead by 1 %.
#ifndef TMG_LEAN128_WAVES
#define TMG_LEAN128_WAVES 8
#endif
constexpr int kLean128Waves = TMG_LEAN128_WAVES;
constexpr int kLean128GenericWaves = 7;   // the generic lean instantiations (8 spills 48-56 B there)
constexpr int kGen128Waves = 5;      // step_kernel<128, true>: c3 (96 VGPRs; 6 / 7 spill and lose, also specialised)
#ifndef TMG_RESET512_WAVES
#define TMG_RESET512_WAVES 8
#endif
#ifndef TMG_RESET128_WAVES
#define TMG_RESET128_WAVES 8
#endif
constexpr int kReset512Waves = TMG_RESET512_WAVES;   // reset_kernel<512>: c5's regeneration (7: 0.8 % slower, profiles/r04/s7)
constexpr int kReset128Waves = TMG_RESET128_WAVES;   // reset_kernel<128> specialised for 10x10 k4 (c3): 63 VGPRs
// envs per wave of a masked reset_kernel launch (the deferred autoreset after a
// general step; 29 of 30 find no finished env).  10x10 boards: 1 / 2 / 4 / 8 /
// 16 measured c3 6.97 / 7.10 / 7.19 / 7.17 / 7.15 x 10^8; 20x20 boards, whose
// regenerations are long: 2 (4 made the storm 4 % slower).
constexpr int kMaskedResetEnvs128 = 8;
constexpr int kMaskedResetEnvs512 = 2;
constexpr int kC5StepWaves = 4;      // step_kernel<512, true> specialised for c5 (128 VGPRs; 3 measured the same)

// compiler-only ordering point between a wave's LDS loads and later stores
#define WFENCE() __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront")

// dynamic LDS of the workgroup (overridable only by the host-side wave
// emulator in tools/wave_emu, which runs this file under AddressSanitizer)
#ifndef TMG_SMEM_DECL
#define TMG_SMEM_DECL(name) extern __shared__ __align__(16) unsigned char name[]
#endif

enum : int { SP_COOKIE = 1, SP_VLASER = 2, SP_HLASER = 4, SP_BOMB = 8 };
enum : int { M_NORMAL = 0, M_VLASER = 1, M_HLASER = 2, M_BOMB = 3, M_COOKIE = 4 };
enum : int { FL_DONE = 1, FL_COMBO = 2, FL_SHUF = 4, FL_RESET = 8, FL_OVF = 0x40, FL_ERR = 0x80 };
// The general step runs in two tiers (step_env's TIER): the step kernel with
// its lane-0 lists in LDS (WsSerial), and, for the steps whose cascade
// outgrows those, spill_kernel, which re-runs them on worst-case
// global-memory lists (WsSerialBig).
enum : int { TIER_MAIN = 0, TIER_SPILL = 2 };
// sticky status (tmg_status): what any env met since the last clear
enum : uint32_t { ST_INTERNAL = 1, ST_OVERFLOW = 2, ST_CALLER = 4 };

// Safety cap of the "while not possible_move() or lines" loop (board.py:102-109,
// 381-391).  Its redraw part ends with probability 1 on every shape tmg_create
// accepts (a full redraw, row R-1, can always come out line-free, and every
// line found lets the next redraw reach its rows), so it is not counted.  The
// shuffle part can spin forever on a colour multiset that has no playable
// line-free arrangement (e.g. 3x3 with at most two tiles of each colour): there
// the reference loops forever; here the wave ends the loop with FL_ERR.
constexpr int kMaxShuffles = 1 << 12;   // shuffles per loop

// Per-stream queue of the envs whose step ran out of LDS list space
// (step_env), drained by spill_kernel.  Sized by the host for the envs of
// the launch (cap >= n), so every such env fits: no step is ever dropped.
constexpr int kSpillWaves = 16;          // spill_kernel workgroups (one wave, one WsSerialBig each)
struct SpillQ {
    uint32_t count, done;        // queued envs; spill_kernel waves finished
    unsigned long long total;    // envs re-run so far (diagnostic, tmg_spills)
    int64_t cap;                 // entries of env[] (>= the envs of any launch on this stream)
    int64_t env[1];              // [cap]
};

// Diagnostic build only (TMG_COVER=1, never the product library): per-branch
// hit counters of the cascade step forms (tmg_debug_cover), so tests can show
// that every wave-parallel form and the lane-0 fallback ran.
#ifndef TMG_COVER
#define TMG_COVER 0
#endif
enum : int {
    CV_SB_LEAN = 0,      // lean bitboard cascade step (no specials enabled)
    CV_SB_NORMAL,        // sb_simple_step: plain normal matches only
    CV_SB_LASER,         // sb_simple_step: a laser created
    CV_SB_PERP_BOMB,     // sb_simple_step: a bomb with a perpendicular (crossing) run
    CV_SB_ROW_BOMB,      // sb_simple_step: a bomb with a row-rs run (bomb_plan)
    CV_SB_CLOSURE,       // sb_simple_step: matched specials activated (closure)
    CV_SB_FALLBACK,      // sb_simple_step declined: lane-0 list step follows
    CV_LDS_NORMAL,       // simple_step_lds (512-cell kernels): normal matches only
    CV_LDS_LASER,        // simple_step_lds: a laser created
    CV_LDS_BOMB,         // simple_step_lds: a bomb (bomb_plan)
    CV_LDS_FALLBACK,     // simple_step_lds declined on a plain board
    CV_SERIAL_STEP,      // lane-0 list step (get_colour_lines / process / resolve)
    CV_SERIAL_ACT,       // activate_special entered on the lane-0 path
    CV_SERIAL_COOKIE,    // a cookie activated on the lane-0 path
    CV_COMBO,            // combination_match
    CV_SPILL,            // step queued for spill_kernel
    CV_SPILL_RUN,        // step re-run by spill_kernel
    CV_SHUFFLE,          // shuffle in a move's ensure-playable loop (board.py:381-391)
    CV_REJECT,           // Lemire rejection: serial replay of a draw batch (draw_colours)
    CV_FAST,             // fast_clear step (general kernel, no specials enabled)
    CV_SHUFFLE_GEN,      // shuffle in generate_board's loop (board.py:102-106)
    CV_REJECT_GEN,       // Lemire rejection in the row-plane generate (bp_generate): exact redo
    CV_COUNT = 32
};
#if TMG_COVER
#define COVER(site)                                                                                     \
    do {                                                                                                \
        if (lane == 0 && P.cover) atomicAdd(P.cover + (site), 1ULL);                                   \
    } while (0)
#define COVER_L0(site)                                                                                  \
    do {                                                                                                \
        if (P.cover) atomicAdd(P.cover + (site), 1ULL);                                                \
    } while (0)
#else
#define COVER(site) ((void)0)
#define COVER_L0(site) ((void)0)
#endif

struct Params {
    int R, C, N, A, W, k, smask, num_moves;
    uint32_t thr;                 // Lemire threshold (2^32 - k) % k; 0 for powers of two
    uint32_t cmag, cm1mag;        // ceil(2^20 / C), ceil(2^20 / (C-1)): exact x / C for x < 2^10
    const uint64_t *jump;         // [64][4] jump-ahead table
    // scalar-bitboard geometry (tmg_sb.hip; boards of <= 128 cells): cell p is
    // bit p>>1 of word p&1.  [0] even cells, [1] odd cells.
    uint64_t sb_nl[2];            // column <= C-2 (a right neighbour exists)
    uint64_t sb_nf[2];            // column >= 1
    uint64_t sb_h[2];             // column <= C-3 (a horizontal line may start)
    uint64_t sb_z;                // one column's cells of one word, from bit 0
    uint64_t sb_in[2], sb_u[2], sb_v[2];   // cells of the board / of rows >= 1 / of rows >= 2
    const uint64_t *sb_rows;      // [R][4]: row r's cells (a, b), rows 0..r's cells (a, b)
    uint32_t *status;             // sticky status words, one per ST_* bit
    void *oh;                     // fused OneHotWrapper output [n][oh_ch][R][C], or null (tmg_step_onehot)
    int oh_dtype, oh_ch, oh_nsel; // TMG_DTYPE_*; channels = k + nsel
    uint32_t oh_sel;              // type ids of the special channels, int8 each (wrappers.py:37-46)
    SpillQ *spill;                // this launch's stream's spill queue (general kernels)
    void *spill_ws;               // kSpillWaves WsSerialBig<MAXN> for spill_kernel
    unsigned long long *cover;    // TMG_COVER builds: CV_COUNT hit counters (null otherwise)
    // Gymnasium vector-env outputs of tmg_step_groups, written in the step's
    // own write-back (each null unless asked for)
    uint8_t *vo_term;             // [n][4] bytes: terminated, is_combination_match, shuffled, error
    uint8_t *vo_mask;             // [n][A] bytes: the action mask (tile_match_env.py:118-124), rewritten
                                  // only where the effective-action bitmask changes
    int64_t *vo_left;             // [n]: num_moves_left after the call (tile_match_env.py:114-116)
    int8_t *vo_final;             // [n][2][R][C]: same-step autoreset, the last board of each env whose
                                  // episode ended, before its regeneration
    int32_t *vo_obs;              // [n][2][R][C]: the board as int32 (the reference's observation dtype),
                                  // rewritten where the board changes
    // in-kernel policy (tmg_step_groups with a policy key): actions[e] <- uniform
    // over env e's effective actions, the stream of tmg_sample_effective
    int sample;
    int32_t pol_t;
    int64_t pol_first;            // global index of env 0 of the launch
    uint64_t pol_key;
};

// The kernels take Params by value as their FIRST argument and read it
// through the kernarg segment pointer, field by field where each is used.
// Used as a by-value argument, the whole block is loaded into SGPRs in the
// entry block (AMDGPULowerKernelArguments) and spilled to VGPR lanes before
// anything else runs, e.g. before the ineffective-move exit of a step.
#ifndef TMG_KERNARG_PARAMS
#if defined(__HIP_DEVICE_COMPILE__)
#define TMG_KERNARG_PARAMS(p) (*(const Params *)__builtin_amdgcn_kernarg_segment_ptr())
#else
#define TMG_KERNARG_PARAMS(p) (p)          // the host pass of the kernel templates (never executed)
#endif
#endif

// host: the per-row masks of Params::sb_rows (boards of <= 128 cells)
inline void build_sb_rows(int R, int C, uint64_t *tab) {
    for (int r = 0; r < R; r++) {
        uint64_t m[4] = {0, 0, 0, 0};
        for (int p = 0; p < (r + 1) * C && p < 128; p++) {
            if (p >= r * C) m[p & 1] |= 1ULL << (p >> 1);
            m[2 + (p & 1)] |= 1ULL << (p >> 1);
        }
        for (int i = 0; i < 4; i++) tab[r * 4 + i] = m[i];
    }
}

inline Params make_params(int R, int C, int k, int smask, int num_moves, const uint64_t *jump) {
    Params P;
    P.R = R; P.C = C; P.N = R * C;
    P.A = 2 * R * C - R - C;
    P.W = (P.A + 63) / 64;
    P.k = k; P.smask = smask; P.num_moves = num_moves;
    const uint32_t rng = (uint32_t)(k - 1), excl = rng + 1;
    P.thr = rng ? (UINT32_MAX - rng) % excl : 0u;
    P.cmag = ((1u << 20) + (uint32_t)C - 1) / (uint32_t)C;
    P.cm1mag = C > 1 ? ((1u << 20) + (uint32_t)C - 2) / (uint32_t)(C - 1) : 0u;
    P.jump = jump;
    for (int w = 0; w < 2; w++) P.sb_nl[w] = P.sb_nf[w] = P.sb_h[w] = P.sb_in[w] = P.sb_u[w] = P.sb_v[w] = 0;
    P.sb_z = 0;
    P.sb_rows = nullptr;
    P.status = nullptr;
    P.spill = nullptr;
    P.spill_ws = nullptr;
    P.cover = nullptr;
    P.oh = nullptr;
    P.oh_dtype = P.oh_ch = P.oh_nsel = 0;
    P.oh_sel = 0;
    P.vo_term = nullptr;
    P.vo_mask = nullptr;
    P.vo_left = nullptr;
    P.vo_final = nullptr;
    P.vo_obs = nullptr;
    P.sample = 0;
    P.pol_t = 0;
    P.pol_first = 0;
    P.pol_key = 0;
    if (P.N <= 128) {
        for (int p = 0; p < P.N; p++) {
            const int c = p % C, w = p & 1, b = p >> 1;
            P.sb_in[w] |= 1ULL << b;
            if (p >= C) P.sb_u[w] |= 1ULL << b;
            if (p >= 2 * C) P.sb_v[w] |= 1ULL << b;
            if (c <= C - 2) P.sb_nl[w] |= 1ULL << b;
            if (c >= 1) P.sb_nf[w] |= 1ULL << b;
            if (c <= C - 3) P.sb_h[w] |= 1ULL << b;
        }
        // even C: a column sits in one word with stride C/2; odd C: it alternates
        // words, stride C within each
        const int stride = (C & 1) ? C : C / 2;
        for (int b = 0; b < 64; b += stride) P.sb_z |= 1ULL << b;
    }
    return P;
}

// x / C and x / (C-1) for 0 <= x < 1024, C <= 64 (error < 2^-10 < 1/C)
__device__ __forceinline__ int div_c(const Params &P, int x) { return (int)(((uint32_t)x * P.cmag) >> 20); }
__device__ __forceinline__ int div_cm1(const Params &P, int x) { return (int)(((uint32_t)x * P.cm1mag) >> 20); }


// Workgroup -> env.  The dispatcher hands workgroup b to XCD b % 8; the host
// pads the grid to a multiple of 8 and XCD x gets the contiguous env block
// [x*G/8, (x+1)*G/8), so the per-env arrays (actions, timer, outputs, masks)
// are touched by one XCD's L2 per cache line instead of eight (speed only:
// correctness never depends on the placement).
__device__ __forceinline__ int64_t wg_env() {
    const int64_t per = gridDim.x >> 3;
    return (int64_t)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
}

// scalar slots in LDS (lane-0 sections publish through these)
enum : int { SC_NACT = 0, SC_NNEW, SC_ERR, SC_NZ, SC_A, SC_B, SC_C, SC_D, SC_COUNT = 16 };

template <int MAXN_>
struct WsCore {
    static constexpr int MAXN = MAXN_;
    static constexpr int NP = MAXN / 64;            // 64-cell passes
    static constexpr int MAXW = (2 * MAXN) / 64 + 2;
    uint64_t effw[MAXW];
    int32_t sc[SC_COUNT];
    // brd sits >= 128 bytes into the workspace, so the effective-action scan's
    // neighbour reads at p - 2C (C <= 64) stay inside it without clamping
    static constexpr int PRE = MAXW * 8 + SC_COUNT * 4;
    int8_t lpad[PRE >= 128 ? 1 : 128 - PRE];
    alignas(4) int8_t brd[2 * MAXN];   // [colour plane N][type plane N], runtime N (same layout as HBM)
    uint8_t mark[MAXN];
    alignas(8) int8_t trash[4 * 64];   // target of predicated-off stores (keeps hot loops branch-free)
    union alignas(16) {
        uint32_t draw[MAXN + 128];                  // refill colours; generate_board's colour ring (bp_ring)
        struct { int8_t tmp[2 * MAXN]; int16_t perm[MAXN]; } sh;   // shuffle
    } u;
};

// The lane-0 list machinery (general variant only): lines of get_colour_lines
// (pool / ls / ll), the process queue (q), matches (ms / mlen / mname / mcol /
// mpool), the activation DFS (f*), special placement (valid / taken / q*).
template <int POOL_, int MLINES_, int MQ_, int MM_, int MPOOL_, int MSTK_>
struct ListStore {
    static constexpr int POOL = POOL_;              // coords of lines
    static constexpr int MLINES = MLINES_;          // lines
    static constexpr int MQ = MQ_;                  // process queue
    static constexpr int MM = MM_;                  // matches
    static constexpr int MPOOL = MPOOL_;            // coords of matches
    static constexpr int MSTK = MSTK_;              // activation DFS frames
    static constexpr int MV = 96;                   // coords of one match: a line (<= 64) + 3 bomb cells
    int16_t pool[POOL];
    int16_t ls[MLINES], ll[MLINES];
    int16_t q[MQ];
    int16_t mpool[MPOOL];
    int16_t ms[MM], mlen[MM];
    int8_t mname[MM], mcol[MM];
    int16_t fcell[MSTK], fidx[MSTK];
    int8_t ftype[MSTK], faux[MSTK];
    int16_t valid[MV];
    int16_t taken[MM], qpos[MM];
    int8_t qname[MM], qcol[MM];
    int32_t counts[16];
    int16_t pick[4];
};

// The LDS lists of the general kernels.  A cascade step of a real board uses a
// few dozen entries; the 512-cell workspace is sized at half the cell count so
// the general 20x20 kernel fits twice the waves per CU in LDS.  A step that
// runs out (FL_OVF from the list machinery) is not written back: the env goes
// to the spill queue and spill_kernel re-runs the step on WsSerialBig.
constexpr int kCap128 = 64;              // lane-0 list capacity of the <= 128-cell general kernels (cells)
// lane-0 list capacity of the 512-cell general kernels (cells): at 80 the
// general workspace is 10 048 B, so 16 waves fit a CU's LDS and the
// specialised c5 step kernel runs at its VGPR occupancy (4 waves/SIMD); at 128
// (12 064 B) LDS held it to 13 waves per CU.  c5 1.56 -> 1.61 x 10^8
// (profiles/r04/s9); a step that outgrows the lists re-runs exactly in the
// spill tier.
constexpr int kCap512 = 80;
template <int MAXN, int CAP = (MAXN > 128 ? kCap512 : kCap128)>
using WsSerial = ListStore<4 * CAP + 256, CAP + 64, 2 * CAP + 64, CAP + 32, 4 * CAP + 256, CAP + 8>;

// Global-memory lists sized at the worst case of any board of <= MAXN cells
// (R, C <= 64), so the spill re-run cannot run out.  One get_colour_lines
// call (board.py:149-215) holds: first-pass lines of the bottom row, <= C
// vertical + C/3 horizontal ones over <= N + C coords (a coord may be listed
// twice); perpendicular lines, each holding exactly one coord (walks stop at
// coords), so <= 2 per distinct coord (one per axis; a coord listed twice
// repeats its lines, which the "not in lines" test drops), i.e. <= 2N; their
// cells: every coord <= 2 times, every other cell <= 4 times (only the coords
// closest to it along an axis, <= 2 per axis, reach it), i.e. <= 4N.  So the
// pool holds <= 5N + C coords plus the R + C + 1 of the line being built.
// process_colour_lines (:269-327) re-queues the tail of a cookie line (<= one
// new line per 5 pooled coords), pops each queued line once and makes <= one
// match per pop, whose coords are that line's plus <= 3 bomb cells.  The
// activation DFS (:473-556) pushes a frame per special it enters, and entering
// clears the cell, so <= N + 1 frames.
template <int MAXN, int POOLB = 5 * MAXN + 3 * 64 + 64, int LINESB = 2 * MAXN + 2 * 64 + POOLB / 5 + 16>
using WsSerialBig = ListStore<POOLB, LINESB, LINESB, LINESB, POOLB + 3 * LINESB, MAXN + 8>;

template <int MAXN, bool GEN>
struct Ws : WsCore<MAXN> {};
template <int MAXN>
struct Ws<MAXN, true> : WsCore<MAXN> {
    WsSerial<MAXN> s;
};

// Integer predicate helpers: keep per-lane logic in VALU registers (a boolean
// "&" of two lane compares would be an s_and_b64 on lane masks, i.e. SALU).
// A predicate is encoded as "zero means true".
__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint32_t umin3(uint32_t a, uint32_t b, uint32_t c) { return umin(umin(a, b), c); }
__device__ __forceinline__ uint32_t ne(int a, int b) { return (uint32_t)(a ^ b); }      // 0 iff a == b

// Wave64 max via DPP (row_shr 1/2/4/8 + row_bcast 15/31, GFX9 encoding): an
// inclusive scan whose lane 63 holds the maximum; ~7 VALU, no SALU.
__device__ __forceinline__ int wave_max(int v) {
    const int lo = (int)0x80000000;
    v = max(v, __builtin_amdgcn_update_dpp(lo, v, 0x111, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(lo, v, 0x112, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(lo, v, 0x114, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(lo, v, 0x118, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(lo, v, 0x142, 0xa, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(lo, v, 0x143, 0xc, 0xf, false));
    return __builtin_amdgcn_readlane(v, 63);
}

// popcount of the bits of m below this lane (v_mbcnt: no lane mask kept in registers)
__device__ __forceinline__ int popc_below(uint64_t m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// The lane index as a value the compiler cannot hoist: values derived from it
// inside the cascade loop are recomputed per iteration (a few VALU ops)
// instead of being kept live, or spilled, across the whole loop.
#ifndef TMG_OPAQUE_V
#define TMG_OPAQUE_V(x) asm volatile("" : "+v"(x))
#endif
// a use of a VGPR value here (its load has to land before this point)
#ifndef TMG_KEEP_V
#define TMG_KEEP_V(x) asm volatile("" ::"v"(x))
#endif
__device__ __forceinline__ int loop_lane(int lane) {
    int l = lane;
    TMG_OPAQUE_V(l);
    return l;
}

__device__ __forceinline__ uint64_t rdlane64(uint64_t v, int l) {
    uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
    uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t bcast64(uint64_t v) {
    uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// ------------------------------------------------------------------- RNG
// numpy PCG64 state of one env, wave-uniform: s (128), inc (128),
// h = has_uint32 << 32 | uinteger.
struct Rng {
    uint64_t slo, shi, ilo, ihi, h;
};
__device__ __forceinline__ void rng_bcast(Rng &g) {
    g.slo = bcast64(g.slo); g.shi = bcast64(g.shi); g.ilo = bcast64(g.ilo); g.ihi = bcast64(g.ihi); g.h = bcast64(g.h);
}

struct LaneJump {
    U128 Aj, Gj, incG;    // A^{lane+1}, G_{lane+1}, G_{lane+1} * inc
};

// jump128's f operand goes through SGPRs (pcg64.h): it must be wave-uniform,
// or the compiler silently takes lane 0's value.  TMG_COVER builds check every
// call site's f and raise ST_INTERNAL on a divergent one.
__device__ __forceinline__ void cover_uniform(const Params &P, int lane, U128 f) {
#if TMG_COVER
    const bool div = f.lo != bcast64(f.lo) || f.hi != bcast64(f.hi);
    if (__ballot(div) != 0 && lane == 0) P.status[0] = 1u;
#else
    (void)P; (void)lane; (void)f;
#endif
}

// single-lane stream (serial replays, shuffle)
__device__ __forceinline__ uint64_t r_next64(Rng &g) {
    U128 s = add128(mul128(U128{g.slo, g.shi}, U128{PCG_A_LO, PCG_A_HI}), U128{g.ilo, g.ihi});
    g.slo = s.lo; g.shi = s.hi;
    return xsl_rr(s);
}
__device__ __forceinline__ uint32_t r_next32(Rng &g) {                      // half-word buffer (numpy next_uint32)
    if (g.h >> 32) { g.h = (uint32_t)g.h; return (uint32_t)g.h; }
    uint64_t n = r_next64(g);
    g.h = (1ULL << 32) | (n >> 32);
    return (uint32_t)n;
}
__device__ __forceinline__ int r_colour(const Params &P, Rng &g) {         // integers(1, k+1), one value
    uint32_t excl = (uint32_t)P.k;
    uint64_t m = (uint64_t)r_next32(g) * excl;
    uint32_t left = (uint32_t)m;
    if (left < excl) {
        while (left < P.thr) { m = (uint64_t)r_next32(g) * excl; left = (uint32_t)m; }
    }
    return 1 + (int)(m >> 32);
}
__device__ __forceinline__ uint32_t r_interval(Rng &g, uint32_t max) {     // random_interval
    if (max == 0) return 0;
    uint32_t mask = max;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t v;
    while ((v = (r_next32(g) & mask)) > max) {}
    return v;
}

// dst[0..M) <- Generator.integers(1, k+1, M) (board.py:97,129,239), lane-parallel:
// lane j evaluates PCG output j of the batch by jump-ahead; the caller syncs.
// ONE: M <= 128, i.e. one batch of 64 outputs (no loop-carried state)
template <bool ONE = false, class T>
__device__ __forceinline__ void draw_colours(const Params &P, int lane, const LaneJump &J, Rng &g, int M, T *dst,
                                             int8_t *trash) {
    if (M <= 0) return;
    const uint32_t k = (uint32_t)P.k;
    if (k == 1) {                                          // rng == 0: numpy draws nothing
        for (int i = lane; i < M; i += 64) dst[i] = (T)1;
        return;
    }
    const Rng g0 = g;
    const int off = (int)(g.h >> 32) & 1;
    bool rej = false;
    {                                                      // the buffered half-word, if any, is draw 0
        const uint64_t m = (uint64_t)(uint32_t)g.h * k;
        const bool st = off & (lane == 0);
        *(st ? dst : reinterpret_cast<T *>(trash) + lane) = (T)(1 + (m >> 32));
        rej = st & ((uint32_t)m < P.thr);
    }
    const int need = M - off;
    const int n64 = (need + 1) >> 1;
    U128 s{g.slo, g.shi};
    uint64_t last_hi = 0;
    U128 sj{0, 0};
    uint64_t out = 0;
    for (int base = 0; base < n64; base += 64) {
        cover_uniform(P, lane, s);
        sj = jump128(J.Aj, s, J.incG);
        out = xsl_rr(sj);
        const int j = base + lane;
        const uint64_t m0 = (uint64_t)(uint32_t)out * k, m1 = (out >> 32) * k;
        const bool ok0 = j < n64, ok1 = 2 * j + 1 < need;          // ok1 implies ok0
        T *d0 = ok0 ? dst + off + 2 * j : reinterpret_cast<T *>(trash) + lane;
        T *d1 = ok1 ? dst + off + 2 * j + 1 : reinterpret_cast<T *>(trash) + lane;
        *d0 = (T)(1 + (m0 >> 32));
        *d1 = (T)(1 + (m1 >> 32));
        rej |= (ok0 & ((uint32_t)m0 < P.thr)) | (ok1 & ((uint32_t)m1 < P.thr));
        const int cnt = n64 - base < 64 ? n64 - base : 64;
        s.lo = rdlane64(sj.lo, cnt - 1);                   // the stream position after the batch
        s.hi = rdlane64(sj.hi, cnt - 1);
        last_hi = rdlane64(out >> 32, cnt - 1);
        if constexpr (ONE) break;
    }
    if (P.thr != 0u && __ballot(rej) != 0ULL) {            // Lemire rejection: exact serial replay
        COVER(CV_REJECT);
        WFENCE();
        if (lane == 0) {
            Rng r = g0;
            for (int i = 0; i < M; i++) dst[i] = (T)r_colour(P, r);
            g = r;
        }
        rng_bcast(g);
        return;
    }
    if (n64 > 0) {
        g.slo = s.lo; g.shi = s.hi;
        g.h = ((uint64_t)(need & 1) << 32) | (uint32_t)last_hi;
    } else {
        g.h = (uint32_t)g0.h;                              // only the buffered half was used
    }
}

// --------------------------------------------------------------- board helpers
__host__ __device__ __forceinline__ void action_coords(int R, int C, int a, int &r1, int &c1, int &r2, int &c2) {  // board.py:77-93
    if (a < C * (R - 1)) { r1 = a / C; c1 = a % C; r2 = r1 + 1; c2 = c1; }
    else { int i = a - C * (R - 1); r1 = i / (C - 1); c1 = i % (C - 1); r2 = r1; c2 = c1 + 1; }
}
// per-lane cell coordinates of each 64-cell pass, computed once per kernel
template <int NP>
struct Cells {
    // per 64-cell pass, one word per lane: key base ((r << 8) | (255 - c)) << 1
    // in bits 0..14 (the first-line key of remove_colour_lines' search), vbad
    // in bit 15, hbad in bit 16 (0 iff a vertical / horizontal triple can be
    // anchored here).  One VGPR per pass instead of four (the 512-cell
    // kernels are VGPR-bound).
    uint32_t pk[NP];
    __device__ __forceinline__ int key(int i) const { return (int)(pk[i] & 0x7fffu); }
    __device__ __forceinline__ int r(int i) const { return (int)((pk[i] >> 9) & 63u); }
    __device__ __forceinline__ int c(int i) const { return 255 - (int)((pk[i] >> 1) & 255u); }
    __device__ __forceinline__ uint32_t vbad(int i) const { return (pk[i] >> 15) & 1u; }
    __device__ __forceinline__ uint32_t hbad(int i) const { return (pk[i] >> 16) & 1u; }
};
template <int NP>
__device__ __forceinline__ Cells<NP> make_cells(const Params &P, int lane) {
    Cells<NP> cl;
#pragma unroll
    for (int i = 0; i < NP; i++) {
        const int p = i * 64 + lane;
        const int r = div_c(P, p), c = p - r * P.C;
        const uint32_t vbad = (p < P.N && r >= 2) ? 0u : 1u;
        const uint32_t hbad = (p < P.N && c + 2 < P.C) ? 0u : 1u;
        cl.pk[i] = ((uint32_t)(((r & 63) << 8) | (255 - (c & 255))) << 1) | (vbad << 15) | (hbad << 16);
    }
    return cl;
}

template <class WS>
__device__ __forceinline__ void load_board(const Params &P, WS &w, int lane, const int8_t *src) {
    const int nb = 2 * P.N;
    if ((nb & 3) == 0) {
        const uint32_t *s = reinterpret_cast<const uint32_t *>(src);
        uint32_t *d = reinterpret_cast<uint32_t *>(w.brd);
        for (int i = lane; i < (nb >> 2); i += 64) d[i] = s[i];
    } else {
        for (int i = lane; i < nb; i += 64) w.brd[i] = src[i];
    }
}
template <class WS>
__device__ __forceinline__ void store_board(const Params &P, const WS &w, int lane, int8_t *dst) {
    const int nb = 2 * P.N;
    if ((nb & 3) == 0) {
        uint32_t *d = reinterpret_cast<uint32_t *>(dst);
        const uint32_t *s = reinterpret_cast<const uint32_t *>(w.brd);
        for (int i = lane; i < (nb >> 2); i += 64) d[i] = s[i];
    } else {
        for (int i = lane; i < nb; i += 64) dst[i] = w.brd[i];
    }
}

// OneHotWrapper._one_hot_encode_board (wrappers.py:56-69) of env e's board in
// LDS, written in the step's own write-back: channel c < k is (colour == c+1),
// channel k + j is (type == oh_sel[j]); each channel's stores are coalesced.
// A one is 1.0f (0x3f800000) for f32, 1 for u8 / i32.
template <class WS>
__device__ __forceinline__ void store_onehot(const Params &P, const WS &w, int lane, int64_t e) {
    const int N = P.N, k = P.k, ch = P.oh_ch;
    const bool bytes = P.oh_dtype == 1;
    const uint32_t one = P.oh_dtype == 0 ? 0x3f800000u : 1u;
    uint8_t *o8 = reinterpret_cast<uint8_t *>(P.oh) + e * (int64_t)ch * N;
    uint32_t *o32 = reinterpret_cast<uint32_t *>(P.oh) + e * (int64_t)ch * N;
    for (int p = lane; p < N; p += 64) {
        const int x = w.brd[p], y = w.brd[N + p];
        for (int c = 0; c < ch; c++) {
            const bool on = c < k ? x == c + 1 : y == (int)(int8_t)(P.oh_sel >> (8 * (c - k)));
            if (bytes) o8[c * N + p] = on ? 1 : 0;
            else o32[c * N + p] = on ? one : 0u;
        }
    }
}

// The action mask bytes of env e (Params::vo_mask, [n][A] bools): byte a =
// bit a of the effective-action bitmask in LDS (w.effw), or all zero.  Four
// actions per lane and dword store when A is a multiple of 4: the nibble's
// bits spread to the low bit of each byte by one multiply.
template <class WS>
__device__ __forceinline__ void store_mask(const Params &P, const WS &w, int lane, int64_t e, bool zero) {
    const int A = P.A;
    uint8_t *m = P.vo_mask + e * (int64_t)A;
    if ((A & 3) == 0) {
        uint32_t *m4 = reinterpret_cast<uint32_t *>(m);
        for (int i = lane; i < (A >> 2); i += 64) {
            const uint32_t b = zero ? 0u : (uint32_t)(w.effw[i >> 4] >> ((4 * i) & 63)) & 0xFu;
            m4[i] = (b * 0x00204081u) & 0x01010101u;
        }
    } else {
        for (int i = lane; i < A; i += 64) m[i] = zero ? (uint8_t)0 : (uint8_t)((w.effw[i >> 6] >> (i & 63)) & 1ULL);
    }
}

// The board of env e in LDS as the int32 observation (Params::vo_obs)
template <class WS>
__device__ __forceinline__ void store_obs(const Params &P, const WS &w, int lane, int64_t e) {
    int32_t *o = P.vo_obs + e * 2 * (int64_t)P.N;
    for (int p = lane; p < 2 * P.N; p += 64) o[p] = w.brd[p];
}

// Per-env outputs of tmg_step_groups besides the step's own (lane 0)
__device__ __forceinline__ void store_vo(const Params &P, int64_t e, int flags, int tnew) {
    if (P.vo_term) {
        const uint32_t v = ((flags & FL_DONE) ? 1u : 0u) | ((flags & FL_COMBO) ? 1u << 8 : 0u) |
                           ((flags & FL_SHUF) ? 1u << 16 : 0u) |
                           ((flags & (FL_ERR | FL_OVF)) ? 1u << 24 : 0u);
        reinterpret_cast<uint32_t *>(P.vo_term)[e] = v;
    }
    if (P.vo_left) P.vo_left[e] = (int64_t)(P.num_moves - tnew);
}

// The examples' policy (src/examples/q_learning.py:19-25), counter-based:
// h = splitmix64(splitmix64(key K + global env) ^ t G) >> 32 (shard.synthetic_actions'
// stream), shared by sample_effective_kernel and the step kernel's own
// sampling (sample_action)
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}
__host__ __device__ __forceinline__ uint64_t policy_draw(uint64_t key, uint64_t gid, int32_t t) {
    const uint64_t base = splitmix64(key * 0xD1B54A32D192ED03ULL + gid);
    return splitmix64(base ^ ((uint64_t)t * 0x9E3779B97F4A7C15ULL)) >> 32;
}

// tmg_sample_effective's draw for env e inside the step (Params::sample):
// the r-th set bit of the env's mask, r = h * count >> 32, or h * A >> 32 when
// no action is effective.  effrow: lane i holds mask word i (W <= 64).
// The word holding bit r by readlanes of the per-lane popcounts; inside it,
// the lane whose bit is set with r set bits below it (v_mbcnt) is the action:
// a handful of VALU and one ballot instead of a scalar binary search (the
// scalar unit is the step kernels' busiest pipe).
__device__ __forceinline__ int sample_action(const Params &P, uint64_t effrow, int64_t e, int lane) {
#ifndef TMG_DRAW_VALU
#define TMG_DRAW_VALU 0
#endif
#if TMG_DRAW_VALU
    // the counter hash on the VALU (an opaque lane value), read back once: the
    // scalar unit is the busiest pipe of an effective step
    uint64_t gid = (uint64_t)(P.pol_first + e);
    TMG_OPAQUE_V(gid);
    const uint32_t h = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)policy_draw(P.pol_key, gid, P.pol_t));
#else
#ifndef TMG_KO
#define TMG_KO 0
#endif
    const uint32_t h = (TMG_KO & 2) ? (uint32_t)(e * 2654435761u) : (uint32_t)policy_draw(P.pol_key, (uint64_t)(P.pol_first + e), P.pol_t);
#endif
    const int W = P.W;
    const int pc = __popcll(effrow);                    // 0 on lanes >= W
    int count = 0;
    for (int j = 0; j < W; j++) count += __builtin_amdgcn_readlane(pc, j);
    if (count == 0) return (int)(((uint64_t)h * (uint64_t)P.A) >> 32);
    int r = (int)(((uint64_t)h * (uint64_t)count) >> 32);
    int j = 0;
    for (; j < W - 1; j++) {
        const int c = __builtin_amdgcn_readlane(pc, j);
        if (r < c) break;
        r -= c;
    }
    const uint64_t x = rdlane64(effrow, j);
    const bool hit = ((x >> lane) & 1ULL) && popc_below(x) == r;
    return j * 64 + __ffsll((unsigned long long)__ballot(hit)) - 1;
}

// The r-th set bit of x (r < popcount(x)): a branch-free binary search on the
// popcounts of its halves, 6 steps (not a loop over the set bits)
__device__ __forceinline__ int nth_set_bit(uint64_t x, int r) {
    int pos = 0;
#pragma unroll
    for (int sh = 32; sh > 0; sh >>= 1) {
        const int c = __popcll(x & ((1ULL << sh) - 1ULL));
        const bool up = r >= c;
        r -= up ? c : 0;
        x = up ? x >> sh : x;
        pos += up ? sh : 0;
    }
    return pos;
}
// tmg_sample_effective's draw for one env by one lane: m = the env's W mask words
__device__ __forceinline__ int32_t draw_row(const uint64_t *m, int W, int A, uint64_t h) {
    int count = 0;
    for (int j = 0; j < W; j++) count += __popcll(m[j]);
    if (count == 0) return (int32_t)((h * (uint64_t)A) >> 32);
    int r = (int)((h * (uint64_t)count) >> 32);
    int j = 0;
    uint64_t x = m[0];
    for (int c = __popcll(x); r >= c && j < W - 1; c = __popcll(x)) {
        r -= c;
        x = m[++j];
    }
    return j * 64 + nth_set_bit(x, r);
}

// is_move_effective, board.py:735-787 — exact windowed scan (any board)
__device__ __forceinline__ bool eff_exact(const Params &P, const int8_t *brd, int a) {
    const int R = P.R, C = P.C, N = P.N;
    int r1, c1, r2, c2;
    action_coords(R, C, a, r1, c1, r2, c2);
    const int8_t *col = brd, *typ = brd + N;
    const int p = r1 * C + c1, q = r2 * C + c2;
    const int tp = typ[p], tq = typ[q];
    if ((tp != 0 && tp != 1) && (tq != 0 && tq != 1)) return true;
    if (tp < 0 || tq < 0) return true;
    const int cp = col[p], cq = col[q];
    auto CO = [&](int x) -> int { return x == p ? cq : (x == q ? cp : (int)col[x]); };
    auto TY = [&](int x) -> int { return x == p ? tq : (x == q ? tp : (int)typ[x]); };
    int rmin = (r1 < r2 ? r1 : r2) - 2; if (rmin < 0) rmin = 0;
    int rmax = (r1 > r2 ? r1 : r2) + 2; if (rmax > R - 1) rmax = R - 1;
    int cmin = (c1 < c2 ? c1 : c2) - 2; if (cmin < 0) cmin = 0;
    int cmax = (c1 > c2 ? c1 : c2) + 2; if (cmax > C - 1) cmax = C - 1;
    if (cmin + 2 <= cmax)
        for (int r = rmin; r <= rmax; r++)
            for (int c = cmin; c + 2 <= cmax; c++) {
                int x = r * C + c;
                int a0 = CO(x);
                if (a0 == CO(x + 1) && a0 == CO(x + 2) && TY(x + 2) >= 0) return true;
            }
    if (rmin + 2 <= rmax)
        for (int r = rmin; r + 2 <= rmax; r++)
            for (int c = cmin; c <= cmax; c++) {
                int x = r * C + c;
                int a0 = CO(x);
                if (a0 == CO(x + C) && a0 == CO(x + 2 * C) && TY(x + 2 * C) >= 0) return true;
            }
    return false;
}

// is_move_effective for every action of a clean board (no empty cell, no
// coloured cookie, no pre-existing colour triple, checked by the caller; a
// swap with a colourless cookie is effective by type): only triples through
// exactly one of the two swapped cells can appear, all inside the window.  Pass i
// takes vertical action i and horizontal action nv + i on every lane; within
// a direction each swapped pair's 14 neighbours sit at the same offsets (±1,
// ±2, ±C, ±2C), so each is an LDS byte read at a uniform offset (WsCore::lpad
// keeps the negative ones inside the workspace) and a validity term.
// Swapping p (top / left) with q: p takes q's colour x2, q takes x1, and
// either needs a triple away from the other cell or across its own axis
// (tile_match_env.py:118-124, board.py:735-787).  Predicates are "zero means
// true" integers (VALU, no lane-mask SALU).  TYPES = false: every type is 1.
// Fills w.effw.
template <bool TYPES, class WS>
__device__ __forceinline__ bool scan_effective_clean(const Params &P, WS &w, int lane) {
    const int R = P.R, C = P.C, N = P.N;
    const int8_t *col = w.brd, *typ = w.brd + N;
    const int nv = C * (R - 1), nh = R * (C - 1);            // board.py:77-93
    if (lane < P.W) w.effw[lane] = 0ULL;
    WFENCE();
    const auto neg = [](int v) -> uint32_t { return (uint32_t)(v >> 31); };               // ~0 iff v < 0
    const auto nq = [](int a, int b, uint32_t inv) -> uint32_t { return (uint32_t)(a ^ b) | inv; };
    const auto place = [&](uint64_t m, int at) {             // lane 0: OR ballot m into bits [at, at + 64)
        const int wi = at >> 6, sh = at & 63;
        w.effw[wi] |= m << sh;
        const uint64_t hi = sh ? m >> (64 - sh) : 0ULL;
        if (hi) w.effw[wi + 1] |= hi;
    };
    uint64_t any = 0;
    for (int base = 0; base < (nv > nh ? nv : nh); base += 64) {
        // an opaque lane index: the per-lane geometry below stays inside the
        // pass (with a constant board shape the passes unroll, and values
        // hoisted out of them would stay live across the callers' loops)
        const int i = base + loop_lane(lane);
        uint32_t fv, fh;                                     // 0 iff effective
        {   // vertical action i: p = i (top cell), q = p + C
            const int p = i < nv ? i : 0, q = p + C;
            const int r = div_c(P, p), c = p - r * C;
            const int x1 = col[p], x2 = col[q];
            const uint32_t l1 = neg(c - 1), l2 = neg(c - 2), g1 = neg(C - 2 - c), g2 = neg(C - 3 - c);
            const uint32_t hp = umin3(nq(col[p - C], x2, neg(r - 1)) | nq(col[p - 2 * C], x2, neg(r - 2)),
                                      nq(col[p - 1], x2, l1) | umin(nq(col[p - 2], x2, l2), nq(col[p + 1], x2, g1)),
                                      nq(col[p + 1], x2, g1) | nq(col[p + 2], x2, g2));
            const uint32_t hq = umin3(nq(col[q + C], x1, neg(R - 3 - r)) | nq(col[q + 2 * C], x1, neg(R - 4 - r)),
                                      nq(col[q - 1], x1, l1) | umin(nq(col[q - 2], x1, l2), nq(col[q + 1], x1, g1)),
                                      nq(col[q + 1], x1, g1) | nq(col[q + 2], x1, g2));
            uint32_t sp = 1u;            // 0 iff both are specials (type not in {0, 1}) or one is a cookie (type < 0)
            if constexpr (TYPES) {
                const uint32_t tp = (uint32_t)(int)typ[p], tq = (uint32_t)(int)typ[q];
                sp = (umin(tp, tq) > 1u || ((tp | tq) >> 31)) ? 0u : 1u;
            }
            fv = umin3(sp, hp, hq) | neg(nv - 1 - i);
        }
        {   // horizontal action nv + i: i = r*(C-1) + c, p = r*C + c, q = p + 1
            const int ih = i < nh ? i : 0;
            const int r = div_cm1(P, ih), c = ih - r * (C - 1);
            const int p = r * C + c, q = p + 1;
            const int x1 = col[p], x2 = col[q];
            const uint32_t u1 = neg(r - 1), u2 = neg(r - 2), d1 = neg(R - 2 - r), d2 = neg(R - 3 - r);
            const uint32_t hp = umin3(nq(col[p - 1], x2, neg(c - 1)) | nq(col[p - 2], x2, neg(c - 2)),
                                      nq(col[p - C], x2, u1) | umin(nq(col[p - 2 * C], x2, u2), nq(col[p + C], x2, d1)),
                                      nq(col[p + C], x2, d1) | nq(col[p + 2 * C], x2, d2));
            const uint32_t hq = umin3(nq(col[q + 1], x1, neg(C - 3 - c)) | nq(col[q + 2], x1, neg(C - 4 - c)),
                                      nq(col[q - C], x1, u1) | umin(nq(col[q - 2 * C], x1, u2), nq(col[q + C], x1, d1)),
                                      nq(col[q + C], x1, d1) | nq(col[q + 2 * C], x1, d2));
            uint32_t sp = 1u;
            if constexpr (TYPES) {
                const uint32_t tp = (uint32_t)(int)typ[p], tq = (uint32_t)(int)typ[q];
                sp = (umin(tp, tq) > 1u || ((tp | tq) >> 31)) ? 0u : 1u;
            }
            fh = umin3(sp, hp, hq) | neg(nh - 1 - i);
        }
        const uint64_t mv = __ballot(fv == 0u), mh = __ballot(fh == 0u);
        any |= mv | mh;
        if (lane == 0) {
            if (mv) place(mv, base);
            if (mh) place(mh, nv + base);
        }
    }
    return any != 0ULL;
}

// ------------------------------------------ effective-action scan on row bit-planes
// scan_effective_clean's predicate (and scan_effective's precheck), row-parallel:
// lane r holds row r of the board as NBV bit-planes of the colour VALUE (bit c
// of plane b = bit b of the colour of cell (r, c); 0 = colourless or outside
// the board), so a lane decides the C vertical actions (r, c)-(r+1, c) and the
// C-1 horizontal actions (r, c)-(r, c+1) of its row at once with 32-bit mask
// logic, and one pass covers every action of the board (scan_effective_clean:
// one action per lane and direction, ~14 byte reads each, ceil(A / 128)
// passes: 2 at 10x10, 6 at 20x20).
// D(x, y) = columns where two (shifted) rows differ in colour; a pattern of two
// cells matches the moved colour where the OR of its two D masks is 0, and an
// action is effective where one of its eight patterns matches (or by type: both
// swapped tiles special, or one a cookie; board.py:735-787).  Cells outside the
// board read colour 0, which differs from every coloured tile; a colourless
// cookie may "match" them, but a swap moving a cookie is effective by type
// anyway.  D masks moved sideways shift in ones (outside = differ), moved across
// lanes (DPP wave shifts) lanes off the board read all ones.  Each D mask is
// computed once and reused by the patterns that look at the same cell pair from
// the other side (a pair of rows one lane up, a column shift).
// C <= kRowScanMaxC: the horizontal patterns reach column c + 3 and the shifted
// masks column C + 1, inside 32 bits.
constexpr int kRowScanMaxC = 28;
__host__ __device__ constexpr int rs_planes(int k) { return k < 2 ? 1 : k < 4 ? 2 : k < 8 ? 3 : 4; }

// bit b of each byte of x as 4 bits (byte i -> bit i): the masked bits sit 8
// apart, so one multiply moves each to bit 28 + i with no carries
__device__ __forceinline__ uint32_t byte_bits(uint32_t x, int b) {
    return ((x & (0x01010101u << b)) * (0x10204080u >> b)) >> 28;
}
// bit 0 of each byte = OR of that byte's 8 bits (the shifts stay inside the byte for bit 0)
__device__ __forceinline__ uint32_t byte_any(uint32_t x) {
    x |= x >> 4;
    x |= x >> 2;
    return x | (x >> 1);
}
// lane l <- lane l+1 (DPP wave_shl:1; lane 63 <- old) / lane l <- lane l-1 (wave_shr:1; lane 0 <- old)
__device__ __forceinline__ uint32_t from_next_lane(uint32_t v, uint32_t old) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x130, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t from_prev_lane(uint32_t v, uint32_t old) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xf, 0xf, false);
}
// bytes [off, off + 4 nd) of the LDS board (nd <= 8), realigned to dwords
template <class WS>
__device__ __forceinline__ void lds_row(const WS &w, int off, int nd, uint32_t (&d)[8]) {
    const uint32_t *b = reinterpret_cast<const uint32_t *>(w.brd + (off & ~3));
    const uint32_t sh = (uint32_t)(off & 3) * 8u;
    uint32_t raw[9];
#pragma unroll
    for (int i = 0; i < 9; i++) raw[i] = i <= nd ? b[i] : 0u;
#pragma unroll
    for (int i = 0; i < 8; i++) d[i] = i < nd ? __builtin_amdgcn_alignbit(raw[i + 1], raw[i], sh) : 0u;
}

// Fills w.effw (bit a = action a effective); returns 1 if any action is
// effective, 0 if none, -1 (clean = false only) when the board is not one the
// predicate covers — an empty cell, a coloured cookie, a colour outside 0..2^NBV-1
// or a colour triple — and the caller must run the exact scan.  TYPES = false:
// every type is 1 (the lean kernels).
template <bool TYPES, int NBV, class WS>
__device__ __forceinline__ int scan_rows_nb(const Params &P, WS &w, int lane_, bool clean) {
    const int R = P.R, C = P.C, N = P.N;
    const int r = loop_lane(lane_);
    const bool on = r < R;
    const int rr = on ? r : 0;
    const int nd = (C + 3) >> 2;
    // ---- row r as bit-planes (and, with specials, its special / cookie / empty masks)
    uint32_t X[NBV];
    bool odd = false;
    {
        uint32_t d[8];
        lds_row(w, rr * C, nd, d);
#pragma unroll
        for (int b = 0; b < NBV; b++) X[b] = 0u;
        uint32_t hi = 0u;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if (j < nd) {
#pragma unroll
                for (int b = 0; b < NBV; b++) X[b] |= byte_bits(d[j], b) << (4 * j);
                hi |= d[j];
            }
        }
        // a colour with bits above the planes (a hand-edited board) would alias
        if (!clean) odd = (hi & (0x01010101u * (0xFFu & (0xFFu << NBV)))) != 0u;
    }
    const uint32_t cm = on ? (C >= 32 ? ~0u : (1u << C) - 1u) : 0u;    // the row's columns
#pragma unroll
    for (int b = 0; b < NBV; b++) X[b] &= cm;
    uint32_t NS = 0u, CK = 0u, Z = 0u;             // type not in {0, 1} / cookie (type < 0) / empty (type 0)
    if constexpr (TYPES) {
        uint32_t d[8];
        lds_row(w, N + rr * C, nd, d);
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if (j < nd) {
                NS |= byte_bits(byte_any(d[j] & 0xFEFEFEFEu), 0) << (4 * j);
                CK |= byte_bits(d[j] >> 7, 0) << (4 * j);
                if (!clean) Z |= byte_bits(~byte_any(d[j]), 0) << (4 * j);
            }
        }
        NS &= cm; CK &= cm; Z &= cm;
    }
    // ---- rows r+1 .. r+3 (lanes off the board hold 0: colour 0 = outside)
    uint32_t X1[NBV], X2[NBV], X3[NBV];
#pragma unroll
    for (int b = 0; b < NBV; b++) {
        X1[b] = from_next_lane(X[b], 0u);
        X2[b] = from_next_lane(X1[b], 0u);
        X3[b] = from_next_lane(X2[b], 0u);
    }
    const auto D = [&](const uint32_t (&x)[NBV], int sx, const uint32_t (&y)[NBV], int sy) -> uint32_t {
        uint32_t m = 0u;      // columns c where colour(x row, c + sx) != colour(y row, c + sy)
#pragma unroll
        for (int b = 0; b < NBV; b++) {
            const uint32_t xs = sx >= 0 ? x[b] >> sx : x[b] << -sx;
            const uint32_t ys = sy >= 0 ? y[b] >> sy : y[b] << -sy;
            m |= xs ^ ys;
        }
        return m;
    };
    // the D masks (bit c: the two cells named differ)
    const uint32_t E1 = D(X1, -1, X, 0);      // (r+1, c-1) vs (r, c)
    const uint32_t E2 = D(X1, -2, X, 0);      // (r+1, c-2) vs (r, c)
    const uint32_t F1 = D(X1, 1, X, 0);       // (r+1, c+1) vs (r, c)
    const uint32_t F2 = D(X1, 2, X, 0);       // (r+1, c+2) vs (r, c)
    const uint32_t V2d = D(X2, 0, X, 0);      // (r+2, c) vs (r, c)
    const uint32_t V3d = D(X3, 0, X, 0);      // (r+3, c) vs (r, c)
    const uint32_t G2 = D(X, 2, X, 0);        // (r, c+2) vs (r, c)
    const uint32_t G3 = D(X, 3, X, 0);        // (r, c+3) vs (r, c)
    const uint32_t W2 = D(X2, 1, X, 0);       // (r+2, c+1) vs (r, c)
    const uint32_t Dn2 = D(X2, 0, X, 1);      // (r+2, c) vs (r, c+1)
    // the same pairs seen from lanes above (off the board: all ones = differ)
    const uint32_t A = from_prev_lane(V2d, ~0u);                       // (r-1, c) vs (r+1, c)
    const uint32_t B = from_prev_lane(from_prev_lane(V3d, ~0u), ~0u);  // (r-2, c) vs (r+1, c)
    const uint32_t U1 = from_prev_lane(F1, ~0u);                       // (r-1, c) vs (r, c+1)
    const uint32_t U2 = from_prev_lane(from_prev_lane(W2, ~0u), ~0u);  // (r-2, c) vs (r, c+1)
    const uint32_t V1 = from_prev_lane(E1, ~0u) >> 1;                  // (r-1, c+1) vs (r, c)
    const uint32_t V2 = from_prev_lane(from_prev_lane(Dn2, ~0u), ~0u); // (r-2, c+1) vs (r, c)
    // vertical action (r, c): p = (r, c) takes x2 = colour(r+1, c), q = (r+1, c) takes x1 = colour(r, c)
    const uint32_t F1l = (F1 << 1) | 1u, F2l = (F2 << 2) | 3u;         // (r, c-1) / (r, c-2) vs (r+1, c)
    const uint32_t E1r = E1 >> 1, E2r = E2 >> 2;                       // (r, c+1) / (r, c+2) vs (r+1, c)
    const uint32_t nv_ = (A | B) & (F1l | F2l) & (F1l | E1r) & (E1r | E2r)     // p: up-up, left-left, left-right, right-right
                       & (V2d | V3d) & (E1 | E2) & (E1 | F1) & (F1 | F2);      // q: down-down, left-left, left-right, right-right
    // horizontal action (r, c): p = (r, c) takes x2 = colour(r, c+1), q = (r, c+1) takes x1 = colour(r, c)
    const uint32_t G2l = (G2 << 1) | 1u, G3l = (G3 << 2) | 3u;         // (r, c-1) / (r, c-2) vs (r, c+1)
    const uint32_t Dn1 = E1 >> 1;                                      // (r+1, c) vs (r, c+1)
    const uint32_t nh_ = (G2l | G3l) & (U1 | U2) & (U1 | Dn1) & (Dn1 | Dn2)    // p: left-left, up-up, up-down, down-down
                       & (G2 | G3) & (V1 | V2) & (V1 | F1) & (F1 | W2);        // q: right-right, up-up, up-down, down-down
    uint32_t tv = 0u, th = 0u;                 // effective by type
    if constexpr (TYPES) {
        const uint32_t NS1 = from_next_lane(NS, 0u), CK1 = from_next_lane(CK, 0u);
        tv = (NS & NS1) | CK | CK1;
        th = (NS & (NS >> 1)) | CK | (CK >> 1);
    }
    const uint32_t mv = (~nv_ | tv) & (r < R - 1 ? cm : 0u);
    const uint32_t mh = (~nh_ | th) & (cm >> 1);
    if (!clean) {
        // scan_effective's precheck: an empty cell, a coloured cookie, or a
        // triple (c, c+1, c+2) / (r, r+1, r+2) whose third cell is not a cookie
        uint32_t nz = 0u;
#pragma unroll
        for (int b = 0; b < NBV; b++) nz |= X[b];
        const uint32_t G1 = D(X, 1, X, 0), V1d = D(X1, 0, X, 0);
        const uint32_t CK2 = from_next_lane(from_next_lane(CK, 0u), 0u);
        const uint32_t th3 = ~(G1 | G2) & ~(CK >> 2) & (cm >> 2);
        const uint32_t tv3 = ~(V1d | V2d) & ~CK2 & (r < R - 2 ? cm : 0u);
        odd |= (Z | (CK & nz) | th3 | tv3) != 0u;
        if (__ballot(odd) != 0ULL) return -1;
    }
    // the rows' masks into w.effw: bit r*C + c (vertical), nv + r*(C-1) + c (horizontal)
    if (lane_ < P.W) w.effw[lane_] = 0ULL;
    WFENCE();
    const auto put = [&](uint32_t m, int pos) {
        const int wi = pos >> 6, sh = pos & 63;
        if (m) {
            atomicOr(reinterpret_cast<unsigned long long *>(&w.effw[wi]), (unsigned long long)m << sh);
            const uint64_t up = sh > 32 ? (uint64_t)m >> (64 - sh) : 0ULL;
            if (up) atomicOr(reinterpret_cast<unsigned long long *>(&w.effw[wi + 1]), (unsigned long long)up);
        }
    };
    put(mv, rr * C);
    put(mh, C * (R - 1) + rr * (C - 1));
    WFENCE();
    return __ballot((mv | mh) != 0u) != 0ULL ? 1 : 0;
}

// scan_rows_nb for the env's colour count (one instantiation survives in the
// shape-specialised kernels)
template <bool TYPES, class WS>
__device__ __forceinline__ int scan_rows(const Params &P, WS &w, int lane, bool clean) {
    switch (rs_planes(P.k)) {
    case 1: return scan_rows_nb<TYPES, 1>(P, w, lane, clean);
    case 2: return scan_rows_nb<TYPES, 2>(P, w, lane, clean);
    case 3: return scan_rows_nb<TYPES, 3>(P, w, lane, clean);
    default: return scan_rows_nb<TYPES, 4>(P, w, lane, clean);
    }
}

// Where the row-plane scan replaces the per-action one (A/B switch, bits):
// 1 = scan_effective (general kernels, hand-edited boards), 2 = the lean /
// scalar-bitboard ensure loop (sb_ensure), 4 = bp_generate's possible_move.
#ifndef TMG_RSCAN
#define TMG_RSCAN 7
#endif

// _get_effective_actions / possible_move (tile_match_env.py:118-124, board.py:558-569):
// fills w.effw, returns whether any action is effective.  `clean` = the caller
// knows the board has no cookie and no colour triple (it just came out of a
// line-free detection with no cookie enabled), which skips the precheck.
template <class WS>
__device__ __forceinline__ bool scan_effective(const Params &P, WS &w, int lane, const Cells<WS::NP> &cl, bool clean) {
    const int R = P.R, C = P.C, N = P.N;
    const int8_t *col = w.brd, *typ = w.brd + N;
    bool exact = false;
    if ((TMG_RSCAN & 1) && C <= kRowScanMaxC) {
        const int r = scan_rows<true>(P, w, lane, clean);         // its own precheck
        if (r >= 0) return r != 0;
        exact = true;
    } else if (!clean) {
        // an empty cell, a cookie that gained a colour or a pre-existing triple ->
        // exact scan.  Colourless cookies are fine: swapping one is effective
        // (board.py:752-753), and colour 0 matches no coloured tile; a cookie
        // triple does not count (its third cell's type is < 0, :763).
        bool odd = false;
#pragma unroll
        for (int i = 0; i < WS::NP; i++) {
            int p = i * 64 + lane;
            if (p < N) {
                int r = cl.r(i), c = cl.c(i), x = col[p];
                odd |= typ[p] == 0 || (typ[p] < 0 && x != 0);
                odd |= (c + 2 < C) && col[p + 1] == x && col[p + 2] == x && typ[p + 2] >= 0;
                odd |= (r + 2 < R) && col[p + C] == x && col[p + 2 * C] == x && typ[p + 2 * C] >= 0;
            }
        }
        exact = __ballot(odd) != 0ULL;
    }
    if (!exact) return scan_effective_clean<true>(P, w, lane);
    uint64_t any = 0;
    for (int base = 0, wi = 0; base < P.A; base += 64, wi++) {
        int a = base + lane;
        const bool e = a < P.A && eff_exact(P, w.brd, a);
        uint64_t m = __ballot(e);
        if (lane == 0) w.effw[wi] = m;
        any |= m;
    }
    return any != 0ULL;
}

// Line masks (get_colour_lines' first pass, board.py:158-193): bit p of v/h =
// a vertical line is anchored at cell p / a horizontal line may start at p.
template <int NP>
struct Det {
    uint64_t v[NP], h[NP];
};

template <int NP>
__device__ __forceinline__ uint64_t bits_at(const uint64_t (&m)[NP], int start, int len) {   // len <= 64
    const int wi = start >> 6, off = start & 63;
    uint64_t lo = 0, hi = 0;
#pragma unroll
    for (int i = 0; i < NP; i++) {
        if (i == wi) lo = m[i];
        if (i == wi + 1) hi = m[i];
    }
    uint64_t r = lo >> off;
    if (off && off + len > 64) r |= hi << (64 - off);
    return len >= 64 ? r : (r & ((1ULL << len) - 1));
}

// Returns the bottom-most row holding a line, or -1 (get_colour_lines == []).
// lim: no anchor lies below row lim (the caller's bound).  The 64-cell passes
// are scanned bottom-up from the one holding row lim's last cell; the scan
// stops one pass above the first pass holding an anchor, so the masks of the
// bottom-most anchor row rs (<= 64 cells: that pass and the one above) are
// complete — the callers read only row rs's bits.  Unscanned passes read 0.
template <class WS>
__device__ __forceinline__ int detect(const Params &P, const WS &w, int lane, const Cells<WS::NP> &cl, Det<WS::NP> &d,
                                      int lim) {
    const int C = P.C, N = P.N, N1 = P.N - 1;
    const int8_t *col = w.brd, *typ = w.brd + N;
    const int last = min((lim + 1) * C, N) - 1;
    int pmax = -1, stop = -2;
#pragma unroll
    for (int i = WS::NP - 1; i >= 0; i--) {
        d.v[i] = 0; d.h[i] = 0;
        if (i * 64 > last || i < stop) continue;                             // wave-uniform
        const int p = i * 64 + lane;
        const int pc = min(p, N1);
        const int x = col[pc];
        const int u1 = col[max(pc - C, 0)], u2 = col[max(pc - 2 * C, 0)];
        const int h1 = col[min(pc + 1, N1)], h2 = col[min(pc + 2, N1)];
        const uint32_t tbad = (uint32_t)((int)typ[pc] - 1) >> 31;            // 1 iff type <= 0
        const uint32_t vb = cl.vbad(i) | tbad | ne(u1, x) | ne(u2, x);
        const uint32_t hb = cl.hbad(i) | tbad | ne(h1, x) | ne(h2, x);
        d.v[i] = __ballot(vb == 0);
        d.h[i] = __ballot(hb == 0);
        const uint64_t m = d.v[i] | d.h[i];
        if (m && pmax < 0) { pmax = i * 64 + 63 - __clzll(m); stop = i - 1; }
    }
    return pmax < 0 ? -1 : div_c(P, pmax);
}

// top row of the same-colour run ending at (rs, c) (vertical line start)
template <class WS>
__device__ __forceinline__ int run_top(const Params &P, const WS &w, int lane, int rs, int c) {
    const int C = P.C;
    const int x = w.brd[rs * C + c];
    const int rr = min(lane, rs);
    uint64_t mn = __ballot(lane < rs ? w.brd[rr * C + c] != x : false);
    return mn ? (63 - __clzll(mn)) + 1 : 0;
}

// For remove_colour_lines (board.py:120-131): row of the first coord of the
// first line get_colour_lines would return, or -1 when it returns [].
// get_colour_lines scans rows bottom-up and, in the first row holding a line,
// columns left to right with the vertical check first; so the first line is
// the maximum of key = (row, -col, is_vertical) over anchor cells: one DPP
// max-reduction instead of mask bookkeeping.
//
// lim: no anchor lies below row lim.  The 64-cell passes are scanned from the
// one holding row lim's last cell upwards and the scan stops one pass above
// the first pass holding an anchor: the bottom-most anchor row (C <= 64
// cells) lies in that pass and the one above it.  ra: the anchor row found.
// ALL1: every type is 1 (generate_board's loop), so the type plane is not read.
template <bool ROLL, bool ALL1 = false, class WS>
__device__ __forceinline__ int first_line_row(const Params &P, const WS &w, int lane, const Cells<WS::NP> &cl,
                                              int lim, int &ra) {
    const int C = P.C, N = P.N, N1 = P.N - 1;
    const int8_t *col = w.brd, *typ = w.brd + N;
    const int last = min((lim + 1) * C, N) - 1;          // highest cell that may anchor a line
    int best = -1, stop = -2;                            // stop: lowest pass still to scan, once found
    if constexpr (!ROLL || WS::NP <= 2) {
#pragma unroll
        for (int i = WS::NP - 1; i >= 0; i--) {
            if (i * 64 > last || i < stop) continue;     // wave-uniform
            const int p = i * 64 + lane;
            const int pc = min(p, N1);
            const int x = col[pc];
            const int u1 = col[max(pc - C, 0)], u2 = col[max(pc - 2 * C, 0)];
            const int h1 = col[min(pc + 1, N1)], h2 = col[min(pc + 2, N1)];
            const uint32_t tbad = ALL1 ? 0u : (uint32_t)((int)typ[pc] - 1) >> 31;
            const uint32_t vb = cl.vbad(i) | tbad | ne(u1, x) | ne(u2, x);
            const uint32_t hb = cl.hbad(i) | tbad | ne(h1, x) | ne(h2, x);
            const int base = cl.key(i);
            best = max(best, max(vb == 0 ? base | 1 : -1, hb == 0 ? base : -1));
            if (stop == -2 && __ballot(best >= 0) != 0ULL) stop = i - 1;
        }
    } else {
        // ROLL (512-cell step kernels): a rolled loop from the pass holding
        // `last` down to the stop pass, the cell's row / column recomputed per
        // pass.  The unrolled scan keeps eight passes' loads and cells live:
        // 187 -> 166 VGPRs, 2 -> 3 waves/SIMD for the step kernel; the reset
        // kernel keeps the unrolled form (its loads overlap: faster there).
        (void)cl;
        for (int i = last >> 6; i >= 0 && i >= stop; i--) {
            const int p = i * 64 + lane;
            const int pc = min(p, N1);
            const int r = div_c(P, p), c = p - r * C;
            const int x = col[pc];
            const int u1 = col[max(pc - C, 0)], u2 = col[max(pc - 2 * C, 0)];
            const int h1 = col[min(pc + 1, N1)], h2 = col[min(pc + 2, N1)];
            const uint32_t tbad = ALL1 ? 0u : (uint32_t)((int)typ[pc] - 1) >> 31;
            const uint32_t vbad = (p < N && r >= 2) ? 0u : 1u, hbad = (p < N && c + 2 < C) ? 0u : 1u;
            const uint32_t vb = vbad | tbad | ne(u1, x) | ne(u2, x);
            const uint32_t hb = hbad | tbad | ne(h1, x) | ne(h2, x);
            const int base = (((r & 63) << 8) | (255 - (c & 255))) << 1;
            best = max(best, max(vb == 0 ? base | 1 : -1, hb == 0 ? base : -1));
            if (stop == -2 && __ballot(best >= 0) != 0ULL) stop = i - 1;
        }
    }
    if (stop == -2) return -1;
    const int key = wave_max(best);
    const int rs = key >> 9;
    ra = rs;
    if (!(key & 1)) return rs;                            // horizontal line at (rs, c0..)
    const int c0 = 255 - ((key >> 1) & 255);
    return run_top(P, w, lane, rs, c0);                   // vertical: starts at the top of its run
}

// gravity, board.py:217-229 — stable partition of each column (empties to
// the top).  Lanes are laid out column-major (64/R columns per pass) so one
// ballot holds whole columns: a non-empty cell moves down by the popcount of
// the empties below it, as one scatter.
// cols: the columns that may hold an empty cell (bit c; others are skipped).
template <class WS>
__device__ __forceinline__ void gravity(const Params &P, WS &w, int lane, uint64_t cols = ~0ULL) {
    const int R = P.R, C = P.C, N = P.N;
    int8_t *col = w.brd, *typ = w.brd + N;
    const int cpp = 64 / R;
    const int lc = lane / R, r = lane - lc * R;
    const uint64_t colmask = (R == 64 ? ~0ULL : ((1ULL << R) - 1)) << (lc * R);
    const uint64_t above = lane == 63 ? 0ULL : ~((2ULL << lane) - 1);    // lanes > lane: lower rows
    const uint64_t grp = cpp >= 64 ? ~0ULL : (1ULL << cpp) - 1;
    for (int c0 = 0; c0 < C; c0 += cpp) {
        if (!((cols >> c0) & grp)) continue;                                 // wave-uniform
        const int c = c0 + lc;
        const bool in = (lc < cpp) & (c < C);
        const int p = in ? r * C + c : 0;
        const int8_t a = col[p], t = typ[p];
        const uint32_t occ = in ? (uint32_t)(uint8_t)(a | t) : 1u;            // 0 iff empty cell
        const uint64_t E = __ballot(occ == 0u);
        if (!E) continue;
        const int below = __popcll(E & colmask & above);
        const int total = __popcll(E & colmask);
        const bool mv = (in ? umin(occ, (uint32_t)below) : 0u) != 0u;       // non-empty cell that falls
        const bool clr = (in ? max(total - r, 0) : 0) != 0;                  // top `total` rows become empty
        const int d = p + below * C;
        WFENCE();
        *(mv ? col + d : w.trash + lane) = a;
        *(mv ? typ + d : w.trash + 64 + lane) = t;
        *(clr ? col + p : w.trash + 128 + lane) = 0;
        *(clr ? typ + p : w.trash + 192 + lane) = 0;
        WFENCE();
    }
}

// refill, board.py:231-241 — empties in row-major order get consecutive draws
// rows: empties lie in rows < rows only (after gravity: the most cells
// cleared in one column); the passes below are skipped.
template <class WS>
__device__ __forceinline__ void refill(const Params &P, WS &w, int lane, const LaneJump &J, Rng &g, int rows = 64) {
    const int N = P.N;
    int8_t *col = w.brd, *typ = w.brd + N;
    const int lastp = min(rows * P.C, N);                                   // cells that may be empty
    uint64_t E[WS::NP];
    int total = 0;
#pragma unroll
    for (int i = 0; i < WS::NP; i++) {
        int p = i * 64 + lane;
        E[i] = i * 64 < lastp ? __ballot(p < N && col[p] == 0 && typ[p] == 0) : 0ULL;
        total += __popcll(E[i]);
    }
    if (total == 0) return;
    draw_colours<WS::MAXN <= 128>(P, lane, J, g, total, w.u.draw, w.trash);
    WSYNC();
    int base = 0;
#pragma unroll
    for (int i = 0; i < WS::NP; i++) {
        const int p = i * 64 + lane;
        const bool e = (E[i] >> lane) & 1;
        const int idx = base + popc_below(E[i]);
        const int8_t v = (int8_t)w.u.draw[e ? idx : 0];
        *(e ? col + p : w.trash + lane) = v;
        *(e ? typ + p : w.trash + 64 + lane) = 1;
        base += __popcll(E[i]);
    }
    WSYNC();
}

// shuffle, board.py:114-118 (both planes)
template <class WS>
__device__ __forceinline__ void shuffle(const Params &P, WS &w, int lane, Rng &g) {
    const int N = P.N;
    for (int p = lane; p < N; p += 64) w.u.sh.perm[p] = (int16_t)p;   // arange(R*C), :115
    WSYNC();
    if (lane == 0) {
        Rng r = g;
        for (int i = N - 1; i >= 1; i--) {
            int j = (int)r_interval(r, (uint32_t)i);
            int16_t x = w.u.sh.perm[i]; w.u.sh.perm[i] = w.u.sh.perm[j]; w.u.sh.perm[j] = x;
        }
        g = r;
    }
    rng_bcast(g);
    for (int i = lane; i < 2 * N; i += 64) w.u.sh.tmp[i] = w.brd[i];
    WSYNC();
    for (int p = lane; p < N; p += 64) {
        int s = w.u.sh.perm[p];
        w.brd[p] = w.u.sh.tmp[s];
        w.brd[N + p] = w.u.sh.tmp[N + s];
    }
    WSYNC();
}

// generate_board's / move's "while not possible_move() or lines" loop
// (board.py:102-109, 381-391, remove_colour_lines :120-131).  Leaves the final
// board's effective mask in w.effw.  Returns FL_SHUF when a shuffle ran, FL_ERR
// when the shuffle cap ended the loop.
// noline: the board is known to hold no line (the cascade loop just found
// none), so the first line search is skipped.
// GEN: the loop of generate_board (the cover counters tell the two apart).
template <bool ROLL = true, bool ALL1 = false, bool GEN = false, class WS>
__device__ __forceinline__ int ensure_playable(const Params &P, WS &w, int lane, const LaneJump &J, Rng &g,
                                const Cells<WS::NP> &cl, bool noline = false) {
    int fl = 0;
    for (int shuffles = 0;; shuffles++) {
        // Redrawing rows 0..row leaves every cell an anchor test reads in rows
        // > row + 2 unchanged, so after it no anchor lies below max(row + 2, ra).
        int lim = P.R - 1;
        for (; !noline;) {
            int ra = 0;
            int r0 = first_line_row<ROLL, ALL1>(P, w, lane, cl, lim, ra);
            if (r0 < 0) break;
            int row = P.R - 1 < r0 + 1 ? P.R - 1 : r0 + 1;   // colour plane only, rows 0..row
            draw_colours(P, lane, J, g, (row + 1) * P.C, w.brd, w.trash);
            WSYNC();
            lim = min(P.R - 1, max(row + 2, ra));
        }
        // generate_board's boards (ALL1: every type 1, no cookie) are line-free
        // here, so the scan needs no precheck
        if (scan_effective(P, w, lane, cl, ALL1 || (P.smask & SP_COOKIE) == 0)) break;
        if (shuffles >= kMaxShuffles) return fl | FL_ERR;
        COVER(GEN ? CV_SHUFFLE_GEN : CV_SHUFFLE);
        WSYNC();
        shuffle(P, w, lane, g);
        fl = FL_SHUF;
        noline = false;
    }
    WSYNC();
    return fl;
}

// generate_board, board.py:95-109, draw by draw (boards of C > 32 columns and
// the exact redo after a Lemire rejection; bp_generate otherwise); returns
// FL_ERR when a safety cap was hit
template <bool ROLL = true, class WS>
__device__ __forceinline__ int generate_board(const Params &P, WS &w, int lane, const LaneJump &J, Rng &g, const Cells<WS::NP> &cl) {
    const int N = P.N;
    draw_colours(P, lane, J, g, N, w.brd, w.trash);
    for (int p = lane; p < N; p += 64) w.brd[N + p] = 1;
    WSYNC();
    return ensure_playable<ROLL, true, true>(P, w, lane, J, g, cl) & FL_ERR;   // types all 1
}

// ------------------------------------------------------------ row bit-planes
// generate_board (board.py:95-131) with one board row per lane, for boards of
// C <= 32 columns (every reset and autoreset path): lane r < R holds NB
// bit-planes of row r, bit c of plane b = bit b of (colour - 1) of cell (r, c)
// (colours 1..k, k <= 15); lanes >= R hold 0.  remove_colour_lines' line
// search (get_colour_lines' first pass, :158-193, every type 1) is then a few
// VALU ops on the lane's own row plus one DPP wave_shr:1 for the row above:
//   neR = OR_b P_b ^ (P_b >> 1)          (cell c differs from c + 1)
//   h   = ~(neR | neR >> 1) & cols<=C-3  (a horizontal run of 3 starts at c)
//   eqU = ~OR_b P_b ^ P_b[r-1]            (cell (r, c) equals (r-1, c))
//   v   = eqU & eqU[r-1] & rows>=2        (a vertical run of 3 ends at (r, c))
// The first line of get_colour_lines is in the bottom-most row holding an
// anchor (one ballot), at its leftmost anchor column, vertical before
// horizontal; a vertical line starts at the top of its run (one ballot of
// eqU's column).  No LDS access in the search at all.
//
// The colours come from the env's stream as one sequence: every
// Generator.integers(1, k+1, M) call takes the next M colours of it (:97,
// :129), whatever M is, so each jump-ahead batch of 64 PCG64 outputs appends
// 128 colours to a 1024-colour ring held as NB bit-strings in LDS (colour i
// is bit i mod 1024 of each plane's string), and a redraw of rows 0..row
// hands lane r its C colours [cons + rC, cons + rC + C) as one funnel shift
// (v_alignbit) of two ring dwords per plane.  Batches start at multiples of
// 128 (a buffered half-word, the sequence's first colour, sits at index 127),
// so a batch's planes are four whole dwords each.
//
// The batches advance lane-locally: lane l holds the PCG64 state X of its
// output bp_out(l) of the next batch, and a fill takes that output and steps
// X by 64 outputs, X <- A^64 X + G_64 inc (a wave-uniform multiplier), so a
// batch's jump-ahead depends only on the lane's own previous one, not on a
// readlane of the last lane, and it is issued before the batch's colours are
// processed.  The exact stream position at the end is recovered from the
// lane holding the last consumed colour by a backward jump of the batches
// filled since (jump-table rows 64.., build_jump_table).
constexpr int kBpRingDw = 32;                    // dwords per plane string (1024 colours)
constexpr int kBpPlaneDw = 36;                   // + a guard copy of dwords 0..3, so [d, d+1] never wraps
template <int NB>
struct RowPlanes {
    uint32_t p[NB];
};
struct BpRing {
    int fill, cons, cons0;                       // colour indices: filled, consumed, consumed at init
    uint32_t rmin;                               // per lane: the smallest Lemire low word filled (a
                                                 // rejected word was drawn iff some lane's < thr)
};
template <class WS>
__device__ __forceinline__ uint32_t *bp_ring(WS &w) { return reinterpret_cast<uint32_t *>(w.u.draw); }   // [4][36]

// The batch's lane order: lane l computes PCG64 output bp_out(l) of the batch
// (outputs o and 32 + o on lanes 2o and 2o + 1), so that the codes of colours l
// and 64 + l (output l >> 1 resp. 32 + (l >> 1), half l & 1) are on lane l or
// its quad neighbour l ^ 1: one DPP swap each instead of a cross-lane gather.
__device__ __forceinline__ int bp_out(int lane) { return (lane >> 1) + ((lane & 1) << 5); }
__device__ __forceinline__ int bp_lane(int out) { return out < 32 ? 2 * out : 2 * (out - 32) + 1; }   // inverse
struct BpJump {
    U128 X;                                      // per lane: state after output bp_out(lane) of the next batch
    U128 c64;                                    // G_64 inc (wave-uniform, kept in VGPRs: the multiply-add's addend)
    U128 A64;                                    // A^64 (wave-uniform, SGPRs)
};
__device__ __forceinline__ BpJump load_bp_jump(const Params &P, const Rng &g) {
    const uint64_t *t = P.jump + 63 * 4;                             // row 63: A^64, G_64
    BpJump J;
    J.A64 = U128{bcast64(t[0]), bcast64(t[1])};                    // loaded as VMEM (the kernel writes global
                                                                     // memory): said uniform, so SGPRs
    J.c64 = mul128(U128{g.ilo, g.ihi}, U128{t[2], t[3]});
    uint32_t c[4] = {(uint32_t)J.c64.lo, (uint32_t)(J.c64.lo >> 32), (uint32_t)J.c64.hi, (uint32_t)(J.c64.hi >> 32)};
#pragma unroll
    for (int i = 0; i < 4; i++) TMG_OPAQUE_V(c[i]);                 // in VGPRs once, not copied per fill
    J.c64 = U128{((uint64_t)c[1] << 32) | c[0], ((uint64_t)c[3] << 32) | c[2]};
    J.X = U128{0, 0};
    return J;
}

template <int NB, class WS>
__device__ __forceinline__ void bp_ring_init(const Params &P, WS &w, int lane, const Rng &g, BpRing &r, BpJump &J) {
    r.fill = r.cons = 0;
    r.rmin = 0xffffffffu;
    if ((g.h >> 32) & 1) {                                   // the buffered half-word is colour 127
        const uint64_t m = (uint64_t)(uint32_t)g.h * (uint32_t)P.k;
        r.rmin = (uint32_t)m;
        const uint32_t code = (uint32_t)(m >> 32);
        uint32_t *ring = bp_ring(w);
        if (lane == 0) {
#pragma unroll
            for (int b = 0; b < NB; b++) ring[b * kBpPlaneDw + 3] = ((code >> b) & 1u) << 31;
        }
        r.cons = 127;
        r.fill = 128;
    }
    r.cons0 = r.cons;
    // the first batch's states: s_{o+1} = A^{o+1} s + G_{o+1} inc, o = bp_out(lane)
    // (an opaque lane: after a shuffle the loop calls this again, and the
    // table row and its product with inc would otherwise be hoisted out of
    // the loop and held in 8 VGPRs through every redraw)
    const uint64_t *t = P.jump + bp_out(loop_lane(lane)) * 4;
    cover_uniform(P, lane, U128{g.slo, g.shi});
    J.X = jump128(U128{t[0], t[1]}, U128{g.slo, g.shi}, mul128(U128{g.ilo, g.ihi}, U128{t[2], t[3]}));
}

// the next 128 colours (64 PCG64 outputs, Lemire-32 on each half) appended
// to the plane strings: lane l gets the codes of colours l and 64 + l from
// itself and its quad neighbour, and one ballot per plane and half gives the
// batch's bits in sequence order; lane 0 stores them
template <int NB, class WS>
__device__ __forceinline__ void bp_ring_fill(const Params &P, WS &w, int lane, BpJump &J, BpRing &r) {
    const uint32_t k = (uint32_t)P.k;
    const uint64_t out = xsl_rr(J.X);
    cover_uniform(P, lane, J.A64);
    J.X = jump128(J.X, J.A64, J.c64);                                // the next batch (A^64: uniform, SGPRs)
    const uint64_t m0 = (uint64_t)(uint32_t)out * k, m1 = (out >> 32) * k;
    if (P.thr != 0u) r.rmin = umin3(r.rmin, (uint32_t)m0, (uint32_t)m1);   // tested once, after the redraws
    const uint32_t c0 = (uint32_t)(m0 >> 32), c1 = (uint32_t)(m1 >> 32);   // codes of colours 2o, 2o + 1
    const uint32_t n0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c0, 0xb1, 0xf, 0xf, true);   // quad_perm [1,0,3,2]
    const uint32_t n1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c1, 0xb1, 0xf, 0xf, true);
    const bool odd = lane & 1;
    const uint32_t x0 = odd ? n1 : c0, x1 = odd ? c1 : n0;        // codes of colours l, 64 + l (< 2^NB)
    uint64_t b0[NB], b1[NB];
#pragma unroll
    for (int b = 0; b < NB; b++) {
        if (b == NB - 1) {                                        // the top bit: one compare
            b0[b] = __ballot(x0 >= (1u << b));
            b1[b] = __ballot(x1 >= (1u << b));
        } else {
            b0[b] = __ballot((x0 >> b) & 1u);
            b1[b] = __ballot((x1 >> b) & 1u);
        }
    }
    const int q = (r.fill >> 5) & (kBpRingDw - 1);
    if constexpr (WS::NP > 2) {
        // 512-cell kernels: one VGPR base (ring + q) for every store.  The
        // planes and their guard copies sit at immediate offsets from it,
        // where separate scalar bases each needed a v_mov.  (The 128-cell
        // kernels measured the same either way, profiles/r04/s8.)
        uint32_t *ws = reinterpret_cast<uint32_t *>(&w);
        int at = (int)(bp_ring(w) - ws) + q;                         // dword index of ring + q (scalar)
        TMG_OPAQUE_V(at);
        if (lane == 0) {
            uint64_t *d = reinterpret_cast<uint64_t *>(ws + at);
#pragma unroll
            for (int b = 0; b < NB; b++) {
                d[b * kBpPlaneDw / 2] = b0[b];
                d[b * kBpPlaneDw / 2 + 1] = b1[b];
            }
            if (q == 0) {                                            // guard copy
#pragma unroll
                for (int b = 0; b < NB; b++) {
                    d[b * kBpPlaneDw / 2 + kBpRingDw / 2] = b0[b];
                    d[b * kBpPlaneDw / 2 + kBpRingDw / 2 + 1] = b1[b];
                }
            }
        }
    } else if (lane == 0) {
        uint32_t *ring = bp_ring(w);
#pragma unroll
        for (int b = 0; b < NB; b++) {
            uint64_t *d = reinterpret_cast<uint64_t *>(ring + b * kBpPlaneDw + q);
            d[0] = b0[b];
            d[1] = b1[b];
            if (q == 0) { d[kBpRingDw / 2] = b0[b]; d[kBpRingDw / 2 + 1] = b1[b]; }   // guard copy
        }
    }
    r.fill += 128;
}

// Whether a filled word was Lemire-rejected (some lane's running minimum
// below thr; a word filled but never consumed counts too, which only sends
// the board to the exact path needlessly)
__device__ __forceinline__ bool bp_rejected(const Params &P, const BpRing &r) {
    return P.thr != 0u && __ballot(r.rmin < P.thr) != 0ULL;
}

// The exact PCG64 state after the last consumed colour i: lane L = the lane
// of its output o holds X = s_{n+1} for output n = o of the next unfilled
// batch, m = (fill >> 7) - (i >> 7) batches after i's (1 <= m <= 6: the
// redraw loop keeps fewer than N + 128 <= 640 colours filled ahead), so s = A^{-64m} X - A^{-64m}
// G_{64m} inc (jump-table row 63 + m).
// Colours filled ahead of the consume position: bp_prefetch fills while fewer
// than maxM <= N <= 512 (C <= 32, N <= 512) are ahead, 128 at a time.
constexpr int kBpMaxAhead = 512 + 128;
static_assert(kBpMaxAhead / 128 + 1 <= kJumpRows - 64,
              "bp_ring_state's backward jump needs a jump-table row for every batch count the ring can reach");
__device__ __forceinline__ void bp_ring_state(const Params &P, const BpJump &J, const BpRing &r, Rng &g) {
    if (r.cons == r.cons0) return;                                   // nothing taken since bp_ring_init(g)
    const int i = r.cons - 1, local = i & 127;                       // i >= 128: a take draws >= 2 colours
    const int m = __builtin_amdgcn_readfirstlane((r.fill >> 7) - (i >> 7));
#if TMG_COVER
    if (m < 1 || m > kJumpRows - 64) P.status[0] = 1u;              // (m wave-uniform) the table has no such row
#endif
    const int l = bp_lane(local >> 1);
    const U128 x{rdlane64(J.X.lo, l), rdlane64(J.X.hi, l)};
    const uint64_t *t = P.jump + (63 + m) * 4;
    const U128 s = add128(mul128(U128{bcast64(t[0]), bcast64(t[1])}, x),         // wave-uniform: SALU
                          mul128(U128{bcast64(t[2]), bcast64(t[3])}, U128{g.ilo, g.ihi}));
    g.slo = bcast64(s.lo);
    g.shi = bcast64(s.hi);
    g.h = ((uint64_t)((local & 1) ^ 1) << 32) | (uint32_t)(xsl_rr(U128{g.slo, g.shi}) >> 32);   // lo half taken: hi half buffered
}

// The next redraw's colours start at the ring's consume position whatever rows
// it redraws (lane r's row at cons + rC), so its reads can be issued before the
// line search that decides the rows: bp_prefetch keeps at least maxM colours
// filled ahead and issues every plane's two ring dwords, bp_apply merges rows
// 0..row once the search has returned.  The LDS latency then overlaps the
// search instead of following it.
template <int NB>
struct BpReads {
    uint32_t lo[NB], hi[NB], sh;
};
template <int NB, class WS>
__device__ __forceinline__ BpReads<NB> bp_prefetch(const Params &P, WS &w, int lane, BpJump &J, BpRing &r, int maxM) {
    r.fill = __builtin_amdgcn_readfirstlane(r.fill);
    r.cons = __builtin_amdgcn_readfirstlane(r.cons);
    while (r.fill - r.cons < maxM) bp_ring_fill<NB>(P, w, lane, J, r);
    // One wave per workgroup, and a wave's LDS instructions execute in order:
    // the reads below see lane 0's ring stores (bp_ring_fill) without waiting
    // for those stores to complete, so a compiler-only fence, not WSYNC's wait
    WFENCE();
    const uint32_t *ring = bp_ring(w);
    const int o = r.cons + lane * P.C;
    const int d = (o >> 5) & (kBpRingDw - 1);
    BpReads<NB> x;
    x.sh = (uint32_t)o & 31u;
#pragma unroll
    for (int b = 0; b < NB; b++) {
        x.lo[b] = ring[b * kBpPlaneDw + d];
        x.hi[b] = ring[b * kBpPlaneDw + d + 1];
    }
    return x;
}
template <int NB>
__device__ __forceinline__ void bp_apply(const Params &P, int lane, BpRing &r, const BpReads<NB> &x, int row, uint32_t cm,
                                         RowPlanes<NB> &pl) {
    const uint32_t in = lane <= row ? cm : 0u;
#pragma unroll
    for (int b = 0; b < NB; b++) {
        const uint32_t v = __builtin_amdgcn_alignbit(x.hi[b], x.lo[b], x.sh);
        pl.p[b] = (v & in) | (pl.p[b] & ~in);
    }
    r.cons += (row + 1) * P.C;
}

// rows 0..row <- the ring's next (row + 1) * C colours (colour plane only)
template <int NB, class WS>
__device__ __forceinline__ void bp_take(const Params &P, WS &w, int lane, BpJump &J, BpRing &r, int row,
                                        uint32_t cm, RowPlanes<NB> &pl) {
    const BpReads<NB> x = bp_prefetch<NB>(P, w, lane, J, r, (row + 1) * P.C);
    bp_apply<NB>(P, lane, r, x, row, cm, pl);
}

// The row of the first coord of the first line get_colour_lines would return
// (remove_colour_lines, board.py:120-131), or -1 when it returns [].
// hml / vml: this lane's valid horizontal-start / vertical-anchor columns.
template <int NB>
__device__ __forceinline__ int bp_first_line_row(const RowPlanes<NB> &pl, uint32_t hml, uint32_t vml) {
    uint32_t neR = 0, neU = 0;
#pragma unroll
    for (int b = 0; b < NB; b++) {
        const uint32_t x = pl.p[b];
        neR |= x ^ (x >> 1);
        neU |= x ^ (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xf, 0xf, true);   // wave_shr:1: row r-1
    }
    const uint32_t eqU = ~neU;
    const uint32_t h = ~(neR | (neR >> 1)) & hml;
    const uint32_t v = eqU & (uint32_t)__builtin_amdgcn_update_dpp(0, (int)eqU, 0x138, 0xf, 0xf, true) & vml;
    const uint32_t any = h | v;
    const uint64_t rows = __ballot(any != 0u);
    if (!rows) return -1;
    const int rs = 63 - __clzll(rows);                           // bottom-most row holding a line
    const uint32_t av = (uint32_t)__builtin_amdgcn_readlane((int)any, rs);
    const uint32_t vv = (uint32_t)__builtin_amdgcn_readlane((int)v, rs);
    const int c0 = __builtin_ctz(av);                            // leftmost line, vertical checked first
    if (!((vv >> c0) & 1u)) return rs;                           // horizontal: starts at (rs, c0)
    const uint64_t m = __ballot((eqU >> c0) & 1u);               // (r, c0) == (r-1, c0)
    const uint64_t low = rs >= 63 ? ~0ULL : (2ULL << rs) - 1ULL;
    return 63 - __clzll((~m & low) | 1ULL);                       // vertical: the top of its run
}

// the LDS colour plane from the row planes (cell p: row r's planes by bpermute)
template <int NB, class WS>
__device__ __forceinline__ void bp_to_lds(const Params &P, WS &w, int lane, const RowPlanes<NB> &pl) {
    const int N = P.N, C = P.C;
#pragma unroll
    for (int i = 0; i < WS::NP; i++) {
        if (i * 64 >= N) break;                                  // wave-uniform
        const int p = min(i * 64 + lane, N - 1);
        const int r = div_c(P, p), c = p - r * C;
        int code = 0;
#pragma unroll
        for (int b = 0; b < NB; b++) code |= (int)((((uint32_t)__builtin_amdgcn_ds_bpermute(r << 2, (int)pl.p[b])) >> c) & 1u) << b;
        if (i * 64 + lane < N) w.brd[p] = (int8_t)(code + 1);
    }
}

// the row planes from the LDS colour plane (after a shuffle)
template <int NB, class WS>
__device__ __forceinline__ RowPlanes<NB> bp_from_lds(const Params &P, const WS &w, int lane) {
    RowPlanes<NB> pl;
#pragma unroll
    for (int b = 0; b < NB; b++) pl.p[b] = 0;
    const int r = lane < P.R ? lane : 0;
    for (int c = 0; c < P.C; c++) {
        const uint32_t x = lane < P.R ? (uint32_t)(w.brd[r * P.C + c] - 1) : 0u;
#pragma unroll
        for (int b = 0; b < NB; b++) pl.p[b] |= ((x >> b) & 1u) << c;
    }
    return pl;
}

// generate_board (board.py:95-109) on row bit-planes (C <= 32, colours of at
// most NB planes).  Returns FL_ERR when the shuffle cap was hit, 0 otherwise;
// -1 on a Lemire rejection anywhere in the colours drawn (Generator.integers'
// bounded draw, p = thr / 2^32 per word): g is then back at its starting
// state and the caller redoes the board on an exact draw-by-draw path.
// Leaves the board in LDS (colour plane; types 1) and its mask in w.effw.
// PRIO: the regenerating wave goes first at issue.  A launch that regenerates
// boards lasts as long as its slowest board, one serial chain of redraws on
// one wave, while the other streams' steps share its SIMD (measured: the lean
// kernels' inline autoreset and the 512-cell reset kernel gain; the 128-cell
// masked reset, beside the c3 step kernels, loses 0.6 %: not raised there).
template <int NB, bool PRIO = true, class WS>
__device__ __forceinline__ int bp_generate(const Params &P, WS &w, int lane, Rng &g) {
    const int R = P.R, C = P.C, N = P.N;
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(3);
    // g is wave-uniform; said so explicitly, since where the divergence analysis
    // cannot see it (the lean step kernel's inline autoreset) the ring's
    // counters and state otherwise go to VGPRs and its loops run exec-masked
    rng_bcast(g);
    const Rng g0 = g;
    BpJump J = load_bp_jump(P, g);
    const uint32_t cm = C >= 32 ? ~0u : (1u << C) - 1u;
    const uint32_t hml = (lane < R && C >= 3) ? cm >> 2 : 0u;          // columns <= C-3
    const uint32_t vml = (lane >= 2 && lane < R) ? cm : 0u;            // rows >= 2
    for (int p = lane; p < N; p += 64) w.brd[N + p] = 1;
    BpRing r;
    bp_ring_init<NB>(P, w, lane, g, r, J);
    RowPlanes<NB> pl;
#pragma unroll
    for (int b = 0; b < NB; b++) pl.p[b] = 0;
    bp_take<NB>(P, w, lane, J, r, R - 1, cm, pl);                       // :97
    int fl = 0;
    bool rej = false;
    for (int shuffles = 0;; shuffles++) {
        // remove_colour_lines, :120-131.  A Lemire rejection is looked for
        // once the redraws end: until then the colours of a stream with a
        // rejected word are still colours, the loop ends as it would on any
        // other board, and the board is then redone exactly.
        for (;;) {
            const BpReads<NB> x = bp_prefetch<NB>(P, w, lane, J, r, N);          // the next redraw's colours
            const int r0 = bp_first_line_row<NB>(pl, hml, vml);
            if (r0 < 0) break;
            bp_apply<NB>(P, lane, r, x, R - 1 < r0 + 1 ? R - 1 : r0 + 1, cm, pl);   // rows 0..min(R-1, r0+1)
        }
        if ((rej = bp_rejected(P, r))) break;
        bp_to_lds<NB>(P, w, lane, pl);
        WSYNC();
        if ((TMG_RSCAN & 4) && P.C <= kRowScanMaxC ? scan_rows<false>(P, w, lane, true) != 0
                                                    : scan_effective_clean<false>(P, w, lane))
            break;                                                       // possible_move, :102
        if (shuffles >= kMaxShuffles) { fl = FL_ERR; break; }
        COVER(CV_SHUFFLE_GEN);
        bp_ring_state(P, J, r, g);                                       // shuffle draws from the stream itself
        WSYNC();
        shuffle(P, w, lane, g);                                          // :105-106
        pl = bp_from_lds<NB>(P, w, lane);
        fl = FL_SHUF;
        bp_ring_init<NB>(P, w, lane, g, r, J);
    }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
    if (rej) {
        COVER(CV_REJECT_GEN);
        g = g0;
        WSYNC();
        return -1;
    }
    bp_ring_state(P, J, r, g);
    WSYNC();
    return fl & FL_ERR;
}

// Queue env e for spill_kernel.  The host sizes the queue for every env of
// the launch, so this cannot fail; false only if that sizing were broken.
__device__ __forceinline__ bool queue_env(SpillQ *q, int lane, int64_t e) {
    int ok = 0;
    if (lane == 0) {
        const uint32_t i = atomicAdd(&q->count, 1u);
        if ((int64_t)i < q->cap) { q->env[i] = e; ok = 1; }
    }
    return __ballot(ok) != 0ULL;
}

// lane 0 records st in the sticky status words (a rare path: error / overflow)
__device__ __forceinline__ void note_status(const Params &P, int lane, uint32_t st) {
    // one word per status bit, each only ever set to 1: plain stores, no atomics
    if (st && lane == 0) {
        if (st & ST_INTERNAL) P.status[0] = 1u;
        if (st & ST_OVERFLOW) P.status[1] = 1u;
        if (st & ST_CALLER) P.status[2] = 1u;
    }
}

template <class WS>
__device__ __forceinline__ int count_type_zero(const Params &P, const WS &w, int lane) {
    int z = 0;
#pragma unroll
    for (int i = 0; i < WS::NP; i++) {
        int p = i * 64 + lane;
        z += __popcll(__ballot(p < P.N && w.brd[P.N + p] == 0));
    }
    return z;
}

template <class WS>
__device__ __forceinline__ int count_colour_nonzero(const Params &P, const WS &w, int lane) {
    int z = 0;
#pragma unroll
    for (int i = 0; i < WS::NP; i++) {
        int p = i * 64 + lane;
        z += __popcll(__ballot(p < P.N && w.brd[p] != 0));
    }
    return z;
}

// ---------------------------------------------------------------- fast cascade
// One cascade iteration when no special can exist (no specials enabled and
// every type is 1): the reference then turns every line of get_colour_lines
// (first pass + perpendicular pass, board.py:149-215) into a normal match
// (process_colour_lines :269-327) and clears their union
// (resolve_colour_match :460-471).  Returns the number of cleared cells.
template <class WS>
__device__ __forceinline__ int fast_clear(const Params &P, WS &w, int lane, const Cells<WS::NP> &cl, const Det<WS::NP> &d, int rs) {
    const int R = P.R, C = P.C, N = P.N;
    int8_t *col = w.brd, *typ = w.brd + N;
    // mark bit0: first-pass coord (the static `coords` list), bit1: cleared
    for (int p = lane; p < N; p += 64) w.mark[p] = 0;
    WSYNC();
    // horizontal lines of row rs: runs of >= 3 starting at their h bits
    const uint64_t hb = bits_at(d.h, rs * C, C);
    const uint64_t cov = hb | (hb << 1) | (hb << 2);
    if (lane < C && ((cov >> lane) & 1)) w.mark[rs * C + lane] = 3;
    // vertical lines anchored in row rs: the whole run above
    uint64_t vb = bits_at(d.v, rs * C, C);
    while (vb) {
        int c = __ffsll((unsigned long long)vb) - 1;
        vb &= vb - 1;
        int top = run_top(P, w, lane, rs, c);
        if (lane >= top && lane <= rs) w.mark[lane * C + c] = 3;
    }
    WSYNC();
    // perpendicular pass: from every first-pass coord walk both axes over
    // non-coord cells of the same colour; a run of >= 3 is a line
    for (int p = lane; p < N; p += 64) {
        if (!(w.mark[p] & 1)) continue;
        int r = p / C, c = p - r * C, x = col[p];
        int lft = 0, rgt = 0, up = 0, dn = 0;
        while (c - lft - 1 >= 0 && !(w.mark[p - lft - 1] & 1) && col[p - lft - 1] == x) lft++;
        while (c + rgt + 1 < C && !(w.mark[p + rgt + 1] & 1) && col[p + rgt + 1] == x) rgt++;
        while (r - up - 1 >= 0 && !(w.mark[p - (up + 1) * C] & 1) && col[p - (up + 1) * C] == x) up++;
        while (r + dn + 1 < R && !(w.mark[p + (dn + 1) * C] & 1) && col[p + (dn + 1) * C] == x) dn++;
        if (1 + lft + rgt >= 3) {
            for (int i = 1; i <= lft; i++) w.mark[p - i] |= 2;
            for (int i = 1; i <= rgt; i++) w.mark[p + i] |= 2;
        }
        if (1 + up + dn >= 3) {
            for (int i = 1; i <= up; i++) w.mark[p - i * C] |= 2;
            for (int i = 1; i <= dn; i++) w.mark[p + i * C] |= 2;
        }
    }
    WSYNC();
    int cleared = 0;
#pragma unroll
    for (int i = 0; i < WS::NP; i++) {
        int p = i * 64 + lane;
        bool clr = p < N && (w.mark[p] & 2);
        if (clr) { col[p] = 0; typ[p] = 0; }
        cleared += __popcll(__ballot(clr));
    }
    WSYNC();
    return cleared;
}

// process_colour_lines' bomb rule (board.py:304-320) for the first-pass lines
// of one row rs, as column masks of that row: hb = horizontal anchor columns
// (a run of L cells holds L-2 consecutive bits), x = the columns where a
// vertical line ending in row rs meets a horizontal run (the shared cell).
// The verticals sort first (their first coord lies above row rs), so each such
// vertical makes a bomb with the run it meets: its cells + the two run cells
// nearest the shared one (by distance, then column, :309-312), and a run of
// < 6 cells then leaves the list with its other cells uncleared (:314-315).
// The bomb goes to the shared cell: get_special_creation_pos' corner
// (:437-447), the bomb's most common row (rs) and column (the vertical's).
// Handled when every vertical is 3 or >= 5 long (the caller's check), each run
// meets one vertical and is at most 5 long; false otherwise.  keep: the run
// cells that stay on the board (vcols: the vertical lines' columns, whose
// cells go with those lines); gone: the runs the bombs took.
__device__ __forceinline__ bool bomb_plan(uint64_t hb, uint64_t x, uint64_t &keep, uint64_t vcols, uint64_t &gone) {
    const uint64_t st = hb & ~(hb << 1);                                     // run starts
    keep = 0;
    gone = 0;
    for (uint64_t m = x; m; m &= m - 1) {
        const int c = __ffsll((unsigned long long)m) - 1;
        const uint64_t le = st & (c >= 63 ? ~0ULL : (2ULL << c) - 1);        // starts <= c
        if (!le) return false;
        const int s = 63 - __clzll(le);
        const int len = __ffsll((unsigned long long)~(hb >> s)) + 1;         // anchors + 2
        if (len > 5) return false;
        const uint64_t run = ((1ULL << len) - 1) << s;
        if (__popcll(x & run) != 1) return false;
        const int e = s + len - 1;
        const uint64_t take = (1ULL << c) | (c > s && c < e ? (5ULL << (c - 1)) : c == s ? (3ULL << (c + 1)) : (3ULL << (c - 2)));
        keep |= run & ~take & ~vcols;                                        // other verticals' cells go with them
        gone |= run;
    }
    return true;
}

// Whether every cell is a coloured tile of type >= 1 with colour 1..k or a
// colourless cookie: then equal colours >= 1 imply types >= 1, so the line
// runs of get_colour_lines (which extend by colour only, board.py:163-193) are
// exactly the anchored runs of detect().  Empties and cookies that gained a
// colour (remove_colour_lines after a shuffle, :129) fail it.  A cascade keeps
// it: refill draws type-1 tiles, create_special gives a cookie colour 0.
template <class WS>
__device__ __forceinline__ bool plain_board(const Params &P, const WS &w, int lane) {
    const int N = P.N;
    bool odd = false;
    for (int p = lane; p < N; p += 64) {
        const int x = w.brd[p], y = w.brd[N + p];
        odd |= y == 0 || (y < 0 && x != 0) || (y > 0 && (x < 1 || x > P.k));
    }
    return __ballot(odd) == 0ULL;
}

// One cascade step of the general kernel (board.py:367-376) on the LDS board,
// wave-parallel, when it needs none of the lane-0 list machinery — the form of
// sb_simple_step for boards without a bitboard path (the 512-cell kernels).
// Requires plain_board().  The step qualifies when get_colour_lines (:149-215)
// yields no perpendicular line, process_colour_lines (:269-327) makes every
// first-pass line of row rs a normal match, a laser or a bomb of bomb_plan (no
// 5+-line when cookies are enabled; no two lines sharing a cell when a laser
// is created) and no line cell holds a special (resolve_colour_match :460-471).
// A straight 4-line's laser goes to its second cell in (row, col) order
// (get_special_creation_pos :429-458, nothing taken): (rs, s+1) / (top+1, c).
// Returns 0 when the step does not qualify (LDS board and marks untouched),
// otherwise the number of cleared cells (cleared in LDS, lasers placed,
// SC_NNEW counted); gravity and refill are the caller's.
template <class WS>
__device__ __forceinline__ int simple_step_lds(const Params &P, WS &w, int lane, const Det<WS::NP> &d, int rs,
                                               uint64_t &cols, int &rows) {
    const int C = P.C, R = P.R, N = P.N, S = P.smask;
    int8_t *col = w.brd, *typ = w.brd + N;
    const uint64_t cm = C >= 64 ? ~0ULL : (1ULL << C) - 1;
    // horizontal runs of row rs: an L-run holds L-2 consecutive anchor bits
    const uint64_t hb = bits_at(d.h, rs * C, C), vb = bits_at(d.v, rs * C, C);
    const uint64_t st = hb & ~(hb << 1);
    const uint64_t h4 = st & (hb >> 1) & ~(hb >> 2), h5 = st & (hb >> 1) & (hb >> 2);
    if (h5 && (S & SP_COOKIE)) return 0;
    const uint64_t cov = (hb | (hb << 1) | (hb << 2)) & cm;
    const uint64_t hl = (S & (SP_HLASER | SP_VLASER)) ? h4 << 1 : 0ULL;   // laser cells (columns of row rs)
    // vertical runs ending in row rs: lane c keeps the top row of column c's run
    int vt = R;
    uint64_t vl = 0;                                                         // columns of vertical 4-lines
    bool v4 = false;
    cols = cov | vb;
    rows = cov ? 1 : 0;
    int ptop = rs;                                                           // top row of the coords
    for (uint64_t m = vb; m; m &= m - 1) {
        const int c = __ffsll((unsigned long long)m) - 1;
        const int top = run_top(P, w, lane, rs, c);
        const int L = rs - top + 1;
        rows = max(rows, L);
        ptop = min(ptop, top);
        if (L >= 5 && (S & SP_COOKIE)) return 0;
        v4 |= L == 4;
        if (L == 4 && (S & SP_VLASER)) vl |= 1ULL << c;
        vt = lane == c ? top : vt;
    }
    // shared cells: lines sharing a cell are separate normal matches without
    // bombs; with bombs they follow bomb_plan
    const uint64_t x = vb & cov, bombc = (S & SP_BOMB) ? x : 0ULL;
    uint64_t keepc = 0;
    if (x && (hl || vl)) return 0;
    uint64_t gonec = 0;
    if (bombc && (h4 || v4 || !bomb_plan(hb, bombc, keepc, vb, gonec))) return 0;
    // coords K: lane-parallel over the cells, K = row rs's runs + the column runs
    const int th = (S & SP_HLASER) ? 3 : 2;
    bool bad = false;
    // the coords lie in rows ptop..rs: only the passes holding those rows
    const int plo = (ptop * C) & ~63, phi = min((rs + 1) * C, N);
    for (int p0 = plo; p0 < phi; p0 += 64) {                                // uniform passes (bpermute)
        const int p = p0 + lane;
        const int r = div_c(P, p), c = p - r * C;
        const int top = __builtin_amdgcn_ds_bpermute((c & 63) << 2, vt);
        const bool k = p < N && ((r == rs && ((cov >> c) & 1)) || (((vb >> c) & 1) && r >= top && r <= rs));
        bad |= k && typ[p] != 1;
        if (k) w.mark[p] = 1;
    }
    WSYNC();
    // get_colour_lines' perpendicular pass (:195-214): from every coord walk each
    // axis over non-coord cells of the same colour; a run of >= 3 is a line
    for (int p = plo + lane; p < phi; p += 64) {
        if (!w.mark[p]) continue;
        const int r = div_c(P, p), c = p - r * C, x = col[p];
        int lft = 0, rgt = 0, up = 0, dn = 0;
        while (c - lft - 1 >= 0 && !w.mark[p - lft - 1] && col[p - lft - 1] == x) lft++;
        while (c + rgt + 1 < C && !w.mark[p + rgt + 1] && col[p + rgt + 1] == x) rgt++;
        while (r - up - 1 >= 0 && !w.mark[p - (up + 1) * C] && col[p - (up + 1) * C] == x) up++;
        while (r + dn + 1 < R && !w.mark[p + (dn + 1) * C] && col[p + (dn + 1) * C] == x) dn++;
        bad |= lft + rgt >= 2 || up + dn >= 2;
    }
    const bool ok = __ballot(bad) == 0ULL;
    WSYNC();
    // resolve: clear the coords (no special among them), then place the lasers
    int cleared = 0;
    for (int p0 = plo; p0 < phi; p0 += 64) {
        const int p = p0 + lane;
        const bool k = p < phi && w.mark[p];
        const int r = div_c(P, p), c = p - r * C;
        const int top = __builtin_amdgcn_ds_bpermute((c & 63) << 2, vt);
        bool pos = false, keep = false;
        int t = 2;
        if (k) {
            const bool ph = r == rs && ((hl >> c) & 1);
            const bool pv = ((vl >> c) & 1) && r == top + 1;
            const bool pb = r == rs && ((bombc >> c) & 1);
            keep = r == rs && ((keepc >> c) & 1);
            pos = ph || pv || pb;
            t = ph ? th : pb ? 4 : 2;
            w.mark[p] = 0;
            if (ok) {
                if (pos) typ[p] = (int8_t)t;
                else if (!keep) { col[p] = 0; typ[p] = 0; }
            }
        }
        cleared += __popcll(__ballot(k && !pos && !keep));
    }
    if (!ok) { WSYNC(); return 0; }
    if (lane == 0) w.sc[SC_NNEW] += __popcll(hl) + __popcll(vl) + __popcll(bombc);
    if (hl | vl) COVER(CV_LDS_LASER);
    if (bombc) COVER(CV_LDS_BOMB);
    if (!(hl | vl | bombc)) COVER(CV_LDS_NORMAL);
    WSYNC();
    return cleared;
}

// ------------------------------------------------------------ general (lane 0)
// Everything below runs on lane 0 only, against LDS.
template <int MAXN, class LS = WsSerial<MAXN>>
struct Serial {
    const Params &P;
    WsCore<MAXN> &w;
    LS &s;
    int8_t *col, *typ;
    int R, C, N;
    int nl, np;        // lines / pool fill
    int nm, nmp;       // matches / match-pool fill
    bool ovf;

    __device__ __forceinline__ Serial(const Params &P_, WsCore<MAXN> &w_, LS &s_) : P(P_), w(w_), s(s_) {
        R = P.R; C = P.C; N = P.N;
        col = w.brd; typ = w.brd + N;
        nl = np = nm = nmp = 0;
        ovf = false;
    }

    __device__ __forceinline__ void clr(int p) {
        if (col[p] != 0) w.sc[SC_NZ]--;
        col[p] = 0; typ[p] = 0;
    }

    // ---- get_colour_lines, board.py:149-215 (rs = bottom-most row with a line)
    __device__ __forceinline__ void build_lines(int rs) {
        nl = 0; np = 0;
        uint64_t hcov = 0;
        const int row = rs;
        for (int c = 0; c < C; c++) {
            int p = row * C + c;
            if (row > 1 && typ[p] > 0 && col[p] == col[p - C]) {                 // :163-177
                int start = row - 1;
                while (start > 0 && col[(start - 1) * C + c] == col[p]) start--;
                if (row - start >= 2) {
                    if (nl >= LS::MLINES || np + (row - start + 1) > LS::POOL) { ovf = true; return; }
                    s.ls[nl] = (int16_t)np; s.ll[nl] = (int16_t)(row - start + 1);
                    for (int i = start; i <= row; i++) s.pool[np++] = (int16_t)(i * C + c);
                    nl++;
                }
            }
            if (c < C - 2 && !((hcov >> c) & 1) && typ[p] > 0 && col[p] == col[p + 1]) {   // :179-193
                int end = c + 1;
                while (end < C - 1 && col[row * C + end + 1] == col[p]) end++;
                if (end - c >= 2) {
                    if (nl >= LS::MLINES || np + (end - c + 1) > LS::POOL) { ovf = true; return; }
                    s.ls[nl] = (int16_t)np; s.ll[nl] = (int16_t)(end - c + 1);
                    for (int i = c; i <= end; i++) { s.pool[np++] = (int16_t)(row * C + i); hcov |= 1ULL << i; }
                    nl++;
                }
            }
        }
        // perpendicular pass over the static coord list, :195-214
        const int ncoords = np;
        for (int i = 0; i < ncoords; i++) w.mark[s.pool[i]] = 1;
        // directions (0,1),(1,0),(0,-1),(-1,0): the last two walk the same cells
        // as the first two, so their sorted lines are always duplicates
        for (int ci = 0; ci < ncoords && !ovf; ci++) {
            const int cp = s.pool[ci];
            const int cr = cp / C, cc = cp - cr * C;
            for (int d = 0; d < 2; d++) {
                const int st = np;
                if (np + R + C + 1 > LS::POOL || nl >= LS::MLINES) { ovf = true; break; }
                s.pool[np++] = (int16_t)cp;
                for (int sd = 0; sd < 2; sd++) {
                    int dr = d == 1 ? (sd ? -1 : 1) : 0, dc = d == 0 ? (sd ? -1 : 1) : 0;
                    int nr = cr + dr, nc = cc + dc;
                    while (nr >= 0 && nr < R && nc >= 0 && nc < C) {
                        int cell = nr * C + nc;
                        if (w.mark[cell]) break;                                    // n in coords
                        if (!(col[cp] == col[cell] && typ[cp] > 0 && typ[cell] > 0)) break;   // match_color
                        s.pool[np++] = (int16_t)cell;
                        nr += dr; nc += dc;
                    }
                }
                const int len = np - st;
                if (len >= 3) {
                    for (int i = st + 1; i < np; i++) {                             // sorted()
                        int16_t x = s.pool[i]; int j = i - 1;
                        while (j >= st && s.pool[j] > x) { s.pool[j + 1] = s.pool[j]; j--; }
                        s.pool[j + 1] = x;
                    }
                    bool dup = false;                                               // not in lines
                    for (int l = 0; l < nl && !dup; l++) {
                        if (s.ll[l] != len) continue;
                        bool same = true;
                        for (int i = 0; i < len; i++) if (s.pool[s.ls[l] + i] != s.pool[st + i]) { same = false; break; }
                        dup = same;
                    }
                    if (dup) np = st;
                    else { s.ls[nl] = (int16_t)st; s.ll[nl] = (int16_t)len; nl++; }
                } else {
                    np = st;
                }
            }
        }
        for (int i = 0; i < ncoords; i++) w.mark[s.pool[i]] = 0;
    }

    __device__ __forceinline__ bool line_has(int l, int cell) {
        for (int i = 0; i < s.ll[l]; i++) if (s.pool[s.ls[l] + i] == cell) return true;
        return false;
    }

    __device__ __forceinline__ int add_match(int name, int colour) {
        if (nm >= LS::MM) { ovf = true; return -1; }
        s.ms[nm] = (int16_t)nmp; s.mlen[nm] = 0; s.mname[nm] = (int8_t)name; s.mcol[nm] = (int8_t)colour;
        return nm++;
    }
    __device__ __forceinline__ void match_push(int m, int cell) {
        if (nmp >= LS::MPOOL) { ovf = true; return; }
        s.mpool[nmp++] = (int16_t)cell; s.mlen[m]++;
    }

    // ---- process_colour_lines, board.py:269-327
    __device__ __forceinline__ void process_lines() {
        const int S = P.smask;
        nm = 0; nmp = 0;
        // lines are already sorted internally; stable sort by first row (:282)
        int qn = 0;
        for (int l = 0; l < nl; l++) {
            int key = s.pool[s.ls[l]] / C, j = qn - 1;
            while (j >= 0 && s.pool[s.ls[s.q[j]]] / C > key) { s.q[j + 1] = s.q[j]; j--; }
            s.q[j + 1] = (int16_t)l;
            qn++;
        }
        int head = 0;
        while (head < qn && !ovf) {
            const int L = s.q[head++];                                              // pop(0)
            const int ls = s.ls[L], ln = s.ll[L];
            if (ln >= 5 && (S & SP_COOKIE)) {                                       // :287-292
                int m = add_match(M_COOKIE, 0); if (m < 0) return;
                for (int i = 0; i < 5; i++) match_push(m, s.pool[ls + i]);
                if (ln - 5 > 2) {
                    if (nl >= LS::MLINES || qn >= LS::MQ) { ovf = true; return; }
                    s.ls[nl] = (int16_t)(ls + 5); s.ll[nl] = (int16_t)(ln - 5);
                    s.q[qn++] = (int16_t)nl; nl++;
                }
            } else if (ln == 4) {                                                   // :294-302
                int name;
                if (s.pool[ls] / C == s.pool[ls + 1] / C && (S & SP_HLASER)) name = M_HLASER;
                else if (S & SP_VLASER) name = M_VLASER;
                else name = M_NORMAL;
                int m = add_match(name, col[s.pool[ls]]); if (m < 0) return;
                for (int i = 0; i < 4; i++) match_push(m, s.pool[ls + i]);
            } else {
                bool shared_any = false;
                if (S & SP_BOMB)
                    for (int h = head; h < qn && !shared_any; h++)
                        for (int i = 0; i < ln; i++) if (line_has(s.q[h], s.pool[ls + i])) { shared_any = true; break; }
                if (shared_any) {                                                   // :304-320
                    for (int h = head; h < qn; h++) {
                        const int O = s.q[h];
                        int shared = -1;
                        for (int i = 0; i < ln; i++) if (line_has(O, s.pool[ls + i])) { shared = s.pool[ls + i]; break; }
                        if (shared < 0) continue;
                        const int sr = shared / C, scc = shared - sr * C;
                        const int os = s.ls[O], on = s.ll[O];
                        // three closest coords of O (stable sort by manhattan distance)
                        int16_t *pick = s.pick; int npk = 0;
                        {
                            int lastd = -1, lasti = -1;
                            for (int t = 0; t < 3 && t < on; t++) {
                                int bd = 1 << 30, bi = -1;
                                for (int i = 0; i < on; i++) {
                                    int v = s.pool[os + i];
                                    int d = abs(v / C - sr) + abs(v % C - scc);
                                    bool after = d > lastd || (d == lastd && i > lasti);
                                    if (after && d < bd) { bd = d; bi = i; }
                                }
                                pick[npk++] = s.pool[os + bi];
                                lastd = bd; lasti = bi;
                            }
                        }
                        int m = add_match(M_BOMB, col[s.pool[ls]]); if (m < 0) return;
                        for (int i = 0; i < ln; i++) match_push(m, s.pool[ls + i]);
                        for (int t = 0; t < npk; t++) {
                            bool inl = false;
                            for (int i = 0; i < ln; i++) if (s.pool[ls + i] == pick[t]) { inl = true; break; }
                            if (!inl) match_push(m, pick[t]);
                        }
                        if (on < 6) {                                               // lines.remove(l)
                            for (int j = h; j < qn - 1; j++) s.q[j] = s.q[j + 1];
                            qn--;
                        } else {                                                    // l.remove(c) in place
                            for (int t = 0; t < npk; t++) {
                                int n = s.ll[O];
                                for (int i = 0; i < n; i++)
                                    if (s.pool[os + i] == pick[t]) {
                                        for (int u = i; u < n - 1; u++) s.pool[os + u] = s.pool[os + u + 1];
                                        s.ll[O] = (int16_t)(n - 1);
                                        break;
                                    }
                            }
                        }
                        break;
                    }
                } else if (ln >= 3) {                                               // :322-325
                    int m = add_match(M_NORMAL, col[s.pool[ls]]); if (m < 0) return;
                    for (int i = 0; i < ln; i++) match_push(m, s.pool[ls + i]);
                }
            }
        }
    }

    // ---- activate_special, board.py:473-556, as an explicit DFS
    // frame kinds: 2 v-laser sweep, 3 h-laser sweep, 4 bomb 3x3, -1 cookie scan
    int sp;
    __device__ __forceinline__ void enter(int cell, int t, bool combo) {
        if (w.sc[SC_NZ] == 0) return;                        // :488-489 np.all(colour == 0)
        if (t == 0 || t == 1) { w.sc[SC_ERR] = 1; return; }  // :491-492
        clr(cell);                                           // :496
        if (!combo) w.sc[SC_NACT]++;                         // :498-499
        COVER_L0(t == -1 ? CV_SERIAL_COOKIE : CV_SERIAL_ACT);
        if (sp >= LS::MSTK) { ovf = true; return; }
        if (t == 2 || t == 3 || t == 4) {
            s.fcell[sp] = (int16_t)cell; s.ftype[sp] = (int8_t)t; s.fidx[sp] = 0; s.faux[sp] = 0; sp++;
        } else if (t == -1) {                                // :530-545
            int32_t *counts = s.counts;
            for (int i = 0; i < 16; i++) counts[i] = 0;
            int any = 0, big = 0;
            for (int p = 0; p < N; p++) {
                int v = col[p];
                if (v != 0) { any = 1; if (v > 0 && v < 16) counts[v]++; else big = 1; }
            }
            if (!any) return;
            if (big) { w.sc[SC_ERR] = 2; return; }
            int mcc = 0;
            for (int v = 1; v < 16; v++) if (counts[v] > counts[mcc]) mcc = v;
            for (int p = 0; p < N; p++) if (col[p] == mcc && typ[p] == 1) clr(p);
            s.fcell[sp] = (int16_t)cell; s.ftype[sp] = -1; s.fidx[sp] = 0; s.faux[sp] = (int8_t)mcc; sp++;
        } else {
            w.sc[SC_ERR] = 3;                                // :555-556
        }
    }
    __device__ __forceinline__ void run_dfs() {
        while (sp > 0 && !ovf && !w.sc[SC_ERR]) {
            const int f = sp - 1;
            const int t = s.ftype[f];
            const int cell = s.fcell[f];
            const int r = cell / C, c = cell - r * C;
            int idx = s.fidx[f];
            int target = -1;
            if (t == 2) {                                    // :502-507 column sweep
                if (idx >= R) { sp--; continue; }
                target = idx * C + c;
            } else if (t == 3) {                             // :510-515 row sweep
                if (idx >= C) { sp--; continue; }
                target = r * C + idx;
            } else if (t == 4) {                             // :517-528 clipped 3x3
                int r0 = r > 0 ? r - 1 : 0, r1 = r < R - 1 ? r + 1 : R - 1;
                int c0 = c > 0 ? c - 1 : 0, c1 = c < C - 1 ? c + 1 : C - 1;
                int wdt = c1 - c0 + 1;
                if (idx >= (r1 - r0 + 1) * wdt) { sp--; continue; }
                target = (r0 + idx / wdt) * C + c0 + idx % wdt;
            } else {                                         // :546-554 cookie: same-colour specials
                const int mcc = s.faux[f];
                while (idx < N && !(typ[idx] > 1 && col[idx] == mcc)) idx++;
                if (idx >= N) { sp--; continue; }
                s.fidx[f] = (int16_t)(idx + 1);
                enter(idx, typ[idx], false);
                continue;
            }
            s.fidx[f] = (int16_t)(idx + 1);
            int tt = typ[target];
            if (tt != 0 && tt != 1) enter(target, tt, false);
            else clr(target);
        }
    }
    __device__ __forceinline__ void activate(int cell, int t, bool combo) {
        sp = 0;
        enter(cell, t, combo);
        run_dfs();
    }

    // ---- get_special_creation_pos, board.py:429-458
    __device__ __forceinline__ int creation_pos(int m, const int16_t *taken, int nt, bool straight) {
        const int ms = s.ms[m], ml = s.mlen[m];
        int16_t *valid = s.valid; int nv = 0;
        for (int i = 0; i < ml; i++) {
            int v = s.mpool[ms + i]; bool tk = false;
            for (int j = 0; j < nt; j++) if (taken[j] == v) { tk = true; break; }
            if (!tk && nv < LS::MV) valid[nv++] = (int16_t)v;
        }
        if (!straight) {
            int br = -1, bc = -1, bnr = -1, bnc = -1;
            for (int i = 0; i < ml; i++) {
                int v = s.mpool[ms + i], r = v / C, c = v % C, nr = 0, nc = 0;
                for (int j = 0; j < ml; j++) { int u = s.mpool[ms + j]; nr += (u / C == r); nc += (u % C == c); }
                if (nr > bnr) { bnr = nr; br = r; }
                if (nc > bnc) { bnc = nc; bc = c; }
            }
            int corner = br * C + bc;
            for (int i = 0; i < nv; i++) if (valid[i] == corner) return corner;
            if (nv == 0) { w.sc[SC_ERR] = 4; return s.mpool[ms]; }
            int best = 0, bd = 1 << 30;
            for (int i = 0; i < nv; i++) {
                int dr = valid[i] / C - br, dc = valid[i] % C - bc, d = dr * dr + dc * dc;
                if (d < bd) { bd = d; best = i; }
            }
            return valid[best];
        }
        if (nv == 0) { w.sc[SC_ERR] = 4; return s.mpool[ms]; }
        for (int i = 1; i < nv; i++) {
            int16_t x = valid[i]; int j = i - 1;
            while (j >= 0 && valid[j] > x) { valid[j + 1] = valid[j]; j--; }
            valid[j + 1] = x;
        }
        return (nv % 2 == 0) ? valid[nv / 2 - 1] : valid[nv / 2];
    }

    // ---- resolve_colour_matches, board.py:397-427 (+ resolve_colour_match :460-471, create_special :572-597)
    __device__ __forceinline__ void resolve() {
        int16_t *taken = s.taken; int nt = 0;
        int16_t *qpos = s.qpos; int8_t *qname = s.qname, *qcol = s.qcol; int nq = 0;
        for (int m = 0; m < nm; m++) {
            if (s.mname[m] == M_NORMAL) continue;
            if (nq >= LS::MM) { ovf = true; return; }
            int pos = creation_pos(m, taken, nt, s.mname[m] != M_BOMB);
            bool dup = false;
            for (int j = 0; j < nt; j++) if (taken[j] == pos) dup = true;
            if (!dup) taken[nt++] = (int16_t)pos;
            qpos[nq] = (int16_t)pos; qname[nq] = s.mname[m]; qcol[nq] = s.mcol[m]; nq++;
        }
        for (int m = 0; m < nm && !ovf && !w.sc[SC_ERR]; m++) {
            const int ms = s.ms[m], ml = s.mlen[m];
            for (int i = 0; i < ml; i++) {
                int p = s.mpool[ms + i], t = typ[p];
                if (t != 0 && t != 1) activate(p, t, false);
                else clr(p);
            }
        }
        for (int i = 0; i < nq; i++) {
            w.sc[SC_NNEW]++;
            int p = qpos[i];
            if (col[p] == 0 && qcol[i] != 0) w.sc[SC_NZ]++;
            else if (col[p] != 0 && qcol[i] == 0) w.sc[SC_NZ]--;
            col[p] = (int8_t)qcol[i];
            const int nmq = qname[i];
            typ[p] = (int8_t)(nmq == M_VLASER ? 2 : nmq == M_HLASER ? 3 : nmq == M_BOMB ? 4 : nmq == M_COOKIE ? -1 : 0);
        }
    }

    // ---- combination_match, board.py:600-719
    __device__ __forceinline__ void combination(int p1, int p2) {
        w.sc[SC_NACT] += 2;                                                 // :609
        int t1 = typ[p1], k1 = col[p1], t2 = typ[p2], k2 = col[p2];
        int r1 = p1 / C, c1 = p1 % C, r2 = p2 / C, c2 = p2 % C;
        if (t1 == -1 && t2 == -1) {                                         // :615-616
            for (int p = 0; p < N; p++) { col[p] = 0; typ[p] = 0; }
            w.sc[SC_NZ] = 0;
        } else if ((t1 == -1 && t2 == 1) || (t1 == 1 && t2 == -1)) {        // :619-641
            if (t1 == 1) { int x = p1; p1 = p2; p2 = x; x = k1; k1 = k2; k2 = x; x = t1; t1 = t2; t2 = x; }
            clr(p1);
            for (int p = 0; p < N; p++) {                                   // colour_mask & normal_mask
                w.mark[p] = (col[p] == k2);
                if (w.mark[p] && typ[p] == 1) clr(p);
            }
            for (int p = 0; p < N; p++) w.mark[p] = w.mark[p] && typ[p] > 1;
            for (int p = 0; p < N && !ovf; p++) {                           // activate_specials_in_mask
                if (!w.mark[p]) continue;
                int t = typ[p];
                if (t != 0 && t != 1) activate(p, t, true);
            }
            for (int p = 0; p < N; p++) w.mark[p] = 0;
            w.sc[SC_NACT] -= 1;
        } else if ((t1 == -1 && t2 >= 2) || (t1 >= 2 && t2 == -1)) {        // :644-660
            if (t2 == -1) { int x = p1; p1 = p2; p2 = x; x = k1; k1 = k2; k2 = x; x = t1; t1 = t2; t2 = x; }
            clr(p1);
            for (int p = 0; p < N; p++) {
                w.mark[p] = (col[p] == k2);
                if (w.mark[p] && typ[p] == 1) typ[p] = (int8_t)t2;
            }
            for (int p = 0; p < N && !ovf; p++) {
                if (!w.mark[p]) continue;
                int t = typ[p];
                if (t != 0 && t != 1) activate(p, t, true);
            }
            for (int p = 0; p < N; p++) w.mark[p] = 0;
        } else if ((t1 == 2 || t1 == 3) && (t2 == 2 || t2 == 3)) {          // :663-674
            clr(p1); clr(p2);
            int r = r1 < r2 ? r1 : r2, c = c1 < c2 ? c1 : c2;
            activate(r * C + c, 2, true);
            activate(r * C + c, 3, true);
        } else if ((t1 == 4 && t2 >= 2 && t2 <= 3) || (t2 == 4 && t1 >= 2 && t1 <= 3)) {   // :677-696
            clr(p1); clr(p2);
            int r = r1 < r2 ? r1 : r2, c = c1 < c2 ? c1 : c2;
            int a0 = r > 0 ? r - 1 : 0, a1 = r < R - 1 ? r + 1 : R - 1;
            int b0 = c > 0 ? c - 1 : 0, b1 = c < C - 1 ? c + 1 : C - 1;
            for (int i = a0; i <= a1; i++) activate(i * C + c, 3, true);
            for (int j = b0; j <= b1; j++) activate(r * C + j, 2, true);
        } else if (t1 == 4 && t2 == 4) {                                    // :699-719
            clr(p1); clr(p2);
            int r = r1 < r2 ? r1 : r2, c = c1 < c2 ? c1 : c2;
            int a0 = r > 1 ? r - 2 : 0, a1 = r < R - 2 ? r + 2 : R - 1;
            int b0 = c > 1 ? c - 2 : 0, b1 = c < C - 2 ? c + 2 : C - 1;
            for (int i = a0; i <= a1; i++)
                for (int j = b0; j <= b1; j++) {
                    int p = i * C + j, t = typ[p];
                    if (t == 1) clr(p);
                    else if (t != 0) activate(p, t, true);
                }
        }
    }
};


#include "tmg_sb.hip"

// ------------------------------------------------------------------ move()
// Board.move, board.py:330-395 (the effectiveness test :352 is done by the
// caller).  Returns eliminations; leaves the effective mask of the final
// board in w.effw.
// clean: the board held no line before the swap (it came out of this file's
// ensure-playable loop), which bounds the first line search.
template <int MAXN, bool GEN, int SBNB, bool CODD, int TIER, class WS, class L>
__device__ __forceinline__ int board_move(const Params &P, WS &w, int lane, const LaneJump &J, Rng &g,
                          const Cells<MAXN / 64> &cl, int p1, int p2, int &flags, int &nn, int &na, int64_t e,
                          L *lists, bool clean) {
    // <= 128 cells: the per-lane cell coordinates are rebuilt where they are
    // used (a few VALU ops) rather than kept live across the cascade loop,
    // which spilled the 128-cell general kernels to scratch; 512 cells: eight
    // passes' worth, kept (rebuilding them there measured neutral at c5)
    const auto cells = [&]() {
        if constexpr (MAXN > 128) return cl;
        else return make_cells<MAXN / 64>(P, loop_lane(lane));
    };
    const int N = P.N;
    // Bound of the bottom-most line (detect's lim): after the swap of a
    // line-free board a line holds a swapped cell, so it is anchored at most two
    // rows below it; after a step that cleared only cells of rows <= rs (no
    // activation) the rows below rs are unchanged, so at most at rs + 2.
    int lim = P.R - 1;
    if (clean) lim = min(P.R - 1, div_c(P, max(p1, p2)) + 2);
    int8_t *col = w.brd, *typ = w.brd + N;
    int elim = 0;
    if (lane == 0) {                                                        // swap_coords :355
        int8_t x = col[p1]; col[p1] = col[p2]; col[p2] = x;
        x = typ[p1]; typ[p1] = typ[p2]; typ[p2] = x;
        w.sc[SC_NACT] = 0; w.sc[SC_NNEW] = 0; w.sc[SC_ERR] = 0; w.sc[SC_A] = 0;
    }
    WSYNC();
    const int t1 = typ[p1], t2 = typ[p2];
    bool ovf = false, err = false;
    if (((t1 != 0 && t1 != 1) && (t2 != 0 && t2 != 1)) || t1 < 0 || t2 < 0) {   // :357-364
        flags |= FL_COMBO;
        if constexpr (GEN) {
            COVER(CV_COMBO);
            int nz = count_colour_nonzero(P, w, lane);
            if (lane == 0) {
                w.sc[SC_NZ] = nz;
                Serial<MAXN, L> S(P, w, *lists);
                S.combination(p1, p2);
                w.sc[SC_A] = S.ovf;
            }
            WSYNC();
            ovf |= w.sc[SC_A] != 0;
            elim += count_type_zero(P, w, lane);
            gravity(P, w, lane);
            WSYNC();
            refill(P, w, lane, J, g);
            lim = P.R - 1;
        } else {
            err = true;                                                     // lean variant never sees specials
        }
    }
    // wave-parallel cascade only when no special can exist on the board
    bool fast = !GEN;
    if (GEN && P.smask == 0) {
        bool ok = true;
        for (int p = lane; p < N; p += 64) ok &= typ[p] == 1;
        fast = __ballot(!ok) == 0ULL;
    }
    // 512-cell general kernels (no bitboard path): wave-parallel steps while
    // the board stays plain (plain_board is kept by every cascade step)
    bool plain = false;
    if constexpr (GEN && SBNB == 0) plain = !fast && !ovf && !err && plain_board(P, w, lane);
    int iters = 0;
    (void)e;
    while (!ovf && !err) {                                                  // :367-376
        if (w.sc[SC_ERR]) break;
        if constexpr (GEN && SBNB > 0) {
            if (!fast) {                    // bitboard step when it provably creates / activates no special
                const int r = sb_simple_step<SBNB, CODD>(P, w, lane, J, g);
                if (r < 0) break;
                if (r > 0) { elim += r; iters++; lim = P.R - 1; continue; }
                COVER(CV_SB_FALLBACK);
            }
        }
        Det<MAXN / 64> d;
        const int rs = detect(P, w, lane, cells(), d, lim);
        if (rs < 0) break;
        lim = P.R - 1;
        if (fast) {
            COVER(CV_FAST);
            elim += fast_clear(P, w, lane, cells(), d, rs);      // clears rows <= rs only (a deeper run would be a lower line)
            lim = min(P.R - 1, rs + 2);
        } else {
            if constexpr (GEN && SBNB == 0) {
                uint64_t cols = 0;
                int rows = 0;
                const int r = plain ? simple_step_lds(P, w, lane, d, rs, cols, rows) : 0;
                if (r > 0) {
                    elim += r;
                    gravity(P, w, lane, cols);
                    WSYNC();
                    refill(P, w, lane, J, g, rows);
                    iters++;
                    lim = min(P.R - 1, rs + 2);
                    continue;
                }
                if (plain) COVER(CV_LDS_FALLBACK);
            }
            if constexpr (GEN) {
                int nz = count_colour_nonzero(P, w, lane);
                COVER(CV_SERIAL_STEP);
                if (lane == 0) {
                    w.sc[SC_NZ] = nz;
                    Serial<MAXN, L> S(P, w, *lists);
                    S.build_lines(rs);
                    if (!S.ovf) S.process_lines();
                    if (!S.ovf) S.resolve();
                    w.sc[SC_A] = S.ovf;
                }
                WSYNC();
                ovf |= w.sc[SC_A] != 0;
                elim += count_type_zero(P, w, lane);
            }
        }
        gravity(P, w, lane);
        WSYNC();
        refill(P, w, lane, J, g);
        iters++;
    }
    (void)iters;
    nn = w.sc[SC_NNEW];
    na = w.sc[SC_NACT];
    elim += nn;                                                             // :378
    if (ovf) flags |= FL_OVF;
    if (err || w.sc[SC_ERR]) flags |= FL_ERR;
    // the cascade loop ends only on a line-free board (or an error / overflow)
    flags |= ensure_playable(P, w, lane, J, g, cells(), !ovf && !err && !w.sc[SC_ERR]);   // :381-391
    return elim;
}

// ------------------------------------------------------------------ kernels
__device__ __forceinline__ LaneJump load_jump(const Params &P, int lane, const Rng &g) {
    const uint64_t *t = P.jump + lane * 4;
    LaneJump J;
    J.Aj = U128{t[0], t[1]};
    J.Gj = U128{t[2], t[3]};
    J.incG = mul128(U128{g.ilo, g.ihi}, J.Gj);
    return J;
}

__device__ __forceinline__ Rng load_rng(const uint64_t *p) {
    Rng g;
    g.slo = bcast64(p[0]); g.shi = bcast64(p[1]); g.ilo = bcast64(p[2]); g.ihi = bcast64(p[3]); g.h = bcast64(p[4]);
    return g;
}
__device__ __forceinline__ void store_rng(uint64_t *p, const Rng &g, int lane) {
    if (lane == 0) { p[0] = g.slo; p[1] = g.shi; p[2] = g.ilo; p[3] = g.ihi; p[4] = g.h; }
}

// TileMatchEnv.step for env e on one wave (tile_match_env.py:93-112).
// GEN=false: lean variant for boards that can hold no special (no specials
// enabled, cached effective mask trusted).  SBNB > 0 (<= 128 cells): the
// scalar-bitboard path of tmg_sb.hip with SBNB colour planes (the move in the
// lean variant, board generation in both); CODD = C is odd.  autoreset:
//   0  none: an ended env writes an all-zero mask, a further step is an error;
//   1  same step, inline: the env whose episode ends is regenerated here;
//   2  same step, deferred: a following reset_kernel launch masked by
//      FL_RESET regenerates it (the general and 512-cell kernels: the reset
//      kernel's occupancy is far higher than theirs);
//   3 / 4  next step (gymnasium's default), inline / deferred: an ending env
//      is left as with 0, and the call after it regenerates it instead of
//      stepping (its action ignored, reward 0, not terminated).
// Returns the ST_* bits this step raises for the sticky status word.
template <int MAXN, bool GEN, int SBNB, bool CODD, int TIER = TIER_MAIN, class WS = Ws<MAXN, GEN>,
          class L = WsSerial<MAXN>>
__device__ __forceinline__ uint32_t step_env(
    const Params &P, WS &w, int lane, int64_t e, int8_t *__restrict__ board, uint64_t *__restrict__ rng, int32_t *__restrict__ timer,
    const int32_t *__restrict__ actions, int32_t *__restrict__ reward, int32_t *__restrict__ n_new,
    int32_t *__restrict__ n_act, uint8_t *__restrict__ flags_out, uint64_t *__restrict__ eff, int trust_eff,
    int autoreset, L *lists) {
    const int N = P.N, W = P.W;
    // Only the 128-cell lean kernels regenerate a finished board inline
    // (autoreset 1 / 3); do_step (tmg_capi.hip) hands every other kernel
    // autoreset 2 / 4, a masked reset_kernel launch after the step, so they
    // carry no generate_board code
    constexpr bool INLINE_GEN = !GEN && MAXN == 128;
    const bool same = autoreset == 1 || autoreset == 2;
    const bool regen_inline = autoreset == 1 || autoreset == 3;
    // wave-uniform loads (the action too with the in-kernel policy, where the
    // draw below replaces it: no wait for the flag before the load goes out)
    int a = __builtin_amdgcn_readfirstlane(actions[e]);
    const int t0 = __builtin_amdgcn_readfirstlane(timer[e]);
    // Issued beside the two loads above, not depending on the action: the
    // env's cached mask row (lane i holds word i).  The ineffective-move exit
    // then waits for one memory latency instead of the chain action -> mask
    // word.  (The mask row is allocated memory whatever trust_eff says; it is
    // only read as a mask when trust_eff != 0.)  Loading the board and RNG
    // state there too measured slower: the quick waves wait for those loads.
    const uint64_t effrow = lane < W ? eff[e * W + lane] : 0ULL;
    TMG_KEEP_V(effrow);
    if (P.sample) {                                                         // the policy's action, from the mask
        a = __builtin_amdgcn_readfirstlane(sample_action(P, effrow, e, lane));
        if (lane == 0) const_cast<int32_t *>(actions)[e] = a;
    }
    // The common ineffective move (board.py:352-353; ~76 % of uniform moves at
    // c2): a live env, a trusted mask, not the episode's last move — only the
    // timer and the zero outputs are written.  Tested ahead of everything else
    // with as little wave-uniform logic as possible (the autoreset mode, the
    // board / mask addresses and the rare outputs stay in the general path
    // below), and the per-env arrays are addressed by the VALU (SGPR base +
    // an opaque 64-bit VGPR index, one v_lshl_add each) instead of a 64-bit
    // SALU add pair per array: the scalar unit is the c2 kernel's busiest pipe.
#ifndef TMG_QEXIT
#define TMG_QEXIT 1
#endif
    if (TMG_QEXIT && trust_eff && t0 < P.num_moves - 1 && (unsigned)a < (unsigned)P.A) {
        if (!((rdlane64(effrow, a >> 6) >> (a & 63)) & 1ULL)) {
            if (lane == 0) {
                uint64_t ve = (uint64_t)e;
                TMG_OPAQUE_V(ve);
                timer[ve] = t0 + 1;
                reward[ve] = 0; n_new[ve] = 0; n_act[ve] = 0;
                flags_out[ve] = (uint8_t)0;
                if (P.vo_term) reinterpret_cast<uint32_t *>(P.vo_term)[ve] = 0u;
                if (P.vo_left) P.vo_left[ve] = (int64_t)(P.num_moves - 1 - t0);
            }
            return 0;
        }
    }
    // an env that ended last call, with next-step autoreset: reset() now
    // (tested only inside the rare branch, so that the common path carries
    // no extra condition into the ineffective-move exit)
    bool pend = false;
    if (t0 >= P.num_moves || a < 0 || a >= P.A) {                           // tile_match_env.py:94-95
        pend = autoreset >= 3 && t0 >= P.num_moves;
    }
    if (!pend && (t0 >= P.num_moves || a < 0 || a >= P.A)) {
        if (lane == 0) {
            reward[e] = 0; n_new[e] = 0; n_act[e] = 0; flags_out[e] = FL_ERR;
            store_vo(P, e, FL_ERR, t0);
        }
        if ((P.oh || P.vo_obs) && !trust_eff) {   // the fused outputs follow every board of an untrusted call
            load_board(P, w, lane, board + e * 2 * N);
            WSYNC();
            if (P.oh) store_onehot(P, w, lane, e);
            if (P.vo_obs) store_obs(P, w, lane, e);
        }
        return ST_CALLER;
    }
    int8_t *gb = board + e * 2 * N;
    uint64_t *ge = eff + e * W;
    const int t1 = t0 + 1;
    const bool done = !pend && t1 == P.num_moves;                           // tile_match_env.py:100-101
    // envs regenerated in this call (here or by the reset launch after it)
    const bool regen = pend || (done && same);
    int flags = done ? FL_DONE : 0;
    bool effective = false;
    if (trust_eff && !pend) {                                               // board.py:352 via cached mask
        effective = (rdlane64(effrow, a >> 6) >> (a & 63)) & 1ULL;
    }
    if (trust_eff && !effective && !(regen && regen_inline)) {              // no state change at all
        const bool defer = regen;                                           // reset_kernel next
        if (done && !same) {                                                // tile_match_env.py:119-120
            for (int i = lane; i < W; i += 64) ge[i] = 0ULL;
            if (P.vo_mask) store_mask(P, w, lane, e, true);
        }
        if (done && same && P.vo_final) {                                   // the last board, as it stands
            // dwords only when every env's board starts on a dword ((2N) % 4 == 0,
            // as `bwhole` below); an odd N gives 2-byte-aligned boards: bytes
            const int nbw = ((2 * N) & 3) == 0 ? (2 * N) >> 2 : 0;
            const uint32_t *src = reinterpret_cast<const uint32_t *>(gb);
            uint32_t *dst = reinterpret_cast<uint32_t *>(P.vo_final + e * 2 * N);
            for (int i = lane; i < nbw; i += 64) dst[i] = src[i];
            for (int i = 4 * nbw + lane; i < 2 * N; i += 64) P.vo_final[e * 2 * N + i] = gb[i];
        }
        if (lane == 0) {
            const int tn = defer ? 0 : t1;
            timer[e] = tn; reward[e] = 0; n_new[e] = 0; n_act[e] = 0;
            flags_out[e] = (uint8_t)(flags | (defer ? FL_RESET : 0));
            store_vo(P, e, flags, tn);
        }
        return 0;
    }
    int r1, c1, r2, c2;
    action_coords(P.R, P.C, a, r1, c1, r2, c2);
    const int p1 = r1 * P.C + c1, p2 = r2 * P.C + c2;

    // The effective path's loads issued together, before anything waits on
    // one: the board (when whole dwords), the RNG state and this lane's
    // jump-table row.  One memory round trip instead of three dependent ones
    // (board -> LDS -> precondition -> RNG -> jump table).  (Issued with the
    // mask row instead when the in-kernel policy makes every move effective:
    // measured the same, c2 4.76 vs 4.75 x 10^8, and it cost the quick exit.)
    const int nbw = (2 * N) >> 2;
    const bool bwhole = ((2 * N) & 3) == 0 && nbw <= 64;
    const uint32_t bw = bwhole ? reinterpret_cast<const uint32_t *>(gb)[lane < nbw ? lane : 0] : 0u;
    const uint64_t *rp = rng + e * 5;
    const uint64_t q0 = rp[0], q1 = rp[1], q2 = rp[2], q3 = rp[3], q4 = rp[4];
    const uint64_t *jt = P.jump + lane * 4;
    const uint64_t j0 = jt[0], j1 = jt[1], j2 = jt[2], j3 = jt[3];
    if (bwhole) {
        if (lane < nbw) reinterpret_cast<uint32_t *>(w.brd)[lane] = bw;
    } else {
        load_board(P, w, lane, gb);
    }
    if constexpr (GEN) {
        for (int p = lane; p < N; p += 64) w.mark[p] = 0;
    }
    if constexpr (TIER == TIER_SPILL) COVER(CV_SPILL_RUN);
    WSYNC();
    if constexpr (!GEN) {                                                   // lean variant precondition
        bool ok = true;
        for (int p = lane; p < N; p += 64) ok &= w.brd[N + p] == 1;
        if (__ballot(!ok) != 0ULL) {
            if (lane == 0) {
                reward[e] = 0; n_new[e] = 0; n_act[e] = 0; flags_out[e] = FL_ERR;
                store_vo(P, e, FL_ERR, t0);
            }
            return ST_INTERNAL;
        }
    }
    if (!trust_eff && !pend) {
        bool ex = lane == 0 ? eff_exact(P, w.brd, a) : false;
        effective = __ballot(ex) != 0ULL;
    }
    Rng g;
    g.slo = bcast64(q0); g.shi = bcast64(q1); g.ilo = bcast64(q2); g.ihi = bcast64(q3); g.h = bcast64(q4);
    LaneJump J;
    J.Aj = U128{j0, j1};
    J.Gj = U128{j2, j3};
    J.incG = mul128(U128{g.ilo, g.ihi}, J.Gj);
    const Cells<MAXN / 64> cl = make_cells<MAXN / 64>(P, lane);
    int elim = 0, nn = 0, na = 0;
    bool changed = false;
    if (effective) {
        if constexpr (SBNB > 0 && !GEN) elim = sb_move<SBNB, CODD>(P, w, lane, J, g, cl, p1, p2, flags, e);
        else elim = board_move<MAXN, GEN, SBNB, CODD, TIER>(P, w, lane, J, g, cl, p1, p2, flags, nn, na, e, lists,
                                                             trust_eff != 0);
        changed = true;
        if constexpr (GEN) {
            if (flags & FL_OVF) {
                // the LDS lists ran out: nothing of this env has been written;
                // queue it for spill_kernel, which re-runs the whole step on
                // lists sized for the worst case (WsSerialBig).  The queue holds
                // every env of the launch and WsSerialBig cannot run out, so the
                // fall-through is unreachable; were it reached, the step is
                // flagged as an internal error, never written back as exact.
                if constexpr (TIER == TIER_MAIN) {
                    if (queue_env(P.spill, lane, e)) { COVER(CV_SPILL); return 0; }
                }
                flags = (flags & ~FL_OVF) | FL_ERR;
            }
        }
    }
    int tnew = t1;
    if (regen) {                                                            // reset() without a seed
        if (done && P.vo_final) store_board(P, w, lane, P.vo_final + e * 2 * N);   // same step: the last board
        if constexpr (INLINE_GEN) {
            if (regen_inline) {
                int fg = -1;
                if constexpr (SBNB > 0) {
                    if (P.C <= 32) fg = bp_generate<SBNB>(P, w, lane, g);
                    if (fg < 0) fg = sb_generate_exact<SBNB, CODD>(P, w, lane, J, g, cl);
                } else {
                    fg = generate_board(P, w, lane, J, g, cl);
                }
                flags |= fg;
                changed = true;
            }
        }                                      // autoreset 2 / 4: reset_kernel regenerates FL_RESET envs next
        tnew = 0;
        flags |= FL_RESET;
    }
    if (changed) {
        store_board(P, w, lane, gb);
        store_rng(rng + e * 5, g, lane);
    }
    // fused one-hot planes: every board this step changed (or, with an
    // untrusted mask, any board: it may have been edited by hand)
    if (P.oh && (changed || !trust_eff)) store_onehot(P, w, lane, e);
    if (P.vo_obs && (changed || !trust_eff)) store_obs(P, w, lane, e);
    if (done && !same) {
        for (int i = lane; i < W; i += 64) ge[i] = 0ULL;                   // tile_match_env.py:119-120
        if (P.vo_mask) store_mask(P, w, lane, e, true);
    } else if (changed) {
        for (int i = lane; i < W; i += 64) ge[i] = w.effw[i];
        if (P.vo_mask) store_mask(P, w, lane, e, false);
    } else if (!trust_eff) {
        scan_effective(P, w, lane, cl, false);
        WSYNC();
        for (int i = lane; i < W; i += 64) ge[i] = w.effw[i];
        if (P.vo_mask) store_mask(P, w, lane, e, false);
    }
    if (lane == 0) {
        timer[e] = tnew;
        reward[e] = elim;
        n_new[e] = nn;
        n_act[e] = na;
        flags_out[e] = (uint8_t)flags;
        store_vo(P, e, flags, tnew);
    }
    return ((flags & FL_ERR) ? ST_INTERNAL : 0u) | ((flags & FL_OVF) ? ST_OVERFLOW : 0u);
}

// TileMatchEnv.step over a batch, one wave per env.
// Shape-specialised kernels: for the benchmark shapes the launcher picks an
// instantiation that tells the compiler the board geometry (R, C, k and what
// follows from them), so every cell offset, division by C, loop bound and
// bitboard mask folds to a constant.  The values are asserted to the compiler
// only; Params still holds them (the host picks the kernel by comparing).
#if defined(__clang__)
#define TMG_ASSUME(x) __builtin_assume(x)
#else
#define TMG_ASSUME(x) do { if (!(x)) __builtin_unreachable(); } while (0)   // the host wave emulator (g++)
#endif
// A fixed shape is encoded as one int, R << 24 | C << 16 | k << 8 | specials
// mask (0: the generic kernel; specials 255: any, for the reset kernels).
constexpr int shape_fix(int R, int C, int k, int smask) { return (R << 24) | (C << 16) | (k << 8) | smask; }
constexpr int kNoFix = 0;
constexpr int kFixAnySpecials = 255;
constexpr int kFixC2 = shape_fix(10, 10, 4, 0);                           // BASELINE configs[1] / [3]
constexpr int kFixC3 = shape_fix(10, 10, 4, SP_VLASER | SP_HLASER | SP_BOMB);   // configs[2]
constexpr int kFixC5 = shape_fix(20, 20, 6, SP_COOKIE | SP_VLASER | SP_HLASER | SP_BOMB);   // configs[4]
constexpr int kFixReset10 = shape_fix(10, 10, 4, kFixAnySpecials);
constexpr int kFixReset20 = shape_fix(20, 20, 6, kFixAnySpecials);
__host__ __device__ constexpr uint64_t fix_mask(int R, int C, int w, int what) {   // make_params' sb_* masks
    uint64_t m = 0;
    for (int p = 0; p < R * C && p < 128; p++) {
        const int c = p % C;
        if ((p & 1) != w) continue;
        const bool on = what == 0 ? true : what == 1 ? p >= C : what == 2 ? p >= 2 * C : what == 3 ? c <= C - 2
                      : what == 4 ? c >= 1 : c <= C - 3;
        if (on) m |= 1ULL << (p >> 1);
    }
    return m;
}
template <int FIX>
__device__ __forceinline__ void assume_shape(const Params &P) {
    if constexpr (FIX != kNoFix) {
        constexpr struct { int R, C, K, smask; } F{FIX >> 24, (FIX >> 16) & 255, (FIX >> 8) & 255, FIX & 255};
        TMG_ASSUME(P.R == F.R);
        TMG_ASSUME(P.C == F.C);
        TMG_ASSUME(P.N == F.R * F.C);
        TMG_ASSUME(P.A == 2 * F.R * F.C - F.R - F.C);
        TMG_ASSUME(P.W == (2 * F.R * F.C - F.R - F.C + 63) / 64);
        TMG_ASSUME(P.k == F.K);
        if constexpr (F.smask != kFixAnySpecials) TMG_ASSUME(P.smask == F.smask);
        TMG_ASSUME(P.thr == (F.K > 1 ? (0xffffffffu - (uint32_t)(F.K - 1)) % (uint32_t)F.K : 0u));
        TMG_ASSUME(P.cmag == ((1u << 20) + (uint32_t)F.C - 1) / (uint32_t)F.C);
        TMG_ASSUME(P.cm1mag == ((1u << 20) + (uint32_t)F.C - 2) / (uint32_t)(F.C - 1));
        if constexpr (F.R * F.C <= 128) {
#define TMG_ASSUME_MASK(field, what)                                          \
    {                                                                         \
        constexpr uint64_t m0 = fix_mask(F.R, F.C, 0, what), m1 = fix_mask(F.R, F.C, 1, what); \
        TMG_ASSUME(P.field[0] == m0);                                   \
        TMG_ASSUME(P.field[1] == m1);                                   \
    }
            TMG_ASSUME_MASK(sb_in, 0)
            TMG_ASSUME_MASK(sb_u, 1)
            TMG_ASSUME_MASK(sb_v, 2)
            TMG_ASSUME_MASK(sb_nl, 3)
            TMG_ASSUME_MASK(sb_nf, 4)
            TMG_ASSUME_MASK(sb_h, 5)
#undef TMG_ASSUME_MASK
        }
    }
}

template <int MAXN, bool GEN, int SBNB = 0, bool CODD = false, int FIX = kNoFix>
__global__ __launch_bounds__(64, MAXN == 128 ? (GEN ? kGen128Waves : (FIX != kNoFix ? kLean128Waves : kLean128GenericWaves))
                                            : (FIX == kFixC5 ? kC5StepWaves : 1)) void step_kernel(
    Params P_, int64_t n, int8_t *__restrict__ board, uint64_t *__restrict__ rng, int32_t *__restrict__ timer,
    const int32_t *__restrict__ actions, int32_t *__restrict__ reward, int32_t *__restrict__ n_new,
    int32_t *__restrict__ n_act, uint8_t *__restrict__ flags_out, uint64_t *__restrict__ eff, int trust_eff,
    int autoreset) {
    TMG_SMEM_DECL(smem);
    using WS = Ws<MAXN, GEN>;
    const Params &P = TMG_KERNARG_PARAMS(P_);
    assume_shape<FIX>(P);
    const int lane = threadIdx.x & 63;
    WS &w = *reinterpret_cast<WS *>(smem);
    const int64_t e = wg_env();
    if (e >= n) return;
    WsSerial<MAXN> *lists = nullptr;
    if constexpr (GEN) lists = &w.s;
    const uint32_t st = step_env<MAXN, GEN, SBNB, CODD, TIER_MAIN, WS, WsSerial<MAXN>>(
        P, w, lane, e, board, rng, timer, actions, reward, n_new, n_act, flags_out, eff, trust_eff, autoreset, lists);
    note_status(P, lane, st);
}

// Re-runs the steps the general step kernel queued on running out of LDS list
// space (step_env, FL_OVF), on global-memory lists sized for the worst case
// (WsSerialBig): launched right after every general step launch on the same
// stream with the same buffers, kSpillWaves one-wave workgroups, each
// with its own WsSerialBig.  An empty queue costs one load per wave.  The
// generic (non-bitboard) path: bit-identical results by construction.
// Small footprint on purpose (no LDS lists, at most 8 waves/SIMD's worth of
// VGPRs, spilling to scratch instead): the launch follows every
// general step on its stream and must find room on a chip busy with the
// other streams' kernels at once, or it holds its stream back; the rare
// steps it re-runs may go slowly.
template <int MAXN>
__global__ __launch_bounds__(64, 8) void spill_kernel(
    Params P, int64_t n, int8_t *__restrict__ board, uint64_t *__restrict__ rng, int32_t *__restrict__ timer,
    const int32_t *__restrict__ actions, int32_t *__restrict__ reward, int32_t *__restrict__ n_new,
    int32_t *__restrict__ n_act, uint8_t *__restrict__ flags_out, uint64_t *__restrict__ eff, int trust_eff,
    int autoreset) {
    TMG_SMEM_DECL(smem);
    using WS = Ws<MAXN, false>;                   // the lists are global (WsSerialBig)
    const int lane = threadIdx.x & 63;
    WS &w = *reinterpret_cast<WS *>(smem);
    SpillQ *q = P.spill;
    WsSerialBig<MAXN> *lists = reinterpret_cast<WsSerialBig<MAXN> *>(P.spill_ws) + blockIdx.x;
    const int64_t queued = (int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)q->count);
    const int cnt = (int)(queued < q->cap ? queued : q->cap);
    int done = 0;
    for (int i = (int)blockIdx.x; i < cnt; i += (int)gridDim.x) {
        const int64_t e = (int64_t)bcast64((uint64_t)q->env[i]);
        if (e < 0 || e >= n) continue;
        WSYNC();
        const uint32_t st = step_env<MAXN, true, 0, false, TIER_SPILL, WS, WsSerialBig<MAXN>>(
            P, w, lane, e, board, rng, timer, actions, reward, n_new, n_act, flags_out, eff, trust_eff, autoreset, lists);
        note_status(P, lane, st);
        done++;
    }
    if (lane == 0) {
        if (done) atomicAdd(&q->total, (unsigned long long)done);
        __threadfence();
        if (atomicAdd(&q->done, 1u) == gridDim.x - 1) { q->count = 0u; q->done = 0u; }   // the last wave empties the queue
    }
}

// TileMatchEnv.reset without a seed (tile_match_env.py:84-91) of env e
template <int MAXN, int SBNB, bool CODD, class WS>
__device__ __forceinline__ void reset_env(const Params &P, WS &w, int lane, int64_t e, int8_t *__restrict__ board,
                                          uint64_t *__restrict__ rng, int32_t *__restrict__ timer,
                                          uint64_t *__restrict__ eff) {
    const int N = P.N, W = P.W;
    Rng g = load_rng(rng + e * 5);
    const Cells<MAXN / 64> cl = make_cells<MAXN / 64>(P, lane);
    // board.py:95-109: on row bit-planes (C <= 32); a Lemire rejection or a
    // wider board takes the exact draw-by-draw path
    int fl = -1;
    if constexpr (SBNB > 0) {
        if (P.C <= 32) fl = bp_generate<SBNB, (MAXN > 128)>(P, w, lane, g);
    }
    if (fl < 0) {
        const LaneJump J = load_jump(P, lane, g);
        if constexpr (MAXN == 128 && SBNB > 0) fl = sb_generate_exact<SBNB, CODD>(P, w, lane, J, g, cl);
        else fl = generate_board(P, w, lane, J, g, cl);
    }
    note_status(P, lane, fl ? ST_INTERNAL : 0u);
    store_board(P, w, lane, board + e * 2 * N);
    store_rng(rng + e * 5, g, lane);
    if (P.oh) store_onehot(P, w, lane, e);
    if (P.vo_obs) store_obs(P, w, lane, e);
    for (int i = lane; i < W; i += 64) eff[e * W + i] = w.effw[i];
    if (P.vo_mask) store_mask(P, w, lane, e, false);
    if (lane == 0) {
        timer[e] = 0;
        if (P.vo_left) P.vo_left[e] = P.num_moves;
    }
}

template <int MAXN, int SBNB = 0, bool CODD = false, int FIX = kNoFix>
__global__ __launch_bounds__(64, MAXN > 128 ? kReset512Waves : (FIX != kNoFix ? kReset128Waves : 1)) void reset_kernel(Params P_, int64_t n, int8_t *__restrict__ board,
                                                             uint64_t *__restrict__ rng, int32_t *__restrict__ timer,
                                                             uint64_t *__restrict__ eff,
                                                             const uint8_t *__restrict__ env_mask, int mask_bits,
                                                             int epw) {
    TMG_SMEM_DECL(smem);
    using WS = Ws<MAXN, false>;
    const Params &P = TMG_KERNARG_PARAMS(P_);
    assume_shape<FIX>(P);
    const int lane = threadIdx.x & 63;
    WS &w = *reinterpret_cast<WS *>(smem);
    // epw consecutive envs per wave (1 for a full reset; a masked reset, where
    // most launches find nothing to do, dispatches epw times fewer waves and
    // regenerates the envs it finds one after another)
    const int64_t e0 = wg_env() * epw;
    if (e0 >= n) return;
    const int64_t el = e0 + lane;
    uint64_t todo = __ballot(lane < epw && el < n && (!env_mask || (env_mask[el] & mask_bits)));
    while (todo) {
        const int k = __builtin_ctzll(todo);
        todo &= todo - 1;
        reset_env<MAXN, SBNB, CODD>(P, w, loop_lane(lane), e0 + k, board, rng, timer, eff);
        WSYNC();                                                         // the next board reuses the workspace
    }
}

// TileMatchEnv._get_effective_actions for arbitrary boards (tile_match_env.py:118-124)
template <int MAXN>
__global__ __launch_bounds__(64) void effective_kernel(Params P, int64_t n, const int8_t *__restrict__ board,
                                                                 uint64_t *__restrict__ eff) {
    TMG_SMEM_DECL(smem);
    using WS = Ws<MAXN, false>;
    const int lane = threadIdx.x & 63;
    WS &w = *reinterpret_cast<WS *>(smem);
    const int64_t e = wg_env();
    if (e >= n) return;
    load_board(P, w, lane, board + e * 2 * P.N);
    WSYNC();
    const Cells<MAXN / 64> cl = make_cells<MAXN / 64>(P, lane);
    scan_effective(P, w, lane, cl, false);
    WSYNC();
    for (int i = lane; i < P.W; i += 64) eff[e * P.W + i] = w.effw[i];
}

}  // namespace tmg
