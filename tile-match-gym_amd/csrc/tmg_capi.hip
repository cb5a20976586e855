// tmg_capi.hip — extern "C" entry points of libtmg.so (declared in include/tmg.h).
// Host code only: the kernels and their launchers live in tmg_kernels.hip
// (one translation unit per kernel group, tmg_launch.h).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "tmg.h"
#include "tmg_board.hip"
#include "tmg_launch.h"

#ifndef TMG_SRC_SHA
#define TMG_SRC_SHA "unknown"
#endif
#ifndef TMG_VARIANT
#define TMG_VARIANT "product"
#endif

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

int hip_check(hipError_t e, const char *what) {
    if (e != hipSuccess) return fail(-5, std::string(what) + ": " + hipGetErrorString(e));
    return 0;
}

}  // namespace

struct tmg_ctx {
    int device;
    tmg::Params P;
    uint64_t *d_jump;
    uint64_t *d_sbrows;
    uint32_t *d_status;  // sticky status words (tmg_status): one per TMG_STATUS_* bit
    unsigned long long *d_cover;   // TMG_COVER builds only
    int maxn;
    int sb;              // scalar-bitboard kernels (<= 128 cells, C <= 63)
    int scan_only;       // tmg_create_scan: tmg_effective only
    // spill queue of the general kernels, one per stream the context steps on
    // (a queue is only ever touched by the launches of its own stream, in
    // order), holding at least as many entries as the largest launch on it
    struct Spill {
        hipStream_t stream;
        tmg::SpillQ *q;
        int64_t cap;
        void *ws;
    };
    std::vector<Spill> spills;
    std::mutex mu;       // guards `spills` (calls on different streams may come from several threads)
};

using tmg::Params;
using tmg::StepArgs;

namespace tmg {
dim3 env_grid(int64_t n) {
    return dim3((unsigned)((n + 7) & ~(int64_t)7));   // one wave per env, 8 equal XCD blocks (wg_env)
}
size_t spill_ws_bytes(int maxn) {
    return maxn <= 128 ? sizeof(WsSerialBig<128>) : sizeof(WsSerialBig<512>);
}
}  // namespace tmg

// A queue of cap entries with its running total, written on s.
static int new_queue(hipStream_t s, int64_t cap, unsigned long long total, tmg::SpillQ **out) {
    const size_t bytes = sizeof(tmg::SpillQ) + (size_t)cap * sizeof(int64_t);
    int rc = hip_check(hipMalloc(out, bytes), "hipMalloc");
    if (rc) return rc;
    tmg::SpillQ h{};
    h.total = total;
    h.cap = cap;
    // written in order on s itself (a copy on the null stream is not ordered
    // with respect to a non-blocking stream's launches)
    rc = hip_check(hipMemcpyAsync(*out, &h, offsetof(tmg::SpillQ, env), hipMemcpyHostToDevice, s), "hipMemcpyAsync");
    if (!rc) rc = hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");   // h leaves scope
    return rc;
}

// The stream's spill queue, holding at least n entries (zeroed on s).
// Growing waits for s first: the old queue may still be read by a queued
// launch.
static int spill_for(tmg_ctx *ctx, hipStream_t s, int64_t n, tmg::SpillQ **q, void **ws) {
    std::lock_guard<std::mutex> lock(ctx->mu);
    tmg_ctx::Spill *sp = nullptr;
    for (auto &x : ctx->spills)
        if (x.stream == s) sp = &x;
    if (!sp) {
        ctx->spills.push_back(tmg_ctx::Spill{s, nullptr, 0, nullptr});
        sp = &ctx->spills.back();
        int rc = hip_check(hipMalloc(&sp->ws, tmg::spill_ws_bytes(ctx->maxn) * tmg::kSpillWaves), "hipMalloc");
        if (rc) { ctx->spills.pop_back(); return rc; }
    }
    if (sp->cap < n) {
        int rc = 0;
        unsigned long long total = 0;
        if (sp->q) {
            rc = hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
            if (!rc) rc = hip_check(hipMemcpy(&total, &sp->q->total, sizeof total, hipMemcpyDeviceToHost), "hipMemcpy");
            (void)hipFree(sp->q);
            sp->q = nullptr;
            sp->cap = 0;
        }
        const int64_t cap = n < 64 ? 64 : n;
        if (!rc) rc = new_queue(s, cap, total, &sp->q);
        if (rc) return rc;
        sp->cap = cap;
    }
    *q = sp->q;
    *ws = sp->ws;
    return 0;
}

static int set_device(tmg_ctx *ctx) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev != ctx->device) return hip_check(hipSetDevice(ctx->device), "hipSetDevice");
    return 0;
}

static int do_reset(tmg_ctx *ctx, const Params &P, int64_t n, int8_t *board, uint64_t *rng, int32_t *timer,
                    uint64_t *eff, const uint8_t *env_mask, int mask_bits, hipStream_t s, int epw_masked = 0) {
    // a masked reset (the deferred autoreset after every general step; most
    // find no finished env) takes several envs per wave
    const int epw = !env_mask ? 1 : epw_masked ? epw_masked
                  : ctx->maxn == 128 ? tmg::kMaskedResetEnvs128 : tmg::kMaskedResetEnvs512;
    const dim3 grid = tmg::env_grid((n + epw - 1) / epw);
    if (ctx->maxn == 128) tmg::launch_reset128(ctx->sb, grid, s, P, n, board, rng, timer, eff, env_mask, mask_bits, epw);
    else tmg::launch_reset512(grid, s, P, n, board, rng, timer, eff, env_mask, mask_bits, epw);
    return hip_check(hipGetLastError(), "kernel launch");
}

// a.autoreset: 0 none, 1 same step, 2 next step (tmg_plan_config); the
// kernels' codes are 1 / 3 inline and 2 / 4 deferred (step_env)
static int do_step(tmg_ctx *ctx, Params P, StepArgs a, hipStream_t s) {
    // lean kernels: no special can exist (none enabled) and the cached mask
    // came from this library's own step / reset of the current boards
    const bool lean = ctx->P.smask == 0 && a.trust_eff;
    const dim3 grid = tmg::env_grid(a.n);
    const int mode = a.autoreset;
    // the lane-per-board kernel (tmg_lane.h) takes the lean steps of the
    // shapes it is built for, unless a fused output (one-hot, vector-env
    // outputs) is asked for, when its lanes are busy: the in-kernel policy
    // (every move effective) or a launch of >= kLaneMinEnvs envs.  With given
    // actions on smaller launches the wave-per-board kernels are faster (a
    // lane's wave runs as long as its longest cascade, and at c2's 65 536
    // envs there is one such wave per SIMD: DESIGN.md §7.7)
#ifndef TMG_LANE
#define TMG_LANE 1
#endif
#ifndef TMG_LANE_MIN_ENVS
#define TMG_LANE_MIN_ENVS 131072
#endif
    const bool lanek = TMG_LANE && lean && ctx->maxn == 128 && tmg::lane_shape(P) && !P.oh && !P.vo_term &&
                       !P.vo_mask && !P.vo_left && !P.vo_final && !P.vo_obs &&
                       (P.sample || a.n >= TMG_LANE_MIN_ENVS);
    // the general and 512-cell kernels (and the lane kernel) leave finished
    // boards to a reset launch masked by FL_RESET, which runs at several
    // times their occupancy
    const int deferred = mode && (ctx->maxn == 512 || !lean || lanek);
    if (!lean) {
        int rc = spill_for(ctx, s, a.n, &P.spill, &P.spill_ws);
        if (rc) return rc;
    }
    a.autoreset = mode == 0 ? 0 : mode == 1 ? (deferred ? 2 : 1) : (deferred ? 4 : 3);
    if (lanek) {
        tmg::launch_step_lane(s, P, a);
    } else if (ctx->maxn == 128) {
        if (lean) tmg::launch_step_lean128(ctx->sb, grid, s, P, a);
        else if (ctx->sb && (P.C & 1)) tmg::launch_step_gen128_odd(grid, s, P, a);
        else tmg::launch_step_gen128_even(ctx->sb, grid, s, P, a);
    } else {
        tmg::launch_step512(!lean, grid, s, P, a);
    }
    int rc = hip_check(hipGetLastError(), "kernel launch");
    if (rc) return rc;
    if (!lean) {                                   // re-run the steps that ran out of LDS list space
        if (ctx->maxn == 128) tmg::launch_spill128(s, P, a);
        else tmg::launch_spill512(s, P, a);
        rc = hip_check(hipGetLastError(), "kernel launch");
        if (rc) return rc;
    }
    if (!deferred) return 0;
    // after a lane step the masked reset takes 2 envs per wave, not 8: the
    // block storms (a whole env group's regeneration) dominate its time there
    // (c2-eff 5.45 vs 5.19, c4-eff 9.9 vs 9.45 x 10^8 on one box; 1 / 4 in
    // between, profiles/r06/s13/)
#ifndef TMG_LANE_RESET_EPW
#define TMG_LANE_RESET_EPW 2
#endif
    return do_reset(ctx, P, a.n, a.board, a.rng, a.timer, a.eff, a.flags, tmg::FL_RESET, s,
                    lanek ? TMG_LANE_RESET_EPW : 0);
}

static int check_call(tmg_ctx *ctx, int64_t n) {
    if (!ctx) return fail(-1, "null context");
    if (n < 0) return fail(-2, "negative batch size");
    return set_device(ctx);
}

static int check_full(tmg_ctx *ctx, int64_t n) {
    int rc = check_call(ctx, n);
    if (!rc && ctx->scan_only) return fail(-2, "context made by tmg_create_scan: tmg_effective only");
    return rc;
}

// ---------------------------------------------------------------- viability
// The reference's generate_board / move loop "while not possible_move() or
// lines" (board.py:102-109, 381-391) never ends on a shape where no board is
// both line-free and playable (e.g. 2x2, or one colour); on the device that
// would be a wave that never retires.  tmg_create therefore asks for one such
// board first.  All-normal boards: a line is 3 equal colours in a row or
// column (board.py:158-193), an effective move a swap that makes one
// (is_move_effective, board.py:735-787).
namespace {

bool has_line(const int *b, int R, int C) {
    for (int r = 0; r < R; r++)
        for (int c = 0; c < C; c++) {
            const int x = b[r * C + c];
            if (c + 2 < C && b[r * C + c + 1] == x && b[r * C + c + 2] == x) return true;
            if (r + 2 < R && b[(r + 1) * C + c] == x && b[(r + 2) * C + c] == x) return true;
        }
    return false;
}

bool playable(int *b, int R, int C) {                 // possible_move on a line-free board
    for (int a = 0; a < 2 * R * C - R - C; a++) {
        int r1, c1, r2, c2;
        tmg::action_coords(R, C, a, r1, c1, r2, c2);
        const int p = r1 * C + c1, q = r2 * C + c2;
        if (b[p] == b[q]) continue;
        std::swap(b[p], b[q]);
        const bool l = has_line(b, R, C);
        std::swap(b[p], b[q]);
        if (l) return true;
    }
    return false;
}

// Whether some R x C board with colours < k is line-free and playable:
// exhaustively when there are at most 2^21 colourings, else by a randomised
// depth-first search over line-free row-major fillings (a cell takes a colour
// that completes no triple with the two cells left of / above it; a dead end
// backtracks instead of restarting, so 2-colour boards, where a cell can have
// both colours forbidden, are found too), testing each complete filling for a
// playable swap.
bool shape_viable(int R, int C, int k) {
    if (k < 2 || (R < 3 && C < 3)) return false;
    const int N = R * C;
    std::vector<int> b(N, 0);
    double total = 1.0;
    for (int i = 0; i < N; i++) total *= k;
    if (total <= (double)(1 << 21)) {
        for (;;) {
            if (!has_line(b.data(), R, C) && playable(b.data(), R, C)) return true;
            int i = N - 1;                            // odometer
            while (i >= 0 && ++b[i] == k) b[i--] = 0;
            if (i < 0) return false;
        }
    }
    uint64_t x = 0x9E3779B97F4A7C15ULL;
    auto rnd = [&x]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
    const int kk = k < 16 ? k : 16;
    std::vector<int> order(N * 16), next(N, 0);       // per cell: a random colour order, the next one to try
    long budget = 1L << 22;                            // cell assignments over the whole search
    for (int restart = 0; restart < 64 && budget > 0; restart++) {
        int p = 0, complete = 0;
        next[0] = 0;
        for (int v = 0; v < kk; v++) order[v] = v;
        for (int v = kk - 1; v > 0; v--) std::swap(order[v], order[rnd() % (v + 1)]);
        while (p >= 0 && budget-- > 0) {
            if (p == N) {
                if (playable(b.data(), R, C)) return true;
                // backtracking only varies the last cells: after many line-free
                // boards with no playable swap, try another random order
                if (++complete > 4096) break;
                p--;
                continue;
            }
            const int r = p / C, c = p - r * C;
            bool placed = false;
            while (next[p] < kk) {
                const int v = order[p * 16 + next[p]++];
                if (c >= 2 && b[p - 1] == v && b[p - 2] == v) continue;
                if (r >= 2 && b[p - C] == v && b[p - 2 * C] == v) continue;
                b[p] = v;
                placed = true;
                break;
            }
            if (!placed) { p--; continue; }              // dead end: backtrack
            if (++p < N) {
                next[p] = 0;
                for (int v = 0; v < kk; v++) order[p * 16 + v] = v;
                for (int v = kk - 1; v > 0; v--) std::swap(order[p * 16 + v], order[p * 16 + rnd() % (v + 1)]);
            }
        }
        // backtracked past the first cell: every line-free board was tried
        // (none playable), so the shape is not viable; only a search cut off
        // by the 4096-board cap restarts with another colour order
        if (p < 0 && complete <= 4096) return false;
    }
    return false;
}

int alloc_tables(tmg_ctx *c) {
    Params &P = c->P;
    uint64_t tab[tmg::kJumpRows * 4];
    tmg::build_jump_table(tab);
    int rc = hip_check(hipMalloc(&c->d_jump, sizeof tab), "hipMalloc");
    if (!rc) rc = hip_check(hipMemcpy(c->d_jump, tab, sizeof tab, hipMemcpyHostToDevice), "hipMemcpy");
    if (!rc) rc = hip_check(hipMalloc(&c->d_status, 16), "hipMalloc");
    if (!rc) rc = hip_check(hipMemset(c->d_status, 0, 16), "hipMemset");
    if (!rc && P.N <= 128) {
        uint64_t rows[64 * 4];
        tmg::build_sb_rows(P.R, P.C, rows);
        rc = hip_check(hipMalloc(&c->d_sbrows, sizeof rows), "hipMalloc");
        if (!rc) rc = hip_check(hipMemcpy(c->d_sbrows, rows, sizeof rows, hipMemcpyHostToDevice), "hipMemcpy");
    }
#if TMG_COVER
    if (!rc) rc = hip_check(hipMalloc(&c->d_cover, tmg::CV_COUNT * sizeof(unsigned long long)), "hipMalloc");
    if (!rc) rc = hip_check(hipMemset(c->d_cover, 0, tmg::CV_COUNT * sizeof(unsigned long long)), "hipMemset");
#endif
    if (!rc) rc = hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    P.jump = c->d_jump;
    P.status = c->d_status;
    P.sb_rows = c->d_sbrows;
    P.cover = c->d_cover;
    return rc;
}

void free_ctx(tmg_ctx *c) {
    if (c->d_jump) (void)hipFree(c->d_jump);
    if (c->d_status) (void)hipFree(c->d_status);
    if (c->d_sbrows) (void)hipFree(c->d_sbrows);
    if (c->d_cover) (void)hipFree(c->d_cover);
    for (const auto &x : c->spills) {
        if (x.q) (void)hipFree(x.q);
        if (x.ws) (void)hipFree(x.ws);
    }
    delete c;
}

int new_ctx(tmg_ctx **out, int device, int rows, int cols, int colours, uint32_t specials_mask, int num_moves,
            int scan_only) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(-3, "no HIP device available");
    if (device < 0 || device >= ndev) return fail(-3, "bad device index");
    int rc = hip_check(hipSetDevice(device), "hipSetDevice");
    if (rc) return rc;
    tmg_ctx *c = new tmg_ctx();
    c->device = device;
    c->d_jump = nullptr; c->d_sbrows = nullptr; c->d_status = nullptr; c->d_cover = nullptr;
    c->P = tmg::make_params(rows, cols, colours, (int)specials_mask, num_moves, nullptr);
    c->maxn = c->P.N <= 128 ? 128 : 512;
    c->sb = c->P.N <= 128 && c->P.C <= 63;
    c->scan_only = scan_only;
    rc = alloc_tables(c);
    if (rc) { free_ctx(c); return rc; }
    *out = c;
    return 0;
}

}  // namespace

extern "C" {

int tmg_create(tmg_ctx **out, int device, int rows, int cols, int colours, uint32_t specials_mask, int num_moves) {
    if (!out) return fail(-1, "null output pointer");
    *out = nullptr;
    if (rows < 1 || cols < 1) return fail(-2, "board must be at least 1x1");
    if (rows > 64 || cols > 64 || rows * cols > 512) return fail(-2, "board too large (R,C <= 64, R*C <= 512)");
    if (colours < 1 || colours > 15) return fail(-2, "num_colours must be in [1, 15]");
    if (specials_mask > 15u) return fail(-2, "bad specials mask");
    if (num_moves < 1) return fail(-2, "num_moves must be >= 1");
    if (!shape_viable(rows, cols, colours))
        return fail(-2, "no playable board exists for this shape and colour count (the reference's "
                        "generate_board would loop forever, board.py:102-109)");
    return new_ctx(out, device, rows, cols, colours, specials_mask, num_moves, 0);
}

int tmg_create_scan(tmg_ctx **out, int device, int rows, int cols) {
    if (!out) return fail(-1, "null output pointer");
    *out = nullptr;
    if (rows < 1 || cols < 1) return fail(-2, "board must be at least 1x1");
    if (rows > 64 || cols > 64 || rows * cols > 512) return fail(-2, "board too large (R,C <= 64, R*C <= 512)");
    if (2 * rows * cols - rows - cols < 1) return fail(-2, "a 1x1 board has no action");
    return new_ctx(out, device, rows, cols, 15, 15u, 1, 1);
}

int tmg_destroy(tmg_ctx *ctx) {
    if (!ctx) return 0;
    free_ctx(ctx);
    return 0;
}

int tmg_spills(tmg_ctx *ctx, uint64_t *count) {
    if (!count) return fail(-1, "null output pointer");
    int rc = check_call(ctx, 0);
    if (rc) return rc;
    rc = hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    uint64_t tot = 0;
    std::lock_guard<std::mutex> lock(ctx->mu);
    for (const auto &x : ctx->spills) {
        if (rc) break;
        if (!x.q) continue;
        unsigned long long t = 0;
        rc = hip_check(hipMemcpy(&t, &x.q->total, sizeof t, hipMemcpyDeviceToHost), "hipMemcpy");
        tot += t;
    }
    if (!rc) *count = tot;
    return rc;
}

int tmg_status(tmg_ctx *ctx, uint32_t *status, int clear) {
    if (!status) return fail(-1, "null output pointer");
    int rc = check_call(ctx, 0);
    if (rc) return rc;
    rc = hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    uint32_t words[4] = {0, 0, 0, 0};      // one word per status bit (note_status in tmg_board.hip)
    if (!rc) rc = hip_check(hipMemcpy(words, ctx->d_status, sizeof words, hipMemcpyDeviceToHost), "hipMemcpy");
    if (rc) return rc;
    *status = (words[0] ? TMG_STATUS_INTERNAL : 0u) | (words[1] ? TMG_STATUS_OVERFLOW : 0u) |
              (words[2] ? TMG_STATUS_CALLER : 0u);
    if (clear) rc = hip_check(hipMemset(ctx->d_status, 0, sizeof words), "hipMemset");
    if (clear && !rc) rc = hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    return rc;
}

int tmg_viable(int rows, int cols, int colours) {
    if (rows < 1 || cols < 1 || rows > 64 || cols > 64 || rows * cols > 512 || colours < 1 || colours > 15) return 0;
    return shape_viable(rows, cols, colours) ? 1 : 0;
}

// OneHotWrapper channel selection (wrappers.py:39-46): enabled specials as
// type ids, in the order of sorted(id + 1)
static int onehot_sel(uint32_t smask, int ids[4]) {
    int n = 0;
    if (smask & TMG_SPECIAL_COOKIE) ids[n++] = -1;
    if (smask & TMG_SPECIAL_VLASER) ids[n++] = 2;
    if (smask & TMG_SPECIAL_HLASER) ids[n++] = 3;
    if (smask & TMG_SPECIAL_BOMB) ids[n++] = 4;
    return n;
}

// Params of a call with the fused one-hot output `onehot` (null: none)
static int onehot_params(tmg_ctx *ctx, void *onehot, int dtype, Params &P) {
    P = ctx->P;
    if (!onehot) return 0;
    if (dtype != TMG_DTYPE_F32 && dtype != TMG_DTYPE_U8 && dtype != TMG_DTYPE_I32)
        return fail(-2, "unknown one-hot output dtype");
    int ids[4] = {0, 0, 0, 0};
    P.oh_nsel = onehot_sel((uint32_t)P.smask, ids);
    P.oh_sel = 0;
    for (int i = 0; i < 4; i++) P.oh_sel |= (uint32_t)(uint8_t)(int8_t)ids[i] << (8 * i);
    P.oh_ch = P.k + P.oh_nsel;
    P.oh_dtype = dtype;
    P.oh = onehot;
    return 0;
}

int tmg_reset(tmg_ctx *ctx, int64_t n, int8_t *board, uint64_t *rng, int32_t *timer, uint64_t *eff,
              const uint8_t *env_mask, void *stream) {
    return tmg_reset_onehot(ctx, n, board, rng, timer, eff, env_mask, nullptr, 0, stream);
}

int tmg_reset_onehot(tmg_ctx *ctx, int64_t n, int8_t *board, uint64_t *rng, int32_t *timer, uint64_t *eff,
                     const uint8_t *env_mask, void *onehot, int onehot_dtype, void *stream) {
    if (!board || !rng || !timer || !eff) return fail(-1, "null state buffer");
    int rc = check_full(ctx, n);
    if (rc || n == 0) return rc;
    Params P;
    rc = onehot_params(ctx, onehot, onehot_dtype, P);
    if (rc) return rc;
    return do_reset(ctx, P, n, board, rng, timer, eff, env_mask, 0xFF, reinterpret_cast<hipStream_t>(stream));
}

int tmg_step(tmg_ctx *ctx, int64_t n, int8_t *board, uint64_t *rng, int32_t *timer, const int32_t *actions,
             int32_t *reward, int32_t *n_new, int32_t *n_act, uint8_t *flags, uint64_t *eff, int trust_eff,
             int autoreset, void *stream) {
    return tmg_step_onehot(ctx, n, board, rng, timer, actions, reward, n_new, n_act, flags, eff, trust_eff, autoreset,
                           nullptr, 0, stream);
}

int tmg_step_onehot(tmg_ctx *ctx, int64_t n, int8_t *board, uint64_t *rng, int32_t *timer, const int32_t *actions,
                    int32_t *reward, int32_t *n_new, int32_t *n_act, uint8_t *flags, uint64_t *eff, int trust_eff,
                    int autoreset, void *onehot, int onehot_dtype, void *stream) {
    if (!board || !rng || !timer || !actions || !reward || !n_new || !n_act || !flags || !eff)
        return fail(-1, "null buffer");
    int rc = check_full(ctx, n);
    if (rc || n == 0) return rc;
    Params P;
    rc = onehot_params(ctx, onehot, onehot_dtype, P);
    if (rc) return rc;
    const StepArgs a{n, board, rng, timer, actions, reward, n_new, n_act, flags, eff, trust_eff, autoreset ? 1 : 0};
    return do_step(ctx, P, a, reinterpret_cast<hipStream_t>(stream));
}

// ------------------------------------------------------------- step plans
struct tmg_plan {
    tmg_ctx *ctx;
    int64_t n;
    int8_t *board;
    uint64_t *rng;
    int32_t *timer, *reward, *n_new, *n_act;
    uint8_t *flags;
    uint64_t *eff;
    std::vector<int64_t> bounds;          // groups + 1
    std::vector<hipStream_t> streams;     // one per group
    hipEvent_t fork;
    std::vector<hipEvent_t> joins;
    int autoreset, policy;
    uint64_t key;
    int64_t first_env;
    Params P;                             // outputs of tmg_plan_config (one-hot, vector-env outputs)
    size_t oh_env_bytes;
};

int tmg_plan_create(tmg_plan **out, tmg_ctx *ctx, int64_t n, int8_t *board, uint64_t *rng, int32_t *timer,
                    int32_t *reward, int32_t *n_new, int32_t *n_act, uint8_t *flags, uint64_t *eff, int groups,
                    const int64_t *bounds, void *const *streams) {
    if (!out) return fail(-1, "null output pointer");
    *out = nullptr;
    if (!board || !rng || !timer || !reward || !n_new || !n_act || !flags || !eff) return fail(-1, "null buffer");
    int rc = check_full(ctx, n);
    if (rc) return rc;
    if (groups < 1 || !bounds || !streams) return fail(-2, "a plan needs >= 1 group, its bounds and streams");
    if (bounds[0] != 0 || bounds[groups] != n) return fail(-2, "group bounds must run from 0 to n");
    for (int g = 0; g < groups; g++)
        if (bounds[g + 1] < bounds[g]) return fail(-2, "group bounds must be non-decreasing");
    tmg_plan *p = new tmg_plan();
    p->ctx = ctx; p->n = n; p->board = board; p->rng = rng; p->timer = timer; p->reward = reward;
    p->n_new = n_new; p->n_act = n_act; p->flags = flags; p->eff = eff;
    p->bounds.assign(bounds, bounds + groups + 1);
    for (int g = 0; g < groups; g++) p->streams.push_back(reinterpret_cast<hipStream_t>(streams[g]));
    p->autoreset = 1; p->policy = 0; p->key = 0; p->first_env = 0;
    p->P = ctx->P;
    p->oh_env_bytes = 0;
    rc = hip_check(hipEventCreateWithFlags(&p->fork, hipEventDisableTiming), "hipEventCreateWithFlags");
    for (int g = 0; g < groups && !rc; g++) {
        hipEvent_t ev;
        rc = hip_check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreateWithFlags");
        if (!rc) p->joins.push_back(ev);
    }
    if (rc) { tmg_plan_destroy(p); return rc; }
    *out = p;
    return 0;
}

int tmg_plan_config(tmg_plan *p, int autoreset, int policy, uint64_t key, int64_t first_env, void *onehot,
                    int onehot_dtype, uint8_t *terminated, uint8_t *action_mask, int64_t *moves_left,
                    int8_t *final_board, int32_t *board32) {
    if (!p) return fail(-1, "null plan");
    if (autoreset < 0 || autoreset > 2) return fail(-2, "autoreset must be 0 (none), 1 (same step) or 2 (next step)");
    if (first_env < 0) return fail(-2, "first_env must be >= 0");
    Params P;
    int rc = onehot_params(p->ctx, onehot, onehot_dtype, P);
    if (rc) return rc;
    P.vo_term = terminated;
    P.vo_mask = action_mask;
    P.vo_left = moves_left;
    P.vo_final = final_board;
    P.vo_obs = board32;
    P.sample = policy ? 1 : 0;
    P.pol_key = key;
    p->P = P;
    p->oh_env_bytes = onehot ? (size_t)P.oh_ch * P.N * (P.oh_dtype == TMG_DTYPE_U8 ? 1 : 4) : 0;
    p->autoreset = autoreset;
    p->policy = policy ? 1 : 0;
    p->key = key;
    p->first_env = first_env;
    return 0;
}

int tmg_plan_step(tmg_plan *p, int32_t *actions, int32_t t, int trust_eff, int fork, void *stream) {
    if (!p) return fail(-1, "null plan");
    if (!actions) return fail(-1, "null actions");
    tmg_ctx *ctx = p->ctx;
    int rc = set_device(ctx);
    if (rc) return rc;
    const hipStream_t cur = reinterpret_cast<hipStream_t>(stream);
    const int G = (int)p->streams.size();
    bool other = false;                     // a NULL group stream is the call's own stream
    for (int g = 0; g < G; g++) other |= p->streams[g] != nullptr && p->streams[g] != cur;
    if (fork && other) {                    // the group streams see the work queued on `stream`
        rc = hip_check(hipEventRecord(p->fork, cur), "hipEventRecord");
        for (int g = 0; g < G && !rc; g++)
            if (p->streams[g] && p->streams[g] != cur)
                rc = hip_check(hipStreamWaitEvent(p->streams[g], p->fork, 0), "hipStreamWaitEvent");
        if (rc) return rc;
    }
    const int W = ctx->P.W, N = ctx->P.N, A = ctx->P.A;
    for (int g = 0; g < G; g++) {
        const int64_t lo = p->bounds[g], m = p->bounds[g + 1] - lo;
        if (m <= 0) continue;
        Params P = p->P;
        if (P.oh) P.oh = static_cast<uint8_t *>(P.oh) + lo * p->oh_env_bytes;
        if (P.vo_term) P.vo_term += 4 * lo;
        if (P.vo_mask) P.vo_mask += lo * A;
        if (P.vo_left) P.vo_left += lo;
        if (P.vo_final) P.vo_final += lo * 2 * N;
        if (P.vo_obs) P.vo_obs += lo * 2 * N;
        P.pol_first = p->first_env + lo;
        P.pol_t = t;
        const hipStream_t gs = p->streams[g] ? p->streams[g] : cur;
#ifndef TMG_GEN_SAMPLE
#define TMG_GEN_SAMPLE 0
#endif
        if (P.sample && !TMG_GEN_SAMPLE && !(ctx->P.smask == 0 && trust_eff)) {
            // the general kernels (low occupancy, long waves) take the draw
            // from the sampler kernel ahead of them; the lean ones sample in
            // their own prologue
            tmg::launch_sample_effective(gs, m, W, A, p->eff + lo * W, p->key, p->first_env + lo, t, actions + lo);
            rc = hip_check(hipGetLastError(), "kernel launch");
            if (rc) return rc;
            P.sample = 0;
        }
        const StepArgs a{m, p->board + lo * 2 * N, p->rng + lo * 5, p->timer + lo, actions + lo, p->reward + lo,
                         p->n_new + lo, p->n_act + lo, p->flags + lo, p->eff + lo * W, trust_eff, p->autoreset};
        rc = do_step(ctx, P, a, gs);
        if (rc) return rc;
    }
    return 0;
}

int tmg_plan_join(tmg_plan *p, void *stream) {
    if (!p) return fail(-1, "null plan");
    int rc = set_device(p->ctx);
    const hipStream_t cur = reinterpret_cast<hipStream_t>(stream);
    const int G = (int)p->streams.size();
    for (int g = 0; g < G && !rc; g++) {
        if (!p->streams[g] || p->streams[g] == cur) continue;
        rc = hip_check(hipEventRecord(p->joins[g], p->streams[g]), "hipEventRecord");
        if (!rc) rc = hip_check(hipStreamWaitEvent(cur, p->joins[g], 0), "hipStreamWaitEvent");
    }
    return rc;
}

// ---------------------------------------------------------- step graphs
struct tmg_graph {
    int device;
    hipGraph_t graph;
    hipGraphExec_t exec;
};

int tmg_graph_destroy(tmg_graph *g) {
    if (!g) return 0;
    if (g->exec) (void)hipGraphExecDestroy(g->exec);
    if (g->graph) (void)hipGraphDestroy(g->graph);
    delete g;
    return 0;
}

int tmg_plan_capture(tmg_plan *p, int steps, int32_t *const *actions, const int32_t *t, int trust_eff, void *stream,
                     tmg_graph **out) {
    if (!out) return fail(-1, "null output pointer");
    *out = nullptr;
    if (!p) return fail(-1, "null plan");
    if (steps < 1 || !actions || !t) return fail(-2, "a capture needs >= 1 step, its actions and step counters");
    if (!stream) return fail(-2, "capture on a created stream (the NULL stream cannot be captured)");
    int rc = set_device(p->ctx);
    if (rc) return rc;
    const hipStream_t cur = reinterpret_cast<hipStream_t>(stream);
    // the general kernels' spill queues must exist before the capture (no
    // allocation or synchronisation inside it)
    if (!(p->ctx->P.smask == 0 && trust_eff)) {
        for (size_t g = 0; g < p->streams.size() && !rc; g++) {
            tmg::SpillQ *q;
            void *ws;
            rc = spill_for(p->ctx, p->streams[g] ? p->streams[g] : cur, p->bounds[g + 1] - p->bounds[g], &q, &ws);
        }
        if (rc) return rc;
    }
    tmg_graph *gr = new tmg_graph();
    gr->device = p->ctx->device;
    rc = hip_check(hipStreamBeginCapture(cur, hipStreamCaptureModeThreadLocal), "hipStreamBeginCapture");
    if (rc) { delete gr; return rc; }
    for (int k = 0; k < steps && !rc; k++) rc = tmg_plan_step(p, actions[k], t[k], k ? 1 : trust_eff, k == 0, stream);
    if (!rc) rc = tmg_plan_join(p, stream);
    const int rc_end = hip_check(hipStreamEndCapture(cur, &gr->graph), "hipStreamEndCapture");
    if (!rc) rc = rc_end;
    if (!rc) rc = hip_check(hipGraphInstantiate(&gr->exec, gr->graph, nullptr, nullptr, 0), "hipGraphInstantiate");
    if (rc) { tmg_graph_destroy(gr); return rc; }
    *out = gr;
    return 0;
}

int tmg_graph_launch(tmg_graph *g, void *stream) {
    if (!g) return fail(-1, "null graph");
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev != g->device) {
        int rc = hip_check(hipSetDevice(g->device), "hipSetDevice");
        if (rc) return rc;
    }
    return hip_check(hipGraphLaunch(g->exec, reinterpret_cast<hipStream_t>(stream)), "hipGraphLaunch");
}

int tmg_plan_destroy(tmg_plan *p) {
    if (!p) return 0;
    if (p->fork) (void)hipEventDestroy(p->fork);
    for (auto ev : p->joins) (void)hipEventDestroy(ev);
    delete p;
    return 0;
}

int tmg_effective(tmg_ctx *ctx, int64_t n, const int8_t *board, uint64_t *eff, void *stream) {
    if (!board || !eff) return fail(-1, "null buffer");
    int rc = check_call(ctx, n);
    if (rc || n == 0) return rc;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const dim3 grid = tmg::env_grid(n);
    if (ctx->maxn == 128) tmg::launch_effective128(grid, s, ctx->P, n, board, eff);
    else tmg::launch_effective512(grid, s, ctx->P, n, board, eff);
    return hip_check(hipGetLastError(), "kernel launch");
}

int tmg_onehot_channels(const tmg_ctx *ctx) {
    if (!ctx) return -1;
    int ids[4];
    return ctx->P.k + onehot_sel((uint32_t)ctx->P.smask, ids);
}

int tmg_onehot(tmg_ctx *ctx, int64_t n, const int8_t *board, void *out, int out_dtype, void *stream) {
    if (!board || !out) return fail(-1, "null buffer");
    int rc = check_full(ctx, n);
    if (rc || n == 0) return rc;
    if (out_dtype != TMG_DTYPE_F32 && out_dtype != TMG_DTYPE_U8 && out_dtype != TMG_DTYPE_I32)
        return fail(-2, "unknown one-hot output dtype");
    int ids[4] = {0, 0, 0, 0};
    const int nsel = onehot_sel((uint32_t)ctx->P.smask, ids);
    tmg::launch_onehot(reinterpret_cast<hipStream_t>(stream), n, ctx->P.N, ctx->P.k, nsel,
                       make_int4(ids[0], ids[1], ids[2], ids[3]), board, out, out_dtype);
    return hip_check(hipGetLastError(), "kernel launch");
}

int tmg_sample_effective(tmg_ctx *ctx, int64_t n, const uint64_t *eff, uint64_t key, int64_t first_env, int32_t t,
                         int32_t *actions, void *stream) {
    if (!eff || !actions) return fail(-1, "null buffer");
    int rc = check_call(ctx, n);
    if (rc || n == 0) return rc;
    if (first_env < 0) return fail(-2, "first_env must be >= 0");
    tmg::launch_sample_effective(reinterpret_cast<hipStream_t>(stream), n, ctx->P.W, ctx->P.A, eff, key, first_env, t,
                                 actions);
    return hip_check(hipGetLastError(), "kernel launch");
}

int tmg_count_states(int device, int rows, int cols, int colours, uint64_t *num_playable, uint64_t *num_line_free) {
    if (!num_playable || !num_line_free) return fail(-1, "null output pointer");
    if (rows < 1 || cols < 1 || rows * cols > 16) return fail(-2, "count_states needs R*C <= 16");
    if (colours < 1 || colours > 15) return fail(-2, "num_colours must be in [1, 15]");
    double total_d = 1.0;
    for (int i = 0; i < rows * cols; i++) total_d *= colours;
    if (total_d > 1.1e12) return fail(-2, "too many boards to enumerate (k^(R*C) > 1.1e12)");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(-3, "no HIP device available");
    if (device < 0 || device >= ndev) return fail(-3, "bad device index");
    int rc = hip_check(hipSetDevice(device), "hipSetDevice");
    if (rc) return rc;
    uint64_t total = 1;
    for (int i = 0; i < rows * cols; i++) total *= (uint64_t)colours;
    // >= ~256k threads when there is work for them, runs of >= 1 board
    uint64_t per = total / (1ULL << 18);
    if (per < 1) per = 1;
    const uint64_t threads = (total + per - 1) / per;
    unsigned long long *d = nullptr;
    rc = hip_check(hipMalloc(&d, 2 * sizeof(unsigned long long)), "hipMalloc");
    if (rc) return rc;
    rc = hip_check(hipMemset(d, 0, 2 * sizeof(unsigned long long)), "hipMemset");
    if (!rc) {
        tmg::launch_count_states(rows, cols, colours, total, per, threads, d);
        rc = hip_check(hipGetLastError(), "kernel launch");
    }
    unsigned long long h[2] = {0, 0};
    if (!rc) rc = hip_check(hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost), "hipMemcpy");
    (void)hipFree(d);
    if (rc) return rc;
    *num_playable = h[0];
    *num_line_free = h[1];
    return 0;
}

#if TMG_COVER
// diagnostic build only: the CV_* branch hit counters of this context
__attribute__((visibility("default"))) int tmg_debug_cover(tmg_ctx *ctx, uint64_t *host, int n, int clear) {
    if (!ctx || !ctx->d_cover) return fail(-1, "no cover counters");
    if (n > tmg::CV_COUNT) n = tmg::CV_COUNT;
    int rc = hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    if (!rc) rc = hip_check(hipMemcpy(host, ctx->d_cover, (size_t)n * 8, hipMemcpyDeviceToHost), "hipMemcpy");
    if (!rc && clear) rc = hip_check(hipMemset(ctx->d_cover, 0, tmg::CV_COUNT * 8), "hipMemset");
    return rc;
}
#endif

int tmg_num_actions(const tmg_ctx *ctx) { return ctx ? ctx->P.A : -1; }
int tmg_mask_words(const tmg_ctx *ctx) { return ctx ? ctx->P.W : -1; }
const char *tmg_last_error(void) { return g_err.c_str(); }
int tmg_abi_version(void) { return 4; }
const char *tmg_build_info(void) { return "src=" TMG_SRC_SHA ";variant=" TMG_VARIANT; }

}  // extern "C"
