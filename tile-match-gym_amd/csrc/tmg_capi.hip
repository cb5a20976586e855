// tmg_capi.hip — extern "C" entry points of libtmg.so (declared in include/tmg.h).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "tmg.h"
#include "tmg_board.hip"
#include "tmg_aux.hip"

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
    int maxn;
    int sb;          // scalar-bitboard kernels usable (<= 128 cells, C <= 63); TMG_SB=0 disables (A/B)
    int defer_general;   // 128-cell general kernel: autoreset by a masked reset launch (TMG_DEFER=0 disables)
    // spill queues of the general kernels, one per stream the context steps on
    // (a queue is only ever touched by the launches of its own stream, in order)
    struct Spill {
        hipStream_t stream;
        tmg::SpillQ *q;
        void *ws;
        tmg::ResetQ *rq;     // deferred-autoreset queue of this stream
        int64_t rq_cap;
    };
    std::vector<Spill> spills;
    int spill_launch;    // TMG_SPILL=0 skips the spill launches (cost A/B only: overflowing steps are then lost)
    int reset_queue;     // deferred autoresets through a queue (TMG_RESETQ=1) instead of an FL_RESET-masked launch
};

using tmg::Params;

struct StepArgs {
    int64_t n;
    int8_t *board;
    uint64_t *rng;
    int32_t *timer;
    const int32_t *actions;
    int32_t *reward, *n_new, *n_act;
    uint8_t *flags;
    uint64_t *eff;
    int trust_eff, autoreset;
};

template <int MAXN, bool GEN, int NB, bool CODD>
static void launch_step(dim3 grid, hipStream_t s, const Params &P, const StepArgs &a) {
    const size_t lds = sizeof(tmg::Ws<MAXN, GEN>) * TMG_WPB;
    hipLaunchKernelGGL((tmg::step_kernel<MAXN, GEN, NB, CODD>), grid, dim3(64 * TMG_WPB), lds, s, P, a.n, a.board,
                       a.rng, a.timer, a.actions, a.reward, a.n_new, a.n_act, a.flags, a.eff, a.trust_eff, a.autoreset);
}

// the stream's spill queue (allocated zeroed on first use)
static int spill_for(tmg_ctx *ctx, hipStream_t s, tmg::SpillQ **q, void **ws) {
    for (const auto &x : ctx->spills)
        if (x.stream == s) { *q = x.q; *ws = x.ws; return 0; }
    const size_t wsz = ctx->maxn == 128 ? sizeof(tmg::WsSerialBig<128>) : sizeof(tmg::WsSerialBig<512>);
    tmg_ctx::Spill sp{s, nullptr, nullptr, nullptr, 0};
    int rc = hip_check(hipMalloc(&sp.q, sizeof(tmg::SpillQ)), "hipMalloc");
    if (!rc) rc = hip_check(hipMalloc(&sp.ws, wsz * TMG_SPILL_WAVES), "hipMalloc");
    // zeroed in order on s itself (a memset on the null stream is not ordered
    // with respect to a non-blocking stream's launches)
    if (!rc) rc = hip_check(hipMemsetAsync(sp.q, 0, sizeof(tmg::SpillQ), s), "hipMemsetAsync");
    if (rc) {
        if (sp.q) (void)hipFree(sp.q);
        if (sp.ws) (void)hipFree(sp.ws);
        return rc;
    }
    ctx->spills.push_back(sp);
    *q = sp.q;
    *ws = sp.ws;
    return 0;
}

// the stream's deferred-autoreset queue, holding at least n envs (zeroed on s)
static int resetq_for(tmg_ctx *ctx, hipStream_t s, int64_t n, tmg::ResetQ **out) {
    tmg_ctx::Spill *sp = nullptr;
    for (auto &x : ctx->spills)
        if (x.stream == s) sp = &x;
    if (!sp) return fail(-5, "no spill entry for this stream");
    if (sp->rq_cap < n) {
        int rc = 0;
        if (sp->rq) {                                  // grow: the old queue may still be in use on s
            rc = hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
            (void)hipFree(sp->rq);
            sp->rq = nullptr;
            sp->rq_cap = 0;
        }
        const size_t bytes = sizeof(tmg::ResetQ) + (size_t)n * sizeof(int64_t);
        if (!rc) rc = hip_check(hipMalloc(&sp->rq, bytes), "hipMalloc");
        if (!rc) rc = hip_check(hipMemsetAsync(sp->rq, 0, sizeof(tmg::ResetQ), s), "hipMemsetAsync");
        if (rc) return rc;
        sp->rq_cap = n;
    }
    *out = sp->rq;
    return 0;
}

template <int MAXN, int NB, bool CODD>
static void launch_reset_queue(hipStream_t s, const Params &P, int64_t n, int8_t *board, uint64_t *rng,
                               int32_t *timer, uint64_t *eff) {
    // a fixed grid of one-wave workgroups draining the queue: about the waves
    // the chip holds at the kernel's occupancy (the queue holds <= n envs)
    const int64_t full = MAXN > 128 ? 256 * 4 * TMG_RESET512_WAVES : 256 * 4 * TMG_RQ128_WAVES;
    const unsigned g = (unsigned)(n < full ? n : full);
    hipLaunchKernelGGL((tmg::reset_queue_kernel<MAXN, NB, CODD>), dim3(g), dim3(64), sizeof(tmg::Ws<MAXN, false>), s,
                       P, board, rng, timer, eff);
    (void)hipMemsetAsync(P.resetq, 0, 16, s);                // count / next / done for the next launch
}

template <int MAXN>
static void launch_spill(hipStream_t s, const Params &P, const StepArgs &a) {
    const size_t lds = sizeof(tmg::Ws<MAXN, true>);
    hipLaunchKernelGGL((tmg::spill_kernel<MAXN>), dim3(TMG_SPILL_WAVES), dim3(64), lds, s, P, a.n, a.board, a.rng,
                       a.timer, a.actions, a.reward, a.n_new, a.n_act, a.flags, a.eff, a.trust_eff, a.autoreset);
}

template <int MAXN, int NB, bool CODD>
static void launch_reset(dim3 grid, hipStream_t s, const Params &P, int64_t n, int8_t *board, uint64_t *rng,
                         int32_t *timer, uint64_t *eff, const uint8_t *env_mask, int mask_bits) {
    const size_t lds = sizeof(tmg::Ws<MAXN, false>) * TMG_WPB;
    hipLaunchKernelGGL((tmg::reset_kernel<MAXN, NB, CODD>), grid, dim3(64 * TMG_WPB), lds, s, P, n, board, rng, timer,
                       eff, env_mask, mask_bits);
}

// scalar-bitboard variants: NB colour planes, C odd or even
template <bool GEN, bool CODD>
static void launch_step_sb(dim3 grid, hipStream_t s, const Params &P, const StepArgs &a) {
    switch (tmg::sb_planes(P.k)) {
    case 1: launch_step<128, GEN, 1, CODD>(grid, s, P, a); break;
    case 2: launch_step<128, GEN, 2, CODD>(grid, s, P, a); break;
    case 3: launch_step<128, GEN, 3, CODD>(grid, s, P, a); break;
    default: launch_step<128, GEN, 4, CODD>(grid, s, P, a); break;
    }
}
template <bool CODD>
static void launch_reset_sb(dim3 grid, hipStream_t s, const Params &P, int64_t n, int8_t *board, uint64_t *rng,
                            int32_t *timer, uint64_t *eff, const uint8_t *env_mask, int mask_bits) {
    switch (tmg::sb_planes(P.k)) {
    case 1: launch_reset<128, 1, CODD>(grid, s, P, n, board, rng, timer, eff, env_mask, mask_bits); break;
    case 2: launch_reset<128, 2, CODD>(grid, s, P, n, board, rng, timer, eff, env_mask, mask_bits); break;
    case 3: launch_reset<128, 3, CODD>(grid, s, P, n, board, rng, timer, eff, env_mask, mask_bits); break;
    default: launch_reset<128, 4, CODD>(grid, s, P, n, board, rng, timer, eff, env_mask, mask_bits); break;
    }
}

// one wave per env: grid padded to 8 equal XCD blocks (wg_env0)
static dim3 env_grid(int64_t n) {
    int64_t nwg = (n + TMG_WPB - 1) / TMG_WPB;
    if (TMG_XCD) nwg = (nwg + 7) & ~(int64_t)7;
    return dim3((unsigned)nwg);
}

static int set_device(tmg_ctx *ctx) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev != ctx->device) return hip_check(hipSetDevice(ctx->device), "hipSetDevice");
    return 0;
}

static int do_reset(tmg_ctx *ctx, const Params &P, int64_t n, int8_t *board, uint64_t *rng, int32_t *timer,
                    uint64_t *eff, const uint8_t *env_mask, int mask_bits, hipStream_t s) {
    const dim3 grid = env_grid(n);
    if (ctx->maxn == 128) {
        if (ctx->sb) {
            if (P.C & 1) launch_reset_sb<true>(grid, s, P, n, board, rng, timer, eff, env_mask, mask_bits);
            else launch_reset_sb<false>(grid, s, P, n, board, rng, timer, eff, env_mask, mask_bits);
        } else {
            launch_reset<128, 0, false>(grid, s, P, n, board, rng, timer, eff, env_mask, mask_bits);
        }
    } else {
        launch_reset<512, 0, false>(grid, s, P, n, board, rng, timer, eff, env_mask, mask_bits);
    }
    return hip_check(hipGetLastError(), "kernel launch");
}

static int do_step(tmg_ctx *ctx, Params P, StepArgs a, hipStream_t s) {
    const bool lean = ctx->P.smask == 0 && a.trust_eff;
    const dim3 grid = env_grid(a.n);
    a.autoreset = a.autoreset ? 1 : 0;
    const int deferred = a.autoreset && (ctx->maxn == 512 || (ctx->defer_general && !lean) || (TMG_LEAN_DEFER && lean));
    if (!lean || deferred) {                       // this stream's spill / deferred-reset queues
        int rc = spill_for(ctx, s, &P.spill, &P.spill_ws);
        if (!rc && deferred && ctx->reset_queue) rc = resetq_for(ctx, s, a.n, &P.resetq);
        if (rc) return rc;
    }
    // 512-cell kernels (and, with defer_general, the 128-cell general one):
    // finished boards are regenerated by a reset_kernel launch masked by
    // FL_RESET, which runs at several times the step kernel's occupancy
    if (deferred) a.autoreset = 2;
    if (ctx->maxn == 128) {
        if (ctx->sb) {
            if (lean) {
                if (P.C & 1) launch_step_sb<false, true>(grid, s, P, a);
                else launch_step_sb<false, false>(grid, s, P, a);
            } else {
                if (P.C & 1) launch_step_sb<true, true>(grid, s, P, a);
                else launch_step_sb<true, false>(grid, s, P, a);
            }
        } else if (lean) {
            launch_step<128, false, 0, false>(grid, s, P, a);
        } else {
            launch_step<128, true, 0, false>(grid, s, P, a);
        }
    } else if (lean) {
        launch_step<512, false, 0, false>(grid, s, P, a);
    } else {
        launch_step<512, true, 0, false>(grid, s, P, a);
    }
    int rc = hip_check(hipGetLastError(), "kernel launch");
    if (rc) return rc;
    if (!lean && ctx->spill_launch) {              // re-run the steps that ran out of LDS list space
        if (ctx->maxn == 128) launch_spill<128>(s, P, a);
        else launch_spill<512>(s, P, a);
        rc = hip_check(hipGetLastError(), "kernel launch");
        if (rc) return rc;
    }
    if (!deferred) return 0;
    if (!P.resetq) return do_reset(ctx, P, a.n, a.board, a.rng, a.timer, a.eff, a.flags, tmg::FL_RESET, s);
    if (ctx->maxn == 512) {
        launch_reset_queue<512, 0, false>(s, P, a.n, a.board, a.rng, a.timer, a.eff);
    } else if (ctx->sb) {
        const bool codd = P.C & 1;
        switch (tmg::sb_planes(P.k)) {
        case 1: codd ? launch_reset_queue<128, 1, true>(s, P, a.n, a.board, a.rng, a.timer, a.eff)
                     : launch_reset_queue<128, 1, false>(s, P, a.n, a.board, a.rng, a.timer, a.eff); break;
        case 2: codd ? launch_reset_queue<128, 2, true>(s, P, a.n, a.board, a.rng, a.timer, a.eff)
                     : launch_reset_queue<128, 2, false>(s, P, a.n, a.board, a.rng, a.timer, a.eff); break;
        case 3: codd ? launch_reset_queue<128, 3, true>(s, P, a.n, a.board, a.rng, a.timer, a.eff)
                     : launch_reset_queue<128, 3, false>(s, P, a.n, a.board, a.rng, a.timer, a.eff); break;
        default: codd ? launch_reset_queue<128, 4, true>(s, P, a.n, a.board, a.rng, a.timer, a.eff)
                      : launch_reset_queue<128, 4, false>(s, P, a.n, a.board, a.rng, a.timer, a.eff); break;
        }
    } else {
        launch_reset_queue<128, 0, false>(s, P, a.n, a.board, a.rng, a.timer, a.eff);
    }
    return hip_check(hipGetLastError(), "kernel launch");
}

static int do_effective(tmg_ctx *ctx, int64_t n, const int8_t *board, uint64_t *eff, hipStream_t s) {
    const dim3 grid = env_grid(n), block(64 * TMG_WPB);
    if (ctx->maxn == 128)
        hipLaunchKernelGGL(tmg::effective_kernel<128>, grid, block, sizeof(tmg::Ws<128, false>) * TMG_WPB, s, ctx->P,
                           n, board, eff);
    else
        hipLaunchKernelGGL(tmg::effective_kernel<512>, grid, block, sizeof(tmg::Ws<512, false>) * TMG_WPB, s, ctx->P,
                           n, board, eff);
    return hip_check(hipGetLastError(), "kernel launch");
}

static int check_call(tmg_ctx *ctx, int64_t n) {
    if (!ctx) return fail(-1, "null context");
    if (n < 0) return fail(-2, "negative batch size");
    return set_device(ctx);
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
// exhaustively when there are at most 2^21 colourings, else by building
// random line-free boards (row-major, a colour that completes no triple).
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
    for (int attempt = 0; attempt < 4096; attempt++) {
        bool ok = true;
        for (int p = 0; p < N && ok; p++) {
            const int r = p / C, c = p - r * C;
            int choices[16], nc = 0;
            for (int v = 0; v < k && v < 16; v++) {
                if (c >= 2 && b[p - 1] == v && b[p - 2] == v) continue;
                if (r >= 2 && b[p - C] == v && b[p - 2 * C] == v) continue;
                choices[nc++] = v;
            }
            if (nc == 0) ok = false;
            else b[p] = choices[rnd() % nc];
        }
        if (ok && playable(b.data(), R, C)) return true;
    }
    return false;
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
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(-3, "no HIP device available");
    if (device < 0 || device >= ndev) return fail(-3, "bad device index");
    int rc = hip_check(hipSetDevice(device), "hipSetDevice");
    if (rc) return rc;
    tmg_ctx *c = new tmg_ctx();
    c->device = device;
    c->P = tmg::make_params(rows, cols, colours, (int)specials_mask, num_moves, nullptr);
    Params &P = c->P;
    c->maxn = P.N <= 128 ? 128 : 512;
    const char *denv = getenv("TMG_DEFER");
    const char *sbenv = getenv("TMG_SB");
    c->sb = P.N <= 128 && P.C <= 63 && !(sbenv && sbenv[0] == '0');
    c->defer_general = c->sb && !(denv && denv[0] == '0');
    const char *spenv = getenv("TMG_SPILL");
    c->spill_launch = !(spenv && spenv[0] == '0');
    // TMG_RESETQ=1: deferred autoresets through the per-stream queue instead of
    // the FL_RESET-masked launch.  Measured on c3: -54 us per normal step (no
    // wave per env to dispatch) but +2.1 ms per reset storm (the looping queue
    // kernel needs 87 VGPRs, 5 waves/SIMD, against the reset kernel's 69 / 7):
    // -5 % overall, so off by default.
    const char *rqenv = getenv("TMG_RESETQ");
    c->reset_queue = rqenv && rqenv[0] == '1';
    uint64_t tab[64 * 4];
    tmg::build_jump_table(tab);
    rc = hip_check(hipMalloc(&c->d_jump, sizeof tab), "hipMalloc");
    if (rc) { delete c; return rc; }
    rc = hip_check(hipMemcpy(c->d_jump, tab, sizeof tab, hipMemcpyHostToDevice), "hipMemcpy");
    if (rc) { (void)hipFree(c->d_jump); delete c; return rc; }
    P.jump = c->d_jump;
    c->d_sbrows = nullptr;
    c->d_status = nullptr;
    rc = hip_check(hipMalloc(&c->d_status, 16), "hipMalloc");
    if (!rc) rc = hip_check(hipMemset(c->d_status, 0, 16), "hipMemset");
    if (!rc) rc = hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    if (rc) {
        (void)hipFree(c->d_jump);
        if (c->d_status) (void)hipFree(c->d_status);
        delete c;
        return rc;
    }
    P.status = c->d_status;
    if (P.N <= 128) {
        uint64_t rows[64 * 4];
        tmg::build_sb_rows(P.R, P.C, rows);
        rc = hip_check(hipMalloc(&c->d_sbrows, sizeof rows), "hipMalloc");
        if (!rc) rc = hip_check(hipMemcpy(c->d_sbrows, rows, sizeof rows, hipMemcpyHostToDevice), "hipMemcpy");
        if (rc) {
            (void)hipFree(c->d_jump);
            (void)hipFree(c->d_status);
            if (c->d_sbrows) (void)hipFree(c->d_sbrows);
            delete c;
            return rc;
        }
        P.sb_rows = c->d_sbrows;
    }
    *out = c;
    return 0;
}

int tmg_destroy(tmg_ctx *ctx) {
    if (!ctx) return 0;
    (void)hipFree(ctx->d_jump);
    (void)hipFree(ctx->d_status);
    if (ctx->d_sbrows) (void)hipFree(ctx->d_sbrows);
    for (const auto &x : ctx->spills) {
        (void)hipFree(x.q);
        (void)hipFree(x.ws);
        if (x.rq) (void)hipFree(x.rq);
    }
    delete ctx;
    return 0;
}

int tmg_spills(tmg_ctx *ctx, uint64_t *count) {
    if (!count) return fail(-1, "null output pointer");
    int rc = check_call(ctx, 0);
    if (rc) return rc;
    rc = hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    uint64_t tot = 0;
    for (const auto &x : ctx->spills) {
        if (rc) break;
        tmg::SpillQ h;
        rc = hip_check(hipMemcpy(&h, x.q, 16, hipMemcpyDeviceToHost), "hipMemcpy");
        tot += h.total;
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
    int rc = check_call(ctx, n);
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
    int rc = check_call(ctx, n);
    if (rc || n == 0) return rc;
    Params P;
    rc = onehot_params(ctx, onehot, onehot_dtype, P);
    if (rc) return rc;
    const StepArgs a{n, board, rng, timer, actions, reward, n_new, n_act, flags, eff, trust_eff, autoreset};
    return do_step(ctx, P, a, reinterpret_cast<hipStream_t>(stream));
}

int tmg_effective(tmg_ctx *ctx, int64_t n, const int8_t *board, uint64_t *eff, void *stream) {
    if (!board || !eff) return fail(-1, "null buffer");
    int rc = check_call(ctx, n);
    if (rc || n == 0) return rc;
    return do_effective(ctx, n, board, eff, reinterpret_cast<hipStream_t>(stream));
}

int tmg_onehot_channels(const tmg_ctx *ctx) {
    if (!ctx) return -1;
    int ids[4];
    return ctx->P.k + onehot_sel((uint32_t)ctx->P.smask, ids);
}

int tmg_onehot(tmg_ctx *ctx, int64_t n, const int8_t *board, void *out, int out_dtype, void *stream) {
    if (!board || !out) return fail(-1, "null buffer");
    int rc = check_call(ctx, n);
    if (rc || n == 0) return rc;
    int ids[4] = {0, 0, 0, 0};
    const int nsel = onehot_sel((uint32_t)ctx->P.smask, ids);
    const int4 sel = make_int4(ids[0], ids[1], ids[2], ids[3]);
    const int64_t cells = n * ctx->P.N;
    const dim3 grid((unsigned)((cells + 255) / 256)), block(256);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    switch (out_dtype) {
    case TMG_DTYPE_F32:
        hipLaunchKernelGGL(tmg::onehot_kernel<float>, grid, block, 0, s, n, ctx->P.N, ctx->P.k, nsel, sel, board, (float *)out);
        break;
    case TMG_DTYPE_U8:
        hipLaunchKernelGGL(tmg::onehot_kernel<uint8_t>, grid, block, 0, s, n, ctx->P.N, ctx->P.k, nsel, sel, board, (uint8_t *)out);
        break;
    case TMG_DTYPE_I32:
        hipLaunchKernelGGL(tmg::onehot_kernel<int32_t>, grid, block, 0, s, n, ctx->P.N, ctx->P.k, nsel, sel, board, (int32_t *)out);
        break;
    default:
        return fail(-2, "unknown one-hot output dtype");
    }
    return hip_check(hipGetLastError(), "kernel launch");
}

int tmg_sample_effective(tmg_ctx *ctx, int64_t n, const uint64_t *eff, uint64_t key, int64_t first_env, int32_t t,
                         int32_t *actions, void *stream) {
    if (!eff || !actions) return fail(-1, "null buffer");
    int rc = check_call(ctx, n);
    if (rc || n == 0) return rc;
    if (first_env < 0) return fail(-2, "first_env must be >= 0");
    const dim3 grid((unsigned)((n + 255) / 256)), block(256);
    hipLaunchKernelGGL(tmg::sample_effective_kernel, grid, block, 0, reinterpret_cast<hipStream_t>(stream), n,
                       ctx->P.W, ctx->P.A, eff, key, first_env, t, actions);
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
    const tmg::CountGeo G = tmg::make_count_geo(rows, cols, colours);
    // >= ~256k threads when there is work for them, runs of >= 1 board
    uint64_t per = total / (1ULL << 18);
    if (per < 1) per = 1;
    const uint64_t threads = (total + per - 1) / per;
    unsigned long long *d = nullptr;
    rc = hip_check(hipMalloc(&d, 2 * sizeof(unsigned long long)), "hipMalloc");
    if (rc) return rc;
    rc = hip_check(hipMemset(d, 0, 2 * sizeof(unsigned long long)), "hipMemset");
    if (!rc) {
        hipLaunchKernelGGL(tmg::count_states_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, 0, G, total,
                           per, d);
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

#if TMG_STAMPS
// diagnostic build only: copy the per-env phase stamps (uint64 [n][8]) to host memory
__attribute__((visibility("default"))) int tmg_debug_stamps(uint64_t *host, int64_t n) {
    if (n > tmg::kStampEnvs) n = tmg::kStampEnvs;
    return hip_check(hipMemcpyFromSymbol(host, HIP_SYMBOL(tmg::g_stamps), (size_t)n * tmg::kStampSlots * sizeof(uint64_t), 0,
                                         hipMemcpyDeviceToHost), "hipMemcpyFromSymbol");
}
#endif

int tmg_num_actions(const tmg_ctx *ctx) { return ctx ? ctx->P.A : -1; }
int tmg_mask_words(const tmg_ctx *ctx) { return ctx ? ctx->P.W : -1; }
const char *tmg_last_error(void) { return g_err.c_str(); }
int tmg_abi_version(void) { return 2; }

}  // extern "C"
