// tmg_capi.hip — extern "C" entry points of libtmg.so (declared in include/tmg.h).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "tmg.h"
#include "tmg_board.hip"

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
    int maxn;
    int sb;        // scalar-bitboard kernels usable (<= 128 cells, C <= 63); TMG_SB=0 disables (A/B)
};

using tmg::Params;

static size_t lean_lds(const tmg_ctx *) { return sizeof(tmg::Ws<128, false>) * TMG_WPB; }

// lean step / reset on scalar bitboards (tmg_sb.hip), NB colour planes, CODD = C odd
template <int NB, bool CODD>
static void launch_sb(int which, tmg_ctx *ctx, dim3 grid, dim3 block, size_t lds, int64_t n, int8_t *board,
                      uint64_t *rng, int32_t *timer, const int32_t *actions, int32_t *reward, int32_t *n_new,
                      int32_t *n_act, uint8_t *flags, uint64_t *eff, const uint8_t *env_mask, int trust_eff,
                      int autoreset, hipStream_t s) {
    if (which == 0)
        hipLaunchKernelGGL((tmg::step_kernel<128, false, NB, CODD>), grid, block, lds, s, ctx->P, n, board, rng, timer,
                           actions, reward, n_new, n_act, flags, eff, trust_eff, autoreset);
    else
        hipLaunchKernelGGL((tmg::reset_kernel<128, NB, CODD>), grid, block, lds, s, ctx->P, n, board, rng, timer, eff,
                           env_mask);
}

template <bool CODD>
static void launch_sb_nb(int which, tmg_ctx *ctx, dim3 grid, dim3 block, size_t lds, int64_t n, int8_t *board,
                         uint64_t *rng, int32_t *timer, const int32_t *actions, int32_t *reward, int32_t *n_new,
                         int32_t *n_act, uint8_t *flags, uint64_t *eff, const uint8_t *env_mask, int trust_eff,
                         int autoreset, hipStream_t s) {
    switch (tmg::sb_planes(ctx->P.k)) {
    case 1: launch_sb<1, CODD>(which, ctx, grid, block, lds, n, board, rng, timer, actions, reward, n_new, n_act, flags, eff, env_mask, trust_eff, autoreset, s); break;
    case 2: launch_sb<2, CODD>(which, ctx, grid, block, lds, n, board, rng, timer, actions, reward, n_new, n_act, flags, eff, env_mask, trust_eff, autoreset, s); break;
    case 3: launch_sb<3, CODD>(which, ctx, grid, block, lds, n, board, rng, timer, actions, reward, n_new, n_act, flags, eff, env_mask, trust_eff, autoreset, s); break;
    default: launch_sb<4, CODD>(which, ctx, grid, block, lds, n, board, rng, timer, actions, reward, n_new, n_act, flags, eff, env_mask, trust_eff, autoreset, s); break;
    }
}

template <int MAXN>
static int launch_all(int which, tmg_ctx *ctx, int64_t n, int8_t *board, uint64_t *rng, int32_t *timer,
                      const int32_t *actions, int32_t *reward, int32_t *n_new, int32_t *n_act, uint8_t *flags,
                      uint64_t *eff, const uint8_t *env_mask, int trust_eff, int autoreset, hipStream_t s) {
    const dim3 block(64 * TMG_WPB);
    int64_t nwg = (n + TMG_WPB - 1) / TMG_WPB;
    if (TMG_XCD) nwg = (nwg + 7) & ~(int64_t)7;                 // wg_env0(): 8 equal XCD blocks
    const dim3 grid((unsigned)nwg);
    const size_t lean = sizeof(tmg::Ws<MAXN, false>) * TMG_WPB;
    const size_t gen = sizeof(tmg::Ws<MAXN, true>) * TMG_WPB;
    if constexpr (MAXN == 128) {
        const bool lean = which == 0 && ctx->P.smask == 0 && trust_eff;
        if (ctx->sb && (lean || which == 1)) {
            if (ctx->P.C & 1)
                launch_sb_nb<true>(which, ctx, grid, block, lean_lds(ctx), n, board, rng, timer, actions, reward, n_new,
                                   n_act, flags, eff, env_mask, trust_eff, autoreset, s);
            else
                launch_sb_nb<false>(which, ctx, grid, block, lean_lds(ctx), n, board, rng, timer, actions, reward, n_new,
                                    n_act, flags, eff, env_mask, trust_eff, autoreset, s);
            return hip_check(hipGetLastError(), "kernel launch");
        }
    }
    if (which == 0) {
        // lean variant: no special can exist (none enabled) and the cached mask is trusted
        if (ctx->P.smask == 0 && trust_eff)
            hipLaunchKernelGGL((tmg::step_kernel<MAXN, false>), grid, block, lean, s, ctx->P, n, board, rng, timer,
                               actions, reward, n_new, n_act, flags, eff, trust_eff, autoreset);
        else
            hipLaunchKernelGGL((tmg::step_kernel<MAXN, true>), grid, block, gen, s, ctx->P, n, board, rng, timer,
                               actions, reward, n_new, n_act, flags, eff, trust_eff, autoreset);
    } else if (which == 1) {
        hipLaunchKernelGGL(tmg::reset_kernel<MAXN>, grid, block, lean, s, ctx->P, n, board, rng, timer, eff, env_mask);
    } else {
        hipLaunchKernelGGL(tmg::effective_kernel<MAXN>, grid, block, lean, s, ctx->P, n, (const int8_t *)board, eff);
    }
    return hip_check(hipGetLastError(), "kernel launch");
}

static int dispatch(int which, tmg_ctx *ctx, int64_t n, int8_t *board, uint64_t *rng, int32_t *timer,
                    const int32_t *actions, int32_t *reward, int32_t *n_new, int32_t *n_act, uint8_t *flags,
                    uint64_t *eff, const uint8_t *env_mask, int trust_eff, int autoreset, void *stream) {
    if (!ctx) return fail(-1, "null context");
    if (n < 0) return fail(-2, "negative batch size");
    if (n == 0) return 0;
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev != ctx->device) {
        int rc = hip_check(hipSetDevice(ctx->device), "hipSetDevice");
        if (rc) return rc;
    }
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (ctx->maxn == 128)
        return launch_all<128>(which, ctx, n, board, rng, timer, actions, reward, n_new, n_act, flags, eff, env_mask,
                               trust_eff, autoreset, s);
    return launch_all<512>(which, ctx, n, board, rng, timer, actions, reward, n_new, n_act, flags, eff, env_mask,
                           trust_eff, autoreset, s);
}

extern "C" {

int tmg_create(tmg_ctx **out, int device, int rows, int cols, int colours, uint32_t specials_mask, int num_moves) {
    if (!out) return fail(-1, "null output pointer");
    *out = nullptr;
    if (rows < 2 || cols < 2) return fail(-2, "board must be at least 2x2");
    if (rows > 64 || cols > 64 || rows * cols > 512) return fail(-2, "board too large (R,C <= 64, R*C <= 512)");
    if (colours < 1 || colours > 15) return fail(-2, "num_colours must be in [1, 15]");
    if (specials_mask > 15u) return fail(-2, "bad specials mask");
    if (num_moves < 1) return fail(-2, "num_moves must be >= 1");
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
    const char *sbenv = getenv("TMG_SB");
    c->sb = P.N <= 128 && P.C <= 63 && !(sbenv && sbenv[0] == '0');
    uint64_t tab[64 * 4];
    tmg::build_jump_table(tab);
    rc = hip_check(hipMalloc(&c->d_jump, sizeof tab), "hipMalloc");
    if (rc) { delete c; return rc; }
    rc = hip_check(hipMemcpy(c->d_jump, tab, sizeof tab, hipMemcpyHostToDevice), "hipMemcpy");
    if (rc) { (void)hipFree(c->d_jump); delete c; return rc; }
    P.jump = c->d_jump;
    c->d_sbrows = nullptr;
    if (P.N <= 128) {
        uint64_t rows[64 * 4];
        tmg::build_sb_rows(P.R, P.C, rows);
        rc = hip_check(hipMalloc(&c->d_sbrows, sizeof rows), "hipMalloc");
        if (!rc) rc = hip_check(hipMemcpy(c->d_sbrows, rows, sizeof rows, hipMemcpyHostToDevice), "hipMemcpy");
        if (rc) { (void)hipFree(c->d_jump); if (c->d_sbrows) (void)hipFree(c->d_sbrows); delete c; return rc; }
        P.sb_rows = c->d_sbrows;
    }
    *out = c;
    return 0;
}

int tmg_destroy(tmg_ctx *ctx) {
    if (!ctx) return 0;
    (void)hipFree(ctx->d_jump);
    if (ctx->d_sbrows) (void)hipFree(ctx->d_sbrows);
    delete ctx;
    return 0;
}

int tmg_reset(tmg_ctx *ctx, int64_t n, int8_t *board, uint64_t *rng, int32_t *timer, uint64_t *eff,
              const uint8_t *env_mask, void *stream) {
    if (!board || !rng || !timer || !eff) return fail(-1, "null state buffer");
    return dispatch(1, ctx, n, board, rng, timer, nullptr, nullptr, nullptr, nullptr, nullptr, eff, env_mask, 0, 0,
                    stream);
}

int tmg_step(tmg_ctx *ctx, int64_t n, int8_t *board, uint64_t *rng, int32_t *timer, const int32_t *actions,
             int32_t *reward, int32_t *n_new, int32_t *n_act, uint8_t *flags, uint64_t *eff, int trust_eff,
             int autoreset, void *stream) {
    if (!board || !rng || !timer || !actions || !reward || !n_new || !n_act || !flags || !eff)
        return fail(-1, "null buffer");
    return dispatch(0, ctx, n, board, rng, timer, actions, reward, n_new, n_act, flags, eff, nullptr, trust_eff,
                    autoreset, stream);
}

int tmg_effective(tmg_ctx *ctx, int64_t n, const int8_t *board, uint64_t *eff, void *stream) {
    if (!board || !eff) return fail(-1, "null buffer");
    return dispatch(2, ctx, n, const_cast<int8_t *>(board), nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                    nullptr, eff, nullptr, 0, 0, stream);
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
int tmg_abi_version(void) { return 1; }

}  // extern "C"
