// Host wave emulator (test/debug tool, never part of the product): runs the
// kernels of tile-match-gym_amd/csrc/tmg_board.hip with one host thread per
// lane, so AddressSanitizer / gdb see every LDS and global index.
#include "hip/hip_runtime.h"
#include "tmg_board.hip"

#include <setjmp.h>
#include <ucontext.h>

#include <cstdio>
#include <dlfcn.h>
#include <cstring>
#include <vector>

#if defined(__has_feature)
#if __has_feature(address_sanitizer)
#define EMU_ASAN 1
#endif
#endif
#if defined(__SANITIZE_ADDRESS__)
#define EMU_ASAN 1
#endif
#ifdef EMU_ASAN
#include <sanitizer/common_interface_defs.h>
#endif

EmuDim emu_block_idx, emu_grid_dim;

namespace {
constexpr size_t kStack = 1 << 20;
struct Lane {
    ucontext_t ctx;                 // only used to enter the fiber the first time
    jmp_buf jb;                     // later switches: _setjmp/_longjmp (no signal-mask syscalls)
    std::vector<char> stack;
    int done = 0, op = 0, arg = 0, started = 0;
    void *site = nullptr, *site2 = nullptr, *site3 = nullptr;
    uint64_t val = 0, res = 0;
};
Lane g_lanes[64];
jmp_buf g_main_jb;
int g_cur = -1;
unsigned char *g_smem = nullptr;
void (*g_body)(void *) = nullptr;
void *g_body_arg = nullptr;
#ifdef EMU_ASAN
void *g_main_fake = nullptr;
const void *g_main_bottom = nullptr;
size_t g_main_size = 0;
#endif

void switch_to_lane(int l) {
    g_cur = l;
    if (_setjmp(g_main_jb) == 0) {
#ifdef EMU_ASAN
        __sanitizer_start_switch_fiber(&g_main_fake, g_lanes[l].stack.data(), kStack);
#endif
        if (!g_lanes[l].started) { g_lanes[l].started = 1; setcontext(&g_lanes[l].ctx); }
        _longjmp(g_lanes[l].jb, 1);
    }
#ifdef EMU_ASAN
    __sanitizer_finish_switch_fiber(g_main_fake, &g_main_bottom, &g_main_size);
#endif
}
void yield_to_main(bool finished) {
    Lane &L = g_lanes[g_cur];
#ifdef EMU_ASAN
    void *fake = nullptr;
#endif
    if (finished || _setjmp(L.jb) == 0) {
#ifdef EMU_ASAN
        __sanitizer_start_switch_fiber(finished ? nullptr : &fake, g_main_bottom, g_main_size);
#endif
        _longjmp(g_main_jb, 1);
    }
#ifdef EMU_ASAN
    __sanitizer_finish_switch_fiber(fake, nullptr, nullptr);
#endif
}
void lane_entry() {
#ifdef EMU_ASAN
    __sanitizer_finish_switch_fiber(nullptr, &g_main_bottom, &g_main_size);
#endif
    g_body(g_body_arg);
    g_lanes[g_cur].done = 1;
    yield_to_main(true);
}
}  // namespace

EmuDim emu_thread_idx() { EmuDim d; d.x = (unsigned)g_cur; return d; }
unsigned char *emu_smem() { return g_smem; }

static void print_site(void *a) {
    Dl_info di;
    if (a && dladdr(a, &di) && di.dli_fbase)
        fprintf(stderr, "%s+0x%lx", di.dli_fname, (unsigned long)((char *)a - (char *)di.dli_fbase));
    else
        fprintf(stderr, "%p", a);
}

__attribute__((noinline)) uint64_t emu_collective(int op, uint64_t v, int arg) {
    Lane &L = g_lanes[g_cur];
    L.op = op; L.val = v; L.arg = arg;
    L.site = __builtin_return_address(0);
#ifdef EMU_DEEP_SITES
    L.site2 = __builtin_return_address(1);
    L.site3 = __builtin_return_address(2);
#endif
    yield_to_main(false);
    return g_lanes[g_cur].res;
}

// run one workgroup of one wave: every lane to completion, resolving collectives
static void run_wave(void (*body)(void *), void *arg) {
    g_body = body; g_body_arg = arg;
    for (int l = 0; l < 64; l++) {
        Lane &L = g_lanes[l];
        if (L.stack.empty()) L.stack.resize(kStack);
        getcontext(&L.ctx);
        L.ctx.uc_stack.ss_sp = L.stack.data();
        L.ctx.uc_stack.ss_size = kStack;
        L.ctx.uc_link = nullptr;
        makecontext(&L.ctx, lane_entry, 0);
        L.done = 0; L.op = 0; L.started = 0;
    }
    for (;;) {
        int live = 0;
        for (int l = 0; l < 64; l++)
            if (!g_lanes[l].done) { switch_to_lane(l); }
        int op = 0;
        for (int l = 0; l < 64; l++) {
            if (g_lanes[l].done) continue;
            live++;
            if (op == 0) op = g_lanes[l].op;
            else if (g_lanes[l].op != op) {
                fprintf(stderr, "wave_emu: divergent collectives (lane %d op %d vs %d) at ", l, g_lanes[l].op, op);
                print_site(g_lanes[l].site); fprintf(stderr, "\n"); abort();
            }
        }
        if (!live) break;
        if (live != 64) {
            fprintf(stderr, "wave_emu: block %u: %d lanes exited before a collective; waiting lanes at:\n",
                    emu_block_idx.x, 64 - live);
            for (int l = 0; l < 64; l++) {
                if (g_lanes[l].done) { fprintf(stderr, "  lane %d: exited\n", l); continue; }
                fprintf(stderr, "  lane %d: op %d at ", l, g_lanes[l].op); print_site(g_lanes[l].site);
                fprintf(stderr, " <- "); print_site(g_lanes[l].site2); fprintf(stderr, " <- "); print_site(g_lanes[l].site3);
                fprintf(stderr, "\n");
                if (l > 2) break;
            }
            abort();
        }
        if (op == EMU_BALLOT) {
            uint64_t m = 0;
            for (int l = 0; l < 64; l++) m |= (g_lanes[l].val & 1) << l;
            for (int l = 0; l < 64; l++) g_lanes[l].res = m;
        } else if (op == EMU_READLANE) {
            for (int l = 0; l < 64; l++) g_lanes[l].res = g_lanes[g_lanes[l].arg & 63].val;
        } else if (op == EMU_DPP) {
            for (int l = 0; l < 64; l++) {
                const int a = g_lanes[l].arg, ctrl = a & 0xfff, rm = (a >> 12) & 0xf, bm = (a >> 16) & 0xf;
                const bool bc = (a >> 20) & 1;
                const uint32_t old = (uint32_t)(g_lanes[l].val >> 32);
                const int row = l >> 4, bank = (l & 15) >> 2;
                int srcl = -1;
                if (ctrl <= 0xff) srcl = (l & ~3) | ((ctrl >> (2 * (l & 3))) & 3);       // quad_perm
                else if (ctrl >= 0x111 && ctrl <= 0x11f) { int n = ctrl - 0x110; if ((l & 15) >= n) srcl = l - n; }
                else if (ctrl == 0x138) { if (l >= 1) srcl = l - 1; }                 // wave_shr:1
                else if (ctrl == 0x130) { if (l <= 62) srcl = l + 1; }                // wave_shl:1
                else if (ctrl == 0x142) { if (row >= 1) srcl = row * 16 - 1; }
                else if (ctrl == 0x143) { if (row >= 2) srcl = 31; }
                else { fprintf(stderr, "wave_emu: unsupported DPP ctrl 0x%x\n", ctrl); abort(); }
                uint32_t r;
                if (!((rm >> row) & 1) || !((bm >> bank) & 1)) r = old;
                else if (srcl < 0) r = bc ? 0u : old;
                else r = (uint32_t)g_lanes[srcl].val;
                g_lanes[l].res = r;
            }
        }
    }
}

template <class F>
static void body_thunk(void *p) { (*reinterpret_cast<F *>(p))(); }

template <class F>
static void run_grid(int64_t nblocks, size_t lds, F kernel) {
    emu_grid_dim.x = (unsigned)nblocks;
    for (int64_t b = 0; b < nblocks; b++) {
        std::vector<unsigned char> smem(lds ? lds : 1);    // exactly sized: ASan catches any overrun
        memset(smem.data(), 0xA5, smem.size());
        g_smem = smem.data();
        emu_block_idx.x = (unsigned)b;
        run_wave(&body_thunk<F>, &kernel);
    }
}

// one wave per env; the grid is padded to 8 XCD blocks like the host launcher does
template <class F>
static void run_blocks(int64_t n, size_t lds, F kernel) {
    int64_t nblocks = n;
    nblocks = (nblocks + 7) & ~(int64_t)7;
    run_grid(nblocks, lds, kernel);
}

static uint64_t g_sbrows[64 * 4];
static uint32_t g_status[4];
static std::vector<int64_t> g_spill_buf;          // a SpillQ with room for every env of the call
static unsigned long long g_spill_total = 0;
static unsigned long long g_cover[tmg::CV_COUNT];
static std::vector<unsigned char> g_spill_ws(sizeof(tmg::WsSerialBig<512>) * tmg::kSpillWaves);
static tmg::SpillQ *spill_queue(std::vector<int64_t> &buf, int64_t n) {
    const size_t words = (sizeof(tmg::SpillQ) + (size_t)n * 8 + 7) / 8;
    buf.assign(words, 0);
    tmg::SpillQ *q = reinterpret_cast<tmg::SpillQ *>(buf.data());
    q->cap = n;
    q->total = 0;
    return q;
}
static tmg::Params make_params(int R, int C, int k, int smask, int moves, const uint64_t *jump) {
    tmg::Params P = tmg::make_params(R, C, k, smask, moves, jump);
    P.status = g_status;
    P.spill = nullptr;
    P.spill_ws = g_spill_ws.data();
    P.cover = g_cover;
    if (P.N <= 128) {
        tmg::build_sb_rows(R, C, g_sbrows);
        P.sb_rows = g_sbrows;
    }
    return P;
}

static uint64_t g_jump[tmg::kJumpRows * 4];
static bool g_jump_init = false;

static bool sb_ok(const tmg::Params &P) { return P.N <= 128 && P.C <= 63; }

// step variants as tmg_capi.hip's do_step: one wave per env
struct EmuStep {
    const tmg::Params *P;
    int64_t n;
    int8_t *board; uint64_t *rng; int32_t *timer; const int32_t *actions;
    int32_t *reward, *n_new, *n_act; uint8_t *flags; uint64_t *eff;
    int trust_eff, autoreset;
};

template <int MAXN, bool GEN, int NB, bool CODD, int FIX = tmg::kNoFix>
static void emu_step_kernel(EmuStep &S) {
    const tmg::Params &P = *S.P;
    run_blocks(S.n, sizeof(tmg::Ws<MAXN, GEN>), [&] { tmg::step_kernel<MAXN, GEN, NB, CODD, FIX>(P, S.n, S.board, S.rng, S.timer, S.actions, S.reward, S.n_new, S.n_act, S.flags, S.eff, S.trust_eff, S.autoreset); });
}
// tmg_kernels.hip's is_shape: the shape-specialised instantiations the launchers pick
template <int FIX>
static bool emu_is_shape(const tmg::Params &P) {
    const int sm = (FIX & 255) == tmg::kFixAnySpecials ? tmg::kFixAnySpecials : P.smask;
    return tmg::shape_fix(P.R, P.C, P.k, sm) == FIX;
}

// spill_kernel after a general step launch, as tmg_capi.hip's do_step
template <int MAXN>
static void emu_spill(EmuStep &S) {
    const tmg::Params &P = *S.P;
    run_grid(tmg::kSpillWaves, sizeof(tmg::Ws<MAXN, false>), [&] { tmg::spill_kernel<MAXN>(P, S.n, S.board, S.rng, S.timer, S.actions, S.reward, S.n_new, S.n_act, S.flags, S.eff, S.trust_eff, S.autoreset); });
}

template <bool GEN, bool CODD>
static void emu_step_sb(EmuStep &S) {
    switch (tmg::sb_planes(S.P->k)) {
    case 1: emu_step_kernel<128, GEN, 1, CODD>(S); break;
    case 2: emu_step_kernel<128, GEN, 2, CODD>(S); break;
    case 3: emu_step_kernel<128, GEN, 3, CODD>(S); break;
    default: emu_step_kernel<128, GEN, 4, CODD>(S); break;
    }
}

template <int MAXN, int NB, bool CODD, int FIX = tmg::kNoFix>
static void emu_reset_kernel(const tmg::Params &P, int64_t n, int8_t *board, uint64_t *rng, int32_t *timer, uint64_t *eff,
                             const uint8_t *mask, int bits) {
    const int epw = !mask ? 1 : MAXN == 128 ? tmg::kMaskedResetEnvs128 : tmg::kMaskedResetEnvs512;   // as do_reset
    run_blocks((n + epw - 1) / epw, sizeof(tmg::Ws<MAXN, false>),
               [&] { tmg::reset_kernel<MAXN, NB, CODD, FIX>(P, n, board, rng, timer, eff, mask, bits, epw); });
}
template <bool CODD>
static void emu_reset_sb(const tmg::Params &P, int64_t n, int8_t *board, uint64_t *rng, int32_t *timer, uint64_t *eff,
                         const uint8_t *mask, int bits) {
    switch (tmg::sb_planes(P.k)) {
    case 1: emu_reset_kernel<128, 1, CODD>(P, n, board, rng, timer, eff, mask, bits); break;
    case 2: emu_reset_kernel<128, 2, CODD>(P, n, board, rng, timer, eff, mask, bits); break;
    case 3: emu_reset_kernel<128, 3, CODD>(P, n, board, rng, timer, eff, mask, bits); break;
    default: emu_reset_kernel<128, 4, CODD>(P, n, board, rng, timer, eff, mask, bits); break;
    }
}

// as tmg_capi.hip's do_reset
static void emu_do_reset(const tmg::Params &P, int64_t n, int8_t *board, uint64_t *rng, int32_t *timer, uint64_t *eff,
                         const uint8_t *mask, int bits) {
    if (emu_is_shape<tmg::kFixReset10>(P)) {
        emu_reset_kernel<128, 2, false, tmg::kFixReset10>(P, n, board, rng, timer, eff, mask, bits);
    } else if (emu_is_shape<tmg::kFixReset20>(P)) {
        emu_reset_kernel<512, 3, false, tmg::kFixReset20>(P, n, board, rng, timer, eff, mask, bits);
    } else if (sb_ok(P)) {
        if (P.C & 1) emu_reset_sb<true>(P, n, board, rng, timer, eff, mask, bits);
        else emu_reset_sb<false>(P, n, board, rng, timer, eff, mask, bits);
    } else if (P.N <= 128) {
        emu_reset_kernel<128, 0, false>(P, n, board, rng, timer, eff, mask, bits);
    } else {
        switch (tmg::sb_planes(P.k)) {
        case 1: emu_reset_kernel<512, 1, false>(P, n, board, rng, timer, eff, mask, bits); break;
        case 2: emu_reset_kernel<512, 2, false>(P, n, board, rng, timer, eff, mask, bits); break;
        case 3: emu_reset_kernel<512, 3, false>(P, n, board, rng, timer, eff, mask, bits); break;
        default: emu_reset_kernel<512, 4, false>(P, n, board, rng, timer, eff, mask, bits); break;
        }
    }
}

extern "C" {

// autoreset as tmg_plan_config (0 none, 1 same step, 2 next step); policy /
// key / first_env / t and the vector-env outputs as tmg_plan_config (NULL: none)
int emu_step(int R, int C, int k, int smask, int moves, int64_t n, int8_t *board, uint64_t *rng, int32_t *timer,
             int32_t *actions, int32_t *reward, int32_t *n_new, int32_t *n_act, uint8_t *flags, uint64_t *eff,
             int trust_eff, int autoreset, int policy, uint64_t key, int64_t first_env, int32_t t, uint8_t *term,
             uint8_t *mask, int64_t *left, int8_t *final_board, int32_t *board32) {
    if (!g_jump_init) { tmg::build_jump_table(g_jump); g_jump_init = true; }
    tmg::Params P = make_params(R, C, k, smask, moves, g_jump);
    P.spill = spill_queue(g_spill_buf, n);
    P.sample = policy ? 1 : 0;
    P.pol_key = key;
    P.pol_first = first_env;
    P.pol_t = t;
    P.vo_term = term;
    P.vo_mask = mask;
    P.vo_left = left;
    P.vo_final = final_board;
    P.vo_obs = board32;
    EmuStep S;
    S.P = &P; S.n = n; S.board = board; S.rng = rng; S.timer = timer; S.actions = actions; S.reward = reward;
    S.n_new = n_new; S.n_act = n_act; S.flags = flags; S.eff = eff; S.trust_eff = trust_eff; S.autoreset = autoreset;
    const bool lean = smask == 0 && trust_eff;
    // as tmg_capi.hip's do_step: the general and 512-cell kernels leave
    // finished boards to a reset launch masked by FL_RESET
    const int deferred = autoreset && (P.N > 128 || !lean);
    S.autoreset = autoreset == 0 ? 0 : autoreset == 1 ? (deferred ? 2 : 1) : (deferred ? 4 : 3);
    if (P.N <= 128) {
        if (lean) {
            if (sb_ok(P) && emu_is_shape<tmg::kFixC2>(P)) emu_step_kernel<128, false, 2, false, tmg::kFixC2>(S);
            else if (!sb_ok(P)) emu_step_kernel<128, false, 0, false>(S);
            else if (P.C & 1) emu_step_sb<false, true>(S);
            else emu_step_sb<false, false>(S);
        } else {
            if (sb_ok(P) && emu_is_shape<tmg::kFixC3>(P)) emu_step_kernel<128, true, 2, false, tmg::kFixC3>(S);
            else if (!sb_ok(P)) emu_step_kernel<128, true, 0, false>(S);
            else if (P.C & 1) emu_step_sb<true, true>(S);
            else emu_step_sb<true, false>(S);
            emu_spill<128>(S);
        }
    } else if (lean) {
        emu_step_kernel<512, false, 0, false>(S);
    } else {
        if (emu_is_shape<tmg::kFixC5>(P)) emu_step_kernel<512, true, 0, false, tmg::kFixC5>(S);
        else emu_step_kernel<512, true, 0, false>(S);
        emu_spill<512>(S);
    }
    g_spill_total += P.spill->total;
    if (deferred) emu_do_reset(P, n, board, rng, timer, eff, flags, tmg::FL_RESET);
    return 0;
}

unsigned long long emu_spills(void) { return g_spill_total; }
void emu_cover(unsigned long long *out, int clear) {
    for (int i = 0; i < tmg::CV_COUNT; i++) { out[i] = g_cover[i]; if (clear) g_cover[i] = 0; }
}
unsigned emu_status(void) { return (g_status[0] ? 1u : 0u) | (g_status[1] ? 2u : 0u) | (g_status[2] ? 4u : 0u); }

int emu_reset(int R, int C, int k, int smask, int moves, int64_t n, int8_t *board, uint64_t *rng, int32_t *timer,
              uint64_t *eff) {
    if (!g_jump_init) { tmg::build_jump_table(g_jump); g_jump_init = true; }
    tmg::Params P = make_params(R, C, k, smask, moves, g_jump);
    emu_do_reset(P, n, board, rng, timer, eff, nullptr, 0xFF);
    return 0;
}

// reset(env_mask): the masked reset_kernel launch (several envs per wave, as tmg_capi.hip do_reset)
int emu_reset_masked(int R, int C, int k, int smask, int moves, int64_t n, int8_t *board, uint64_t *rng,
                     int32_t *timer, uint64_t *eff, const uint8_t *mask, int bits) {
    if (!g_jump_init) { tmg::build_jump_table(g_jump); g_jump_init = true; }
    tmg::Params P = make_params(R, C, k, smask, moves, g_jump);
    emu_do_reset(P, n, board, rng, timer, eff, mask, bits);
    return 0;
}

int emu_effective(int R, int C, int k, int smask, int64_t n, const int8_t *board, uint64_t *eff) {
    if (!g_jump_init) { tmg::build_jump_table(g_jump); g_jump_init = true; }
    tmg::Params P = make_params(R, C, k, smask, 1, g_jump);
    if (P.N <= 128)
        run_blocks(n, sizeof(tmg::Ws<128, false>), [&] { tmg::effective_kernel<128>(P, n, board, eff); });
    else
        run_blocks(n, sizeof(tmg::Ws<512, false>), [&] { tmg::effective_kernel<512>(P, n, board, eff); });
    return 0;
}

}  // extern "C"
