// Host build of csrc/tmg_lane.h (test infrastructure, tests/test_lane_host.py):
// the lane kernel's per-env step run env by env on the CPU, so its logic is
// checked against the oracle without a GPU.  Not a product path.
#include <stdint.h>
#define __host__
#define __device__
#define __forceinline__ inline
static long long g_iters[64];
// per-env trace of the current step (for wave-level cost models): passes / holes per cascade iteration
static int g_trace_on, g_it, g_pass[64], g_holes[64];
#define TMG_LANE_NOTE_ITERS(n) (g_iters[(n) < 63 ? (n) : 63]++)
#define TMG_LANE_NOTE_PASS() (g_trace_on && g_it < 64 ? (void)g_pass[g_it]++ : (void)0)
#define TMG_LANE_NOTE_HOLES(n) (g_trace_on && g_it < 64 ? (void)(g_holes[g_it++] = (n)) : (void)0)
#include "tmg_lane.h"

using namespace tmg::lane;

static int *g_out;          // [n][1 + 2*64]: iterations, then passes / holes per iteration
template <int R, int C, int K>
static uint32_t run(const StepIO &io, int64_t n) {
    uint8_t scratch[128];
    uint32_t st = 0;
    for (int64_t e = 0; e < n; e++) {
        g_trace_on = g_out != nullptr; g_it = 0;
        for (int i = 0; i < 64; i++) g_pass[i] = g_holes[i] = 0;
        st |= step_env<Board<R, C, K>>(io, e, scratch);
        if (g_out) {
            int *o = g_out + e * 129;
            o[0] = g_it;
            for (int i = 0; i < 64; i++) { o[1 + i] = g_pass[i]; o[65 + i] = g_holes[i]; }
        }
    }
    return st;
}
extern "C" __attribute__((visibility("default"))) void lane_host_trace(int *out) { g_out = out; }

extern "C" __attribute__((visibility("default"))) void lane_host_iters(long long *out, int clear) {
    for (int i = 0; i < 64; i++) { out[i] = g_iters[i]; if (clear) g_iters[i] = 0; }
}

extern "C" __attribute__((visibility("default"))) int lane_host_step(
    int R, int C, int K, int64_t n, int8_t *board, uint64_t *rng, int32_t *timer, int32_t *actions, int32_t *reward,
    int32_t *n_new, int32_t *n_act, uint8_t *flags, uint64_t *eff, int num_moves, int autoreset, int sample,
    uint64_t key, int64_t first, int32_t t) {
    const StepIO io{board, rng, timer, actions, reward, n_new, n_act, flags, eff, num_moves, autoreset, sample, key,
                    first, t};
#define SHAPE(r, c, k) if (R == r && C == c && K == k) return (int)run<r, c, k>(io, n);
    SHAPE(10, 10, 4)
    SHAPE(10, 10, 5)
    SHAPE(6, 8, 3)
    SHAPE(12, 10, 4)
    SHAPE(8, 16, 4)
    SHAPE(7, 8, 6)
    SHAPE(4, 4, 3)
#undef SHAPE
    return -1;
}
