// tmg_launch.h — host-side launchers of the kernels, one group per
// translation unit of tmg_kernels.hip (compiled once per TMG_TU value, in
// parallel), called by tmg_capi.hip.  Each launcher enqueues its kernel(s) on
// `s` and returns nothing; tmg_capi checks hipGetLastError afterwards.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace tmg {

struct Params;

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

// one wave per env: grid padded to 8 equal XCD blocks (wg_env0)
dim3 env_grid(int64_t n);

// TU 1 — lean step kernels (no specials, cached mask trusted), <= 128 cells;
// sb: scalar-bitboard variants (C <= 63)
void launch_step_lean128(bool sb, dim3 grid, hipStream_t s, const Params &P, const StepArgs &a);
// and the lane-per-board lean step (tmg_lane.h) for the shapes lane_shape
// accepts; its autoreset codes are the deferred ones (0, 2, 4)
bool lane_shape(const Params &P);
void launch_step_lane(hipStream_t s, const Params &P, const StepArgs &a);
constexpr int kLaneScratch = 128;      // LDS bytes per lane (a shuffle's index array, N <= 128)
// TU 2 / 3 — general <= 128-cell step kernels, C even / odd (the
// non-bitboard one lives in TU 2)
void launch_step_gen128_even(bool sb, dim3 grid, hipStream_t s, const Params &P, const StepArgs &a);
void launch_step_gen128_odd(dim3 grid, hipStream_t s, const Params &P, const StepArgs &a);
// TU 4 — 512-cell kernels
void launch_step512(bool gen, dim3 grid, hipStream_t s, const Params &P, const StepArgs &a);
// TU 7 — the spill tier (steps whose cascade outgrew the LDS lists)
void launch_spill128(hipStream_t s, const Params &P, const StepArgs &a);
void launch_spill512(hipStream_t s, const Params &P, const StepArgs &a);
void launch_reset512(dim3 grid, hipStream_t s, const Params &P, int64_t n, int8_t *board, uint64_t *rng,
                     int32_t *timer, uint64_t *eff, const uint8_t *env_mask, int mask_bits, int epw);
void launch_effective512(dim3 grid, hipStream_t s, const Params &P, int64_t n, const int8_t *board, uint64_t *eff);
// TU 5 — <= 128-cell reset / effective kernels
void launch_reset128(bool sb, dim3 grid, hipStream_t s, const Params &P, int64_t n, int8_t *board, uint64_t *rng,
                     int32_t *timer, uint64_t *eff, const uint8_t *env_mask, int mask_bits, int epw);
void launch_effective128(dim3 grid, hipStream_t s, const Params &P, int64_t n, const int8_t *board, uint64_t *eff);
// TU 6 — the callers either side (tmg_aux.hip)
void launch_onehot(hipStream_t s, int64_t n, int N, int k, int nsel, int4 sel, const int8_t *board, void *out,
                   int dtype);
void launch_sample_effective(hipStream_t s, int64_t n, int W, int A, const uint64_t *eff, uint64_t key,
                             int64_t first_env, int32_t t, int32_t *actions);
void launch_count_states(int R, int C, int k, uint64_t total, uint64_t per, uint64_t threads,
                         unsigned long long *counts);

// bytes of one spill-kernel wave's worst-case global-memory lists
size_t spill_ws_bytes(int maxn);

}  // namespace tmg
