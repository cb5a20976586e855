// tmg_kernels.hip — kernel instantiations and their host launchers
// (tmg_launch.h).  Compiled once per translation unit, TMG_TU = 1..7, so the
// heavy template instantiations build in parallel; each TU registers only its
// own kernels.
#include <hip/hip_runtime.h>

#include "tmg_board.hip"
#include "tmg_launch.h"
#if TMG_TU == 1
#include "tmg_lane.h"
#endif
#if TMG_TU == 6
#include "tmg_aux.hip"      // non-template kernels: one TU only
#endif

#ifndef TMG_TU
#error "compile tmg_kernels.hip with -DTMG_TU=1..7"
#endif

namespace tmg {

namespace {

template <int MAXN, bool GEN, int NB, bool CODD, int FIX = kNoFix>
void step_one(dim3 grid, hipStream_t s, const Params &P, const StepArgs &a) {
    const size_t lds = sizeof(Ws<MAXN, GEN>);
    hipLaunchKernelGGL((step_kernel<MAXN, GEN, NB, CODD, FIX>), grid, dim3(64), lds, s, P, a.n, a.board, a.rng,
                       a.timer, a.actions, a.reward, a.n_new, a.n_act, a.flags, a.eff, a.trust_eff, a.autoreset);
}
// whether P is the shape a FIX instantiation was compiled for
template <int FIX>
bool is_shape(const Params &P) {
    const int sm = (FIX & 255) == kFixAnySpecials ? kFixAnySpecials : P.smask;
    return shape_fix(P.R, P.C, P.k, sm) == FIX;
}

// scalar-bitboard variants: NB colour planes (sb_planes(k))
template <bool GEN, bool CODD>
void step_sb(dim3 grid, hipStream_t s, const Params &P, const StepArgs &a) {
    switch (sb_planes(P.k)) {
    case 1: step_one<128, GEN, 1, CODD>(grid, s, P, a); break;
    case 2: step_one<128, GEN, 2, CODD>(grid, s, P, a); break;
    case 3: step_one<128, GEN, 3, CODD>(grid, s, P, a); break;
    default: step_one<128, GEN, 4, CODD>(grid, s, P, a); break;
    }
}

template <int MAXN>
void spill_one(hipStream_t s, const Params &P, const StepArgs &a) {
    const size_t lds = sizeof(Ws<MAXN, false>);
    hipLaunchKernelGGL((spill_kernel<MAXN>), dim3(kSpillWaves), dim3(64), lds, s, P, a.n, a.board, a.rng, a.timer,
                       a.actions, a.reward, a.n_new, a.n_act, a.flags, a.eff, a.trust_eff, a.autoreset);
}

template <int MAXN, int NB, bool CODD, int FIX = kNoFix>
void reset_one(dim3 grid, hipStream_t s, const Params &P, int64_t n, int8_t *board, uint64_t *rng, int32_t *timer,
               uint64_t *eff, const uint8_t *env_mask, int mask_bits, int epw) {
    const size_t lds = sizeof(Ws<MAXN, false>);
    hipLaunchKernelGGL((reset_kernel<MAXN, NB, CODD, FIX>), grid, dim3(64), lds, s, P, n, board, rng, timer, eff,
                       env_mask, mask_bits, epw);
}

template <int MAXN>
void effective_one(dim3 grid, hipStream_t s, const Params &P, int64_t n, const int8_t *board, uint64_t *eff) {
    hipLaunchKernelGGL(effective_kernel<MAXN>, grid, dim3(64), sizeof(Ws<MAXN, false>), s, P, n,
                       board, eff);
}

}  // namespace

#if TMG_TU == 1
// The lane-per-board lean step (tmg_lane.h): EPW envs per one-wave
// workgroup (lane i < EPW = env EPW * group + i), the groups in wg_env's
// XCD-blocked order.  Each lane keeps kLaneScratch bytes of LDS for a
// shuffle's index array (the rare path).  A wave lasts as long as its longest
// cascade, so a launch too small to give each SIMD two waves of 64 takes 32
// envs per wave (c2's 21 845-env group launches: c2-eff +4.5 %; at c4's
// 43 690 the 64-env waves are 4.5 % faster, profiles/r06/s12/).
#ifndef TMG_LANE_WPE
#define TMG_LANE_WPE 0          // amdgpu_waves_per_eu(WPE, WPE) when > 0 (A/B)
#endif
#ifndef TMG_LANE_LDS
#define TMG_LANE_LDS 0          // extra LDS bytes per workgroup (A/B: caps workgroups per CU)
#endif
#ifndef TMG_LANE_SMALL
#define TMG_LANE_SMALL 32768    // launches below this many envs: 32 envs per wave
#endif
template <int R, int C, int K, int EPW>
__global__ __launch_bounds__(64)
#if TMG_LANE_WPE > 0
__attribute__((amdgpu_waves_per_eu(TMG_LANE_WPE, TMG_LANE_WPE)))
#endif
void lane_step_kernel(Params P_, int64_t n, int8_t *__restrict__ board, uint64_t *__restrict__ rng,
                      int32_t *__restrict__ timer, int32_t *__restrict__ actions, int32_t *__restrict__ reward,
                      int32_t *__restrict__ n_new, int32_t *__restrict__ n_act, uint8_t *__restrict__ flags,
                      uint64_t *__restrict__ eff, int autoreset) {
    __shared__ uint8_t scratch[EPW * kLaneScratch + TMG_LANE_LDS];
    const Params &P = TMG_KERNARG_PARAMS(P_);
    const int lane = threadIdx.x & 63;
    const int64_t e = wg_env() * EPW + lane;
    if (lane >= EPW || e >= n) return;
    const lane::StepIO io{board, rng, timer, actions, reward, n_new, n_act, flags, eff,
                          P.num_moves, autoreset, P.sample, P.pol_key, P.pol_first, P.pol_t};
    const uint32_t st = lane::step_env<lane::Board<R, C, K>>(io, e, scratch + lane * kLaneScratch);
    if (st & lane::LS_INTERNAL) P.status[0] = 1u;
    if (st & lane::LS_CALLER) P.status[2] = 1u;
}

bool lane_shape(const Params &P) {
    return P.smask == 0 && P.R == 10 && P.C == 10 && (P.k == 4 || P.k == 5);
}

template <int K, int EPW>
void lane_one(hipStream_t s, const Params &P, const StepArgs &a) {
    const dim3 grid = env_grid((a.n + EPW - 1) / EPW);
    int32_t *act = const_cast<int32_t *>(a.actions);            // the policy writes its draws back
    hipLaunchKernelGGL((lane_step_kernel<10, 10, K, EPW>), grid, dim3(64), 0, s, P, a.n, a.board, a.rng, a.timer,
                       act, a.reward, a.n_new, a.n_act, a.flags, a.eff, a.autoreset);
}

void launch_step_lane(hipStream_t s, const Params &P, const StepArgs &a) {
    const bool small = a.n < TMG_LANE_SMALL;
    if (P.k == 4) small ? lane_one<4, 32>(s, P, a) : lane_one<4, 64>(s, P, a);
    else small ? lane_one<5, 32>(s, P, a) : lane_one<5, 64>(s, P, a);
}

void launch_step_lean128(bool sb, dim3 grid, hipStream_t s, const Params &P, const StepArgs &a) {
    if (sb && is_shape<kFixC2>(P)) { step_one<128, false, 2, false, kFixC2>(grid, s, P, a); return; }
    if (!sb) step_one<128, false, 0, false>(grid, s, P, a);
    else if (P.C & 1) step_sb<false, true>(grid, s, P, a);
    else step_sb<false, false>(grid, s, P, a);
}
#endif

#if TMG_TU == 2
void launch_step_gen128_even(bool sb, dim3 grid, hipStream_t s, const Params &P, const StepArgs &a) {
    if (sb && is_shape<kFixC3>(P)) step_one<128, true, 2, false, kFixC3>(grid, s, P, a);
    else if (sb) step_sb<true, false>(grid, s, P, a);
    else step_one<128, true, 0, false>(grid, s, P, a);
}
#endif

#if TMG_TU == 7
void launch_spill128(hipStream_t s, const Params &P, const StepArgs &a) { spill_one<128>(s, P, a); }
void launch_spill512(hipStream_t s, const Params &P, const StepArgs &a) { spill_one<512>(s, P, a); }
#endif

#if TMG_TU == 3
void launch_step_gen128_odd(dim3 grid, hipStream_t s, const Params &P, const StepArgs &a) {
    step_sb<true, true>(grid, s, P, a);
}
#endif

#if TMG_TU == 4
void launch_step512(bool gen, dim3 grid, hipStream_t s, const Params &P, const StepArgs &a) {
    if (gen && is_shape<kFixC5>(P)) step_one<512, true, 0, false, kFixC5>(grid, s, P, a);
    else if (gen) step_one<512, true, 0, false>(grid, s, P, a);
    else step_one<512, false, 0, false>(grid, s, P, a);
}

void launch_reset512(dim3 grid, hipStream_t s, const Params &P, int64_t n, int8_t *board, uint64_t *rng,
                     int32_t *timer, uint64_t *eff, const uint8_t *env_mask, int mask_bits, int epw) {
    // NB = colour bit-planes of the row-plane generate (bp_generate)
    if (is_shape<kFixReset20>(P)) { reset_one<512, 3, false, kFixReset20>(grid, s, P, n, board, rng, timer, eff, env_mask, mask_bits, epw); return; }
    switch (sb_planes(P.k)) {
    case 1: reset_one<512, 1, false>(grid, s, P, n, board, rng, timer, eff, env_mask, mask_bits, epw); break;
    case 2: reset_one<512, 2, false>(grid, s, P, n, board, rng, timer, eff, env_mask, mask_bits, epw); break;
    case 3: reset_one<512, 3, false>(grid, s, P, n, board, rng, timer, eff, env_mask, mask_bits, epw); break;
    default: reset_one<512, 4, false>(grid, s, P, n, board, rng, timer, eff, env_mask, mask_bits, epw); break;
    }
}
void launch_effective512(dim3 grid, hipStream_t s, const Params &P, int64_t n, const int8_t *board, uint64_t *eff) {
    effective_one<512>(grid, s, P, n, board, eff);
}
#endif

#if TMG_TU == 5
void launch_reset128(bool sb, dim3 grid, hipStream_t s, const Params &P, int64_t n, int8_t *board, uint64_t *rng,
                     int32_t *timer, uint64_t *eff, const uint8_t *env_mask, int mask_bits, int epw) {
    if (!sb) { reset_one<128, 0, false>(grid, s, P, n, board, rng, timer, eff, env_mask, mask_bits, epw); return; }
    if (is_shape<kFixReset10>(P)) { reset_one<128, 2, false, kFixReset10>(grid, s, P, n, board, rng, timer, eff, env_mask, mask_bits, epw); return; }
    const bool codd = P.C & 1;
    switch (sb_planes(P.k)) {
    case 1: codd ? reset_one<128, 1, true>(grid, s, P, n, board, rng, timer, eff, env_mask, mask_bits, epw)
                 : reset_one<128, 1, false>(grid, s, P, n, board, rng, timer, eff, env_mask, mask_bits, epw); break;
    case 2: codd ? reset_one<128, 2, true>(grid, s, P, n, board, rng, timer, eff, env_mask, mask_bits, epw)
                 : reset_one<128, 2, false>(grid, s, P, n, board, rng, timer, eff, env_mask, mask_bits, epw); break;
    case 3: codd ? reset_one<128, 3, true>(grid, s, P, n, board, rng, timer, eff, env_mask, mask_bits, epw)
                 : reset_one<128, 3, false>(grid, s, P, n, board, rng, timer, eff, env_mask, mask_bits, epw); break;
    default: codd ? reset_one<128, 4, true>(grid, s, P, n, board, rng, timer, eff, env_mask, mask_bits, epw)
                  : reset_one<128, 4, false>(grid, s, P, n, board, rng, timer, eff, env_mask, mask_bits, epw); break;
    }
}
void launch_effective128(dim3 grid, hipStream_t s, const Params &P, int64_t n, const int8_t *board, uint64_t *eff) {
    effective_one<128>(grid, s, P, n, board, eff);
}
#endif

#if TMG_TU == 6
void launch_onehot(hipStream_t s, int64_t n, int N, int k, int nsel, int4 sel, const int8_t *board, void *out,
                   int dtype) {
    const int64_t cells = n * N;
    const dim3 grid((unsigned)((cells + 255) / 256)), block(256);
    switch (dtype) {
    case 0: hipLaunchKernelGGL(onehot_kernel<float>, grid, block, 0, s, n, N, k, nsel, sel, board, (float *)out); break;
    case 1: hipLaunchKernelGGL(onehot_kernel<uint8_t>, grid, block, 0, s, n, N, k, nsel, sel, board, (uint8_t *)out); break;
    default: hipLaunchKernelGGL(onehot_kernel<int32_t>, grid, block, 0, s, n, N, k, nsel, sel, board, (int32_t *)out); break;
    }
}
void launch_sample_effective(hipStream_t s, int64_t n, int W, int A, const uint64_t *eff, uint64_t key,
                             int64_t first_env, int32_t t, int32_t *actions) {
    constexpr int BS = TMG_SAMPLE_BS;
    const dim3 grid((unsigned)((n + BS - 1) / BS)), block(BS);
    hipLaunchKernelGGL((sample_effective_kernel<BS, TMG_SAMPLE_LDS != 0>), grid, block, 0, s, n, W, A, eff, key,
                       first_env, t, actions);
}
void launch_count_states(int R, int C, int k, uint64_t total, uint64_t per, uint64_t threads,
                         unsigned long long *counts) {
    const CountGeo G = make_count_geo(R, C, k);
    hipLaunchKernelGGL(count_states_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, 0, G, total, per,
                       counts);
}
#endif

}  // namespace tmg
