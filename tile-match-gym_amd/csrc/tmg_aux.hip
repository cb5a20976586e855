// tmg_aux.hip — the callers either side of the Board transition (SURVEY.md
// §8(d,f)): the one-hot observation encoding of OneHotWrapper, the examples'
// uniform-over-effective-actions policy and the brute-force state count of
// utils.compute_num_states.  Included by
// tmg_capi.hip.  Both are plain HBM-streaming / integer kernels, one thread
// per (env, cell) and one thread per run of boards respectively.

namespace tmg {

// OneHotWrapper._one_hot_encode_board (src/tile_match_gym/wrappers.py:56-69):
// channels 0..k-1 = colour 1..k; then one channel per enabled special, in the
// order of sorted(id + 1) over {cookie: -1, v-laser: 2, h-laser: 3, bomb: 4}
// (wrappers.py:9-10, 39-46), i.e. cookie, v-laser, h-laser, bomb.  A colour-0
// (colourless / empty) cell and a normal tile set no channel of their kind.
// out: T [n][k + nsel][R][C].  One thread per cell: byte loads and each
// channel's stores are coalesced across the wave.
template <class T>
__global__ __launch_bounds__(256) void onehot_kernel(int64_t n, int N, int k, int nsel, int4 sel,
                                                     const int8_t *__restrict__ board, T *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n * N) return;
    const int64_t e = i / N;
    const int p = (int)(i - e * N);
    const int colour = board[e * 2 * N + p], type = board[e * 2 * N + N + p];
    T *o = out + e * (int64_t)(k + nsel) * N + p;
    for (int c = 0; c < k; c++) o[(int64_t)c * N] = (T)(colour == c + 1 ? 1 : 0);
    const int ids[4] = {sel.x, sel.y, sel.z, sel.w};
    for (int j = 0; j < nsel; j++) o[(int64_t)(k + j) * N] = (T)(type == ids[j] ? 1 : 0);
}

// The examples' policy (src/examples/q_learning.py:19-25: rng.choice over
// info["effective_actions"]): one action per env, uniform over the env's
// effective actions (ascending, tile_match_env.py:118-124), from a
// counter-based draw h = splitmix64(splitmix64(key * K + global env) ^ t * G)
// — the same stream as shard.synthetic_actions, so any shard layout picks the
// same actions.  The r-th set bit, r = hi32(h) * count >> 32; with no
// effective action (a finished env without autoreset) hi32(h) * A >> 32.
// One thread per env; W <= 16 mask words (A < 2 * 512); draw_row
// (tmg_board.hip) picks the r-th set bit by a branch-free binary search on
// popcounts.  The lean step kernels sample the same way in their prologue
// (sample_action); the general ones take this kernel's draw.
// One-wave workgroups: the launch sits between the group's step launches
// while the other streams' step waves fill the CUs, and a 64-thread block
// gets a slot sooner than a 256-thread one (c3-eff 2.37 vs 2.32 x 10^8,
// profiles/r06/s4).  Staging the block's mask rows through LDS for coalesced
// loads (STAGE) measured the same (2.36) and stays a template option.
constexpr int kSampleMaxW = 16;
#ifndef TMG_SAMPLE_BS
#define TMG_SAMPLE_BS 64
#endif
#ifndef TMG_SAMPLE_LDS
#define TMG_SAMPLE_LDS 0
#endif
template <int BS, bool STAGE>
__global__ __launch_bounds__(BS) void sample_effective_kernel(int64_t n, int W, int A, const uint64_t *__restrict__ eff,
                                                              uint64_t key, int64_t first_env, int32_t t,
                                                              int32_t *__restrict__ actions) {
    __shared__ uint64_t rows[STAGE ? BS * (kSampleMaxW + 1) : 1];
    const int64_t base = (int64_t)blockIdx.x * BS;
    const int64_t i = base + threadIdx.x;
    const uint64_t *m;
    if constexpr (STAGE) {
        const int Wp = W | 1;
        const int cnt = (int)((n - base) < BS ? (n - base) : BS);
        const uint64_t *src = eff + base * W;
        for (int q = threadIdx.x; q < cnt * W; q += BS) {
            const int row = q / W;
            rows[row * Wp + (q - row * W)] = src[q];
        }
        __syncthreads();
        m = rows + threadIdx.x * Wp;
    } else {
        m = eff + (i < n ? i : 0) * W;
    }
    if (i >= n) return;
    actions[i] = draw_row(m, W, A, policy_draw(key, (uint64_t)(first_env + i), t));
}

// utils.compute_num_states / is_valid_state (src/tile_match_gym/utils/utils.py:6-26):
// over every colouring of an all-normal R x C board with colours 1..k (the
// itertools.product order: cell 0 is the most significant digit), count the
// boards with no colour line (get_colour_lines() == [], board.py:149-215) and,
// of those, the ones with an effective move (possible_move, board.py:558-569).
// A board is 4-bit nibbles of one uint64 (cell p at bits 4p..4p+3, N <= 16).
// Each thread walks `per` consecutive boards with an odometer.
struct CountGeo {
    int R, C, N, k;
    uint64_t ones;      // 0x1 in every cell nibble
    uint64_t hmask;     // cells with c <= C-3
    uint64_t vmask;     // cells with r <= R-3
};

__device__ __forceinline__ uint64_t nib_eq(uint64_t d, uint64_t ones) {   // bit 4p set iff nibble p of d is 0
    return ~(d | (d >> 1) | (d >> 2) | (d >> 3)) & ones;
}

__device__ __forceinline__ bool has_line(const CountGeo &G, uint64_t x) {
    const uint64_t eh = nib_eq(x ^ (x >> 4), G.ones);                    // cell p == cell p+1
    const uint64_t ev = nib_eq(x ^ (x >> (4 * G.C)), G.ones);            // cell p == cell p+C
    const uint64_t h3 = eh & (eh >> 4) & G.hmask;
    const uint64_t v3 = ev & (ev >> (4 * G.C)) & G.vmask;
    return (h3 | v3) != 0ULL;
}

__global__ __launch_bounds__(256) void count_states_kernel(CountGeo G, uint64_t total, uint64_t per,
                                                           unsigned long long *counts) {
    __shared__ unsigned long long sh[2][256];
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t b0 = t * per;
    uint64_t playable = 0, linefree = 0;
    if (b0 < total) {
        // digits of b0, cell N-1 least significant; stored as colour - 1
        uint64_t x = 0, v = b0;
        for (int p = G.N - 1; p >= 0; p--) {
            x |= (v % (uint64_t)G.k) << (4 * p);
            v /= (uint64_t)G.k;
        }
        const uint64_t end = b0 + per < total ? b0 + per : total;
        for (uint64_t b = b0; b < end; b++) {
            if (!has_line(G, x)) {
                linefree++;
                bool mv = false;
                // vertical swaps (p, p+C), then horizontal (p, p+1) with c <= C-2
                for (int p = 0; p + G.C < G.N && !mv; p++) {
                    const uint64_t d = ((x >> (4 * p)) ^ (x >> (4 * (p + G.C)))) & 0xF;
                    mv = d && has_line(G, x ^ (d << (4 * p)) ^ (d << (4 * (p + G.C))));
                }
                for (int p = 0; p + 1 < G.N && !mv; p++) {
                    if (p % G.C == G.C - 1) continue;
                    const uint64_t d = ((x >> (4 * p)) ^ (x >> (4 * (p + 1)))) & 0xF;
                    mv = d && has_line(G, x ^ (d << (4 * p)) ^ (d << (4 * (p + 1))));
                }
                playable += mv ? 1 : 0;
            }
            // odometer: next colouring
            for (int p = G.N - 1; p >= 0; p--) {
                const uint64_t dg = (x >> (4 * p)) & 0xF;
                if (dg + 1 < (uint64_t)G.k) { x += 1ULL << (4 * p); break; }
                x &= ~(0xFULL << (4 * p));
            }
        }
    }
    sh[0][threadIdx.x] = playable;
    sh[1][threadIdx.x] = linefree;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            sh[0][threadIdx.x] += sh[0][threadIdx.x + s];
            sh[1][threadIdx.x] += sh[1][threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        atomicAdd(&counts[0], sh[0][0]);
        atomicAdd(&counts[1], sh[1][0]);
    }
}

inline CountGeo make_count_geo(int R, int C, int k) {
    CountGeo G;
    G.R = R; G.C = C; G.N = R * C; G.k = k;
    G.ones = G.hmask = G.vmask = 0;
    for (int p = 0; p < G.N; p++) {
        G.ones |= 1ULL << (4 * p);
        if (p % C <= C - 3) G.hmask |= 1ULL << (4 * p);
        if (p / C <= R - 3) G.vmask |= 1ULL << (4 * p);
    }
    return G;
}

}  // namespace tmg
