/*
 * tmg.h — C ABI of libtmg.so, the MI355X (gfx950) batched tile-match Board.
 *
 * The reference (akshilpatel/tile-match-gym v1.0.6) has no FFI: its hot path is
 * the Python class API below, and this ABI is what a binding of that path
 * binds (the ctypes stub lives in tile_match_gym_amd/_native.py; see
 * INTEGRATION.md).  Each entry point cites the reference interface it replaces.
 *
 * Batched state (device memory, owned by the caller, e.g. PyTorch tensors):
 *   board  int8   [n][2][R][C]   plane 0 colour (0 empty/colourless, 1..k),
 *                                plane 1 type (0 empty, 1 normal, 2 v-laser,
 *                                3 h-laser, 4 bomb, -1 cookie)   board.py:18-25,96
 *   rng    uint64 [n][5]         numpy PCG64 per env: state lo/hi, inc lo/hi,
 *                                has_uint32<<32 | uinteger       tile_match_env.py:49
 *   timer  int32  [n]            moves taken this episode         tile_match_env.py:88,100
 *   eff    uint64 [n][W]         effective-action bitmask, W = ceil(A/64),
 *                                A = 2RC-R-C; bit a of word a/64  tile_match_env.py:118-124
 * Per-step outputs (device memory):
 *   reward int32 [n]   num_eliminations                            board.py:330-395
 *   n_new  int32 [n]   info["num_new_specials"]
 *   n_act  int32 [n]   info["num_specials_activated"]
 *   flags  uint8 [n]   bit0 done, bit1 is_combination_match, bit2 shuffled,
 *                      bit3 autoreset ran, bit7 error (step after done / bad
 *                      action, or an internal safety cap)  tile_match_env.py:94-95
 *                      (bit6, capacity overflow, is no longer produced: a step
 *                      whose cascade outgrows the kernels' LDS lists is re-run
 *                      on worst-case lists, and the queue of such steps holds
 *                      every env of the launch)
 *
 * Errors: 0 = ok, negative = error; tmg_last_error() gives a thread-local
 * message.  All launches are asynchronous on `stream` (a hipStream_t; NULL =
 * default stream).  Not re-entrant per context.
 */
#ifndef TMG_H
#define TMG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tmg_ctx tmg_ctx;

#if defined(__GNUC__) || defined(__clang__)
#define TMG_API __attribute__((visibility("default")))
#else
#define TMG_API
#endif

/* Special-tile mask bits (Board(colourless_specials=..., colour_specials=...), board.py:42-61). */
#define TMG_SPECIAL_COOKIE 1u
#define TMG_SPECIAL_VLASER 2u
#define TMG_SPECIAL_HLASER 4u
#define TMG_SPECIAL_BOMB   8u

#define TMG_FLAG_DONE      0x01u
#define TMG_FLAG_COMBO     0x02u
#define TMG_FLAG_SHUFFLED  0x04u
#define TMG_FLAG_RESET     0x08u
#define TMG_FLAG_OVERFLOW  0x40u   /* not produced since ABI 3 (kept for old callers) */
#define TMG_FLAG_ERROR     0x80u

/* Replaces TileMatchEnv.__init__ / Board.__init__ (tile_match_env.py:17-77,
 * board.py:42-93): fixes the shape, colours, specials and episode length for a
 * batch, builds the action->coords table (board.py:77-93) and the PCG64
 * jump-ahead table on `device`. */
TMG_API int tmg_create(tmg_ctx **out, int device, int rows, int cols, int colours,
               uint32_t specials_mask, int num_moves);

/* A context for tmg_effective only, on any rows x cols board of up to 512
 * cells (no viability test, no colours or specials): the module-level
 * is_move_effective(board, c1, c2) / Board.possible_move(grid) of the
 * reference (board.py:558-569, 735-787), which accept any board.  Every other
 * call on it fails. */
TMG_API int tmg_create_scan(tmg_ctx **out, int device, int rows, int cols);

/* Frees the context's device tables.  Never frees caller buffers. */
TMG_API int tmg_destroy(tmg_ctx *ctx);

/* Replaces TileMatchEnv.reset (tile_match_env.py:84-91 -> Board.generate_board,
 * board.py:95-131) for every env i with env_mask == NULL or env_mask[i] != 0:
 * generates a board from the env's RNG stream (continuing it, like reset()
 * without a seed), sets timer = 0 and writes the effective-action mask. */
TMG_API int tmg_reset(tmg_ctx *ctx, int64_t n, int8_t *board, uint64_t *rng, int32_t *timer,
              uint64_t *eff, const uint8_t *env_mask, void *stream);

/* Replaces TileMatchEnv.step (tile_match_env.py:93-112 -> Board.move,
 * board.py:330-395) for n envs at once.  actions[i] in [0, A).
 * trust_eff != 0: eff holds the mask a tmg_step / tmg_reset of this library
 *   wrote for the current boards (the effectiveness test of board.py:352 is
 *   then a bit lookup, and the boards are known to hold no line, which bounds
 *   the first line search); pass 0 after editing boards by hand, also when the
 *   mask was then recomputed by tmg_effective.
 * autoreset != 0: an env whose episode ends is regenerated in the same call
 *   (continuing its RNG stream, == reset() without a seed); reward / flags
 *   still describe the final move and flag bit3 is set.  With autoreset == 0
 *   a finished env writes an all-zero eff mask (tile_match_env.py:119-120) and
 *   a further step sets TMG_FLAG_ERROR without touching its state. */
TMG_API int tmg_step(tmg_ctx *ctx, int64_t n, int8_t *board, uint64_t *rng, int32_t *timer,
             const int32_t *actions, int32_t *reward, int32_t *n_new, int32_t *n_act,
             uint8_t *flags, uint64_t *eff, int trust_eff, int autoreset, void *stream);

/* Step plans: one host call per batched step of a fixed set of buffers
 * (TileMatchEnv.step, tile_match_env.py:93-124, for every env of the batch),
 * with the batch split into env groups on their own streams, the callers'
 * per-step outputs written in the kernels' own write-back, and optionally
 * the examples' policy sampled inside the step.
 *
 * tmg_plan_create binds the state / output buffers (as for tmg_step) and
 * `groups` contiguous env groups: group g = envs [bounds[g], bounds[g+1])
 * (bounds[0] = 0, bounds[groups] = n), stepped on streams[g] (NULL: the
 * stream of each tmg_plan_step / tmg_plan_join call).  The plan keeps
 * the pointers; the caller keeps the buffers and streams alive until
 * tmg_plan_destroy. */
typedef struct tmg_plan tmg_plan;
TMG_API int tmg_plan_create(tmg_plan **out, tmg_ctx *ctx, int64_t n, int8_t *board, uint64_t *rng, int32_t *timer,
                            int32_t *reward, int32_t *n_new, int32_t *n_act, uint8_t *flags, uint64_t *eff,
                            int groups, const int64_t *bounds, void *const *streams);

/* What each tmg_plan_step does (default: autoreset 1, no policy, no extra
 * outputs).
 *   autoreset: 0 none (as tmg_step's 0); 1 same step (as tmg_step's 1);
 *     2 next step (gymnasium.vector's default): an env whose episode ends is
 *     left as with 0 (terminated, all-zero mask), and the next call resets it
 *     (Board regenerated from its stream) instead of stepping it: its action
 *     is ignored, reward / n_new / n_act / flags 0 but TMG_FLAG_RESET.
 *   policy != 0: actions[] is an output: env i plays a uniform draw over its
 *     effective actions, exactly tmg_sample_effective(key, first_env + i, t)
 *     (src/examples/q_learning.py:19-25), drawn inside the step (the lean
 *     kernels) or by the sampler kernel enqueued right before it.
 *   onehot / onehot_dtype: fused OneHotWrapper planes, as tmg_step_onehot.
 *   terminated [n][4] bytes: terminated, is_combination_match, shuffled,
 *     error (0/1 each; the reference's step info, tile_match_env.py:102-112).
 *   action_mask [n][A] bytes: 0/1 of the effective-action bitmask (the
 *     reference's info["effective_actions"] as a mask), kept up to date: a
 *     call rewrites the rows whose mask changed.  The caller initialises it
 *     (e.g. after tmg_reset) from the bitmask.
 *   moves_left [n]: num_moves - timer after the call (tile_match_env.py:114-116).
 *   final_board [n][2][R][C]: with autoreset 1, the board each env whose
 *     episode ended had before its regeneration (rows of other envs untouched).
 *   board32 [n][2][R][C] int32: the boards in the reference's observation
 *     dtype (tile_match_env.py:52-77), kept up to date like action_mask
 *     (initialise it after a reset).
 * Any output pointer may be NULL (not written). */
TMG_API int tmg_plan_config(tmg_plan *plan, int autoreset, int policy, uint64_t key, int64_t first_env,
                            void *onehot, int onehot_dtype, uint8_t *terminated, uint8_t *action_mask,
                            int64_t *moves_left, int8_t *final_board, int32_t *board32);

/* One step of every env: with fork != 0 the group streams first wait for
 * the work queued on `stream` (an event; fork = 0 when nothing queued there
 * since the previous step is read by this one, e.g. back-to-back steps on
 * actions staged beforehand), then each group's launches are enqueued on its
 * stream.  Nothing waits for them: call tmg_plan_join before reading the
 * results on `stream`.  actions [n] (input, or the policy's output) must stay
 * valid until then.  t: the step counter of the policy draw.  trust_eff: as
 * tmg_step. */
TMG_API int tmg_plan_step(tmg_plan *plan, int32_t *actions, int32_t t, int trust_eff, int fork, void *stream);

/* `stream` waits for every group's queued work (events). */
TMG_API int tmg_plan_join(tmg_plan *plan, void *stream);
TMG_API int tmg_plan_destroy(tmg_plan *plan);

/* `steps` consecutive tmg_plan_step calls (step k: actions[k], t[k]; trust_eff
 * for the first, 1 after it) and the final tmg_plan_join, captured on
 * `stream` (a created stream, not NULL) into a HIP graph: tmg_graph_launch
 * then enqueues all of them on a stream with one call, the env groups'
 * launches still overlapping across the steps inside it.  Nothing runs at
 * capture time.  The graph keeps the plan's buffers, the action pointers and
 * the configuration of the moment; re-capture after tmg_plan_config. */
typedef struct tmg_graph tmg_graph;
TMG_API int tmg_plan_capture(tmg_plan *plan, int steps, int32_t *const *actions, const int32_t *t, int trust_eff,
                             void *stream, tmg_graph **out);
TMG_API int tmg_graph_launch(tmg_graph *graph, void *stream);
TMG_API int tmg_graph_destroy(tmg_graph *graph);

/* Replaces TileMatchEnv._get_effective_actions (tile_match_env.py:118-124,
 * is_move_effective board.py:735-787) as a bitmask, ignoring the timer. */
TMG_API int tmg_effective(tmg_ctx *ctx, int64_t n, const int8_t *board, uint64_t *eff, void *stream);

/* Output element types of tmg_onehot. */
#define TMG_DTYPE_F32 0
#define TMG_DTYPE_U8  1
#define TMG_DTYPE_I32 2

/* Replaces OneHotWrapper._one_hot_encode_board (src/tile_match_gym/wrappers.py:56-69)
 * for n boards: out[n][C_oh][R][C] with C_oh = tmg_onehot_channels(ctx) =
 * colours + #enabled specials.  Channel c < colours is (colour == c + 1); then
 * one channel per enabled special in the order cookie, v-laser, h-laser, bomb
 * (sorted(type id + 1), wrappers.py:39-46), set where the type equals it.
 * The reference builds float64; out_dtype picks f32 / u8 / i32 (TMG_DTYPE_*).
 * Asynchronous on `stream`. */
TMG_API int tmg_onehot(tmg_ctx *ctx, int64_t n, const int8_t *board, void *out, int out_dtype, void *stream);
TMG_API int tmg_onehot_channels(const tmg_ctx *ctx);

/* tmg_step / tmg_reset with the one-hot planes fused into the kernels' own
 * write-back (OneHotWrapper.observation, wrappers.py:50-69,
 * applied to every step's obs): `onehot` is out[n][C_oh][R][C] as for
 * tmg_onehot and must already hold the planes of the current boards (from a
 * tmg_reset_onehot or a tmg_onehot call); a step rewrites the planes of every
 * board it changes (any board when trust_eff == 0), tmg_reset_onehot those of
 * every board it generates.  onehot == NULL: plain tmg_step / tmg_reset. */
TMG_API int tmg_step_onehot(tmg_ctx *ctx, int64_t n, int8_t *board, uint64_t *rng, int32_t *timer,
                            const int32_t *actions, int32_t *reward, int32_t *n_new, int32_t *n_act,
                            uint8_t *flags, uint64_t *eff, int trust_eff, int autoreset, void *onehot,
                            int onehot_dtype, void *stream);
TMG_API int tmg_reset_onehot(tmg_ctx *ctx, int64_t n, int8_t *board, uint64_t *rng, int32_t *timer,
                             uint64_t *eff, const uint8_t *env_mask, void *onehot, int onehot_dtype, void *stream);

/* The examples' policy over info["effective_actions"] (src/examples/q_learning.py:19-25,
 * qrdqn.py:58), on device: actions[i] uniform over env i's effective actions
 * (the ascending list of tile_match_env.py:118-124, read from the bitmask eff
 * [n][W]), picked by a counter-based draw of (key, first_env + i, t) — the
 * stream of the bench's synthetic actions, so shard layouts agree.  An env with
 * no effective action gets the uniform draw over all A actions.  Asynchronous
 * on `stream`. */
TMG_API int tmg_sample_effective(tmg_ctx *ctx, int64_t n, const uint64_t *eff, uint64_t key, int64_t first_env,
                                 int32_t t, int32_t *actions, void *stream);

/* Replaces utils.compute_num_states (src/tile_match_gym/utils/utils.py:6-26) on
 * `device`: over all colours^(rows*cols) colourings of an all-normal board,
 * num_line_free = boards with no colour line, num_playable = those that also
 * have an effective move (the reference's two returned sums, in the order
 * (playable, line_free)).  Needs rows*cols <= 16.  Synchronous. */
TMG_API int tmg_count_states(int device, int rows, int cols, int colours, uint64_t *num_playable,
                             uint64_t *num_line_free);

/* Sticky status of the context: the OR, over every env of every call since
 * the last clear, of TMG_STATUS_INTERNAL (a safety cap or an inconsistent
 * board ended a step with TMG_FLAG_ERROR), TMG_STATUS_OVERFLOW (not produced
 * since ABI 3) and TMG_STATUS_CALLER (a step after done / a bad action).
 * Waits for the device; clear != 0 then zeroes it.  The reference raises at
 * the point of failure (tile_match_env.py:94-95, board.py:349-350); a batch
 * reports through this word and the per-env flags instead. */
#define TMG_STATUS_INTERNAL 1u
#define TMG_STATUS_OVERFLOW 2u
#define TMG_STATUS_CALLER   4u
TMG_API int tmg_status(tmg_ctx *ctx, uint32_t *status, int clear);

/* Number of steps, since the context was created, whose cascade outgrew the
 * general kernels' LDS lists and was re-run on global-memory lists sized for
 * the worst case (spill_kernel; diagnostic — results are exact either way;
 * the queue of such steps is sized per stream for the largest launch).
 * Waits for the device. */
TMG_API int tmg_spills(tmg_ctx *ctx, uint64_t *count);

/* 1 when some rows x cols board with `colours` colours is line-free and has an
 * effective move, i.e. the reference's generate_board terminates
 * (board.py:102-109); tmg_create refuses the other shapes. */
TMG_API int tmg_viable(int rows, int cols, int colours);

/* Number of actions A = 2RC - R - C (tile_match_env.py:58) and mask words W. */
TMG_API int tmg_num_actions(const tmg_ctx *ctx);
TMG_API int tmg_mask_words(const tmg_ctx *ctx);

/* Message for the last failing call on this thread. */
TMG_API const char *tmg_last_error(void);

/* ABI version (bumped on any signature change). */
TMG_API int tmg_abi_version(void);

/* "src=<sha256 of the library's sources>;variant=<product|diagnostic name>":
 * the loader compares the hash with the sources next to the library and
 * refuses a stale build. */
TMG_API const char *tmg_build_info(void);

#ifdef __cplusplus
}
#endif

#endif /* TMG_H */
