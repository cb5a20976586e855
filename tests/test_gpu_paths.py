"""Rare RNG and playability paths, per kernel variant, on the MI355X.

numpy's Generator.integers(1, k+1) (board.py:97 generate_board, :129
remove_colour_lines, :239 refill) rejects a 32-bit word with probability
<= k / 2^32, so random seeds never reach the device's exact replays of a
rejected draw; and the shuffles of the "while not possible_move()" loops
(board.py:102-106 in generate_board, :381-391 in move) need boards with many
colours and few moves.  Each configuration below runs one kernel variant's
step and reset paths:

* rollouts with the effective-action policy (every step changes the board,
  so in-move shuffles come up) and short episodes (num_moves = 10, so every
  env regenerates its board every 10 steps);
* before every 5th step each env's PCG64 stream is moved
  (tests/rejection_states.py words_rejecting_at) so that one of its next
  draws is a rejected word: near positions land in the step's refill, far
  ones before an autoreset step in generate_board; half of the crafted states
  hold a buffered half-word (so "the draw right after it" is covered);
* on the product library every field of every env at every step equals the
  oracle (tmg_oracle.c, pinned by the reference's goldens);
* the same trajectories on the TMG_COVER build count the branch hits per
  site: shuffles in moves / in generate_board, rejections replayed by
  draw_colours / redone by the row-plane generate.
"""
import os

import numpy as np
import pytest
import torch

from deep_rollouts import COVER_LIB, specials
from oracle import oracle as orc
from rejection_states import words_rejecting_at

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
KEY = 4242
MOVES = 10

# name: (R, C, k, smask, envs, steps, sites that must be hit)
VARIANTS = {
    # step_kernel<128, false, NB> (lean, scalar bitboards) + its inline autoreset (bp_generate)
    "lean_sb_5x6k7": (5, 6, 7, 0, 2048, 40, ("shuffle", "shuffle_gen", "reject", "reject_gen")),
    # step_kernel<128, true, NB> (specials) + the masked reset_kernel<128, NB>
    "gen_sb_6x6k7": (6, 6, 7, 14, 2048, 40, ("shuffle", "shuffle_gen", "reject", "reject_gen")),
    # step_kernel<512, false> + reset_kernel<512, NB>
    "lean_512_9x15k15": (9, 15, 15, 0, 2048, 40, ("shuffle", "shuffle_gen", "reject", "reject_gen")),
    # step_kernel<512, true> (the c5 kernel) + reset_kernel<512, NB>
    "gen_512_11x12k10": (11, 12, 10, 14, 2048, 40, ("shuffle", "reject", "reject_gen")),
    "c5_20x20k6": (20, 20, 6, 15, 1024, 30, ("reject", "reject_gen")),
    # C > 32: generate_board's exact draw-by-draw path (no row planes)
    "wide_512_3x45k7": (3, 45, 7, 9, 2048, 40, ("shuffle", "reject")),
}
FIELDS = ("board", "rng", "timer", "eff", "reward", "n_new", "n_act", "flags")


def _host(env, f):
    if f == "rng":
        return env.rng_words()
    v = getattr(env, f).cpu().numpy()
    return v.view(np.uint64) if f == "eff" else v


def _inject(t, n, rs):
    """Draw positions of the crafted rejections before step t (None: none)."""
    if t % MOVES == MOVES - 1:               # the autoreset step: refill first, then generate_board
        return rs.integers(0, 240, n), rs.random(n) < 0.5
    if t % 5 == 1:                           # a step's refill
        return rs.integers(0, 8, n), rs.random(n) < 0.5
    return None


def _rollout(name, lib_path=None, ref=True):
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    R, C, k, sm, n, steps, _ = VARIANTS[name]
    cl, co = specials(sm)
    base = 20_000 + 10_000 * sorted(VARIANTS).index(name)
    env = TileMatchVecEnv(n, R, C, k, MOVES, cl, co, seeds=range(base, base + n), device=DEV, lib_path=lib_path)
    o = orc.OracleBatch(R, C, k, sm, MOVES, env.rng_words().copy(), threads=16) if ref else None
    env.reset()
    if o is not None:
        o.reset()
    rs = np.random.default_rng(base)
    A = env.num_actions
    shuffled = 0
    for t in range(steps):
        inj = _inject(t, n, rs)
        if inj is not None:
            w = words_rejecting_at(env.rng_words(), inj[0], buffered=inj[1])
            env.rng.copy_(torch.from_numpy(w.view(np.int64)).to(DEV))
            if o is not None:
                o.rng[:] = w
        env.step_effective(t, key=KEY)
        env.join()
        if o is not None:
            from oracle.policy_np import sample_effective_np
            o.step(sample_effective_np(o.eff, A, KEY, 0, t), autoreset=True)
            for f in FIELDS:
                got, want = _host(env, f), getattr(o, f)
                if not np.array_equal(got, want):
                    bad = np.nonzero((got.reshape(n, -1) != want.reshape(n, -1)).any(axis=1))[0]
                    raise AssertionError(f"{name} step {t}: {f} differs in {bad.size} envs, first {bad[:5]}")
            shuffled += int(((o.flags & 4) != 0).sum())
    torch.cuda.synchronize()
    return env, shuffled


@pytest.mark.parametrize("name", sorted(VARIANTS))
def test_rare_paths_vs_oracle(name):
    """Product library: every field of every env at every step equals the oracle."""
    env, shuffled = _rollout(name)
    assert env.status() == 0
    if "shuffle" in VARIANTS[name][6]:
        assert shuffled > 0, "the rollout was meant to shuffle inside moves"
    env.close()


@pytest.mark.parametrize("name", sorted(VARIANTS))
def test_rare_paths_taken(name):
    """TMG_COVER build, same trajectories: each listed site was hit."""
    from tile_match_gym_amd import _native
    assert os.path.exists(COVER_LIB), "build() makes libtmg_cover.so"
    env, _ = _rollout(name, lib_path=COVER_LIB, ref=False)
    c = env.ctx.cover()
    counts = {nm: int(c[i]) for i, nm in enumerate(_native.COVER_NAMES)}
    out = os.environ.get("TMG_EVIDENCE_DIR")
    if out:
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, f"rare_paths_{name}.txt"), "w") as f:
            f.write(repr(counts) + "\n")
    assert env.status() == 0
    missing = {s: counts[s] for s in VARIANTS[name][6] if counts[s] == 0}
    assert not missing, f"{name}: sites never taken: {missing} (counts {counts})"
    env.close()


# (R, C, k, smask): the lean 128-cell reset, the 10x10 k4 reset specialised for c3, the c5 reset
MASKED = [(5, 6, 7, 0), (10, 10, 4, 14), (20, 20, 6, 15)]


@pytest.mark.parametrize("shape", MASKED)
def test_masked_reset_subsets_vs_oracle(shape):
    """reset(env_mask=...) (tile_match_env.py:84-91 for the selected envs only):
    a masked reset_kernel launch takes several envs per wave (kMaskedResetEnvs*);
    random subsets, whole groups and a ragged tail (n not a multiple of 8) all
    regenerate exactly the selected boards, and leave every other env as it was."""
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    R, C, k, sm = shape
    n = 1003
    cl, co = specials(sm)
    env = TileMatchVecEnv(n, R, C, k, 30, cl, co, seeds=range(7000, 7000 + n), device=DEV)
    env.reset()
    for t in range(3):                                    # move the streams on, differently per env
        env.step_effective(t, key=KEY)
    env.join()
    rs = np.random.default_rng(sum(shape))
    mask = rs.random(n) < 0.3
    mask[8:16] = True                                     # one whole group of envs
    mask[16:24] = False
    mask[-3:] = True                                      # the ragged tail
    before = {f: _host(env, f).copy() for f in ("board", "rng", "timer", "eff")}
    o = orc.OracleBatch(R, C, k, sm, 30, env.rng_words().copy(), threads=16)
    o.reset()                                             # every env regenerated from its own stream
    env.reset(env_mask=torch.from_numpy(mask))
    env.join()
    for f in ("board", "rng", "timer", "eff"):
        got = _host(env, f).reshape(n, -1)
        want = np.where(mask[:, None], getattr(o, f).reshape(n, -1), before[f].reshape(n, -1))
        bad = np.nonzero((got != want).any(axis=1))[0]
        assert bad.size == 0, f"{shape}: {f} differs in {bad.size} envs, first {bad[:5]}"
    assert env.status() == 0
    env.close()
