"""BASELINE.json's full sizes (configs c2, c3, c4, c5 at their boards per GPU),
stepped exactly as bench.py steps them: three env groups on three HIP streams,
phases staggered in three blocks, the counter-based synthetic actions (or the
in-kernel effective-action policy), autoreset.  The oracle cannot replay
262 144 boards in seconds, so parity at these sizes rests on

  * exact replay of sampled envs: boards are independent (tile_match_env.py
    steps each env alone), so contiguous blocks of envs — the batch edges, the
    env-group and phase-block boundaries, random interior blocks — replayed on
    the oracle from their own seeds and timers must match every field at every
    step; for c4 the envs are rank 3's shard of 1 048 576 boards (global seeds
    and action streams), so this is also the shard-layout check at full size;
  * size-independent properties of the whole batch after the run: no colour
    line anywhere (board.py:174-176: every move ends on a line-free board),
    the cached effective-action masks equal a fresh tmg_effective over the
    final boards, every board has an effective action (board.py:181-184
    shuffles until one exists; generate_board only returns playable boards),
    colours and types in range, no bits past num_actions, status clear.
"""
import numpy as np
import pytest
import torch

from deep_rollouts import specials
from oracle import oracle as orc

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
KEY = 12345
MOVES = 30
BLOCK = 128

# name: (R, C, k, smask, boards, shard rank) — BASELINE.json configs[1..4]
FULL = {
    "c2": (10, 10, 4, 0, 65536, 0),
    "c3": (10, 10, 4, 14, 262144, 0),
    "c4": (10, 10, 4, 0, 131072, 3),
    "c5": (20, 20, 6, 15, 262144, 0),
    "g1": (10, 10, 5, 0, 65536, 0),
    # one launch of 262 144 envs of the c2 shape (groups = 1): the lane-per-board
    # kernel with given actions (tmg_capi.hip do_step, TMG_LANE_MIN_ENVS)
    "c2x4": (10, 10, 4, 0, 262144, 0),
}
CASES = [("c2", "uniform"), ("c3", "uniform"), ("c4", "uniform"), ("c5", "uniform"),
         ("c2", "effective"), ("c5", "effective"), ("c4", "effective"), ("g1", "effective"),
         ("c2x4", "uniform")]
GROUPS = {"c2x4": 1}


def _blocks(n, rs):
    """Starts of the replayed blocks: both batch edges, both sides of every
    phase-block (and env-group) boundary, four random interior blocks."""
    starts = {0, n - BLOCK}
    for j in (1, 2):
        starts |= {j * n // 3 - BLOCK // 2}
    while len(starts) < 8:
        starts.add(int(rs.integers(0, n - BLOCK)))
    return sorted(starts)


def _line_free(col):
    """(n, R, C) colours -> (n,) bool: no three equal non-zero colours in a row or column."""
    h = (col[:, :, :-2] == col[:, :, 1:-1]) & (col[:, :, 1:-1] == col[:, :, 2:]) & (col[:, :, :-2] > 0)
    v = (col[:, :-2, :] == col[:, 1:-1, :]) & (col[:, 1:-1, :] == col[:, 2:, :]) & (col[:, :-2, :] > 0)
    return ~(h.any(axis=(1, 2)) | v.any(axis=(1, 2)))


@pytest.mark.parametrize("name,policy", CASES)
def test_full_size(name, policy):
    from oracle.policy_np import sample_effective_np
    from tile_match_gym_amd.shard import shard_range, shard_seeds, synthetic_actions
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    R, C, k, sm, n, rank = FULL[name]
    cl, co = specials(sm)
    envs = shard_range(rank, n)
    env = TileMatchVecEnv(n, R, C, k, MOVES, cl, co, seeds=shard_seeds(rank, n), device=DEV,
                          groups=GROUPS.get(name, 3))
    A = env.num_actions
    rs = np.random.default_rng(sum(FULL[name]))
    starts = _blocks(n, rs)
    idx = np.concatenate([np.arange(s, s + BLOCK) for s in starts])
    idx_d = torch.from_numpy(idx).to(DEV)

    o = orc.OracleBatch(R, C, k, sm, MOVES, env.rng_words()[idx].copy(), threads=16)
    env.reset()
    o.reset()
    env.stagger_phases(blocks=3, first_env=envs.start)
    env.join()
    o.timer[:] = env.timer.index_select(0, idx_d).cpu().numpy()
    assert len(set(o.timer.tolist())) == 3                   # the replayed blocks span all three phases

    steps = MOVES + MOVES // 3 + 2                           # every env finishes at least one episode
    acts = torch.from_numpy(synthetic_actions(envs, steps, A)).to(DEV)
    fields = ("board", "rng", "timer", "eff", "reward", "n_new", "n_act", "flags")
    resets = 0
    for t in range(steps):
        if policy == "uniform":
            env.step_raw(acts[t])
            a = acts[t].index_select(0, idx_d).cpu().numpy()
        else:
            env.step_effective(t, key=KEY, first_env=envs.start)
            a = np.concatenate([sample_effective_np(o.eff[j * BLOCK:(j + 1) * BLOCK], A, KEY, envs.start + s, t)
                                for j, s in enumerate(starts)])
        env.join()
        if policy == "effective":
            assert np.array_equal(env.actions.index_select(0, idx_d).cpu().numpy(), a), f"{name} step {t}: actions"
        o.step(a, autoreset=True)
        for f in fields:
            if f == "rng":
                got = env.rng_words()[idx]
            else:
                got = getattr(env, f).index_select(0, idx_d).cpu().numpy()
                if f == "eff":
                    got = got.view(np.uint64)
            want = getattr(o, f)
            bad = np.nonzero((got.reshape(len(idx), -1) != want.reshape(len(idx), -1)).any(axis=1))[0]
            assert bad.size == 0, f"{name}/{policy} step {t}: {f} differs in {bad.size} envs, first {idx[bad[:5]]}"
        resets += int(((o.flags & 8) != 0).sum())
    assert resets >= len(idx), "every replayed env was meant to finish an episode"

    # whole-batch properties
    torch.cuda.synchronize()
    assert env.status() == 0
    board = env.board.cpu().numpy()
    col, typ = board[:, 0], board[:, 1]
    assert _line_free(col).all(), "a board holds a colour line after its step"
    ids = [1] + [t for b, t in ((1, -1), (2, 2), (4, 3), (8, 4)) if sm & b]
    assert np.isin(typ, ids).all(), "type outside the enabled specials"
    cookie = typ == -1
    assert ((col >= 1) & (col <= k) | cookie).all() and (col[cookie] == 0).all(), "colour out of range"
    t_all = env.timer.cpu().numpy()
    assert ((t_all >= 0) & (t_all < MOVES)).all()
    cached = env.eff.cpu().numpy().view(np.uint64).copy()
    fresh = env.compute_effective().cpu().numpy().view(np.uint64)
    bad = np.nonzero((cached != fresh).any(axis=1))[0]
    assert bad.size == 0, f"cached masks differ from tmg_effective in {bad.size} envs, first {bad[:5]}"
    bits = np.unpackbits(fresh.view(np.uint8).reshape(n, -1), axis=1, bitorder="little")
    assert bits[:, :A].any(axis=1).all(), "a board without an effective action"
    assert not bits[:, A:].any(), "mask bits past num_actions"
    env.close()
