"""GPU parity of the §8(f) rows: compute_num_states, the one-hot observation
encoding, checkpoint/restore and the Gymnasium vector-env autoreset modes —
each against the oracle / counts recorded from the reference."""
import os

import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SPECIALS = {1: "cookie", 2: "vertical_laser", 4: "horizontal_laser", 8: "bomb"}


def _lists(sm):
    cl = ["cookie"] if sm & 1 else []
    co = [SPECIALS[b] for b in (2, 4, 8) if sm & b]
    return cl, co


def test_count_states_gpu():
    """utils.compute_num_states (utils.py:6-26) on the GPU vs the reference's counts and the oracle."""
    from tile_match_gym_amd.utils import compute_num_states
    d = np.load(os.path.join(GOLDEN, "fn_count_states.npz"))
    for (R, C, k), p, lf in zip(d["shapes"], d["playable"], d["line_free"]):
        assert compute_num_states(int(R), int(C), int(k), 4) == (int(p), int(lf)), (R, C, k)
    for (R, C, k) in [(4, 3, 3), (4, 4, 2), (3, 5, 3), (5, 3, 3)]:
        assert compute_num_states(R, C, k) == orc.count_states(R, C, k, threads=16), (R, C, k)


def _onehot_ref(board, k, sm):
    """wrappers.py:56-69 restated: colour channels 1..k, then enabled specials'
    type channels in the order cookie, v-laser, h-laser, bomb."""
    ids = [t for b, t in ((1, -1), (2, 2), (4, 3), (8, 4)) if sm & b]
    chans = [board[:, 0] == c for c in range(1, k + 1)] + [board[:, 1] == t for t in ids]
    return np.stack(chans, axis=1).astype(np.float64)


@pytest.mark.parametrize("R,C,k,sm", [(10, 10, 4, 0), (10, 10, 4, 14), (20, 20, 6, 15), (7, 5, 3, 1), (6, 9, 5, 10)])
def test_onehot_gpu(R, C, k, sm):
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    from tile_match_gym_amd.wrappers import VecOneHot
    cl, co = _lists(sm)
    n = 512
    env = TileMatchVecEnv(n, R, C, k, 30, cl, co, seed=3, device=DEV)
    env.reset()
    rs = np.random.default_rng(R * C + sm)
    # arbitrary boards with every colour / type value, incl. empties and cookies
    b = np.stack([rs.integers(0, k + 1, (n, R, C)), rs.integers(-1, 5, (n, R, C))], axis=1).astype(np.int8)
    env.board.copy_(torch.from_numpy(b))
    want = _onehot_ref(b, k, sm)
    for dt in (torch.float32, torch.uint8, torch.int32):
        got = VecOneHot(env, dtype=dt).encode()
        torch.cuda.synchronize()
        assert got.shape == want.shape
        assert np.array_equal(got.cpu().numpy().astype(np.float64), want), dt


def test_onehot_wrapper_facade():
    """OneHotWrapper / ProportionRewardWrapper on the single-env facade (float64 like the reference)."""
    from tile_match_gym_amd.tile_match_env import TileMatchEnv
    from tile_match_gym_amd.wrappers import OneHotWrapper, ProportionRewardWrapper
    env = ProportionRewardWrapper(OneHotWrapper(TileMatchEnv(6, 6, 4, 10, ["cookie"], ["bomb"], seed=5)))
    obs, info = env.reset()
    raw = env.unwrapped.board.board
    want = _onehot_ref(raw[None], 4, 1 | 8)[0]
    assert obs["board"].dtype == np.float64 and np.array_equal(obs["board"], want)
    a = info["effective_actions"][0]
    obs, r, done, trunc, info = env.step(a)
    assert np.array_equal(obs["board"], _onehot_ref(env.unwrapped.board.board[None], 4, 9)[0])
    assert 0 < r <= 1.0


def test_checkpoint_restore_continues_bit_exact(tmp_path):
    from tile_match_gym_amd.shard import synthetic_actions
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    n, R, C, k = 1024, 10, 10, 4
    env = TileMatchVecEnv(n, R, C, k, 30, [], ["vertical_laser", "bomb"], seed=11, device=DEV)
    acts = torch.from_numpy(synthetic_actions(range(n), 40, env.num_actions)).to(DEV)
    env.reset()
    for t in range(17):
        env.step_raw(acts[t])
    p = tmp_path / "ck.npz"
    env.save(p)
    env2 = TileMatchVecEnv.load(p, device=DEV)
    for t in range(17, 40):
        env.step_raw(acts[t])
        env2.step_raw(acts[t])
        for f in ("board", "rng", "timer", "eff", "reward", "flags"):
            assert torch.equal(getattr(env, f), getattr(env2, f)), (t, f)


# (8, 8, 3, 14) / (10, 10, 4, 14): the 128-cell general kernels (deferred
# resets); (10, 10, 4, 0): the lean c2 kernel (inline); (20, 20, 6, 15): the
# 512-cell c5 kernels; (7, 9, 5, 15): an odd cell count (2N % 4 == 2, boards
# not dword-aligned) through the general kernel's same-step final boards.
@pytest.mark.parametrize("cfg", [(8, 8, 3, 14), (10, 10, 4, 0), (10, 10, 4, 14), (20, 20, 6, 15), (7, 9, 5, 15)])
@pytest.mark.parametrize("obs_dtype", ["int32", "int8"])
@pytest.mark.parametrize("groups", [1, 3])
@pytest.mark.parametrize("mode", ["next_step", "same_step"])
def test_vector_env_autoreset_modes(mode, groups, obs_dtype, cfg):
    """TileMatchVectorEnv (gymnasium vector API) vs the oracle driven with the
    same autoreset semantics (tests/vector_ref.py): obs, rewards, terminations,
    infos, action masks, final boards — the general kernels (deferred resets)
    and the lean ones (inline), on one and on three group streams, int32
    (kernel-written) and int8 (the live state) observations.  copy=True (the
    default): every returned tensor keeps its value after the next step."""
    from tile_match_gym_amd.vector import TileMatchVectorEnv
    from vector_ref import VectorOracle
    R, C, k, sm = cfg
    n, moves = (128 if R * C > 128 else 256), 6
    cl, co = _lists(sm)
    odt = torch.int32 if obs_dtype == "int32" else torch.int8
    venv = TileMatchVectorEnv(n, R, C, k, moves, cl, co, seed=40, device=DEV, autoreset_mode=mode, groups=groups,
                              obs_dtype=odt)
    ref = orc.OracleBatch(R, C, k, sm, moves, venv.vec.rng_words().copy())
    obs, info = venv.reset()
    ref.reset()
    assert obs["board"].dtype == odt
    assert np.array_equal(obs["board"].cpu().numpy(), ref.board.astype(np.int32))
    A = venv.single_action_space.n
    assert venv.action_space.shape == (venv.num_envs,) and (venv.action_space.nvec == A).all()
    vo = VectorOracle(ref, mode)
    rs = np.random.default_rng(1)
    kept = None
    for t in range(3 * moves + 2):
        a = rs.integers(0, A, n).astype(np.int32)
        obs, rew, term, trunc, info = venv.step(torch.from_numpy(a).to(DEV))
        if kept is not None:                       # copies of the previous step, untouched by this one
            for got, want_prev in zip(kept[0], kept[1]):
                assert np.array_equal(got.cpu().numpy(), want_prev), t
        kept = ((obs["board"], obs["num_moves_left"], rew, term, info["action_mask"]),
                tuple(x.cpu().numpy().copy() for x in (obs["board"], obs["num_moves_left"], rew, term,
                                                       info["action_mask"])))
        want = vo.step(a)
        want_term = want["terminated"][:, 0].astype(bool)
        if mode == "same_step":
            fb = info["final_obs"]["board"].cpu().numpy()
            assert np.array_equal(info["_final_obs"].cpu().numpy(), want_term)
            assert np.array_equal(fb[want_term], want["final_board"][want_term].astype(np.int32))
        assert np.array_equal(term.cpu().numpy(), want_term), t
        assert not trunc.any()
        assert np.array_equal(rew.cpu().numpy(), want["reward"]), t
        assert np.array_equal(obs["board"].cpu().numpy(), ref.board.astype(np.int32)), t
        assert np.array_equal(obs["num_moves_left"].cpu().numpy(), want["moves_left"]), t
        for i, key in enumerate(("is_combination_match", "shuffled", "error")):
            col = (1, 2, 3)[i]
            assert np.array_equal(info[key].cpu().numpy(), want["terminated"][:, col].astype(bool)), (t, key)
        assert np.array_equal(info["num_new_specials"].cpu().numpy(), want["n_new"]), t
        assert np.array_equal(info["num_specials_activated"].cpu().numpy(), want["n_act"]), t
        assert np.array_equal(info["action_mask"].cpu().numpy(), want["action_mask"].astype(bool)), t


def test_onehot_wrapper_reference_vectors():
    """The reference's own OneHotWrapper expectations (tests/test_wrappers.py:5-41):
    three seeded scenarios — colours after reset, a bomb made by action 33, a
    cookie made by action 2 — replayed through this TileMatchEnv + OneHotWrapper,
    asserting the reference's literal vectors and shapes."""
    from tile_match_gym_amd.tile_match_env import TileMatchEnv
    from tile_match_gym_amd.wrappers import OneHotWrapper
    env = OneHotWrapper(TileMatchEnv(4, 3, 5, 10, [], [], seed=1))
    assert env.observation_space["board"].shape == (5, 4, 3)
    assert env.observation_space["num_moves_left"].n == 11
    obs, info = env.reset()
    assert np.array_equal(obs["board"][:, 0, 0], np.array([0, 0, 1, 0, 0], dtype=np.float32))
    assert np.array_equal(obs["board"][:, 1, 1], np.array([1, 0, 0, 0, 0], dtype=np.float32))
    assert obs["num_moves_left"] == 10

    env = OneHotWrapper(TileMatchEnv(5, 5, 3, 10, [], ["bomb"], seed=2))
    obs, info = env.reset()
    assert np.array_equal(obs["board"][:, 2, 2], np.array([1, 0, 0, 0], dtype=np.float32))
    obs, *_ = env.step(33)                                   # makes a bomb
    assert obs["board"].shape == (4, 5, 5)
    assert obs["num_moves_left"] == 9
    assert np.array_equal(obs["board"][:, 3, 2], np.array([1, 0, 0, 1], dtype=np.float32))

    env = OneHotWrapper(TileMatchEnv(5, 5, 2, 12, ["cookie"], ["vertical_laser"], seed=2))
    obs, info = env.reset()
    assert obs["board"].shape == (4, 5, 5)
    assert obs["num_moves_left"] == 12
    obs, *_ = env.step(2)                                    # makes a cookie
    assert np.array_equal(obs["board"][:, 1, 2], np.array([0, 0, 1, 0], dtype=np.float32))
    assert obs["board"].shape == (4, 5, 5)
    assert obs["num_moves_left"] == 11


@pytest.mark.parametrize("R,C,k,sm,groups", [(10, 10, 4, 0, 3), (10, 10, 4, 14, 2), (20, 20, 6, 15, 2),
                                             (7, 5, 3, 1, 1), (6, 9, 5, 10, 1)])
def test_fused_onehot_matches_separate_encode(R, C, k, sm, groups):
    """tmg_step_onehot (one-hot planes written in the step / reset kernels'
    own write-back, only for changed boards) == tmg_onehot of the boards after
    every step, with autoreset, env groups, every dtype and a hand edit."""
    from tile_match_gym_amd.shard import synthetic_actions
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    from tile_match_gym_amd.wrappers import VecOneHot
    cl, co = _lists(sm)
    n = 1500
    for dt in (torch.float32, torch.uint8, torch.int32):
        env = TileMatchVecEnv(n, R, C, k, 12, cl, co, seed=41, device=DEV, groups=groups)
        env.reset()
        fused = VecOneHot(env, dtype=dt, fused=True)
        sep = VecOneHot(env, dtype=dt)
        acts = torch.from_numpy(synthetic_actions(range(n), 30, env.num_actions)).to(DEV)
        for t in range(30):
            if t == 13:                                          # hand edit -> untrusted mask
                env.join()
                env.board[::7, 0, 0, 0] = 1
                env.board[::7, 1, 0, 0] = 1
                env.invalidate_effective_cache()
            env.step_raw(acts[t])
            got = fused.encode().clone()
            want = sep.encode()
            torch.cuda.synchronize()
            assert torch.equal(got, want), (dt, t)
        env.reset()                                              # tmg_reset_onehot
        assert torch.equal(fused.encode().clone(), sep.encode()), dt


def test_checkpoint_restore_vs_oracle(tmp_path):
    """Save mid-episode on the GPU, load the arrays into the oracle (board, the
    PCG64 words incl. numpy's buffered half-word and its flag, timer, eff) and
    into a fresh TileMatchVecEnv; 35 more steps (two autoresets) must agree
    with the oracle at every step (tile_match_env.py:49 stream format)."""
    from tile_match_gym_amd.shard import synthetic_actions
    from tile_match_gym_amd.vec_env import TileMatchVecEnv, load_state
    n, R, C, k, sm = 2048, 10, 10, 4, 14
    cl, co = _lists(sm)
    env = TileMatchVecEnv(n, R, C, k, 15, cl, co, seed=21, device=DEV, groups=2)
    acts = synthetic_actions(range(n), 60, env.num_actions)
    dacts = torch.from_numpy(acts).to(DEV)
    env.reset()
    for t in range(23):
        env.step_raw(dacts[t])
    p = tmp_path / "ck.npz"
    env.save(p)
    arrays, cfg = load_state(p)
    assert ((arrays["rng"][:, 4] >> np.uint64(32)) & np.uint64(1)).any(), "some env should hold a buffered half-word"
    o = orc.OracleBatch(R, C, k, sm, 15, arrays["rng"].copy(), threads=16)
    o.board[:] = arrays["board"]
    o.timer[:] = arrays["timer"]
    o.eff[:] = arrays["eff"]
    env2 = TileMatchVecEnv.load(p, device=DEV)
    for t in range(23, 58):
        env2.step(dacts[t])
        o.step(acts[t], autoreset=True)
        assert np.array_equal(env2.board.cpu().numpy(), o.board), t
        assert np.array_equal(env2.rng_words(), o.rng), t
        assert np.array_equal(env2.timer.cpu().numpy(), o.timer), t
        assert np.array_equal(env2.reward.cpu().numpy(), o.reward), t
        assert np.array_equal(env2.flags.cpu().numpy(), o.flags), t
        assert np.array_equal(env2.eff.cpu().numpy().view(np.uint64), o.eff), t


@pytest.mark.parametrize("R,C,k,sm", [(10, 10, 4, 0), (10, 10, 4, 14), (20, 20, 6, 15)])
def test_step_effective_after_hand_edit_with_low_line(R, C, k, sm):
    """Boards edited by hand to hold a line in their bottom row, the mask
    invalidated, then TileMatchVecEnv.step_effective: the policy samples from
    tmg_effective's mask, and that step must run untrusted — a mask from
    tmg_effective says nothing about lines already on the board, which the
    reference's cascade clears first (board.py:367-391: get_colour_lines scans
    from the bottom).  Every field equals the oracle for that step and the
    next ones."""
    from oracle.policy_np import sample_effective_np
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    cl, co = _lists(sm)
    n = 2048
    env = TileMatchVecEnv(n, R, C, k, 30, cl, co, seed=61, device=DEV)
    o = orc.OracleBatch(R, C, k, sm, 30, env.rng_words().copy(), threads=16)
    env.reset()
    o.reset()
    b = env.board.cpu().numpy()
    rs = np.random.default_rng(3)
    for i in range(n):                                  # a horizontal 3-line of normals low on the board
        r = R - 1 - int(rs.integers(0, 2))
        c = int(rs.integers(0, C - 2))
        b[i, 0, r, c:c + 3] = 1 + int(rs.integers(0, k))
        b[i, 1, r, c:c + 3] = 1
    env.board.copy_(torch.from_numpy(b))
    o.board[:] = b
    env.invalidate_effective_cache()
    A = env.num_actions
    for i in range(n):                                   # the oracle's view of the edited boards' masks
        m, _ = orc.effective_mask(b[i])
        o.eff[i] = np.packbits(np.concatenate([m, np.zeros(o.W * 64 - A, bool)]), bitorder="little").view(np.uint64)
    for t in range(4):
        a = sample_effective_np(o.eff, A, 4242, 0, t)
        env.step_effective(t, key=4242)
        env.join()
        o.step(a, autoreset=True)
        assert np.array_equal(env.actions.cpu().numpy(), a), t
        for f in ("board", "reward", "n_new", "n_act", "flags", "timer"):
            assert np.array_equal(getattr(env, f).cpu().numpy(), getattr(o, f)), (t, f)
        assert np.array_equal(env.rng_words(), o.rng), t
        assert np.array_equal(env.eff.cpu().numpy().view(np.uint64), o.eff), t
    assert env.status() == 0


@pytest.mark.parametrize("cfg", [(10, 10, 4, 0), (8, 8, 3, 14)])
@pytest.mark.parametrize("policy", [False, True])
def test_captured_steps_match_eager(cfg, policy):
    """TileMatchVecEnv.capture_steps / run_graph (tmg_plan_capture: the plan
    steps of a window in one HIP graph) leaves exactly the state of the same
    steps launched one by one: lean and general kernels, three env groups,
    given actions and the in-kernel policy, across autoresets."""
    from tile_match_gym_amd.shard import synthetic_actions
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    R, C, k, sm = cfg
    n, T = 3000, 24
    cl, co = _lists(sm)
    envs = [TileMatchVecEnv(n, R, C, k, 7, cl, co, seed=3, device=DEV, groups=3) for _ in range(2)]
    A = envs[0].num_actions
    acts = torch.from_numpy(synthetic_actions(range(n), T, A)).to(DEV)
    for e in envs:
        e.reset()
    for t in range(T):
        if policy:
            envs[0].step_effective(t)
        else:
            envs[0].step_raw(acts[t])
    envs[0].join()
    g = (envs[1].capture_steps(ts=range(T), policy=True) if policy else
         envs[1].capture_steps([acts[t] for t in range(T)]))
    envs[1].run_graph(g)
    torch.cuda.synchronize()
    for f in ("board", "rng", "timer", "eff", "reward", "n_new", "n_act", "flags"):
        assert torch.equal(getattr(envs[0], f), getattr(envs[1], f)), (cfg, policy, f)
    if policy:
        assert torch.equal(envs[0].actions, envs[1].actions)
    assert envs[1].status() == 0


def test_vecenv_autoreset_mode_survives_toggle_and_checkpoint(tmp_path):
    """The autoreset mode is one field: toggling the bool keeps next-step mode,
    and a checkpoint taken in next-step mode restores into next-step mode (its
    pending resets are implicit in timer == num_moves)."""
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    n, R, C, k, moves = 64, 8, 8, 3, 4
    env = TileMatchVecEnv(n, R, C, k, moves, [], [], seed=3, device=DEV, autoreset=False)
    assert env.autoreset_mode == "none" and not env.autoreset
    env.set_step_outputs("next_step")
    assert env.autoreset_mode == "next_step" and env.autoreset
    env.autoreset = True
    assert env.autoreset_mode == "next_step"
    env.reset()
    acts = torch.zeros(n, dtype=torch.int32, device=DEV)
    for _ in range(moves):
        env.step_raw(acts)
    env.join()
    p = tmp_path / "ck.npz"
    env.save(p)
    env2 = TileMatchVecEnv.load(p, device=DEV)
    assert env2.autoreset_mode == "next_step"
    env.step_raw(acts)           # every env ended last call: regenerated now, timer 0
    env2.step_raw(acts)
    env.join(); env2.join()
    for f in ("board", "rng", "timer", "eff", "reward", "flags"):
        assert torch.equal(getattr(env, f), getattr(env2, f)), f
    assert (env.timer == 0).all()
    env.autoreset = False
    assert env.autoreset_mode == "none"
    env.autoreset = True
    assert env.autoreset_mode == "same_step"
