"""GPU: the examples' effective-action policy (tmg_sample_effective) and the
multi-GPU shard layout (SURVEY.md §8(d) secondary action mode, §8(e) G=1 vs
G=8 bit-compare), checked against numpy / the CPU oracle."""
import numpy as np
import pytest
import torch

from oracle import oracle as orc
from oracle.policy_np import sample_effective_np

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _specials(sm):
    cl = ["cookie"] if sm & 1 else []
    co = [nm for b, nm in ((8, "bomb"), (2, "vertical_laser"), (4, "horizontal_laser")) if sm & b]
    return cl, co


@pytest.mark.parametrize("R,C", [(10, 10), (20, 20), (3, 4), (22, 23)])   # W = 3, 12, 1, 16 (the maximum)
def test_sample_effective_matches_numpy(R, C):
    from tile_match_gym_amd import _native
    ctx = _native.Context(0, R, C, 4, 0, 30)
    A, W = ctx.num_actions, ctx.mask_words
    rs = np.random.default_rng(R * C)
    n = 3000
    bits = rs.random((n, W * 64)) < rs.choice([0.002, 0.05, 0.5], size=(n, 1))
    bits[:, A:] = False
    bits[:40] = False
    eff = np.packbits(bits, axis=1, bitorder="little").view(np.uint64)
    d_eff = torch.from_numpy(eff.view(np.int64)).to(DEV)
    out = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    for t, first in ((0, 0), (17, 123456), (29, 7)):
        ctx.sample_effective(n, d_eff.data_ptr(), 12345, first, t, out.data_ptr(),
                             torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), sample_effective_np(eff, A, 12345, first, t))


@pytest.mark.parametrize("R,C,k,sm,n,steps", [(10, 10, 4, 0, 2048, 40), (8, 8, 3, 15, 2048, 40),
                                               (20, 20, 6, 15, 256, 32)])
@pytest.mark.parametrize("groups", [1, 3])
def test_step_effective_vs_oracle(R, C, k, sm, n, steps, groups):
    """Every env plays an effective move each step (until its episode ends):
    the device policy + step vs numpy policy + oracle, bit for bit."""
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    cl, co = _specials(sm)
    env = TileMatchVecEnv(n, R, C, k, 30, cl, co, seed=500, device=DEV, groups=groups)
    ref = orc.OracleBatch(R, C, k, sm, 30, env.rng_words().copy(), threads=16)
    env.reset()
    ref.reset()
    A = env.num_actions
    for t in range(steps):
        a = sample_effective_np(ref.eff, A, 99, 0, t)
        env.step_effective(t, key=99)
        ref.step(a, autoreset=True)
        env.join()
        assert np.array_equal(env.actions.cpu().numpy(), a), f"step {t}: actions"
        assert not (env.flags.cpu().numpy() & 0xC0).any()
        assert np.array_equal(env.board.cpu().numpy(), ref.board), f"step {t}: board"
        assert np.array_equal(env.rng_words(), ref.rng), f"step {t}: rng"
        assert np.array_equal(env.reward.cpu().numpy(), ref.reward), f"step {t}: reward"
        assert np.array_equal(env.eff.cpu().numpy().view(np.uint64), ref.eff), f"step {t}: eff"
    assert (ref.reward > 0).mean() > 0.5          # the policy's moves are effective


@pytest.mark.parametrize("policy", ["uniform", "effective"])
def test_shard_layout_g8_matches_g1(policy):
    """bench.py's layout for G = 8 (rank g: envs [g*n, (g+1)*n), seeds = global
    index, actions from the global-index stream) gathers to the G = 1 run."""
    from tile_match_gym_amd.shard import shard_range, shard_seeds, synthetic_actions
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    G, npr, steps = 8, 256, 35
    R, C, k = 10, 10, 4

    def run(envs, seeds):
        env = TileMatchVecEnv(len(envs), R, C, k, 30, seeds=seeds, device=DEV)
        env.reset()
        acts = torch.from_numpy(synthetic_actions(envs, steps, env.num_actions)).to(DEV)
        for t in range(steps):
            if policy == "uniform":
                env.step_raw(acts[t])
            else:
                env.step_effective(t, first_env=envs.start)
        env.join()
        torch.cuda.synchronize()
        return env.board.cpu().numpy(), env.rng_words(), env.reward.cpu().numpy()

    whole = run(range(0, G * npr), range(0, G * npr))
    parts = [run(shard_range(g, npr), shard_seeds(g, npr)) for g in range(G)]
    for i in range(3):
        assert np.array_equal(np.concatenate([p[i] for p in parts]), whole[i])


@pytest.mark.parametrize("k", [4, 5])
def test_policy_no_autoreset_vs_oracle(k):
    """The in-kernel policy without autoreset (the lane-per-board kernel's mode
    0): episodes end at num_moves with an all-zero mask (tile_match_env.py:
    119-120), and a further step is a caller error that leaves the env as it
    was (:94-95)."""
    from oracle.policy_np import sample_effective_np
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    n, M = 3000, 6
    env = TileMatchVecEnv(n, 10, 10, k, M, seeds=range(500, 500 + n), device=DEV, autoreset=False)
    o = orc.OracleBatch(10, 10, k, 0, M, env.rng_words().copy(), threads=16)
    env.reset()
    o.reset()
    A = env.num_actions
    for t in range(M + 2):
        env.step_effective(t, key=99)
        env.join()
        a = sample_effective_np(o.eff, A, 99, 0, t)
        assert np.array_equal(env.actions.cpu().numpy(), a), f"step {t}: actions"
        o.step(a, autoreset=False)
        for f in ("board", "timer", "eff", "reward", "flags"):
            got = getattr(env, f).cpu().numpy()
            got = got.view(np.uint64) if f == "eff" else got
            assert np.array_equal(got, getattr(o, f)), f"step {t}: {f}"
        assert np.array_equal(env.rng_words(), o.rng), f"step {t}: rng"
    assert (env.flags.cpu().numpy() == 0x80).all()             # every env stepped past its end
    assert env.status(clear=True) == 4                          # STATUS_CALLER
    env.close()
