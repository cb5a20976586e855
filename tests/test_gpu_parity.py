"""GPU parity: the HIP path (through the C ABI) against the reference's golden
vectors and against the CPU oracle.  Bit-exact everywhere (integer work)."""
import numpy as np
import pytest
import torch

from golden_io import load_records, load_traj, traj_names, replay_trajectory
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _ctx(R, C, k, smask, moves=1 << 20):
    from tile_match_gym_amd import _native
    return _native.Context(0, R, C, k, smask, moves)


def _stream():
    return torch.cuda.current_stream().cuda_stream


class _VecBackend:
    def __init__(self, d):
        from tile_match_gym_amd.vec_env import TileMatchVecEnv
        from tile_match_gym_amd._native import specials_mask  # noqa: F401
        sm = d["smask"]
        cl = ["cookie"] if sm & 1 else []
        co = [n for b, n in ((8, "bomb"), (2, "vertical_laser"), (4, "horizontal_laser")) if sm & b]
        self.env = TileMatchVecEnv(len(d["seeds"]), d["R"], d["C"], d["k"], d["num_moves"], cl, co,
                                   seeds=[int(s) for s in d["seeds"]], device=DEV)

    def reset(self):
        self.env.reset()

    def step(self, a, autoreset):
        self.env.autoreset = autoreset
        self.env.step(torch.from_numpy(a).to(DEV))

    def get_board(self):
        return self.env.board.cpu().numpy()

    def get_rng(self):
        return self.env.rng_words()

    def get_eff(self):
        return self.env.eff.cpu().numpy().view(np.uint64)

    get_reward = lambda self: self.env.reward.cpu().numpy()
    get_flags = lambda self: self.env.flags.cpu().numpy()
    get_n_new = lambda self: self.env.n_new.cpu().numpy()
    get_n_act = lambda self: self.env.n_act.cpu().numpy()


@pytest.mark.parametrize("name", traj_names())
@pytest.mark.parametrize("autoreset", [False, True])
def test_trajectory_golden_gpu(name, autoreset):
    """Whole reference trajectories (tile_match_env.py:84-124), RNG-exact."""
    d = load_traj(name)
    assert replay_trajectory(d, _VecBackend(d), autoreset) > 0


def _by_shape(recs):
    g = {}
    for r in recs:
        g.setdefault((r["R"], r["C"], r["k"], r["smask"]), []).append(r)
    return g


def test_move_golden_gpu():
    """Board.move (board.py:330-395) from arbitrary boards with specials, RNG-exact."""
    total = 0
    for (R, C, k, sm), recs in _by_shape(load_records("move")).items():
        recs = [r for r in recs if not r["err"]]
        if not recs:
            continue
        n = len(recs)
        ctx = _ctx(R, C, k, sm)
        board = torch.from_numpy(np.stack([r["board"] for r in recs]).astype(np.int8)).to(DEV)
        rng = torch.from_numpy(np.stack([r["rng_in"] for r in recs]).astype(np.uint64).view(np.int64)).to(DEV)
        timer = torch.zeros(n, dtype=torch.int32, device=DEV)
        acts = torch.tensor([int(r["action"]) for r in recs], dtype=torch.int32, device=DEV)
        out = torch.zeros((3, n), dtype=torch.int32, device=DEV)
        flags = torch.zeros(n, dtype=torch.uint8, device=DEV)
        eff = torch.zeros((n, ctx.mask_words), dtype=torch.int64, device=DEV)
        ctx.step(n, board.data_ptr(), rng.data_ptr(), timer.data_ptr(), acts.data_ptr(), out[0].data_ptr(),
                 out[1].data_ptr(), out[2].data_ptr(), flags.data_ptr(), eff.data_ptr(), 0, 0, _stream())
        torch.cuda.synchronize()
        b = board.cpu().numpy()
        rw = rng.cpu().numpy().view(np.uint64)
        o = out.cpu().numpy()
        f = flags.cpu().numpy()
        for i, r in enumerate(recs):
            res = r["res"]
            assert np.array_equal(b[i], r["out"]), f"board mismatch shape {(R, C, k, sm)} rec {i}"
            assert np.array_equal(rw[i], r["rng_out"]), f"rng mismatch shape {(R, C, k, sm)} rec {i}"
            assert (o[0, i], o[1, i], o[2, i]) == (res[0], res[2], res[3]), f"counters {(R, C, k, sm)} rec {i}"
            assert bool(f[i] & 2) == bool(res[1]) and bool(f[i] & 4) == bool(res[4])
            assert not (f[i] & 0xC0)
        total += n
    assert total > 500


def test_effective_golden_gpu():
    """is_move_effective (board.py:735-787) over every action, arbitrary boards."""
    for (R, C, k, sm), recs in _by_shape(load_records("effective")).items():
        ctx = _ctx(R, C, k, sm)
        n = len(recs)
        board = torch.from_numpy(np.stack([r["board"] for r in recs]).astype(np.int8)).to(DEV)
        eff = torch.zeros((n, ctx.mask_words), dtype=torch.int64, device=DEV)
        ctx.effective(n, board.data_ptr(), eff.data_ptr(), _stream())
        torch.cuda.synchronize()
        from golden_io import eff_words_to_bool
        got = eff_words_to_bool(eff.cpu().numpy().view(np.uint64), ctx.num_actions)
        for i, r in enumerate(recs):
            assert np.array_equal(got[i], r["eff"].astype(bool)), f"shape {(R, C, k, sm)} rec {i}"


@pytest.mark.parametrize("R,C,k,sm", [(10, 10, 6, 0), (9, 9, 5, 15), (20, 20, 6, 15), (9, 15, 15, 0)])
def test_generate_lemire_rejection_gpu(R, C, k, sm):
    """generate_board whose first 32-bit draw is a Lemire rejection
    (tests/rejection_states.py): the device's colour-ring generators redo the
    board draw by draw; board, RNG state and mask equal the oracle's."""
    from tile_match_gym_amd.seeding import batch_rng_words
    from rejection_states import rejecting_words
    ctx = _ctx(R, C, k, sm)
    n = 256
    w = rejecting_words(batch_rng_words(range(700, 700 + n)))
    board = torch.zeros((n, 2, R, C), dtype=torch.int8, device=DEV)
    rng = torch.from_numpy(w.view(np.int64).copy()).to(DEV)
    timer = torch.zeros(n, dtype=torch.int32, device=DEV)
    eff = torch.zeros((n, ctx.mask_words), dtype=torch.int64, device=DEV)
    ctx.reset(n, board.data_ptr(), rng.data_ptr(), timer.data_ptr(), eff.data_ptr(), None, _stream())
    torch.cuda.synchronize()
    o = orc.OracleBatch(R, C, k, sm, 30, w)
    o.reset()
    assert np.array_equal(board.cpu().numpy(), o.board)
    assert np.array_equal(rng.cpu().numpy().view(np.uint64), o.rng)
    assert np.array_equal(eff.cpu().numpy().view(np.uint64), o.eff)


def test_generate_golden_gpu():
    """generate_board (board.py:95-131) seeded like tile_match_env.py:49."""
    from tile_match_gym_amd.seeding import rng_words_from_seed
    for (R, C, k, sm), recs in _by_shape(load_records("generate")).items():
        ctx = _ctx(R, C, k, sm)
        n = len(recs)
        board = torch.zeros((n, 2, R, C), dtype=torch.int8, device=DEV)
        rng = torch.from_numpy(np.stack([rng_words_from_seed(int(r["seed"])) for r in recs]).view(np.int64)).to(DEV)
        timer = torch.zeros(n, dtype=torch.int32, device=DEV)
        eff = torch.zeros((n, ctx.mask_words), dtype=torch.int64, device=DEV)
        ctx.reset(n, board.data_ptr(), rng.data_ptr(), timer.data_ptr(), eff.data_ptr(), None, _stream())
        torch.cuda.synchronize()
        b = board.cpu().numpy()
        for i, r in enumerate(recs):
            assert np.array_equal(b[i], r["out"]), f"shape {(R, C, k, sm)} rec {i}"


@pytest.mark.parametrize("cfg", [
    # R, C, k, smask, n_envs, steps
    (10, 10, 4, 0, 8192, 65),
    (10, 10, 4, 14, 4096, 65),
    (20, 20, 6, 15, 512, 35),
    # 512-cell path, rows straddling the 64-cell passes unevenly (bounded line search)
    (16, 24, 7, 0, 256, 35),
    (24, 21, 7, 9, 256, 35),
    (8, 8, 3, 15, 4096, 65),
    (5, 5, 3, 15, 4096, 65),
    (6, 7, 5, 1, 2048, 45),
    # scalar-bitboard lean path (no specials, <= 128 cells): odd C, 1..4 colour planes, C = 63
    (7, 5, 3, 0, 4096, 65),
    (6, 9, 9, 0, 2048, 45),
    (16, 8, 5, 0, 2048, 45),
    (3, 4, 2, 0, 2048, 45),
    (2, 63, 6, 0, 1024, 35),
    (11, 11, 4, 0, 2048, 45),
    # > 128 cells and many colours: generated boards often need a shuffle, so
    # the 512-cell reset kernel's colour ring hands over the exact stream
    # position mid-generation (board.py:102-118)
    (9, 15, 15, 0, 2048, 24),
    (10, 14, 14, 0, 2048, 24),
    # bench.py's generic-shape configs g1 / g2 (no shape-specialised kernel)
    (10, 10, 5, 0, 4096, 65),
    (20, 20, 6, 14, 512, 35),
])
def test_oracle_parity_random_actions(cfg):
    """Batched random-action rollouts with autoreset vs the CPU oracle, every step."""
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    R, C, k, sm, n, steps = cfg
    cl = ["cookie"] if sm & 1 else []
    co = [nm for b, nm in ((8, "bomb"), (2, "vertical_laser"), (4, "horizontal_laser")) if sm & b]
    env = TileMatchVecEnv(n, R, C, k, 30, cl, co, seed=1000, device=DEV)
    ref = orc.OracleBatch(R, C, k, sm, 30, env.rng_words().copy(), threads=16)
    env.reset()
    ref.reset()
    assert np.array_equal(env.board.cpu().numpy(), ref.board)
    rs = np.random.default_rng(R * 1000 + C * 10 + sm)
    A = env.num_actions
    for t in range(steps):
        # half uniform random, half uniform over effective actions (as in examples/random_agent.py)
        a = rs.integers(0, A, n).astype(np.int32)
        effm = np.unpackbits(ref.eff.view(np.uint8).reshape(n, -1), axis=1, bitorder="little")[:, :A]
        pick = rs.random(n) < 0.5
        for i in np.nonzero(pick)[0][:256]:
            nz = np.nonzero(effm[i])[0]
            if nz.size:
                a[i] = nz[rs.integers(nz.size)]
        env.step(torch.from_numpy(a).to(DEV))
        ref.step(a, autoreset=True)
        f = env.flags.cpu().numpy()
        assert not (f & 0xC0).any(), f"error/overflow flag at step {t}"
        b = env.board.cpu().numpy()
        bad = np.nonzero((b.reshape(n, -1) != ref.board.reshape(n, -1)).any(axis=1))[0]
        assert bad.size == 0, f"step {t}: {bad.size} boards differ, first env {bad[0]}"
        assert np.array_equal(env.rng_words(), ref.rng), f"step {t}: rng"
        assert np.array_equal(env.reward.cpu().numpy(), ref.reward), f"step {t}: reward"
        assert np.array_equal(env.n_new.cpu().numpy(), ref.n_new)
        assert np.array_equal(env.n_act.cpu().numpy(), ref.n_act)
        assert np.array_equal(f, ref.flags), f"step {t}: flags"
        assert np.array_equal(env.eff.cpu().numpy().view(np.uint64), ref.eff), f"step {t}: eff"


@pytest.mark.parametrize("R,C,k,sm", [(10, 10, 4, 0), (8, 8, 3, 15), (20, 20, 6, 15)])
def test_env_groups_match_single_stream(R, C, k, sm):
    """TileMatchVecEnv(groups=3) — env groups on separate HIP streams — equals groups=1 bit for bit."""
    from tile_match_gym_amd.shard import synthetic_actions
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    cl = ["cookie"] if sm & 1 else []
    co = [nm for b, nm in ((8, "bomb"), (2, "vertical_laser"), (4, "horizontal_laser")) if sm & b]
    n = 1000
    e1 = TileMatchVecEnv(n, R, C, k, 12, cl, co, seed=77, device=DEV)
    e3 = TileMatchVecEnv(n, R, C, k, 12, cl, co, seed=77, device=DEV, groups=3)
    acts = torch.from_numpy(synthetic_actions(range(n), 30, e1.num_actions)).to(DEV)
    e1.reset()
    e3.reset()
    for t in range(30):
        e1.step_raw(acts[t])
        e3.step_raw(acts[t])
    e3.join()
    torch.cuda.synchronize()
    for f in ("board", "rng", "timer", "eff", "reward", "n_new", "n_act", "flags"):
        assert torch.equal(getattr(e1, f), getattr(e3, f)), f


@pytest.mark.parametrize("blocks", [0, 3])
@pytest.mark.parametrize("R,C,k,sm", [(10, 10, 4, 0), (10, 10, 4, 14)])
def test_bench_phase_stagger_vs_oracle(blocks, R, C, k, sm):
    """The bench's workload: episode phases offset after the reset
    (stagger_phases; blocks=3 with 3 env groups, blocks=0 every env), the
    synthetic action stream, autoreset — vs the oracle given the same timers."""
    from tile_match_gym_amd.shard import synthetic_actions
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    co = [nm for b, nm in ((8, "bomb"), (2, "vertical_laser"), (4, "horizontal_laser")) if sm & b]
    n = 3000
    env = TileMatchVecEnv(n, R, C, k, 30, [], co, seed=5, device=DEV, groups=3)
    ref = orc.OracleBatch(R, C, k, sm, 30, env.rng_words().copy(), threads=16)
    env.reset()
    ref.reset()
    env.stagger_phases(blocks=blocks)
    t0 = env.timer.cpu().numpy()
    if blocks:
        assert sorted(set(t0.tolist())) == [0, 10, 20]
        assert (t0[:1000] == 0).all() and (t0[1000:2000] == 10).all() and (t0[2000:] == 20).all()
    else:
        assert np.array_equal(t0, np.arange(n) % 30)
    ref.timer[:] = t0
    acts = synthetic_actions(range(n), 45, env.num_actions)
    dacts = torch.from_numpy(acts).to(DEV)
    for t in range(45):
        env.step_raw(dacts[t])
        ref.step(acts[t], autoreset=True)
        env.join()
        f = env.flags.cpu().numpy()
        assert np.array_equal(f, ref.flags), f"step {t}: flags"
        assert np.array_equal(env.board.cpu().numpy(), ref.board), f"step {t}: board"
        assert np.array_equal(env.reward.cpu().numpy(), ref.reward), f"step {t}: reward"
    assert np.array_equal(env.rng_words(), ref.rng)
    assert np.array_equal(env.timer.cpu().numpy(), ref.timer)
    assert env.status() == 0
