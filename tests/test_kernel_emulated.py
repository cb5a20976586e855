"""CPU-side check of the HIP kernel *logic*: tools/wave_emu compiles
csrc/tmg_board.hip for the host (one fiber per lane, collectives resolved at
the wavefront's lockstep points) and replays the reference's golden
trajectories through it.  This is a debugging aid that runs without a GPU;
the parity gate proper is tests/test_gpu_parity.py on the MI355X."""
import os
import subprocess
import sys

import numpy as np
import pytest

from golden_io import load_traj, traj_names, replay_trajectory

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMU_DIR = os.path.join(ROOT, "tools", "wave_emu")


@pytest.fixture(scope="module")
def emu_lib():
    asan = os.environ.get("TMG_EMU_ASAN") == "1"
    subprocess.run(["make", "-C", EMU_DIR, "libwave_emu_asan.so" if asan else "libwave_emu.so"], check=True,
                   stdout=subprocess.DEVNULL)
    sys.path.insert(0, EMU_DIR)
    import emu
    return emu, emu.load(asan=asan)


class _EmuBackend:
    def __init__(self, emu, L, d):
        self.b = emu.EmuBatch(L, d["R"], d["C"], d["k"], d["smask"], d["num_moves"], d["init_rng"])

    def reset(self):
        self.b.reset()

    def step(self, a, autoreset):
        self.b.step(a, autoreset)

    get_board = lambda self: self.b.board
    get_rng = lambda self: self.b.rng
    get_eff = lambda self: self.b.eff
    get_reward = lambda self: self.b.reward
    get_flags = lambda self: self.b.flags
    get_n_new = lambda self: self.b.n_new
    get_n_act = lambda self: self.b.n_act


@pytest.mark.parametrize("name", traj_names())
@pytest.mark.parametrize("autoreset", [False, True])
def test_trajectory_golden_emulated(emu_lib, name, autoreset, monkeypatch):
    emu, L = emu_lib
    monkeypatch.setenv("EMU_EPW", "1")      # one env per workgroup, as libtmg launches
    d = load_traj(name)
    assert replay_trajectory(d, _EmuBackend(emu, L, d), autoreset) > 0


@pytest.mark.parametrize("cfg", [
    # R, C, k, smask: the scalar-bitboard lean path (even/odd C, 1..4 colour planes,
    # 128 cells, C = 63) and the general kernel with specials
    (10, 10, 4, 0), (8, 8, 3, 0), (7, 5, 5, 0), (6, 9, 9, 0), (3, 4, 2, 0), (16, 8, 4, 0), (2, 63, 6, 0),
    (11, 11, 4, 0), (10, 10, 4, 14), (8, 8, 3, 15), (5, 12, 6, 15),
    # 512-cell kernels: rows straddle the 64-cell passes unevenly (bounded line search)
    (16, 24, 7, 0), (24, 21, 7, 9),
    # 512-cell general kernels with specials: wave-parallel simple / laser steps
    # (simple_step_lds) beside the lane-0 list machinery
    (20, 20, 6, 15), (12, 12, 5, 15), (16, 16, 6, 6),
])
def test_random_rollouts_emulated(emu_lib, cfg):
    """Random-action rollouts with autoreset: emulated kernels vs the oracle, every field, every step."""
    from oracle import oracle as orc
    from tile_match_gym_amd.seeding import batch_rng_words
    emu, L = emu_lib
    R, C, k, sm = cfg
    n, T = 12, 40
    w = batch_rng_words(range(1000, 1000 + n))
    e = emu.EmuBatch(L, R, C, k, sm, 7, w)
    o = orc.OracleBatch(R, C, k, sm, 7, w)
    e.reset()
    o.reset()
    rs = np.random.default_rng(R * 100 + C + sm)
    A = 2 * R * C - R - C
    for t in range(-1, T):
        if t >= 0:
            a = rs.integers(0, A, n).astype(np.int32)
            e.step(a, True)
            o.step(a, True)
        for f in ("board", "rng", "eff", "reward", "flags", "timer", "n_new", "n_act"):
            assert np.array_equal(getattr(e, f), getattr(o, f)), f"{cfg} step {t}: {f}"


@pytest.mark.parametrize("cfg", [(9, 15, 15, 0), (10, 14, 14, 0)])
def test_generate_shuffles_emulated(emu_lib, cfg):
    """> 128-cell boards with many colours, where a generated line-free board
    often has no effective move: the 512-cell reset kernel's colour ring hands
    the exact stream position to shuffle (board.py:102-118) and resumes after it.
    Emulated kernels vs the oracle, every field, after every reset and step."""
    from oracle import oracle as orc
    from tile_match_gym_amd.seeding import batch_rng_words
    emu, L = emu_lib
    R, C, k, sm = cfg
    n, T = 48, 24
    w = batch_rng_words(range(5000, 5000 + n))
    e = emu.EmuBatch(L, R, C, k, sm, 3, w)
    o = orc.OracleBatch(R, C, k, sm, 3, w)
    e.reset()
    o.reset()
    rs = np.random.default_rng(R * 100 + C)
    A = 2 * R * C - R - C
    shuffled = 0
    for t in range(-1, T):
        if t >= 0:
            a = rs.integers(0, A, n).astype(np.int32)
            e.step(a, True)
            o.step(a, True)
            shuffled += int(((o.flags & 4) != 0).sum())
        for f in ("board", "rng", "eff", "reward", "flags", "timer", "n_new", "n_act"):
            assert np.array_equal(getattr(e, f), getattr(o, f)), f"{cfg} step {t}: {f}"


@pytest.mark.parametrize("cfg", [(10, 10, 6, 0), (9, 9, 5, 15), (20, 20, 6, 15), (16, 16, 6, 6), (9, 15, 15, 0)])
def test_generate_lemire_rejection_emulated(emu_lib, cfg):
    """generate_board whose very first 32-bit draw is a Lemire rejection
    (tests/rejection_states.py): the colour-ring generators must detect it and
    redo the board draw by draw — same board and RNG state as the oracle."""
    from oracle import oracle as orc
    from tile_match_gym_amd.seeding import batch_rng_words
    from rejection_states import rejecting_words
    emu, L = emu_lib
    R, C, k, sm = cfg
    n = 8
    w = rejecting_words(batch_rng_words(range(300, 300 + n)))
    e = emu.EmuBatch(L, R, C, k, sm, 30, w)
    o = orc.OracleBatch(R, C, k, sm, 30, w)
    e.reset()
    o.reset()
    for f in ("board", "rng", "eff", "timer"):
        assert np.array_equal(getattr(e, f), getattr(o, f)), f"{cfg}: {f}"
    assert not np.array_equal(o.rng, w), "the reset consumed the stream"


def test_move_golden_emulated(emu_lib):
    """Board.move (board.py:330-395) from the recorded arbitrary boards (specials, coloured cookies,
    empties), through the emulated general kernel — the CPU twin of test_move_golden_gpu."""
    from golden_io import load_records
    emu, L = emu_lib
    groups = {}
    for r in load_records("move"):
        if not r["err"]:
            groups.setdefault((r["R"], r["C"], r["k"], r["smask"]), []).append(r)
    total = 0
    for (R, C, k, sm), recs in groups.items():
        n = len(recs)
        b = emu.EmuBatch(L, R, C, k, sm, 30, np.stack([r["rng_in"] for r in recs]).astype(np.uint64))
        b.board[:] = np.stack([r["board"] for r in recs]).astype(np.int8)
        b.trust = False
        b.step(np.array([int(r["action"]) for r in recs], np.int32), autoreset=False)
        for i, r in enumerate(recs):
            res = r["res"]
            assert np.array_equal(b.board[i], r["out"]), f"board {(R, C, k, sm)} rec {i}"
            assert np.array_equal(b.rng[i], r["rng_out"]), f"rng {(R, C, k, sm)} rec {i}"
            assert (b.reward[i], b.n_new[i], b.n_act[i]) == (res[0], res[2], res[3]), f"counters {(R, C, k, sm)} rec {i}"
        total += n
    assert total > 500


@pytest.mark.parametrize("name", ["c5_20x20k6", "gen_512_11x12k10", "gen_sb_6x6k7", "lean_512_9x15k15",
                                  "lean_sb_5x6k7", "wide_512_3x45k7"])
def test_rare_paths_emulated(emu_lib, name):
    """tests/test_gpu_paths.py's rollouts (effective-action policy, short
    episodes, crafted Lemire rejections before every 5th step) on the emulated
    kernels vs the oracle, and each listed site (in-move / generate shuffles,
    draw_colours replays, row-plane generate redos) hit."""
    from oracle import oracle as orc
    from oracle.policy_np import sample_effective_np
    from rejection_states import words_rejecting_at
    from test_gpu_paths import MOVES, VARIANTS, _inject
    from tile_match_gym_amd._native import COVER_NAMES
    from tile_match_gym_amd.seeding import batch_rng_words
    emu, L = emu_lib
    R, C, k, sm, _, _, sites = VARIANTS[name]
    n, T = 96, 30
    w = batch_rng_words(range(n))
    e = emu.EmuBatch(L, R, C, k, sm, MOVES, w)
    o = orc.OracleBatch(R, C, k, sm, MOVES, w)
    emu.cover(L, True)
    e.reset()
    o.reset()
    rs = np.random.default_rng(1)
    A = 2 * R * C - R - C
    for t in range(T):
        inj = _inject(t, n, rs)
        if inj is not None:
            ww = words_rejecting_at(o.rng, inj[0], buffered=inj[1])
            o.rng[:] = ww
            e.rng[:] = ww
        a = sample_effective_np(o.eff, A, 7, 0, t)
        e.step(a, True)
        o.step(a, True)
        for f in ("board", "rng", "eff", "reward", "flags", "timer", "n_new", "n_act"):
            assert np.array_equal(getattr(e, f), getattr(o, f)), (name, t, f)
    hits = dict(zip(COVER_NAMES, emu.cover(L, True)))
    missing = [s for s in sites if s != "shuffle_gen" and hits[s] == 0]
    assert not missing, (name, {s: int(hits[s]) for s in sites})


@pytest.mark.parametrize("cfg", [(10, 10, 4, 0), (10, 10, 4, 14), (6, 6, 7, 14), (20, 20, 6, 15)])
def test_masked_reset_subsets_emulated(emu_lib, cfg):
    """reset(env_mask): the masked reset_kernel launch takes several envs per wave
    (kMaskedResetEnvs*); a random subset, a whole group of envs and a ragged tail
    regenerate exactly the selected boards (vs the oracle's reset of the same
    streams) and leave the others untouched."""
    from oracle import oracle as orc
    from tile_match_gym_amd.seeding import batch_rng_words
    emu, L = emu_lib
    R, C, k, sm = cfg
    n = 27 if R * C <= 128 else 11
    w = batch_rng_words(range(3000, 3000 + n))
    e = emu.EmuBatch(L, R, C, k, sm, 30, w)
    e.reset()
    rs = np.random.default_rng(R + C + k + sm)
    A = 2 * R * C - R - C
    for _ in range(2):                                      # move the streams on
        e.step(rs.integers(0, A, n).astype(np.int32), True)
    mask = (rs.random(n) < 0.4).astype(np.uint8)
    if n > 16:
        mask[:8] = 1                                        # a whole group of envs
    mask[-1] = 1                                            # the ragged tail
    before = {f: getattr(e, f).copy() for f in ("board", "rng", "timer", "eff")}
    o = orc.OracleBatch(R, C, k, sm, 30, e.rng.copy())
    o.reset()
    e.reset(mask)
    sel = mask.astype(bool)
    for f in ("board", "rng", "timer", "eff"):
        got = getattr(e, f).reshape(n, -1)
        want = np.where(sel[:, None], getattr(o, f).reshape(n, -1), before[f].reshape(n, -1))
        assert np.array_equal(got, want), f"{cfg}: {f}"


@pytest.mark.parametrize("cfg", [(10, 10, 4, 0), (8, 8, 3, 14), (7, 9, 5, 15), (12, 12, 5, 15)])
@pytest.mark.parametrize("mode", ["next_step", "same_step"])
def test_plan_vector_outputs_emulated(emu_lib, cfg, mode):
    """tmg_plan_config's Gymnasium vector-env step (include/tmg.h): next-step
    autoreset done by the kernels (inline for the lean kernels, by the masked
    reset launch for the others), and the per-env outputs written in the
    kernels' write-back — terminated / info bytes, action-mask bytes and int32
    boards (kept across steps: rows rewritten only where they change), moves
    left, same-step final boards — against the oracle driven with the same semantics."""
    from oracle import oracle as orc
    from tile_match_gym_amd.seeding import batch_rng_words
    from vector_ref import VectorOracle, mask_bytes
    emu, L = emu_lib
    R, C, k, sm = cfg
    n, moves = 12, 5
    A = 2 * R * C - R - C
    w = batch_rng_words(range(700, 700 + n))
    e = emu.EmuBatch(L, R, C, k, sm, moves, w)
    o = orc.OracleBatch(R, C, k, sm, moves, w)
    e.reset()
    o.reset()
    ref = VectorOracle(o, mode)
    outs = {"terminated": np.zeros((n, 4), np.uint8), "action_mask": mask_bytes(e.eff, A),
            "moves_left": np.full(n, moves, np.int64), "final_board": np.zeros((n, 2, R, C), np.int8),
            "board32": e.board.astype(np.int32)}
    rs = np.random.default_rng(R + C + k + sm)
    for t in range(3 * moves + 2):
        a = rs.integers(0, A, n).astype(np.int32)
        want = ref.step(a)
        e.step(a, mode={"same_step": 1, "next_step": 2}[mode], outputs=outs)
        for f in ("board", "rng", "eff", "timer"):
            assert np.array_equal(getattr(e, f), getattr(o, f)), (cfg, mode, t, f)
        for f in ("reward", "n_new", "n_act"):
            assert np.array_equal(getattr(e, f), want[f]), (cfg, mode, t, f)
        for f in ("terminated", "action_mask", "moves_left"):
            assert np.array_equal(outs[f], want[f]), (cfg, mode, t, f)
        assert np.array_equal(outs["board32"], o.board.astype(np.int32)), (cfg, mode, t, "board32")
        if mode == "same_step":
            term = want["terminated"][:, 0].astype(bool)
            assert np.array_equal(outs["final_board"][term], want["final_board"][term]), (cfg, t)


@pytest.mark.parametrize("cfg", [(10, 10, 4, 0), (8, 8, 3, 14), (12, 12, 5, 15)])
def test_plan_policy_in_kernel_emulated(emu_lib, cfg):
    """The examples' policy sampled inside the step kernel (tmg_plan_config
    policy): the actions it writes equal tmg_sample_effective's draw
    (oracle/policy_np.py) for the same (key, first_env, t), and the trajectory
    equals the oracle stepping those actions."""
    from oracle import oracle as orc
    from oracle.policy_np import sample_effective_np
    from tile_match_gym_amd.seeding import batch_rng_words
    emu, L = emu_lib
    R, C, k, sm = cfg
    n, key, first = 10, 99, 1000
    A = 2 * R * C - R - C
    w = batch_rng_words(range(first, first + n))
    e = emu.EmuBatch(L, R, C, k, sm, 7, w)
    o = orc.OracleBatch(R, C, k, sm, 7, w)
    e.reset()
    o.reset()
    acts = np.zeros(n, np.int32)
    for t in range(20):
        want = sample_effective_np(o.eff, A, key, first, t)
        e.step(acts, True, policy=(key, first, t))
        assert np.array_equal(acts, want), (cfg, t)
        o.step(want, True)
        for f in ("board", "rng", "eff", "reward", "flags", "timer", "n_new", "n_act"):
            assert np.array_equal(getattr(e, f), getattr(o, f)), (cfg, t, f)
