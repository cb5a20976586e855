"""Pins the CPU oracle (oracle/tmg_oracle.c) to vectors recorded from the
reference itself (tests/golden/make_goldens.py).  No GPU needed."""
import numpy as np
import pytest

from golden_io import load_records, load_traj, traj_names, replay_trajectory
from oracle import oracle as orc


def test_get_colour_lines_golden():
    """board.py:149-215 — exact list (order matters downstream)."""
    for r in load_records("lines"):
        got = orc.get_colour_lines(r["board"], r["k"], r["smask"])
        C = r["C"]
        exp, o = [], 0
        for L in r["lens"]:
            exp.append([(int(x) // C, int(x) % C) for x in r["cells"][o:o + L]])
            o += L
        assert got == exp


def test_process_colour_lines_golden():
    """board.py:269-327 via detect_colour_matches :133-147."""
    n = 0
    for r in load_records("lines"):
        if r["perr"]:
            continue
        coords, names, cols = orc.process_lines(r["board"], r["k"], r["smask"])
        exp, o = [], 0
        for L in r["plens"]:
            exp.append([int(x) for x in r["pcells"][o:o + L]])
            o += L
        assert coords == exp
        assert np.array_equal(names, r["pnames"])
        assert np.array_equal(cols, r["pcols"])
        n += len(exp)
    assert n > 100


def test_is_move_effective_golden():
    """board.py:735-787 and possible_move :558-569."""
    for r in load_records("effective"):
        m, any_ = orc.effective_mask(r["board"])
        assert np.array_equal(m, r["eff"].astype(bool))
        assert any_ == bool(r["possible"])


def test_gravity_golden():
    """board.py:217-229."""
    for r in load_records("gravity"):
        assert np.array_equal(orc.gravity(r["board"]), r["out"])


def test_activate_special_golden():
    """board.py:473-556 (recursive DFS, cookie argmax)."""
    for r in load_records("activate"):
        out, na, err = orc.activate(r["board"], r["cell"], r["combo"], r["k"], r["smask"])
        assert err == 0
        assert np.array_equal(out, r["out"])
        assert na == r["n_act"]


def test_combination_match_golden():
    """board.py:600-719."""
    for r in load_records("combo"):
        out, na, err = orc.combination(r["board"], r["action"], r["k"], r["smask"])
        assert err == 0
        assert np.array_equal(out, r["out"])
        assert na == r["n_act"]


def test_detect_resolve_golden():
    """board.py:397-471 + 572-597 (one cascade iteration, no gravity/refill)."""
    n = 0
    for r in load_records("resolve"):
        if r["err"]:
            continue
        out, na, nn, err = orc.detect_resolve(r["board"], r["k"], r["smask"])
        assert err == 0
        assert np.array_equal(out, r["out"])
        assert (na, nn) == (r["n_act"], r["n_new"])
        n += 1
    assert n > 100


def test_move_golden():
    """board.py:330-395 incl. refill RNG draws and the ensure-playable loop."""
    n = 0
    for r in load_records("move"):
        if r["err"]:
            continue
        out, rng, res, err = orc.move(r["board"], r["rng_in"], r["action"], r["k"], r["smask"])
        assert err == 0
        assert np.array_equal(out, r["out"])
        assert np.array_equal(rng, r["rng_out"])
        assert np.array_equal(res, r["res"])
        n += 1
    assert n > 500


def test_generate_board_golden():
    """board.py:95-131 seeded exactly like tile_match_env.py:49."""
    for r in load_records("generate"):
        from tile_match_gym_amd.seeding import rng_words_from_seed
        b, _ = orc.generate(r["R"], r["C"], r["k"], r["smask"], rng_words_from_seed(int(r["seed"])))
        assert np.array_equal(b, r["out"])


def test_rng_matches_numpy():
    """RNG contract against numpy's own Generator."""
    from tile_match_gym_amd.seeding import rng_words_from_seed
    for seed in range(10):
        for k in (2, 3, 4, 5, 6, 7, 9):
            g = np.random.default_rng(seed)
            w = rng_words_from_seed(seed)
            for n in (1, 7, 100):
                got, w = orc.rng_colours(w, k, n)
                assert np.array_equal(got, g.integers(1, k + 1, n))
            for n in (9, 64, 100, 400):
                got, w = orc.rng_shuffle(w, n)
                x = np.arange(n)
                g.shuffle(x)
                assert np.array_equal(got, x)


class _OracleBackend:
    def __init__(self, d, threads=1):
        self.o = orc.OracleBatch(d["R"], d["C"], d["k"], d["smask"], d["num_moves"], d["init_rng"], threads)

    def reset(self):
        self.o.reset()

    def step(self, a, autoreset):
        self.o.step(a, autoreset)

    get_board = lambda self: self.o.board
    get_rng = lambda self: self.o.rng
    get_eff = lambda self: self.o.eff
    get_reward = lambda self: self.o.reward
    get_flags = lambda self: self.o.flags
    get_n_new = lambda self: self.o.n_new
    get_n_act = lambda self: self.o.n_act


@pytest.mark.parametrize("name", traj_names())
@pytest.mark.parametrize("autoreset", [False, True])
def test_trajectory_golden(name, autoreset):
    """tile_match_env.py:84-124 whole trajectories (RNG-exact)."""
    d = load_traj(name)
    n = replay_trajectory(d, _OracleBackend(d, threads=2), autoreset)
    assert n > 0
