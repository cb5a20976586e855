"""The reference's own hand-built edge cases (tests/board/test_move.py:35-337,
test_activation.py:9-434, test_combination_match.py:6-417,
test_match_detection.py:15-346, test_gravity, test_generate_board,
test_move_valid, test_possible_move), recorded from the reference itself as
data by tests/golden/make_ref_cases.py into tests/golden/ref_*.npz.

CPU: the oracle against every record.  GPU: the kernels, through the C ABI,
against the records they can be driven with (move by action, effective-action
masks, generate_board from a PCG64 state)."""
import numpy as np
import pytest
import torch

from golden_io import load_records
from oracle import oracle as orc


def test_ref_move_oracle():
    recs = load_records("move", "ref")
    assert len(recs) >= 8
    for r in recs:
        out, rng, res, err = orc.move(r["board"], r["rng_in"], r["action"], r["k"], r["smask"])
        assert err == 0
        assert np.array_equal(out, r["out"]) and np.array_equal(rng, r["rng_out"]) and np.array_equal(res, r["res"])


def test_ref_activate_oracle():
    recs = load_records("activate", "ref")
    assert len(recs) >= 8
    for r in recs:
        out, na, err = orc.activate(r["board"], r["cell"], r["combo"], r["k"], r["smask"])
        assert err == 0
        assert np.array_equal(out, r["out"]) and na == r["n_act"]


def test_ref_combination_oracle():
    recs = load_records("combo", "ref")
    assert len(recs) >= 10
    for r in recs:
        out, na, err = orc.combination(r["board"], r["action"], r["k"], r["smask"])
        assert err == 0
        assert np.array_equal(out, r["out"]) and na == r["n_act"]


def test_ref_lines_oracle():
    recs = load_records("lines", "ref")
    assert len(recs) >= 20
    for r in recs:
        got = orc.get_colour_lines(r["board"], r["k"], r["smask"])
        C, exp, o = r["C"], [], 0
        for L in r["lens"]:
            exp.append([(int(x) // C, int(x) % C) for x in r["cells"][o:o + L]])
            o += L
        assert got == exp
        if not r["perr"]:
            coords, names, cols = orc.process_lines(r["board"], r["k"], r["smask"])
            pexp, o = [], 0
            for L in r["plens"]:
                pexp.append([int(x) for x in r["pcells"][o:o + L]])
                o += L
            assert coords == pexp and np.array_equal(names, r["pnames"]) and np.array_equal(cols, r["pcols"])


def test_ref_gravity_effective_generate_oracle():
    for r in load_records("gravity", "ref"):
        assert np.array_equal(orc.gravity(r["board"]), r["out"])
    for r in load_records("effective", "ref"):
        m, any_ = orc.effective_mask(r["board"])
        assert np.array_equal(m, r["eff"].astype(bool)) and any_ == bool(r["possible"])
    n = 0
    for r in load_records("generate", "ref"):
        b, rng = orc.generate(r["R"], r["C"], r["k"], r["smask"], r["rng_in"])
        assert np.array_equal(b, r["out"]) and np.array_equal(rng, r["rng_out"])
        n += 1
    assert n > 1000


# ------------------------------------------------------------------- GPU
def _by_shape(recs):
    g = {}
    for r in recs:
        g.setdefault((r["R"], r["C"], r["k"], r["smask"]), []).append(r)
    return g


def _ctx(R, C, k, sm):
    from tile_match_gym_amd import _native
    if not _native.viable(R, C, k):
        return None
    return _native.Context(0, R, C, k, sm, 1 << 20)


@pytest.mark.gpu
def test_ref_move_gpu():
    """The reference's RNG-exact move() cases (test_move.py:35-337) on the step kernel."""
    n_all = 0
    for (R, C, k, sm), recs in _by_shape(load_records("move", "ref")).items():
        ctx = _ctx(R, C, k, sm)
        assert ctx is not None
        n = len(recs)
        dev = "cuda:0"
        board = torch.from_numpy(np.stack([r["board"] for r in recs]).astype(np.int8)).to(dev)
        rng = torch.from_numpy(np.stack([r["rng_in"] for r in recs]).astype(np.uint64).view(np.int64)).to(dev)
        timer = torch.zeros(n, dtype=torch.int32, device=dev)
        acts = torch.tensor([int(r["action"]) for r in recs], dtype=torch.int32, device=dev)
        out = torch.zeros((3, n), dtype=torch.int32, device=dev)
        flags = torch.zeros(n, dtype=torch.uint8, device=dev)
        eff = torch.zeros((n, ctx.mask_words), dtype=torch.int64, device=dev)
        ctx.step(n, board.data_ptr(), rng.data_ptr(), timer.data_ptr(), acts.data_ptr(), out[0].data_ptr(),
                 out[1].data_ptr(), out[2].data_ptr(), flags.data_ptr(), eff.data_ptr(), 0, 0,
                 torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        b, rw, o, f = board.cpu().numpy(), rng.cpu().numpy().view(np.uint64), out.cpu().numpy(), flags.cpu().numpy()
        for i, r in enumerate(recs):
            res = r["res"]
            assert np.array_equal(b[i], r["out"]), ((R, C, k, sm), i)
            assert np.array_equal(rw[i], r["rng_out"]), ((R, C, k, sm), i)
            assert (o[0, i], o[1, i], o[2, i]) == (res[0], res[2], res[3])
            assert bool(f[i] & 2) == bool(res[1]) and bool(f[i] & 4) == bool(res[4]) and not (f[i] & 0xC0)
        n_all += n
    assert n_all >= 8


@pytest.mark.gpu
def test_ref_effective_and_generate_gpu():
    """The reference's possible_move / is_move_effective boards
    (test_move_valid.py, test_possible_move.py) on effective_kernel, and its
    generate_board calls (test_generate_board.py) on reset_kernel from the
    recorded PCG64 states."""
    from golden_io import eff_words_to_bool
    dev = "cuda:0"
    s = torch.cuda.current_stream().cuda_stream
    checked = 0
    for (R, C, k, sm), recs in _by_shape(load_records("effective", "ref")).items():
        ctx = _ctx(R, C, k, sm)
        if ctx is None:
            continue
        n = len(recs)
        board = torch.from_numpy(np.stack([r["board"] for r in recs]).astype(np.int8)).to(dev)
        eff = torch.zeros((n, ctx.mask_words), dtype=torch.int64, device=dev)
        ctx.effective(n, board.data_ptr(), eff.data_ptr(), s)
        torch.cuda.synchronize()
        got = eff_words_to_bool(eff.cpu().numpy().view(np.uint64), ctx.num_actions)
        for i, r in enumerate(recs):
            assert np.array_equal(got[i], r["eff"].astype(bool)), ((R, C, k, sm), i)
        checked += n
    assert checked >= 100
    gen = 0
    for (R, C, k, sm), recs in _by_shape(load_records("generate", "ref")).items():
        ctx = _ctx(R, C, k, sm)
        assert ctx is not None
        n = len(recs)
        board = torch.zeros((n, 2, R, C), dtype=torch.int8, device=dev)
        rng = torch.from_numpy(np.stack([r["rng_in"] for r in recs]).astype(np.uint64).view(np.int64)).to(dev)
        timer = torch.zeros(n, dtype=torch.int32, device=dev)
        eff = torch.zeros((n, ctx.mask_words), dtype=torch.int64, device=dev)
        ctx.reset(n, board.data_ptr(), rng.data_ptr(), timer.data_ptr(), eff.data_ptr(), None, s)
        torch.cuda.synchronize()
        b, rw = board.cpu().numpy(), rng.cpu().numpy().view(np.uint64)
        for i, r in enumerate(recs):
            assert np.array_equal(b[i], r["out"]), ((R, C, k, sm), i)
            assert np.array_equal(rw[i], r["rng_out"]), ((R, C, k, sm), i)
        gen += n
    assert gen > 1000


@pytest.mark.gpu
def test_ref_board_facade_gpu():
    """The reference's board-level call pattern (board.py:95,330,558,735) on
    the facade Board: Board(..., np_random=, board=).move(c1, c2) /
    generate_board() / possible_move() / is_move_effective(board, c1, c2),
    against the reference's own recorded cases."""
    from tile_match_gym_amd.seeding import generator_from_words
    from tile_match_gym_amd.tile_match_env import Board, action_to_coords, is_move_effective
    SP = {1: "cookie", 2: "vertical_laser", 4: "horizontal_laser", 8: "bomb"}

    def lists(sm):
        return ([SP[1]] if sm & 1 else []), [SP[b] for b in (2, 4, 8) if sm & b]

    for r in load_records("move", "ref"):
        cl, co = lists(r["smask"])
        b = Board(r["R"], r["C"], r["k"], cl, co, np_random=generator_from_words(r["rng_in"]),
                  board=r["board"].astype(np.int32))
        c1, c2 = action_to_coords(r["R"], r["C"])[int(r["action"])]
        res = b.move(c1, c2)
        assert np.array_equal(b.board, r["out"]) and np.array_equal(b.rng_words, r["rng_out"])
        assert res == (int(r["res"][0]), bool(r["res"][1]), int(r["res"][2]), int(r["res"][3]), bool(r["res"][4]))
        with pytest.raises(ValueError):
            b.move((0, 0), (2, 2))                               # board.py:349-350
    for r in load_records("generate", "ref")[:200]:
        cl, co = lists(r["smask"])
        b = Board(r["R"], r["C"], r["k"], cl, co, np_random=generator_from_words(r["rng_in"]))
        b.generate_board()
        assert np.array_equal(b.board, r["out"]) and np.array_equal(b.rng_words, r["rng_out"])
    n = small = 0
    for r in load_records("effective", "ref"):
        R, C = r["R"], r["C"]
        if max(R, C) < 3 or not _native_viable(R, C, max(2, r["k"])):
            # a shape no generated board can take (e.g. 2x2): the reference's
            # is_move_effective / possible_move still answer for it
            small += 1
            eff = np.zeros(2 * R * C - R - C, bool)
            for a, (c1, c2) in enumerate(action_to_coords(R, C)):
                eff[a] = is_move_effective(r["board"], c1, c2)
            assert np.array_equal(eff, r["eff"].astype(bool)), (R, C)
            continue
        b = Board(R, C, max(2, r["k"]), [], [], board=r["board"].astype(np.int32))
        eff = np.zeros(b.num_actions, bool)
        eff[b.effective_actions()] = True
        assert np.array_equal(eff, r["eff"].astype(bool)) and b.possible_move() == bool(r["possible"])
        if n < 8:
            for a in (0, b.num_actions - 1):
                c1, c2 = b.action_to_coords[a]
                assert is_move_effective(r["board"], c1, c2) == bool(r["eff"][a])
                assert is_move_effective(r["board"], c2, c1) == bool(r["eff"][a])
        n += 1
    assert n >= 100


def _native_viable(R, C, k):
    from tile_match_gym_amd import _native
    return _native.viable(R, C, k)


@pytest.mark.gpu
def test_ref_combination_boards_gpu():
    """The reference's combination_match boards (test_combination_match.py:6-417:
    every special pair) driven through tmg_step with their recorded action on
    the kernels — combination, gravity, refill, the cascade and the
    ensure-playable loop (board.py:357-391, 600-719) — from 16 PCG64 states
    each, against the oracle's move() on the same inputs."""
    from tile_match_gym_amd.seeding import batch_rng_words
    dev = "cuda:0"
    s = torch.cuda.current_stream().cuda_stream
    reps, total = 16, 0
    for (R, C, k, sm), recs in _by_shape(load_records("combo", "ref")).items():
        ctx = _ctx(R, C, k, sm)
        assert ctx is not None, (R, C, k)
        boards = np.stack([r["board"] for r in recs for _ in range(reps)]).astype(np.int8)
        acts = np.array([int(r["action"]) for r in recs for _ in range(reps)], np.int32)
        n = boards.shape[0]
        words = batch_rng_words(range(4000 + total, 4000 + total + n))
        board = torch.from_numpy(boards).to(dev)
        rng = torch.from_numpy(words.view(np.int64).copy()).to(dev)
        timer = torch.zeros(n, dtype=torch.int32, device=dev)
        dacts = torch.from_numpy(acts).to(dev)
        out = torch.zeros((3, n), dtype=torch.int32, device=dev)
        flags = torch.zeros(n, dtype=torch.uint8, device=dev)
        eff = torch.zeros((n, ctx.mask_words), dtype=torch.int64, device=dev)
        ctx.step(n, board.data_ptr(), rng.data_ptr(), timer.data_ptr(), dacts.data_ptr(), out[0].data_ptr(),
                 out[1].data_ptr(), out[2].data_ptr(), flags.data_ptr(), eff.data_ptr(), 0, 0, s)
        torch.cuda.synchronize()
        b, rw, o, f = board.cpu().numpy(), rng.cpu().numpy().view(np.uint64), out.cpu().numpy(), flags.cpu().numpy()
        for i in range(n):
            want_b, want_rng, res, err = orc.move(boards[i], words[i], int(acts[i]), k, sm)
            assert err == 0
            assert res[1] == 1, "a combination record must take the combination branch"
            assert np.array_equal(b[i], want_b), ((R, C, k, sm), i)
            assert np.array_equal(rw[i], want_rng), ((R, C, k, sm), i)
            assert (o[0, i], o[1, i], o[2, i]) == (res[0], res[2], res[3]), ((R, C, k, sm), i)
            assert bool(f[i] & 2) and bool(f[i] & 4) == bool(res[4]) and not (f[i] & 0xC0)
        total += n
    assert total == 13 * reps
