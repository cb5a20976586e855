"""CPU-side checks of the boundary: libtmg.so loads and exports exactly the
entry points include/tmg.h declares (no GPU calls)."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "tmg.h")).read()
    return sorted(set(re.findall(r"TMG_API\s+[\w\s\*]+?\b(tmg_\w+)\s*\(", txt)))


def test_header_declares_exports():
    from tile_match_gym_amd import _native
    assert header_symbols() == sorted(_native.EXPORTS)


def test_library_loads_and_exports():
    from tile_match_gym_amd import _native
    assert os.path.exists(_native.LIB_PATH), "run __graft_entry__.build() first"
    lib = ctypes.CDLL(_native.LIB_PATH)
    for name in header_symbols():
        assert hasattr(lib, name), name
    L = _native.load()
    assert L.tmg_abi_version() == _native.ABI_VERSION


def test_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from tile_match_gym_amd import _native
    with pytest.raises(_native.TmgError):
        _native.Context(0, 10, 10, 4, 0, 30)


def test_specials_mask_and_spaces():
    from tile_match_gym_amd import _native
    from tile_match_gym_amd.spaces import Box, Dict, Discrete
    assert _native.specials_mask(["cookie"], ["bomb", "vertical_laser", "horizontal_laser"]) == 15
    assert _native.specials_mask([], ["vertical_laser"]) == 2
    with pytest.raises(ValueError):
        _native.specials_mask(["bogus"], [])
    d = Discrete(5, seed=1)
    assert d.n == 5 and d.contains(4) and not d.contains(5)
    b = Box(low=np.zeros((2, 3, 4), np.int32), high=np.full((2, 3, 4), 4, np.int32), shape=(2, 3, 4), dtype=np.int32, seed=1)
    assert b.shape == (2, 3, 4) and b.contains(b.sample())
    D = Dict({"board": b, "num_moves_left": d})
    assert D["board"] is b and D.contains(D.sample())
    from tile_match_gym_amd.spaces import MultiDiscrete
    m = MultiDiscrete(np.full(7, 180, np.int64), seed=3)            # batched Discrete(180) over 7 envs
    x = m.sample()
    assert m.shape == (7,) and m.contains(x) and not m.contains(np.full(7, 180)) and not m.contains(x[:3])


def test_action_table_matches_reference_rule():
    """board.py:77-93 (first C(R-1) actions vertical, rest horizontal)."""
    from tile_match_gym_amd.tile_match_env import action_to_coords
    t = action_to_coords(3, 5)
    assert len(t) == 2 * 15 - 8
    assert t[0] == ((0, 0), (1, 0)) and t[9] == ((1, 4), (2, 4))
    assert t[10] == ((0, 0), (0, 1)) and t[-1] == ((2, 3), (2, 4))


def test_seeding_matches_numpy():
    from tile_match_gym_amd.seeding import generator_from_words, rng_words_from_seed
    for s in (0, 1, 3, 12345, 2**40):
        g1 = np.random.default_rng(s)
        g2 = generator_from_words(rng_words_from_seed(s))
        assert np.array_equal(g1.integers(1, 7, 50), g2.integers(1, 7, 50))


def test_viability_matches_state_counts():
    """tmg_viable (the tmg_create guard) == "some board is line-free and
    playable", i.e. compute_num_states' playable count > 0 (oracle restatement
    of utils.py:6-26, pinned by tests/golden/fn_count_states.npz)."""
    from oracle import oracle as orc
    from tile_match_gym_amd import _native
    for R in range(1, 5):
        for C in range(1, 5):
            for k in (1, 2, 3):
                if k ** (R * C) > 600_000:
                    continue
                playable, _ = orc.count_states(R, C, k)
                assert _native.viable(R, C, k) == (playable > 0), (R, C, k, playable)
    for shape in ((10, 10, 4), (20, 20, 6), (8, 8, 3), (1, 13, 2), (2, 64, 2), (64, 8, 15),
                  (16, 16, 2), (20, 20, 2), (12, 30, 2), (64, 8, 2)):     # 2 colours: found by backtracking
        assert _native.viable(*shape), shape


def test_create_refuses_unplayable_shapes():
    """Shapes whose generate_board loop (board.py:102-109) never ends are
    refused at creation instead of hanging a wave."""
    from tile_match_gym_amd import _native
    for shape in ((2, 2, 4), (3, 3, 1), (1, 3, 5), (2, 2, 2)):
        with pytest.raises(_native.TmgError, match="no playable board"):
            _native.Context(0, shape[0], shape[1], shape[2], 0, 30)
