"""tile_match_gym_amd — MI355X-native batched tile-match Board.

Drop-in for akshilpatel/tile-match-gym's hot path: `TileMatchEnv` keeps the
reference's Gymnasium reset/step API and spaces (tile_match_env.py:14-150),
`TileMatchVecEnv` steps N boards per HIP launch, `TileMatchVectorEnv` puts the
Gymnasium vector-env surface on it.  The wrappers (`OneHotWrapper`,
`ProportionRewardWrapper`, batched `VecOneHot`) and `compute_num_states`
mirror the reference's wrappers.py / utils.py.  All run in libtmg.so (csrc/,
C ABI in include/tmg.h); there is no CPU fallback.
"""
from ._native import TmgError, load as load_native  # noqa: F401
from .seeding import rng_words_from_seed, batch_rng_words  # noqa: F401


def __getattr__(name):  # lazy: importing torch-backed classes only when used
    if name == "TileMatchEnv":
        from .tile_match_env import TileMatchEnv
        return TileMatchEnv
    if name == "TileMatchVecEnv":
        from .vec_env import TileMatchVecEnv
        return TileMatchVecEnv
    if name == "TileMatchVectorEnv":
        from .vector import TileMatchVectorEnv
        return TileMatchVectorEnv
    if name in ("OneHotWrapper", "ProportionRewardWrapper", "VecOneHot"):
        from . import wrappers
        return getattr(wrappers, name)
    if name == "compute_num_states":
        from .utils import compute_num_states
        return compute_num_states
    raise AttributeError(name)


try:  # same gym id as the reference (src/tile_match_gym/__init__.py:3)
    from gymnasium.envs.registration import register as _register
    _register(id="TileMatch-v0", entry_point="tile_match_gym_amd.tile_match_env:TileMatchEnv")
except Exception:
    pass
