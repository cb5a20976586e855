"""TileMatchVectorEnv — the Gymnasium (>= 1.0) vector-env surface over
TileMatchVecEnv.

Per env the transition is the reference's TileMatchEnv (tile_match_env.py:84-124);
batching follows gymnasium.vector.VectorEnv:

* ``reset(seed=None, options=None) -> (obs, infos)``;
  ``step(actions) -> (obs, rewards, terminations, truncations, infos)``.
* ``autoreset_mode="next_step"`` (gymnasium's default): the step after an
  env terminates resets it — that call ignores its action and returns the
  reset observation with reward 0 and terminated False.
  ``"same_step"``: a terminating env is reset inside the same call; its last
  observation is in ``infos["final_obs"]`` (board / num_moves_left, valid where
  ``infos["_final_obs"]``).
* Resets continue each env's own PCG64 stream (== the reference's reset()
  without a seed, tile_match_env.py:84-87), so env i seeded with s follows
  TileMatchEnv(..., seed=s).
* obs: ``{"board": (N, 2, R, C), "num_moves_left": (N,)}`` device tensors;
  ``obs_dtype=torch.int32`` (the reference's dtype, a converted copy) or
  ``torch.int8`` (zero-copy view of the live state).
* infos: the reference's step info keys (is_combination_match,
  num_new_specials, num_specials_activated, shuffled) as (N,) tensors, and
  ``action_mask`` — (N, A) bool of effective actions (tile_match_env.py:118-124;
  all False for a terminated env) — when ``action_masks=True``.
* Truncation never happens in the reference (tile_match_env.py:112): all False.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _native
from .spaces import Box, Dict, Discrete, MultiDiscrete
from .vec_env import TileMatchVecEnv


class TileMatchVectorEnv:
    metadata = {"autoreset_mode": "NextStep"}

    def __init__(self, num_envs: int, num_rows: int, num_cols: int, num_colours: int, num_moves: int,
                 colourless_specials=(), colour_specials=(), seed: int = 0, device=None,
                 autoreset_mode: str = "next_step", obs_dtype=torch.int32, action_masks: bool = True):
        if autoreset_mode not in ("next_step", "same_step"):
            raise ValueError("autoreset_mode must be 'next_step' or 'same_step'")
        if obs_dtype not in (torch.int32, torch.int8):
            raise ValueError("obs_dtype must be torch.int32 or torch.int8")
        self.autoreset_mode = autoreset_mode
        self.metadata = {"autoreset_mode": "NextStep" if autoreset_mode == "next_step" else "SameStep"}
        self.obs_dtype = obs_dtype
        self.action_masks = action_masks
        self.vec = TileMatchVecEnv(num_envs, num_rows, num_cols, num_colours, num_moves, colourless_specials,
                                   colour_specials, seed=seed, device=device, autoreset=False)
        self.num_envs = num_envs
        self.device = self.vec.device
        self.num_moves = num_moves
        R, C = num_rows, num_cols
        nsp = len(colour_specials)
        # tile_match_env.py:52-77 (type plane: low = -num_colourless_specials, high = num_colour_specials + 2)
        low = np.array([np.zeros((R, C), np.int32), np.full((R, C), -len(colourless_specials), np.int32)])
        high = np.array([np.full((R, C), num_colours, np.int32), np.full((R, C), nsp + 2, np.int32)])
        self.single_observation_space = Dict({"board": Box(low=low, high=high, shape=(2, R, C), dtype=np.int32),
                                              "num_moves_left": Discrete(num_moves + 1)})
        self.single_action_space = Discrete(self.vec.num_actions)
        # batched as gymnasium.vector.utils.batch_space does: Box -> stacked Box,
        # Discrete(n) -> MultiDiscrete([n] * num_envs)
        self.observation_space = Dict({
            "board": Box(low=np.broadcast_to(low, (num_envs, 2, R, C)), high=np.broadcast_to(high, (num_envs, 2, R, C)),
                         shape=(num_envs, 2, R, C), dtype=np.int32),
            "num_moves_left": MultiDiscrete(np.full(num_envs, num_moves + 1, dtype=np.int64))})
        self.action_space = MultiDiscrete(np.full(num_envs, self.vec.num_actions, dtype=np.int64))
        self._autoreset = torch.zeros(num_envs, dtype=torch.bool, device=self.device)
        self._bits = torch.arange(64, device=self.device, dtype=torch.int64)

    # ---------------------------------------------------------------- helpers
    def _obs(self):
        b = self.vec.board if self.obs_dtype == torch.int8 else self.vec.board.to(torch.int32)
        return {"board": b, "num_moves_left": (self.num_moves - self.vec.timer).to(torch.int64)}

    def _mask(self):
        v = self.vec
        m = ((v.eff.unsqueeze(-1) >> self._bits) & 1).reshape(self.num_envs, -1)[:, :v.num_actions]
        return m.bool()

    def _reset_where(self, m: torch.Tensor):
        v = self.vec
        mm = m.to(torch.uint8).contiguous()
        v.ctx.reset(v.num_envs, v.board.data_ptr(), v.rng.data_ptr(), v.timer.data_ptr(), v.eff.data_ptr(),
                    mm.data_ptr(), v._stream())

    # -------------------------------------------------------------------- API
    def reset(self, seed=None, options=None):
        """Reset every env; `seed` (int) re-seeds env i with seed + i (list: one seed per env)."""
        if seed is not None:
            seeds = list(seed) if isinstance(seed, (list, tuple, np.ndarray)) else range(int(seed), int(seed) + self.num_envs)
            self.vec.set_seed(seeds)
        self.vec.reset()
        self._autoreset.zero_()
        infos = {}
        if self.action_masks:
            infos["action_mask"] = self._mask()
        return self._obs(), infos

    def step(self, actions):
        v = self.vec
        a = torch.as_tensor(actions, device=self.device).to(torch.int32).contiguous()
        if a.shape != (self.num_envs,):
            raise ValueError(f"actions must have shape ({self.num_envs},)")
        prev_reset = self._autoreset.clone()
        v.step_raw(a)                      # envs that ended last step: FLAG_ERROR, state untouched
        flags = v.flags
        term = (flags & _native.FLAG_DONE) != 0
        infos = {}
        if self.autoreset_mode == "next_step":
            self._reset_where(prev_reset)
            term = term & ~prev_reset
            rewards = torch.where(prev_reset, torch.zeros_like(v.reward), v.reward)
            self._autoreset = term.clone()
        else:
            rewards = v.reward.clone()
            if self.obs_dtype == torch.int8:
                final_board = v.board.clone()
            else:
                final_board = v.board.to(torch.int32)
            infos["final_obs"] = {"board": final_board,
                                  "num_moves_left": (self.num_moves - v.timer).to(torch.int64)}
            infos["_final_obs"] = term.clone()
            self._reset_where(term)
        live = ~prev_reset if self.autoreset_mode == "next_step" else torch.ones_like(term)
        zero_i = torch.zeros_like(v.n_new)
        infos["is_combination_match"] = ((flags & _native.FLAG_COMBO) != 0) & live
        infos["num_new_specials"] = torch.where(live, v.n_new, zero_i)
        infos["num_specials_activated"] = torch.where(live, v.n_act, zero_i)
        infos["shuffled"] = ((flags & _native.FLAG_SHUFFLED) != 0) & live
        # a live env whose step met an internal error / capacity overflow (never expected)
        infos["error"] = ((flags & (_native.FLAG_ERROR | _native.FLAG_OVERFLOW)) != 0) & live
        if self.action_masks:
            infos["action_mask"] = self._mask()
        trunc = torch.zeros_like(term)
        return self._obs(), rewards, term, trunc, infos

    def close(self):
        self.vec.close()
