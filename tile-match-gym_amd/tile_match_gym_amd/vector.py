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

One host call per step (a tmg_plan step over the env groups' streams): the
kernels themselves reset the envs due (next-step mode), keep the (N, A) mask
bytes of the envs whose mask changed, and write the terminated / info bytes,
moves left, the int32 observation boards and (same-step mode) the final
boards.  As in gymnasium (its vector envs' ``copy`` flag, default True) the
returned tensors are fresh copies; ``copy=False`` returns views of the env's
live buffers instead, overwritten by the next call (the benchmark's setting).
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
                 autoreset_mode: str = "next_step", obs_dtype=torch.int32, action_masks: bool = True,
                 groups: int = 1, copy: bool = True):
        if autoreset_mode not in ("next_step", "same_step"):
            raise ValueError("autoreset_mode must be 'next_step' or 'same_step'")
        if obs_dtype not in (torch.int32, torch.int8):
            raise ValueError("obs_dtype must be torch.int32 or torch.int8")
        self.autoreset_mode = autoreset_mode
        self.metadata = {"autoreset_mode": "NextStep" if autoreset_mode == "next_step" else "SameStep"}
        self.obs_dtype = obs_dtype
        self.action_masks = action_masks
        self.copy = copy
        self.vec = TileMatchVecEnv(num_envs, num_rows, num_cols, num_colours, num_moves, colourless_specials,
                                   colour_specials, seed=seed, device=device, autoreset=False, groups=groups)
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
        kw = dict(device=self.device)
        A = self.vec.num_actions
        # outputs the step kernels write (tmg_plan_config)
        self._term = torch.zeros((num_envs, 4), dtype=torch.uint8, **kw)   # terminated, combo, shuffled, error
        self._mask = torch.zeros((num_envs, A), dtype=torch.uint8, **kw) if action_masks else None
        self._left = torch.zeros(num_envs, dtype=torch.int64, **kw)
        self._final = (torch.zeros((num_envs, 2, R, C), dtype=torch.int8, **kw)
                       if autoreset_mode == "same_step" else None)
        self._obs32 = torch.zeros((num_envs, 2, R, C), dtype=torch.int32, **kw) if obs_dtype == torch.int32 else None
        self._trunc = torch.zeros(num_envs, dtype=torch.bool, **kw)
        self._zero_left = torch.zeros(num_envs, dtype=torch.int64, **kw)
        self._bits = torch.arange(64, device=self.device, dtype=torch.int64)
        self.vec.set_step_outputs(autoreset_mode, terminated=self._term, action_mask=self._mask,
                                  moves_left=self._left, final_board=self._final, board32=self._obs32)

    # ---------------------------------------------------------------- helpers
    def _c(self, t):
        return t.clone() if self.copy else t

    def _board(self, b):
        return self._c(b) if self.obs_dtype == torch.int8 else b.to(torch.int32)

    def _obs(self):
        b = self._obs32 if self._obs32 is not None else self.vec.board       # int32: kept by the kernels
        return {"board": self._c(b), "num_moves_left": self._c(self._left)}

    # -------------------------------------------------------------------- API
    def reset(self, seed=None, options=None):
        """Reset every env; `seed` (int) re-seeds env i with seed + i (list: one seed per env)."""
        v = self.vec
        if seed is not None:
            seeds = list(seed) if isinstance(seed, (list, tuple, np.ndarray)) else range(int(seed), int(seed) + self.num_envs)
            v.set_seed(seeds)
        v.reset()
        if self._obs32 is not None:        # the step kernels keep it up to date from here on
            self._obs32.copy_(v.board)
        self._term.zero_()
        self._left.fill_(self.num_moves)
        infos = {}
        if self.action_masks:          # the step kernels keep it up to date from here on
            m = ((v.eff.unsqueeze(-1) >> self._bits) & 1).reshape(self.num_envs, -1)[:, :v.num_actions]
            self._mask.copy_(m)
            infos["action_mask"] = self._c(self._mask.view(torch.bool))
        return self._obs(), infos

    def stagger_phases(self, **kw):
        """TileMatchVecEnv.stagger_phases on the envs (episode phases offset by
        timers, e.g. for benchmarking), with moves left updated."""
        self.vec.stagger_phases(**kw)
        self._left.copy_(self.num_moves - self.vec.timer.to(torch.int64))

    def step(self, actions):
        v = self.vec
        a = actions if isinstance(actions, torch.Tensor) else torch.as_tensor(actions)
        if a.device != self.device or a.dtype != torch.int32:
            a = a.to(device=self.device, dtype=torch.int32)
        a = a.contiguous()
        if a.shape != (self.num_envs,):
            raise ValueError(f"actions must have shape ({self.num_envs},)")
        v.step_raw(a)                      # next step: the envs that ended last call are reset in the kernel
        v.join()
        tb = self._term.view(torch.bool)
        infos = {}
        if self.autoreset_mode == "same_step":
            infos["final_obs"] = {"board": self._board(self._final), "num_moves_left": self._c(self._zero_left)}
            infos["_final_obs"] = self._c(tb[:, 0])
        infos["is_combination_match"] = self._c(tb[:, 1])
        infos["num_new_specials"] = self._c(v.n_new)
        infos["num_specials_activated"] = self._c(v.n_act)
        infos["shuffled"] = self._c(tb[:, 2])
        # a live env whose step met an internal error or ran out of list
        # capacity (byte 3: TMG_FLAG_ERROR | TMG_FLAG_OVERFLOW; never expected)
        infos["error"] = self._c(tb[:, 3])
        if self.action_masks:
            infos["action_mask"] = self._c(self._mask.view(torch.bool))
        return self._obs(), self._c(v.reward), self._c(tb[:, 0]), self._c(self._trunc), infos

    def close(self):
        self.vec.close()
