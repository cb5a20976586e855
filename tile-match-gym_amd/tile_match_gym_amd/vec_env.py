"""TileMatchVecEnv — N independent TileMatchEnv boards stepped by one HIP launch.

State lives in PyTorch-ROCm tensors on one device (layout: include/tmg.h);
each reset/step enqueues one kernel on the current torch stream through the
C ABI.  Per env the semantics are the reference's TileMatchEnv
(tile_match_env.py:84-124) with one numpy PCG64 stream per env, so env i
seeded with s follows exactly the trajectory of TileMatchEnv(..., seed=s).

Autoreset (default on): an env whose episode ends is regenerated inside the
same step call, continuing its RNG stream (== the reference's reset() without
a seed, tile_match_env.py:84-87); reward/flags describe the final move,
`info["final_board"]` is not kept (pass autoreset=False to inspect it).

groups > 1: the envs are split into that many contiguous groups, each stepped
on its own HIP stream, so the tail of one group's launch overlaps the next
launch of another (envs are independent; results are identical to
groups=1).  `step_raw` then only enqueues: call `join()` before reading the
state or outputs on the current stream (`step`, `reset` and the other
accessors join themselves).
"""
from __future__ import annotations

import json

import numpy as np
import torch

from . import _native
from .seeding import batch_rng_words, rng_words_from_seed

CHECKPOINT_FORMAT = 1
_STATE_ARRAYS = ("board", "rng", "timer", "eff")


def save_state(path, arrays: dict, config: dict) -> None:
    """Write a batched-env checkpoint: the four state arrays (include/tmg.h
    layout) plus the env config as JSON, in one .npz (no pickled objects)."""
    meta = dict(config, format=CHECKPOINT_FORMAT)
    np.savez(path, config=np.array(json.dumps(meta, sort_keys=True)),
             **{k: np.ascontiguousarray(arrays[k]) for k in _STATE_ARRAYS})


def load_state(path):
    """(arrays, config) of a checkpoint written by save_state (numpy.load with
    allow_pickle=False)."""
    with np.load(path, allow_pickle=False) as z:
        config = json.loads(str(z["config"]))
        if config.get("format") != CHECKPOINT_FORMAT:
            raise ValueError(f"unsupported checkpoint format {config.get('format')!r}")
        arrays = {k: z[k].copy() for k in _STATE_ARRAYS}
    return arrays, config


def _ptr(t: torch.Tensor):
    return t.data_ptr() if t is not None else None


def _raw_stream(device_index: int) -> int:
    """The current HIP stream of the device as a raw handle (the cheap accessor
    when this torch has it)."""
    return torch.cuda.current_stream(device_index).cuda_stream


if hasattr(torch._C, "_cuda_getCurrentRawStream"):
    _raw_stream = torch._C._cuda_getCurrentRawStream        # noqa: F811


class TileMatchVecEnv:
    def __init__(self, num_envs: int, num_rows: int, num_cols: int, num_colours: int, num_moves: int,
                 colourless_specials=(), colour_specials=(), seed: int = 0, seeds=None, device=None,
                 autoreset: bool = True, groups: int = 1, lib_path: str = None):
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        device = torch.device(device)
        if device.type != "cuda":
            raise _native.TmgError("TileMatchVecEnv runs on a HIP device only (no CPU fallback)")
        self.device = device
        self.num_envs = int(num_envs)
        self.num_rows, self.num_cols, self.num_colours, self.num_moves = num_rows, num_cols, num_colours, num_moves
        self.colourless_specials = list(colourless_specials)
        self.colour_specials = list(colour_specials)
        self.specials_mask = _native.specials_mask(colourless_specials, colour_specials)
        # the one source of truth for the autoreset semantics: "none",
        # "same_step" or "next_step" (set_step_outputs); `autoreset` derives from it
        self._autoreset_mode = "same_step" if autoreset else "none"
        # lib_path: another build of libtmg.so (a diagnostic variant) for this env's context
        self.ctx = _native.Context(device.index if device.index is not None else torch.cuda.current_device(),
                                   num_rows, num_cols, num_colours, self.specials_mask, num_moves, lib_path=lib_path)
        self.num_actions = self.ctx.num_actions
        self.mask_words = self.ctx.mask_words
        N = self.num_envs
        kw = dict(device=device)
        self.board = torch.zeros((N, 2, num_rows, num_cols), dtype=torch.int8, **kw)
        if seeds is None:
            seeds = range(int(seed), int(seed) + N)
        self.rng = torch.from_numpy(batch_rng_words(seeds).view(np.int64)).to(device)
        self.timer = torch.zeros(N, dtype=torch.int32, **kw)
        self.eff = torch.zeros((N, self.mask_words), dtype=torch.int64, **kw)
        self.reward = torch.zeros(N, dtype=torch.int32, **kw)
        self.n_new = torch.zeros(N, dtype=torch.int32, **kw)
        self.n_act = torch.zeros(N, dtype=torch.int32, **kw)
        self.flags = torch.zeros(N, dtype=torch.uint8, **kw)
        self.actions = None                     # step_effective's sampled actions (N,) int32
        self.onehot = None                      # fused one-hot planes (attach_onehot)
        self._oh_code = _native.DTYPE_F32
        self._eff_valid = False
        groups = max(1, min(int(groups), N))
        self.groups = groups
        bounds = [g * N // groups for g in range(groups + 1)]
        self._ranges = [(bounds[g], bounds[g + 1]) for g in range(groups) if bounds[g + 1] > bounds[g]]
        self._streams = [torch.cuda.Stream(device) for _ in self._ranges] if groups > 1 else []
        # step plans (tmg_plan_*): one host call per batched step enqueues every
        # group's launches with their fork event; one plan per action source
        # (given actions / the in-kernel effective-action policy), configured
        # with the attached outputs
        bounds = [lo for lo, _ in self._ranges] + [N]
        streams = [st.cuda_stream for st in self._streams] if self._streams else [0]
        self._plans = {pol: _native.Plan(self.ctx, N, _ptr(self.board), _ptr(self.rng), _ptr(self.timer),
                                         _ptr(self.reward), _ptr(self.n_new), _ptr(self.n_act), _ptr(self.flags),
                                         _ptr(self.eff), bounds, streams) for pol in (False, True)}
        self._policy = (12345, 0)                   # (key, first_env) the policy plan is configured with
        self._vout = {}                             # extra outputs (set_step_outputs)
        self._held = []                             # action tensors the queued steps still read
        self._dev_index = device.index if device.index is not None else torch.cuda.current_device()
        self._configure()

    # ----------------------------------------------------------------- API
    @property
    def autoreset(self) -> bool:
        """Whether envs whose episode ends are reset (same step or, after
        set_step_outputs("next_step"), the next one).  Settable: True keeps a
        next-step mode and otherwise selects same-step; False selects none (the
        step plans are reconfigured)."""
        return self._autoreset_mode != "none"

    @property
    def autoreset_mode(self) -> str:
        return self._autoreset_mode

    @autoreset.setter
    def autoreset(self, value):
        mode = ("next_step" if self._autoreset_mode == "next_step" else "same_step") if value else "none"
        if mode != self._autoreset_mode:
            self.join()
            self._autoreset_mode = mode
            self._configure()

    def _stream(self):
        return _raw_stream(self._dev_index)

    def _configure(self):
        """(Re)configure both step plans: autoreset mode, fused one-hot planes,
        vector-env outputs, the policy's key and shard offset."""
        for pol, plan in self._plans.items():
            plan.config(self._autoreset_mode, policy=pol, key=self._policy[0], first_env=self._policy[1],
                        onehot=_ptr(self.onehot), onehot_dtype=self._oh_code, **self._vout)

    def set_step_outputs(self, autoreset_mode: str = None, terminated=None, action_mask=None, moves_left=None,
                         final_board=None, board32=None):
        """Outputs every step writes in the kernels' own write-back (tmg_plan_config):
        terminated (N, 4) uint8 (terminated, is_combination_match, shuffled, error),
        action_mask (N, A) uint8/bool (kept up to date: rows are rewritten where the
        mask changes, so initialise it after a reset), moves_left (N,) int64,
        final_board (N, 2, R, C) int8 (same-step autoreset: the last board of each
        env whose episode ended), board32 (N, 2, R, C) int32 (the boards in the
        reference's observation dtype, kept up to date like action_mask).
        autoreset_mode: "none", "same_step", "next_step"."""
        self.join()
        if autoreset_mode is not None:
            if autoreset_mode not in ("none", "same_step", "next_step"):
                raise ValueError("autoreset_mode must be 'none', 'same_step' or 'next_step'")
            self._autoreset_mode = autoreset_mode
        self._vout = {k: _ptr(v) for k, v in (("terminated", terminated), ("action_mask", action_mask),
                                               ("moves_left", moves_left), ("final_board", final_board),
                                               ("board32", board32))}
        self._vout_refs = (terminated, action_mask, moves_left, final_board, board32)
        self._configure()

    def set_seed(self, seeds):
        """Re-seed every env (== tile_match_env.py:79-82 per env)."""
        self.join()
        w = batch_rng_words(seeds)
        self.rng.copy_(torch.from_numpy(w.view(np.int64)))

    def stagger_phases(self, blocks: int = 0, first_env: int = 0, interleave: bool = False, shift: int = 0):
        """Offset the episode phases right after a reset by setting timers.  A
        timer of m is the state after m ineffective moves (board.py:352-353: no
        board or RNG change; tile_match_env.py:100 counts the move).

        blocks = 0: env i gets (first_env + i) mod num_moves, so every step
        finishes ~N/num_moves episodes (pass the shard's global offset as
        first_env to keep the layout shard-invariant).
        blocks = P > 0: each env group's range is split into Pg = ceil(P / groups)
        contiguous sub-blocks; sub-block j of group g starts at phase
        j * M / Pg + g * M / (Pg * groups) (M = num_moves, floors).  Every
        group then finishes a sub-block's episodes every M / Pg steps, and the
        groups take turns, so a window of a multiple of M / Pg steps holds the
        same reset work on every group's stream.
        interleave=True: env i belongs to block i mod P instead, so every group
        stream holds an equal part of every block's resets.
        shift: every phase advanced by `shift` steps (mod num_moves), i.e. the
        whole reset schedule moved `shift` steps earlier; the reset work per
        window of a multiple of the block spacing is unchanged."""
        self.join()
        N, M = self.num_envs, self.num_moves
        if blocks == 1:
            self.timer.zero_()
        elif blocks and blocks > 0 and interleave:
            # interleaved blocks: env i in block i mod P (every env group holds
            # all P blocks), block b starting at b * M // P
            i = torch.arange(N, device=self.device, dtype=torch.int64)
            self.timer.copy_(((i % blocks) * M // blocks % M).to(torch.int32))
        elif blocks and blocks > 0:
            G = len(self._ranges)
            Pg = max(1, -(-int(blocks) // G))
            t = torch.zeros(N, dtype=torch.int64)
            for g, (lo, hi) in enumerate(self._ranges):
                n = hi - lo
                for j in range(Pg):
                    a, b = lo + j * n // Pg, lo + (j + 1) * n // Pg
                    t[a:b] = (j * M // Pg + g * M // (Pg * G) + shift) % M
            self.timer.copy_(t.to(torch.int32).to(self.device))
        else:
            g = torch.arange(first_env, first_env + N, device=self.device, dtype=torch.int64)
            self.timer.copy_((g % M).to(torch.int32))

    def status(self, clear: bool = False) -> int:
        """Sticky _native.STATUS_* bits: OR over every env of every step since
        the last clear (waits for the device)."""
        self.join()
        return self.ctx.status(clear)

    def record(self, event, group: int = 0):
        """Record `event` on the stream group `group` is stepped on (the current
        stream for groups=1): HIP-event timing of that group's launches."""
        event.record(self._streams[group] if self._streams else torch.cuda.current_stream(self.device))

    def join(self):
        """Make the current stream wait for every group's queued steps (no-op for groups=1)."""
        if self._streams:
            self._plans[False].join(self._stream())
        self._held.clear()

    def reset(self, seed=None, env_mask=None):
        self.join()
        if seed is not None:
            self.set_seed(range(int(seed), int(seed) + self.num_envs))
        m = None
        if env_mask is not None:
            m = torch.as_tensor(env_mask, device=self.device).to(torch.uint8).contiguous()
        self.ctx.reset(self.num_envs, _ptr(self.board), _ptr(self.rng), _ptr(self.timer), _ptr(self.eff),
                       _ptr(m), self._stream(), self._oh(0), self._oh_code)
        self._eff_valid = True
        return self._obs(), {"effective_bits": self.eff}

    def step(self, actions):
        a = torch.as_tensor(actions, device=self.device)
        if a.dtype != torch.int32:
            a = a.to(torch.int32)
        a = a.contiguous()
        if a.shape != (self.num_envs,):
            raise ValueError(f"actions must have shape ({self.num_envs},)")
        self.step_raw(a)
        self.join()
        flags = self.flags
        info = {
            "is_combination_match": (flags & _native.FLAG_COMBO) != 0,
            "num_new_specials": self.n_new,
            "num_specials_activated": self.n_act,
            "shuffled": (flags & _native.FLAG_SHUFFLED) != 0,
            "effective_bits": self.eff,
            "error": (flags & _native.FLAG_ERROR) != 0,
            "overflow": (flags & _native.FLAG_OVERFLOW) != 0,
        }
        done = (flags & _native.FLAG_DONE) != 0
        return self._obs(), self.reward, done, torch.zeros_like(done), info

    def step_raw(self, actions_i32: torch.Tensor, fork: bool = True):
        """Enqueue one batched step (no output post-processing): the bench path.
        actions_i32: contiguous int32 (N,) on the device.  With groups > 1 call
        join() before reading results.  One host call (tmg_plan_step) enqueues
        every group's launches; the actions tensor is held until join().
        fork=False: nothing queued on the current stream since the previous
        step is read by this one (e.g. actions staged beforehand), so the group
        streams need not wait for it (saves the fork event per step)."""
        self._plans[False].step(actions_i32.data_ptr(), 0, int(self._eff_valid), self._stream(), int(fork))
        self._eff_valid = True
        if self._streams:
            self._held.append(actions_i32)
            if len(self._held) > 256:
                self.join()

    def step_effective(self, t: int, key: int = 12345, first_env: int = 0, fork: bool = True):
        """Enqueue one step of the examples' policy (src/examples/q_learning.py:19-25):
        every env takes an action drawn uniformly from its effective actions
        (tmg_sample_effective's draw, counter-based in (key, first_env + env, t),
        so a shard passing its global offset as first_env picks the same actions
        as the unsharded batch), sampled by the step kernel itself from the mask
        it reads anyway.  The sampled actions stay in self.actions."""
        # a mask from tmg_effective (hand-edited boards) may sit beside a line
        # on the board, so that step runs untrusted (tmg.h, trust_eff)
        trust = int(self._eff_valid)
        if not self._eff_valid:
            self.compute_effective()
        if self.actions is None:
            self.actions = torch.zeros(self.num_envs, dtype=torch.int32, device=self.device)
        if self._policy != (int(key), int(first_env)):
            self.join()
            self._policy = (int(key), int(first_env))
            self._configure()
        self._plans[True].step(self.actions.data_ptr(), int(t), trust, self._stream(), int(fork))
        self._eff_valid = True

    def capture_steps(self, actions=None, ts=None, policy: bool = False, key: int = 12345, first_env: int = 0):
        """Capture len(ts) batched steps into a HIP graph (tmg_plan_capture):
        run_graph() then enqueues all of them with one host call, the env
        groups still overlapping across the steps.  actions: a list of (N,)
        int32 device tensors, one per step (kept alive by the graph), or
        policy=True for the in-kernel effective-action policy (step counters
        ts).  Nothing runs at capture time; the graph assumes the state it is
        replayed on has this library's own masks (run it right after steps,
        resets or other graphs of this env)."""
        ts = list(range(len(actions))) if ts is None else [int(t) for t in ts]
        self.join()
        if policy:
            if self.actions is None:
                self.actions = torch.zeros(self.num_envs, dtype=torch.int32, device=self.device)
            if self._policy != (int(key), int(first_env)):
                self._policy = (int(key), int(first_env))
                self._configure()
            ptrs = [self.actions.data_ptr()] * len(ts)
        else:
            if len(actions) != len(ts):
                raise ValueError("one action tensor per step")
            ptrs = [a.data_ptr() for a in actions]
        side = torch.cuda.Stream(self.device)          # the NULL stream cannot be captured
        side.wait_stream(torch.cuda.current_stream(self.device))
        g = self._plans[bool(policy)].capture(ptrs, ts, int(self._eff_valid), side.cuda_stream)
        g.refs = (actions, side)
        return g

    def run_graph(self, graph):
        """Enqueue a captured run of steps (capture_steps) on the current stream."""
        graph.launch(self._stream())
        self._eff_valid = True

    def invalidate_effective_cache(self):
        """Call after editing self.board by hand."""
        self._eff_valid = False

    def compute_effective(self):
        self.join()
        self.ctx.effective(self.num_envs, _ptr(self.board), _ptr(self.eff), self._stream())
        return self.eff

    def effective_mask(self) -> torch.Tensor:
        """(N, A) bool mask of effective actions, unpacked from the bitmask."""
        self.join()
        bits = torch.arange(64, device=self.device, dtype=torch.int64)
        m = ((self.eff.unsqueeze(-1) >> bits) & 1).reshape(self.num_envs, -1)[:, :self.num_actions]
        return m.bool()

    # ------------------------------------------------------ fused one-hot
    def attach_onehot(self, dtype=torch.float32) -> torch.Tensor:
        """Keep OneHotWrapper planes (wrappers.py:56-69) of every board in a
        (N, channels, R, C) tensor that the step / reset kernels update in
        their own write-back (tmg_step_onehot): only boards a step changes are
        rewritten.  Encodes the current boards once (tmg_onehot); returns the
        tensor (also self.onehot).  Call refresh_onehot() after editing boards
        by hand with a trusted mask."""
        codes = {torch.float32: _native.DTYPE_F32, torch.uint8: _native.DTYPE_U8, torch.int32: _native.DTYPE_I32}
        if dtype not in codes:
            raise ValueError(f"dtype must be one of {list(codes)}")
        self.join()
        ch = self.ctx.onehot_channels()
        self.onehot = torch.zeros((self.num_envs, ch, self.num_rows, self.num_cols), dtype=dtype, device=self.device)
        self._oh_code = codes[dtype]
        self.refresh_onehot()
        self._configure()
        return self.onehot

    def refresh_onehot(self):
        self.join()
        self.ctx.onehot(self.num_envs, self.board.data_ptr(), self.onehot.data_ptr(), self._oh_code, self._stream())

    def _oh(self, lo):
        if self.onehot is None:
            return None
        return self.onehot.data_ptr() + lo * self.onehot[0].numel() * self.onehot.element_size()

    def _obs(self):
        return {"board": self.board, "num_moves_left": self.num_moves - self.timer}

    def rng_words(self) -> np.ndarray:
        self.join()
        return self.rng.cpu().numpy().view(np.uint64)

    # ------------------------------------------------------- checkpoint/restore
    def config(self) -> dict:
        return {"num_rows": self.num_rows, "num_cols": self.num_cols, "num_colours": self.num_colours,
                "num_moves": self.num_moves, "colourless_specials": self.colourless_specials,
                "colour_specials": self.colour_specials, "num_envs": self.num_envs, "autoreset": self.autoreset,
                "autoreset_mode": self._autoreset_mode}

    def state_dict(self) -> dict:
        """Host copy of the whole batched state: boards, the exact PCG64 stream
        position of every env (incl. numpy's buffered half-word), timers and the
        effective-action masks; restoring it continues every trajectory
        bit-exactly."""
        self.join()
        torch.cuda.synchronize(self.device)
        return {"board": self.board.cpu().numpy(), "rng": self.rng_words().copy(),
                "timer": self.timer.cpu().numpy(), "eff": self.eff.cpu().numpy().view(np.uint64).copy(),
                "eff_valid": self._eff_valid, "config": self.config()}

    def load_state_dict(self, sd: dict) -> None:
        cfg = sd["config"]
        mine = self.config()
        def norm(v):
            return list(v) if isinstance(v, (list, tuple)) else v

        for k in ("num_rows", "num_cols", "num_colours", "num_moves", "colourless_specials", "colour_specials",
                  "num_envs"):
            if norm(cfg[k]) != norm(mine[k]):
                raise ValueError(f"checkpoint {k}={cfg[k]!r} does not match this env ({mine[k]!r})")
        self.board.copy_(torch.from_numpy(np.ascontiguousarray(sd["board"], dtype=np.int8)))
        self.rng.copy_(torch.from_numpy(np.ascontiguousarray(sd["rng"], dtype=np.uint64).view(np.int64)))
        self.timer.copy_(torch.from_numpy(np.ascontiguousarray(sd["timer"], dtype=np.int32)))
        self.eff.copy_(torch.from_numpy(np.ascontiguousarray(sd["eff"], dtype=np.uint64).view(np.int64)))
        self._eff_valid = bool(sd.get("eff_valid", True))

    def save(self, path) -> None:
        sd = self.state_dict()
        cfg = dict(sd["config"], eff_valid=sd["eff_valid"])
        save_state(path, sd, cfg)

    @classmethod
    def load(cls, path, device=None) -> "TileMatchVecEnv":
        arrays, cfg = load_state(path)
        env = cls(cfg["num_envs"], cfg["num_rows"], cfg["num_cols"], cfg["num_colours"], cfg["num_moves"],
                  cfg["colourless_specials"], cfg["colour_specials"], seeds=range(cfg["num_envs"]), device=device,
                  autoreset=cfg["autoreset"])
        # next-step mode: the pending resets are implicit in timer == num_moves,
        # so the mode must come back with the state (older checkpoints: the bool)
        mode = cfg.get("autoreset_mode")
        if mode is not None and mode != env._autoreset_mode:
            env._autoreset_mode = mode
            env._configure()
        env.load_state_dict(dict(arrays, config=cfg, eff_valid=cfg.get("eff_valid", True)))
        return env

    def close(self):
        self.join()
        for plan in self._plans.values():
            plan.close()
        self.ctx.close()
