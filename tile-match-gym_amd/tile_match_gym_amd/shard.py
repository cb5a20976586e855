"""Multi-GPU layout: one process per GPU, contiguous env shards, no collective
on the data path.

Boards are independent, so rank g of G owns global envs [g*n, (g+1)*n) and
seeds env i with ``base_seed + i`` (tile_match_env.py:49 per env).  Synthetic
actions are a pure function of (t, global env index), so every env follows
the same trajectory for any G.  The only collectives are outside the step
path: one barrier around the timed region and a MAX of the elapsed time.
"""
from __future__ import annotations

import os

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def dist_env():
    """(world_size, rank, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_range(rank: int, boards_per_rank: int) -> range:
    """Global env indices owned by `rank` (weak scaling: fixed boards per rank)."""
    return range(rank * boards_per_rank, (rank + 1) * boards_per_rank)


def shard_seeds(rank: int, boards_per_rank: int, base_seed: int = 0) -> range:
    r = shard_range(rank, boards_per_rank)
    return range(base_seed + r.start, base_seed + r.stop)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def synthetic_actions(env_ids: range, steps: int, num_actions: int, key: int = 12345) -> np.ndarray:
    """(steps, len(env_ids)) int32 actions, uniform in [0, num_actions):
    action[t, i] = hi32(splitmix64(key, t, global i) * A) — a counter-based
    stream, identical whatever the shard layout."""
    g = np.arange(env_ids.start, env_ids.stop, dtype=np.uint64)
    out = np.empty((steps, len(g)), dtype=np.int32)
    with np.errstate(over="ignore"):
        base = _splitmix64(np.uint64(key) * np.uint64(0xD1B54A32D192ED03) + g)
        for t in range(steps):
            h = _splitmix64(base ^ (np.uint64(t) * np.uint64(0x9E3779B97F4A7C15)))
            out[t] = ((h >> np.uint64(32)) * np.uint64(num_actions) >> np.uint64(32)).astype(np.int32)
    return out


def max_over_ranks(value: float, dist=None, device=None) -> float:
    """MAX of a per-rank scalar (bench timing); identity without a process group."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch
    if dist.get_backend() == "gloo":
        device = "cpu"
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
