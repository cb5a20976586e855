"""N>1 path on CPU (gloo, world_size 2): the shard layout bench.py uses.

Each rank steps its own contiguous env shard (seeds = global index, actions a
function of (t, global index)); gathering the shards must give exactly the
single-process trajectory of all envs (G=1 vs G=N bit-equal).
The per-shard stepping here is the oracle — this tests the partition and the
timing reduction, not the kernels (those are tests/test_gpu_parity.py).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as orc
from tile_match_gym_amd.seeding import batch_rng_words
from tile_match_gym_amd.shard import max_over_ranks, shard_range, shard_seeds, synthetic_actions

R, C, K, SMASK, MOVES, STEPS, NPR = 8, 8, 4, 2 | 4 | 8, 10, 25, 48


def _run_shard(envs: range, seeds: range):
    o = orc.OracleBatch(R, C, K, SMASK, MOVES, batch_rng_words(seeds))
    o.reset()
    acts = synthetic_actions(envs, STEPS, orc.num_actions(R, C))
    rew = []
    for t in range(STEPS):
        o.step(acts[t], autoreset=True)
        rew.append(o.reward.copy())
    return o.board.copy(), o.rng.copy(), np.stack(rew)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        board, rng, rew = _run_shard(shard_range(rank, NPR), shard_seeds(rank, NPR))
        parts = [None] * world
        dist.all_gather_object(parts, (board, rng, rew))
        t = max_over_ranks(1.0 + rank, dist)
        if rank == 0:
            q.put((parts, t))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_layout_matches_single_process_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    parts, tmax = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert tmax == 2.0                                      # MAX over ranks of (1 + rank)
    board, rng, rew = _run_shard(range(0, world * NPR), range(0, world * NPR))
    assert np.array_equal(np.concatenate([p[0] for p in parts]), board)
    assert np.array_equal(np.concatenate([p[1] for p in parts]), rng)
    assert np.array_equal(np.concatenate([p[2] for p in parts], axis=1), rew)


def test_synthetic_actions_shard_invariant():
    a = synthetic_actions(range(0, 300), 7, 180)
    b = synthetic_actions(range(100, 200), 7, 180)
    assert np.array_equal(a[:, 100:200], b)
    assert a.min() >= 0 and a.max() < 180
    assert list(shard_seeds(3, 10, base_seed=5)) == list(range(35, 45))


def test_max_over_ranks_without_group():
    assert max_over_ranks(3.5) == 3.5
