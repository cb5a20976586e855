"""One rank of the multi-process shard check (test helper, run by
tests/test_gpu_multiproc.py as WORLD_SIZE fresh processes).

Rank r steps its contiguous shard of the global envs (shard.py: seeds = global
env index, tile_match_env.py:49-50 per env) with TileMatchVecEnv on its device
(all ranks share cuda:0 on a one-GPU box), gathers the shard's final state
over gloo, and rank 0 compares the gathered batch with the single-process
oracle run over the whole range.  Prints one JSON line per rank.

    RANK=.. WORLD_SIZE=.. MASTER_ADDR=127.0.0.1 MASTER_PORT=.. python tests/dist_shard_run.py \
        R C k smask envs_per_rank steps policy
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "tile-match-gym_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)


def main():
    R, C, k, sm, per, steps = (int(x) for x in sys.argv[1:7])
    policy = sys.argv[7]
    import torch
    import torch.distributed as dist
    from tile_match_gym_amd.shard import dist_env, shard_range, shard_seeds, synthetic_actions
    world, rank, local_rank = dist_env()
    dist.init_process_group("gloo")
    torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()))
    dev = torch.device("cuda", torch.cuda.current_device())
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    cl = ["cookie"] if sm & 1 else []
    co = [nm for b, nm in ((8, "bomb"), (2, "vertical_laser"), (4, "horizontal_laser")) if sm & b]
    rng_ = shard_range(rank, per)
    env = TileMatchVecEnv(per, R, C, k, 30, cl, co, seeds=shard_seeds(rank, per), device=dev, groups=2)
    env.reset()
    acts = torch.from_numpy(synthetic_actions(rng_, steps, env.num_actions)).to(dev)
    rew = torch.zeros(per, dtype=torch.int64, device=dev)
    for t in range(steps):
        if policy == "effective":
            env.step_effective(t, first_env=rng_.start)
        else:
            env.step_raw(acts[t])
        env.join()
        rew += env.reward.to(torch.int64)
    torch.cuda.synchronize()
    mine = {"board": env.board.cpu(), "rng": env.rng.cpu(), "timer": env.timer.cpu(), "eff": env.eff.cpu(),
            "reward_sum": rew.cpu(), "flags": env.flags.cpu()}
    status = env.status()
    gathered = {}
    for key, t in mine.items():
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t.contiguous())
        gathered[key] = torch.cat(parts).numpy()
    result = {"rank": rank, "world": world, "envs": [rng_.start, rng_.stop], "status": status}
    if rank == 0:
        from oracle import oracle as orc
        from oracle.policy_np import sample_effective_np
        from tile_match_gym_amd.seeding import batch_rng_words
        n = per * world
        o = orc.OracleBatch(R, C, k, sm, 30, batch_rng_words(range(n)), threads=8)
        o.reset()
        all_acts = synthetic_actions(range(n), steps, env.num_actions)
        rsum = np.zeros(n, np.int64)
        for t in range(steps):
            a = sample_effective_np(o.eff, env.num_actions, 12345, 0, t) if policy == "effective" else all_acts[t]
            o.step(a, autoreset=True)
            rsum += o.reward
        mism = {}
        for key, want in (("board", o.board), ("rng", o.rng.view(np.int64)), ("timer", o.timer),
                          ("eff", o.eff.view(np.int64)), ("reward_sum", rsum), ("flags", o.flags)):
            got = gathered[key]
            bad = np.nonzero((got.reshape(n, -1) != want.reshape(n, -1)).any(axis=1))[0]
            if bad.size:
                mism[key] = int(bad.size)
        result.update(equal=not mism, mismatches=mism, envs_total=n)
    print(json.dumps(result), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
