"""Launch-cost probes for the step kernel (diagnostics, not the bench).

    python tools/microbench.py [--config c2] [--boards N]

quick   : every env takes the ineffective-move exit (cached mask all zero,
          timer kept below num_moves) -> the dispatch + per-env I/O floor.
normal  : the bench's action stream, steps 1..28 of an episode (no autoreset).
storm   : the autoreset step (every env regenerates its board).
policy  : a step of the effective-action policy (bench --policy effective):
          every env plays an effective move.
Times are HIP-event device times per launch (median of the probes).
"""
import argparse
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tile-match-gym_amd")]


def timed(fn, reps):
    out = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b) * 1e3)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--boards", type=int, default=0)
    args = ap.parse_args()
    import bench
    from tile_match_gym_amd.shard import synthetic_actions
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    R, C, k, cl, co, nb, _ = bench.CONFIGS[args.config]
    nb = args.boards or nb
    env = TileMatchVecEnv(nb, R, C, k, 30, cl, co, seed=0, device="cuda:0")
    A = env.num_actions
    acts = torch.from_numpy(synthetic_actions(range(nb), 60, A)).cuda()
    env.reset()
    torch.cuda.synchronize()
    res = {}
    # normal steps 0..27 and the storm at step 29
    norm, storm = [], []
    for t in range(60):
        us = timed(lambda: env.step_raw(acts[t]), 1)[0]
        (storm if t % 30 == 29 else norm).append(us)
    res["normal_us"] = statistics.median(norm)
    res["storm_us"] = statistics.median(storm)
    # quick-exit floor
    saved_eff = env.eff.clone()
    env.eff.zero_()

    def quick():
        env.step_raw(acts[0])

    q = []
    for _ in range(20):
        env.timer.zero_()
        q += timed(quick, 1)
    res["quick_us"] = statistics.median(q)
    env.eff.copy_(saved_eff)
    # the examples' policy: every env plays one of its effective actions
    # (bench --policy effective), timers held below the episode end
    pol = []
    for t in range(20):
        env.timer.zero_()
        pol += timed(lambda: env.step_effective(t), 1)
    res["policy_us"] = statistics.median(pol)
    # back-to-back launches between one event pair (no host enqueue gap):
    # device time per launch of 25 quick-exit steps / 25 policy steps
    steps = {"quick_b2b_us": lambda: [env.step_raw(acts[0]) for _ in range(25)],
             "normal_b2b_us": lambda: [env.step_raw(acts[t]) for t in range(1, 26)],
             "policy_b2b_us": lambda: [env.step_effective(t) for t in range(25)]}
    for name, fn in steps.items():
        r = []
        for rep in range(5):
            env.timer.zero_()
            if name == "quick_b2b_us":
                env.eff.zero_()
            else:
                env.compute_effective()
            torch.cuda.synchronize()
            r += [x / 25 for x in timed(fn, 1)]
        res[name] = statistics.median(r)
    print({k: round(v, 2) for k, v in res.items()}, flush=True)


if __name__ == "__main__":
    main()
