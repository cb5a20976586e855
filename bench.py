#!/usr/bin/env python3
"""Benchmark: batched Board.step (BASELINE.json metric) on 1..8 MI355X.

    python bench.py --gpus N --steps K --warmup W [--config c2|c3|c5]

One "step" = one TileMatchEnv.step for every env of the shard (one HIP launch
per env group; `--groups` groups run on separate HIP streams so one group's
launch tail overlaps the next group's launch — same boards, same work),
uniform random actions pre-staged in HBM, autoreset on (num_moves = 30, so
every 30th step also regenerates every board).  Each rank steps its own
contiguous shard of envs (seed = global env index); there is no collective on
the data path.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "tile-match-gym_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "env-steps/sec (whole node), 65536×10×10 boards, at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0           # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

CONFIGS = {
    # name: (R, C, k, colourless, colour, boards per GPU, description)
    "c2": (10, 10, 4, [], [], 65536, "65536 x 10x10 boards per GPU, 4 colours, no specials"),
    "c3": (10, 10, 4, [], ["vertical_laser", "horizontal_laser", "bomb"], 262144,
           "262144 x 10x10 boards per GPU, 4 colours, v/h-laser + bomb"),
    "c5": (20, 20, 6, ["cookie"], ["vertical_laser", "horizontal_laser", "bomb"], 262144,
           "262144 x 20x20 boards per GPU, 6 colours, all specials"),
}


def algorithmic_bytes_per_env_step(R, C):
    """4RC (int8 colour+type read+write) + 48 (PCG64 state r/w
    + inc read) + 8 (half-word buffer r/w) + 4 (action) + 8 (timer r/w)
    + 16 (reward, n_new, n_act, flags) + 8*ceil(A/64) (effective mask)."""
    A = 2 * R * C - R - C
    return 4 * R * C + 48 + 8 + 4 + 8 + 16 + 8 * ((A + 63) // 64)


def cpu_baseline(R, C, k, smask, moves, budget_s=12.0, policy="uniform"):
    """The oracle (oracle/tmg_oracle.c, a bit-exact C port of the reference
    Board) timed on this host's cores over a bounded sample of the same
    workload (same seeds / action distribution; for the effective-action policy
    the numpy restatement of the sampler picks the actions, inside the timing)."""
    from oracle import oracle as orc
    from tile_match_gym_amd.seeding import batch_rng_words
    threads = min(16, os.cpu_count() or 1)
    n = 2048
    o = orc.OracleBatch(R, C, k, smask, moves, batch_rng_words(range(n)), threads=threads)
    o.reset()
    from tile_match_gym_amd.shard import synthetic_actions
    T = 300
    acts = synthetic_actions(range(n), T, 2 * R * C - R - C)
    steps = 0
    t0 = time.perf_counter()
    while True:
        for t in range(moves):
            if policy == "effective":
                from oracle.policy_np import sample_effective_np
                a = sample_effective_np(o.eff, 2 * R * C - R - C, 12345, 0, steps + t)
            else:
                a = acts[(steps + t) % T]
            o.step(a, autoreset=True)
        steps += moves
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    return {"value": round(n * steps / el, 1), "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"{n} envs x {steps} steps ({steps // moves} episodes incl. autoreset), "
                      f"{el:.1f} s, OpenMP over {threads} threads"}


def load_traffic(config):
    p = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(p):
        return None
    try:
        d = json.load(open(p))
        return d.get(config, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--boards", type=int, default=0, help="override boards per GPU")
    ap.add_argument("--groups", type=int, default=3,
                    help="env groups per GPU, each stepped on its own HIP stream (TileMatchVecEnv(groups=))")
    ap.add_argument("--policy", default="uniform", choices=("uniform", "effective"),
                    help="uniform: random actions over all A (headline); effective: every env samples uniformly "
                         "from its effective actions on device each step (SURVEY §8(d) secondary mode)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    from tile_match_gym_amd.shard import dist_env, max_over_ranks, shard_range, shard_seeds, synthetic_actions
    world, rank, local_rank = dist_env()
    dist = None
    if world > 1:
        import torch.distributed as dist
        # one process per GPU; TMG_DIST_BACKEND=gloo rehearses the N>1 path with
        # several ranks on one device (RCCL refuses duplicate GPUs)
        torch.cuda.set_device(local_rank % torch.cuda.device_count())
        dist.init_process_group(os.environ.get("TMG_DIST_BACKEND", "nccl"))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    R, C, k, cl, co, nb, desc = CONFIGS[args.config]
    if args.boards:
        nb = args.boards
    moves = 30
    env = TileMatchVecEnv(nb, R, C, k, moves, cl, co, seeds=shard_seeds(rank, nb), device=dev, autoreset=True,
                          groups=args.groups)
    A = env.num_actions
    T = 300
    acts = torch.from_numpy(synthetic_actions(shard_range(rank, nb), T, A)).to(dev)
    env.reset()
    first_env = shard_range(rank, nb).start

    def step(t):
        if args.policy == "effective":
            env.step_effective(t, first_env=first_env)       # sampler + step, both on device
        else:
            env.step_raw(acts[t % T])

    for t in range(args.warmup):
        step(t)
    env.join()
    torch.cuda.synchronize()

    # HIP events on the stream the first env group's kernels are launched on,
    # bracketing the timed region: its back-to-back launches' average duration
    # (the dominant kernel's per-launch time for the roofline)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    env.record(ev0)
    for i in range(args.steps):
        step(args.warmup + i)
    env.record(ev1)
    env.join()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / max(1, args.steps)
    launch_envs = env._ranges[0][1] - env._ranges[0][0]
    flags = env.flags.cpu().numpy()
    assert not (flags & 0xC0).any(), "error/overflow flag raised during the bench"
    el = max_over_ranks(el, dist, dev)
    kern_ms = max_over_ranks(kern_ms, dist, dev)

    if rank == 0:
        total = nb * world * args.steps
        value = total / el
        bpu = algorithmic_bytes_per_env_step(R, C)
        achieved = bpu * launch_envs / (kern_ms * 1e-3) / 1e9
        smask = (1 if "cookie" in cl else 0) | (2 if "vertical_laser" in co else 0) | \
                (4 if "horizontal_laser" in co else 0) | (8 if "bomb" in co else 0)
        cpu = None if (args.no_cpu_baseline or world > 1) else cpu_baseline(R, C, k, smask, moves, policy=args.policy)
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int8",
            "data": ("synthetic (uniform random actions, counter-based per (step, global env); seeds = global env index)"
                     if args.policy == "uniform" else
                     "synthetic (each step every env samples uniformly from its effective actions on device, "
                     "counter-based per (step, global env); seeds = global env index)"),
            "config": {"workload": f"{args.config}: {desc}, num_moves=30, autoreset"
                                   + ("" if args.policy == "uniform" else ", effective-action policy"),
                       "boards_per_gpu": nb, "rows": R, "cols": C, "colours": k,
                       "specials": cl + co, "env_groups_per_gpu": env.groups,
                       "parallelism": f"dp{world} (independent env shards, no collective)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": load_traffic(args.config) if args.policy == "uniform" else None,
                         "kernel_ms_per_launch": round(kern_ms, 4), "envs_per_launch": launch_envs,
                         "algorithmic_bytes_per_env_step": bpu,
                         "job_gbs": round(bpu * nb * args.steps / el / 1e9, 2)},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
