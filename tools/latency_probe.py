"""Latency probes (diagnostics, not the bench).

    python tools/latency_probe.py [--config c2]

reset_n   : one reset launch (generate_board for every env) over n boards, for
            growing n -> the single-board regeneration latency (small n) and
            the throughput regime (large n).
stagger   : per-step device time of the bench's staggered workload (timer0 =
            env mod 30, ~1/30 of the envs regenerate every step) vs the aligned
            one (normal steps + one storm step every 30), groups = 1 and 3.
"""
import argparse
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tile-match-gym_amd")]


def ev_time(fn):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--skip-reset", action="store_true")
    args = ap.parse_args()
    import bench
    from tile_match_gym_amd.shard import synthetic_actions
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    R, C, k, cl, co, nb, _ = bench.CONFIGS[args.config]
    if not args.skip_reset:
        for n in (1, 16, 256, 1024, 4096, 16384, nb):
            env = TileMatchVecEnv(n, R, C, k, 30, cl, co, seed=0, device="cuda:0")
            ts = [ev_time(env.reset) for _ in range(5)]
            print(f"reset n={n:7d}  us={statistics.median(ts):10.1f}  per-board-ns={1e3 * statistics.median(ts) / n:9.1f}",
                  flush=True)
            del env
    for groups in (1, 3):
        for stagger in (False, True):
            env = TileMatchVecEnv(nb, R, C, k, 30, cl, co, seed=0, device="cuda:0", groups=groups)
            A = env.num_actions
            acts = torch.from_numpy(synthetic_actions(range(nb), 90, A)).cuda()
            env.reset()
            if stagger:
                env.stagger_phases()
            torch.cuda.synchronize()
            ts = []
            for t in range(90):
                ts.append(ev_time(lambda: (env.step_raw(acts[t]), env.join())))
            ts = ts[30:]
            print(f"groups={groups} stagger={int(stagger)}  mean-us={statistics.mean(ts):8.1f}  median-us="
                  f"{statistics.median(ts):8.1f}  max-us={max(ts):8.1f}", flush=True)
            del env


if __name__ == "__main__":
    main()
