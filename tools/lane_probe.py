"""Launch probe of the c2 step kernels (diagnostics, not the bench): reset, then
`--steps` normal steps back to back (timers held below the episode end, so no
regeneration), uniform actions or the in-kernel policy.  Meant to run under
rocprofv3 (--kernel-trace --stats, or one --pmc pass)."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tile-match-gym_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--boards", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=25)
    ap.add_argument("--policy", action="store_true")
    ap.add_argument("--k", type=int, default=4)
    args = ap.parse_args()
    from tile_match_gym_amd.shard import synthetic_actions
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    n = args.boards
    env = TileMatchVecEnv(n, 10, 10, args.k, 30, seed=0, device="cuda:0")
    acts = torch.from_numpy(synthetic_actions(range(n), args.steps, env.num_actions)).cuda()
    env.reset()
    torch.cuda.synchronize()
    for t in range(args.steps):
        if args.policy:
            env.step_effective(t)
        else:
            env.step_raw(acts[t])
    torch.cuda.synchronize()
    print("status", env.status(), flush=True)


if __name__ == "__main__":
    main()
