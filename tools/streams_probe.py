"""Probe: TileMatchVecEnv(groups=S) step loop cost with/without the per-step
fork (group streams wait on the caller's stream) and per-launch timing
events (diagnostics)."""
import os, sys, time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tile-match-gym_amd")]


def main():
    from tile_match_gym_amd.shard import synthetic_actions
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    n, K = 65536, 300
    acts = None
    for S in (1, 2, 3):
        env = TileMatchVecEnv(n, 10, 10, 4, 30, [], [], seeds=range(n), device="cuda:0", groups=S)
        if acts is None:
            acts = torch.from_numpy(synthetic_actions(range(n), K, env.num_actions)).cuda()
        env.reset()
        for mode in ("plain", "nofork"):
            if S == 1 and mode == "nofork":
                continue
            fork = env._fork
            if mode == "nofork":
                env._fork = lambda: None
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
            env.join(); torch.cuda.synchronize()
            t0 = time.perf_counter()
            for t in range(K):
                env.step_raw(acts[t])
            env.join(); torch.cuda.synchronize()
            el = time.perf_counter() - t0
            env._fork = fork
            print(f"S={S} {mode}: {n * K / el:.3e} env-steps/s", flush=True)


if __name__ == "__main__":
    main()
