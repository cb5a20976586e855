"""Reset-kernel probe (diagnostics): times env.reset() (generate_board for
every env) — the autoreset 'storm' work without the step around it."""
import os, sys, statistics
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tile-match-gym_amd")]


def main():
    import bench
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    R, C, k, cl, co, nb, _ = bench.CONFIGS[cfg]
    env = TileMatchVecEnv(nb, R, C, k, 30, cl, co, seed=0, device="cuda:0")
    ts = []
    for _ in range(6):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); env.reset(); b.record(); torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    print(cfg, "reset_us", [round(t) for t in ts], "median", round(statistics.median(ts)), flush=True)


if __name__ == "__main__":
    main()
