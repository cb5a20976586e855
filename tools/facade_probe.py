"""Per-call cost of the single-env drop-in (TileMatchEnv.step / reset) on the GPU.

The facade uploads the board and RNG state, launches one wave, and downloads the
new state each call (tile_match_env.py, the drop-in for the reference's
tile_match_env.py:84-112), so its rate is host round trips, not kernel work.
Prints one JSON line: steps/s and resets/s for BASELINE configs[0]'s shape.

    python tools/facade_probe.py [--steps 400]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tile-match-gym_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=400)
    a = ap.parse_args()
    import numpy as np
    import torch
    from tile_match_gym_amd.tile_match_env import TileMatchEnv
    env = TileMatchEnv(8, 8, 4, 30, [], [], seed=0)
    env.reset()
    rs = np.random.default_rng(0)
    acts = rs.integers(0, env.num_actions, a.steps + 20)
    for t in range(20):                                  # warm-up
        _, _, done, _, _ = env.step(int(acts[t]))
        if done:
            env.reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    resets = 0
    for t in range(20, 20 + a.steps):
        _, _, done, _, _ = env.step(int(acts[t]))
        if done:
            env.reset()
            resets += 1
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    t1 = time.perf_counter()
    for _ in range(50):
        env.reset()
    torch.cuda.synchronize()
    dr = time.perf_counter() - t1
    print(json.dumps({"probe": "TileMatchEnv facade, 8x8 k4, num_moves 30, uniform actions",
                      "steps": a.steps, "resets_inside": resets, "steps_per_s": round(a.steps / dt, 1),
                      "us_per_step": round(1e6 * dt / a.steps, 1), "resets_per_s": round(50 / dr, 1)}))


if __name__ == "__main__":
    main()
