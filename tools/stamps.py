"""Phase timing from the diagnostic build (libtmg_stamps.so, TMG_STAMPS=1).

    TMG_LIB=.../libtmg_stamps.so python tools/stamps.py [--config c2] [--steps 60]

Per step: the launch's wall span, the spread of wave start times (dispatch),
and per-env phase durations (quick exit / move cascade / ensure-playable /
autoreset), from s_memrealtime (100 MHz) stamps written by lane 0.
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tile-match-gym_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--boards", type=int, default=0)
    args = ap.parse_args()
    import bench
    from tile_match_gym_amd import _native
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    L = _native.load()
    L.tmg_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
    R, C, k, cl, co, nb, _ = bench.CONFIGS[args.config]
    nb = args.boards or min(nb, 1 << 18)
    env = TileMatchVecEnv(nb, R, C, k, 30, cl, co, seed=0, device="cuda:0")
    A = env.num_actions
    acts = torch.from_numpy(np.random.default_rng(12345).integers(0, A, (args.steps, nb)).astype(np.int32)).cuda()
    env.reset()
    st = np.zeros((nb, 8), np.uint64)
    rows = []
    for t in range(args.steps):
        env.step_raw(acts[t])
        torch.cuda.synchronize()
        _native.check(L.tmg_debug_stamps(env.ctx.handle, st.ctypes.data, nb), L)
        rew = env.reward.cpu().numpy()
        fl = env.flags.cpu().numpy()
        s = st.astype(np.int64)
        t0 = s[:, 0].min()
        span = (s[:, 7].max() - t0) / 100.0                      # us
        start_spread = (np.percentile(s[:, 0] - t0, [50, 99, 100]) / 100.0)
        eff = rew > 0
        done = (fl & 1) != 0
        quick = ~eff & ~done
        d = {"t": t, "span_us": span, "start_p50": start_spread[0], "start_max": start_spread[2],
             "n_eff": int(eff.sum()), "done": bool(done.any())}
        if quick.any():
            d["quick_us"] = np.median((s[quick, 7] - s[quick, 0]) / 100.0)
        if eff.any():
            d["load_us"] = np.median((s[eff, 1] - s[eff, 0]) / 100.0)
            d["cascade_us"] = np.median((s[eff, 2] - s[eff, 1]) / 100.0)
            d["ensure_us"] = np.median((s[eff, 3] - s[eff, 2]) / 100.0)
            d["eff_total_us"] = np.median((s[eff, 7] - s[eff, 0]) / 100.0)
            d["eff_p99_us"] = np.percentile((s[eff, 7] - s[eff, 0]) / 100.0, 99)
            d["iters"] = float(np.mean(s[eff, 6]))
        if done.any():
            d["reset_us"] = np.median((s[done, 5] - s[done, 4]) / 100.0)
            d["reset_p99_us"] = np.percentile((s[done, 5] - s[done, 4]) / 100.0, 99)
        rows.append(d)
    keys = ["t", "span_us", "start_p50", "start_max", "n_eff", "quick_us", "load_us", "cascade_us", "ensure_us",
            "eff_total_us", "eff_p99_us", "iters", "reset_us", "reset_p99_us"]
    print(" ".join(f"{k:>10s}" for k in keys))
    for d in rows[-32:]:
        print(" ".join(f"{d.get(k, float('nan')):10.2f}" if not isinstance(d.get(k), bool) else f"{d[k]!s:>10s}" for k in keys))


if __name__ == "__main__":
    main()
