"""Volume rollouts for the wave-parallel cascade steps (test helper).

The same configurations serve two runs with identical trajectories (same
seeds, same action streams):

* tests/test_gpu_deep.py runs them on the product library against the CPU
  oracle (oracle/tmg_oracle.c, pinned by the reference's goldens), every field
  of every env at every step;
* cover_counts() runs them on the GPU only with the TMG_COVER diagnostic
  build (libtmg_cover.so, loaded beside the product library) and returns the
  per-branch hit counters (CV_* in tmg_board.hip), so the test can show that
  every cascade-step form — the
  bitboard normal / laser / perpendicular-bomb / row-bomb / closure steps, the
  512-cell LDS forms, the lane-0 fallback, the spill path — ran on exactly the
  trajectories the parity run checked.

Reference: board.py:269-327 (process_colour_lines), :429-458
(get_special_creation_pos), :473-556 (activate_special).
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "tile-match-gym_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

KEY = 777
# name: (R, C, k, smask, envs, steps, policy)
CONFIGS = {
    "c3_uniform": (10, 10, 4, 14, 32768, 90, "uniform"),
    "c3_effective": (10, 10, 4, 14, 32768, 90, "effective"),
    "c3_cookie_effective": (10, 10, 4, 15, 16384, 90, "effective"),
    "c5_uniform": (20, 20, 6, 15, 16384, 90, "uniform"),
    "c5_effective": (20, 20, 6, 15, 16384, 90, "effective"),
    "s12_effective": (12, 12, 5, 15, 8192, 90, "effective"),
    "s16_effective": (16, 16, 6, 14, 8192, 90, "effective"),
}


def specials(sm):
    cl = ["cookie"] if sm & 1 else []
    co = [nm for b, nm in ((8, "bomb"), (2, "vertical_laser"), (4, "horizontal_laser")) if sm & b]
    return cl, co


def seed_base(name):
    return 100_000 * (1 + sorted(CONFIGS).index(name))


COVER_LIB = os.path.join(ROOT, "tile-match-gym_amd", "tile_match_gym_amd", "_lib", "libtmg_cover.so")


def run(name, device="cuda:0", check=None, threads=16, lib_path=None):
    """Roll config `name` out on the device.  check(t, env, ref) is called
    after every step when given (then the oracle runs beside it)."""
    import torch
    from tile_match_gym_amd.shard import synthetic_actions
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    R, C, k, sm, n, steps, policy = CONFIGS[name]
    cl, co = specials(sm)
    base = seed_base(name)
    env = TileMatchVecEnv(n, R, C, k, 30, cl, co, seeds=range(base, base + n), device=device, groups=2,
                          lib_path=lib_path)
    ref = None
    if check is not None:
        from oracle import oracle as orc
        ref = orc.OracleBatch(R, C, k, sm, 30, env.rng_words().copy(), threads=threads)
    env.reset()
    if ref is not None:
        ref.reset()
        check(-1, env, ref)
    A = env.num_actions
    acts = synthetic_actions(range(n), steps, A, key=KEY) if policy == "uniform" else None
    dacts = torch.from_numpy(acts).to(device) if acts is not None else None
    for t in range(steps):
        if policy == "uniform":
            env.step_raw(dacts[t])
            a = acts[t]
        else:
            env.step_effective(t, key=KEY)
            a = None
            if ref is not None:
                from oracle.policy_np import sample_effective_np
                a = sample_effective_np(ref.eff, A, KEY, 0, t)
        env.join()
        if ref is not None:
            ref.step(a, autoreset=True)
            check(t, env, ref)
    torch.cuda.synchronize()
    return env


def cover_counts(names=None):
    """{name: {"counts": {CV name: hits}, "status": ..., ...}} from the TMG_COVER build."""
    from tile_match_gym_amd import _native
    info = _native.build_info(COVER_LIB)
    if info.get("variant") != "cover":
        raise RuntimeError(f"{COVER_LIB} is not the TMG_COVER build ({info})")
    res = {"build": info, "names": list(_native.COVER_NAMES), "configs": {}}
    for name in names or sorted(CONFIGS):
        t0 = time.time()
        env = run(name, lib_path=COVER_LIB)
        c = env.ctx.cover()
        res["configs"][name] = {"counts": {nm: int(c[i]) for i, nm in enumerate(_native.COVER_NAMES)},
                                "status": env.status(), "seconds": round(time.time() - t0, 2), "spec": CONFIGS[name]}
        env.close()
    return res


def main():
    out = sys.argv[sys.argv.index("--cover") + 1]
    names = [a for a in sys.argv[1:] if a in CONFIGS] or None
    res = cover_counts(names)
    for name, c in res["configs"].items():
        print(name, c, flush=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
