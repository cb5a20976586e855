"""Probe: env groups with staggered episode phases (diagnostics).  Group g is
stepped alone for g*30/S extra steps before the timed region, so the groups'
autoreset steps fall on different launches."""
import os, sys, time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tile-match-gym_amd")]


def step_one(env, g, a):
    lo = env._ranges[g][0]
    p = env._gptr[g]
    st = env._streams[g]
    a.record_stream(st)
    env.ctx.step(p[0], p[1], p[2], p[3], a.data_ptr() + 4 * lo, p[5], p[6], p[7], p[8], p[4], 1, 1, st.cuda_stream)


def main():
    from tile_match_gym_amd.shard import synthetic_actions
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    n, K = 65536, 300
    S, stagger = int(sys.argv[1]), sys.argv[2] == "1"
    if True:
        if True:
            env = TileMatchVecEnv(n, 10, 10, 4, 30, [], [], seeds=range(n), device="cuda:0", groups=S)
            acts = torch.from_numpy(synthetic_actions(range(n), K, env.num_actions)).cuda()
            env.reset()
            env.step_raw(acts[0])
            if stagger:
                for g in range(1, S):
                    for t in range(g * 30 // S):
                        step_one(env, g, acts[1 + t])
            env.join(); torch.cuda.synchronize()
            for rep in range(2):
                t0 = time.perf_counter()
                for t in range(K):
                    env.step_raw(acts[t])
                env.join(); torch.cuda.synchronize()
                el = time.perf_counter() - t0
            print(f"S={S} stagger={stagger}: {n * K / el:.3e} env-steps/s", flush=True)
            del env, acts
            torch.cuda.synchronize()


if __name__ == "__main__":
    main()
