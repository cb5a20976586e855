import sys, time, torch
sys.path[:0]=['/root/repo','/root/repo/tile-match-gym_amd']
from tile_match_gym_amd.vec_env import TileMatchVecEnv
from tile_match_gym_amd.shard import synthetic_actions
for (R,C,k,co,n,groups) in [(10,10,4,["vertical_laser","bomb"],1024,1),(10,10,4,["vertical_laser","bomb"],1024,3)]:
    env = TileMatchVecEnv(n, R, C, k, 30, [], co, seed=11, device="cuda:0", groups=groups)
    acts = torch.from_numpy(synthetic_actions(range(n), 40, env.num_actions)).cuda()
    env.reset(); torch.cuda.synchronize()
    for t in range(40):
        t0=time.time(); env.step_raw(acts[t]); env.join(); torch.cuda.synchronize()
        print(R,C,groups,"step",t,f"{(time.time()-t0)*1e3:.2f} ms", flush=True)
