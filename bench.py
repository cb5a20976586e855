#!/usr/bin/env python3
"""Benchmark: batched Board.step (BASELINE.json metric) on 1..8 MI355X.

    python bench.py --gpus N --steps K --warmup W [--config c2|c3|c5]

One "step" = one TileMatchEnv.step for every env of the shard (one HIP launch
per env group; `--groups` groups run on separate HIP streams so one group's
launch tail overlaps the next group's launch — same boards, same work),
uniform random actions pre-staged in HBM, autoreset on (num_moves = 30).

Episode phases (`--phase-blocks P`, default 3 = the env groups): after the
reset the shard's envs form P contiguous blocks whose episodes are offset by
30/P steps (`TileMatchVecEnv.stagger_phases`: a timer of m is the state after
m ineffective moves).  Every 10 steps one block's episodes end and its boards
are regenerated (tile_match_env.py:84-91 -> board.py:95-131), so any timed
window of a multiple of 10 steps (the driver's 20, the default 300) holds
exactly its share of the reset work (20 steps: 2/3 of the boards), and each
block's regeneration overlaps the other groups' steps on their streams.
`--phase-align 1` (default) moves that schedule so the timed window opens on a
block's reset step: same reset work per window, but no reset right before the
window's end, whose regeneration tail would then have nothing to overlap.
P = 1 is the aligned run (every env resets on the same step); P = 0 staggers
every env (env i at timer i mod 30: each step regenerates N/30 boards, and the
step time is then the slowest of those regenerations).

Multi-GPU: one process per GPU, each stepping its own contiguous shard of envs
(seed = global env index); there is no collective on the data path, only a
barrier around the timed region and a MAX of the elapsed time (gloo, on the
host).  Under torch.distributed.run the ranks come from the environment; a
plain `--gpus N` (N > 1) spawns the N rank processes itself before anything
touches the GPU.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "tile-match-gym_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "env-steps/sec (whole node), 65536×10×10 boards, at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0           # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
# Issue peaks (MI355X_MICROARCH.md: 256 CUs x 4 SIMD-32, 2.4 GHz; a wave64 VALU
# instruction takes 2 cycles of its SIMD; one scalar unit per CU issuing at
# most one SALU instruction per cycle), in wave-instructions per second.
CLOCK_HZ = 2.4e9
VALU_PEAK = 256 * 4 * CLOCK_HZ / 2
SALU_PEAK = 256 * CLOCK_HZ

CONFIGS = {
    # name: (R, C, k, colourless, colour, boards per GPU, what the specials are)
    "c2": (10, 10, 4, [], [], 65536, "no specials"),
    "c3": (10, 10, 4, [], ["vertical_laser", "horizontal_laser", "bomb"], 262144, "v/h-laser + bomb"),
    "c5": (20, 20, 6, ["cookie"], ["vertical_laser", "horizontal_laser", "bomb"], 262144, "all specials"),
    # shapes no kernel is specialised for (tmg_kernels.hip is_shape): the generic instantiations' rate
    "g1": (10, 10, 5, [], [], 65536, "no specials, generic kernels"),
    "g2": (20, 20, 6, [], ["vertical_laser", "horizontal_laser", "bomb"], 262144, "v/h-laser + bomb, generic kernels"),
}


# Profiled runs (tools/issue.py, tools/traffic.py key their counts by these
# names): a config name runs that config; c4 = BASELINE configs[3], one GPU's
# shard of 1 048 576 / 8 boards of the c2 shape; suffixes: "-p1" adds
# --phase-blocks 1 (episodes aligned), "-vec" --api vector (aligned episodes),
# "-eff" --policy effective.
PROFILE_RUNS = {"c4": ("c2", 131072)}
SUFFIXES = (("-eff", ["--policy", "effective"]), ("-vec", ["--api", "vector"]), ("-p1", ["--phase-blocks", "1"]))


def run_args(name):
    """bench.py arguments of a profiled run name."""
    extra = []
    for suf, args in SUFFIXES:
        if name.endswith(suf):
            name, extra = name[:-len(suf)], args + extra
    cfg, boards = PROFILE_RUNS.get(name, (name, 0))
    return ["--config", cfg] + (["--boards", str(boards)] if boards else []) + extra


def run_name(config, boards, policy, api="raw", phase_blocks=3):
    """The profiled-run name of a bench line (the inverse of run_args)."""
    base = config
    for name, (cfg, nb) in PROFILE_RUNS.items():
        if cfg == config and nb == boards:
            base = name
    if api == "vector":
        base += "-vec"
    elif phase_blocks == 1:
        base += "-p1"
    return base + ("-eff" if policy == "effective" else "")


def last_bench_line(path):
    """The JSON line a bench run printed last (its log), or None."""
    try:
        with open(path) as f:
            lines = [ln for ln in f if ln.startswith("{")]
        return json.loads(lines[-1]) if lines else None
    except (OSError, ValueError):
        return None


def run_identity(line):
    """What a profile must share with a bench line to be attached to it: the
    library build (source hash), the policy, the run shape and the API."""
    c = line["config"]
    return {"build_src": line["build"]["src"], "policy": c.get("policy", "uniform"), "api": c.get("api", "raw"),
            "boards_per_gpu": c["boards_per_gpu"], "env_groups_per_gpu": c["env_groups_per_gpu"],
            "phase_blocks": c.get("phase_blocks", 3)}


def workload_desc(R, C, k, nb, specials):
    """The workload of a run as it was actually configured (--boards included)."""
    return f"{nb} x {R}x{C} boards per GPU, {k} colours, {specials}"
# The reference's own Python step() measured in the survey container (BASELINE.md §2,
# 8 vCPU Xeon, numba absent): context for the CPU baseline, not a target.
REF_PY = {"c2": (290, 1976), "c3": (281, 2421), "c5": (69, 492)}


def algorithmic_bytes_per_env_step(R, C):
    """4RC (int8 colour+type read+write) + 48 (PCG64 state r/w
    + inc read) + 8 (half-word buffer r/w) + 4 (action) + 8 (timer r/w)
    + 16 (reward, n_new, n_act, flags) + 8*ceil(A/64) (effective mask)."""
    A = 2 * R * C - R - C
    return 4 * R * C + 48 + 8 + 4 + 8 + 16 + 8 * ((A + 63) // 64)


def host_threads():
    """Host cores this job may use: the affinity set, capped by OMP_NUM_THREADS
    when the launcher sets it (the GPU box gives each GPU a 16-core share)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def _time_oracle(R, C, k, smask, moves, n, threads, budget_s, policy):
    import numpy as np
    from oracle import oracle as orc
    from tile_match_gym_amd.seeding import batch_rng_words
    from tile_match_gym_amd.shard import synthetic_actions
    A = 2 * R * C - R - C
    o = orc.OracleBatch(R, C, k, smask, moves, batch_rng_words(range(n)), threads=threads)
    o.reset()
    o.timer[:] = np.arange(n) % moves              # staggered phases: the amortised reset share every step
    T = 300
    acts = synthetic_actions(range(n), T, A)
    steps = 0
    t0 = time.perf_counter()
    while True:
        for t in range(moves):
            if policy == "effective":
                from oracle.policy_np import sample_effective_np
                a = sample_effective_np(o.eff, A, 12345, 0, steps + t)
            else:
                a = acts[(steps + t) % T]
            o.step(a, autoreset=True)
        steps += moves
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    return n * steps / el, steps, el


def cpu_baseline(config, R, C, k, smask, moves, policy="uniform"):
    """The oracle (oracle/tmg_oracle.c, a bit-exact C restatement of the
    reference Board) timed on this host over a bounded sample of the same
    workload (same seeds, staggered phases and action stream): once on one
    thread and once over every host core this job may use (OpenMP)."""
    threads = host_threads()
    single, s_steps, s_el = _time_oracle(R, C, k, smask, moves, 256, 1, 8.0, policy)
    multi, m_steps, m_el = _time_oracle(R, C, k, smask, moves, 256 * threads, threads, 8.0, policy)
    ref1, ref8 = REF_PY.get(config, (None, None))
    return {"value": round(multi, 1), "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"{256 * threads} envs x {m_steps} steps ({m_steps // moves} episodes incl. autoreset), "
                      f"{m_el:.1f} s, OpenMP over {threads} threads",
            "single_thread": {"value": round(single, 1), "cores": 1,
                              "sample": f"256 envs x {s_steps} steps, {s_el:.1f} s"},
            "reference_python_survey": {"value_1_process": ref1, "value_8_processes": ref8,
                                        "note": "reference TileMatchEnv.step, survey container 8 vCPU, numba absent "
                                                "(BASELINE.md §2); context only"}}


def load_profile(fname, run, ident):
    """The committed rocprofv3 counts of a profiled run (profiles/<fname>, key
    `run`), only if they were taken on the same library build and run shape
    (run_identity); counts of another build or shape would not describe this
    line's launches."""
    p = os.path.join(ROOT, "profiles", fname)
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            prof = json.load(f).get(run)
    except Exception:
        return None
    if not prof or any(prof.get(k) != v for k, v in ident.items()):
        return None
    return prof


def spawn_ranks(n):
    """`bench.py --gpus n` without a launcher: start n rank processes (this
    process touches no GPU) and exit with the worst of their codes."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--boards", type=int, default=0, help="override boards per GPU")
    ap.add_argument("--groups", type=int, default=None,
                    help="env groups per GPU, each stepped on its own HIP stream (TileMatchVecEnv(groups=)); "
                         "default 3 (--api vector: 1, its step joins every group each call)")
    ap.add_argument("--policy", default="uniform", choices=("uniform", "effective"),
                    help="uniform: random actions over all A (headline); effective: every env samples uniformly "
                         "from its effective actions on device each step (SURVEY §8(d) secondary mode)")
    ap.add_argument("--phase-blocks", type=int, default=None,
                    help="episode phase blocks: P contiguous env blocks offset by 30/P steps (1 = aligned, "
                         "0 = every env staggered); default 3, or 1 for --api vector when --steps is a multiple "
                         "of 30 (a vector env reset once keeps every episode in lock-step, tile_match_env.py:84-101; "
                         "the window then holds whole reset storms)")
    ap.add_argument("--phase-align", type=int, default=1,
                    help="1: shift the phase blocks so the timed window opens on a block's reset step (0: phases "
                         "from step 0)")
    ap.add_argument("--phase-interleave", action="store_true",
                    help="env i in phase block i mod P (every env group holds all blocks) instead of contiguous blocks")
    ap.add_argument("--api", default="raw", choices=("raw", "vector"),
                    help="raw: TileMatchVecEnv.step_raw (headline); vector: the Gymnasium vector-env step "
                         "(TileMatchVectorEnv.step: next-step autoreset, action masks, obs / reward / terminated / "
                         "info tensors every step)")
    ap.add_argument("--obs-dtype", default="int32", choices=("int32", "int8"),
                    help="--api vector: the observation board dtype (int32 = the reference's, a converted copy; int8 = "
                         "a view of the live state)")
    ap.add_argument("--graph", type=int, default=0,
                    help="1: the timed steps are captured into one HIP graph beforehand (TileMatchVecEnv.capture_steps: "
                         "the same launches, one host call for the whole window; --api raw)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dry-run", action="store_true", help="print each rank's shard layout and exit (no GPU)")
    args = ap.parse_args()
    if args.groups is None:
        args.groups = 1 if args.api == "vector" else 3

    from tile_match_gym_amd.shard import dist_env, max_over_ranks, shard_range, shard_seeds, synthetic_actions
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world, rank, local_rank = dist_env()
    R, C, k, cl, co, nb, spdesc = CONFIGS[args.config]
    if args.boards:
        nb = args.boards
    rng_ = shard_range(rank, nb)
    if args.dry_run:
        print(json.dumps({"rank": rank, "world": world, "local_rank": local_rank, "envs": [rng_.start, rng_.stop]}),
              flush=True)
        return

    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        # one process per GPU; the only collectives (a barrier and a MAX of the
        # elapsed time) run on the host
        dist.init_process_group(os.environ.get("TMG_DIST_BACKEND", "gloo"))
    ndev = torch.cuda.device_count()
    torch.cuda.set_device(local_rank % max(1, ndev))
    dev = torch.device("cuda", torch.cuda.current_device())

    from tile_match_gym_amd import _native
    from tile_match_gym_amd.vec_env import TileMatchVecEnv
    build = _native.build_info()            # the loader has checked the library against this tree's sources
    moves = 30
    venv = None
    if args.api == "vector":
        from tile_match_gym_amd.vector import TileMatchVectorEnv
        if args.policy != "uniform":
            raise SystemExit("--api vector takes the uniform action stream (actions are the caller's)")
        venv = TileMatchVectorEnv(nb, R, C, k, moves, cl, co, device=dev, autoreset_mode="next_step",
                                  obs_dtype=torch.int32 if args.obs_dtype == "int32" else torch.int8,
                                  action_masks=True, groups=args.groups, copy=False)
        venv.vec.set_seed(shard_seeds(rank, nb))
        env = venv.vec
    else:
        env = TileMatchVecEnv(nb, R, C, k, moves, cl, co, seeds=shard_seeds(rank, nb), device=dev, autoreset=True,
                              groups=args.groups)
    A = env.num_actions
    T = 300
    acts = torch.from_numpy(synthetic_actions(rng_, T, A)).to(dev)
    if venv is not None:
        venv.reset()
    else:
        env.reset()
    # --phase-align: move the reset schedule so that the timed window opens on a
    # block's reset step (the blocks' resets are `spacing` steps apart; any
    # window of a multiple of `spacing` steps holds the same reset work however
    # it is aligned, but one ending just after a reset times that reset's tail
    # with nothing left to overlap it)
    if args.phase_blocks is None:
        args.phase_blocks = 1 if (args.api == "vector" and args.steps % moves == 0) else 3
    spacing = moves // max(1, args.phase_blocks)
    shift = (moves - 1 - args.warmup) % spacing if (args.phase_align and args.phase_blocks > 1
                                                    and not args.phase_interleave) else 0
    if args.phase_blocks != 1:
        (venv or env).stagger_phases(blocks=args.phase_blocks, first_env=rng_.start,
                                     interleave=args.phase_interleave, shift=shift)
    env.status(clear=True)

    rows = [acts[t] for t in range(T)]                    # the staged action rows (views)

    def step(t, fork=True):
        # fork=False: back-to-back steps on staged actions (nothing queued on
        # the current stream in between), so the group streams skip the fork
        if venv is not None:
            venv.step(rows[t % T])                            # obs, rewards, terminations, truncations, infos
        elif args.policy == "effective":
            env.step_effective(t, first_env=rng_.start, fork=fork)   # sampled inside the step
        else:
            env.step_raw(rows[t % T], fork=fork)

    for t in range(args.warmup):
        step(t)
    env.join()
    graph = None
    if args.graph and args.api == "raw":            # capture the timed steps (untimed)
        ts = [args.warmup + i for i in range(args.steps)]
        graph = (env.capture_steps(ts=ts, policy=True, first_env=rng_.start) if args.policy == "effective" else
                 env.capture_steps([acts[t % T] for t in ts], ts))
    torch.cuda.synchronize()

    # HIP events: on the current stream around the whole step (fork ... join:
    # the device time of a step, all groups), and on group 0's stream (its
    # launches' average duration, comparable with rocprofv3's per-kernel stats)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev[0].record()
    if graph is not None:
        env.run_graph(graph)
    else:
        env.record(ev[2])
        for i in range(args.steps):
            step(args.warmup + i, fork=i == 0)
    host_issue_s = time.perf_counter() - t0          # host time to enqueue the window (launch-rate check)
    if graph is None:
        env.record(ev[3])
    env.join()
    ev[1].record()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    step_ms = ev[0].elapsed_time(ev[1]) / max(1, args.steps)
    if graph is not None:
        # the graph's kernels run on the runtime's streams: group 0's launch
        # time from 10 eager steps after the timed window (untimed)
        env.record(ev[2])
        for i in range(10):
            step(args.warmup + args.steps + i)
        env.record(ev[3])
        env.join()
        torch.cuda.synchronize()
        kern_ms = ev[2].elapsed_time(ev[3]) / 10
    else:
        kern_ms = ev[2].elapsed_time(ev[3]) / max(1, args.steps)
    launch_envs = env._ranges[0][1] - env._ranges[0][0]
    st = env.status()                     # sticky: every env of every step, warmup included
    if st & 0x3:
        raise SystemExit(f"bench: internal error / overflow raised during the run (status {st:#x})")
    el = max_over_ranks(el, dist, dev)
    step_ms = max_over_ranks(step_ms, dist, dev)
    kern_ms = max_over_ranks(kern_ms, dist, dev)

    if rank == 0:
        total = nb * world * args.steps
        value = total / el
        bpu = algorithmic_bytes_per_env_step(R, C)
        # roofline.achieved: one GPU's algorithmic bytes per step (bpu x its
        # envs) / the device time of that step (HIP events around the fork ...
        # join of all env groups).  The groups' step launches run at the same
        # time on their own streams, so one launch's bytes over its own
        # duration (per_launch_gbs, comparable with rocprofv3's average for
        # the step kernel) counts a third of the device's work per unit time.
        achieved = bpu * nb / (step_ms * 1e-3) / 1e9
        per_launch_gbs = bpu * launch_envs / (kern_ms * 1e-3) / 1e9
        smask = (1 if "cookie" in cl else 0) | (2 if "vertical_laser" in co else 0) | \
                (4 if "horizontal_laser" in co else 0) | (8 if "bomb" in co else 0)
        cpu = None if (args.no_cpu_baseline or world > 1) else cpu_baseline(args.config, R, C, k, smask, moves,
                                                                             policy=args.policy)
        issue = None
        ident = {"build_src": build["src"][:16], "policy": args.policy, "api": args.api, "boards_per_gpu": nb,
                 "env_groups_per_gpu": env.groups, "phase_blocks": args.phase_blocks}
        run = run_name(args.config, nb, args.policy, args.api, args.phase_blocks)
        prof = load_profile("issue.json", run, ident)
        if prof:
            per_gpu = value / world
            v = prof["valu_per_env_step"] * per_gpu
            s = prof["salu_per_env_step"] * per_gpu
            issue = {"valu_per_env_step": prof["valu_per_env_step"], "salu_per_env_step": prof["salu_per_env_step"],
                     "valu_rate": round(v, 1), "salu_rate": round(s, 1), "valu_peak": VALU_PEAK,
                     "salu_peak": SALU_PEAK, "unit": "wave-instructions/s per GPU",
                     "valu_frac": round(v / VALU_PEAK, 4), "salu_frac": round(s / SALU_PEAK, 4),
                     "source": prof.get("source")}
        traffic = load_profile("traffic.json", run, ident)
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el * 1e3 / args.steps, 4),
            "host_issue_ms_per_step": round(host_issue_s * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int8",
            "data": ("synthetic (uniform random actions, counter-based per (step, global env); seeds = global env index)"
                     if args.policy == "uniform" else
                     "synthetic (each step every env samples uniformly from its effective actions on device, "
                     "counter-based per (step, global env); seeds = global env index)"),
            "config": {"workload": f"{args.config}: {workload_desc(R, C, k, nb, spdesc)}, num_moves=30, autoreset"
                                   + (", episodes aligned" if args.phase_blocks == 1 else
                                      ", every env's episode phase staggered (timer0 = env mod 30)" if args.phase_blocks <= 0
                                      else f", {args.phase_blocks} episode-phase blocks offset by "
                                           f"{moves // args.phase_blocks} steps"
                                           + (f", the timed window opening on a block's reset step (phases + {shift})"
                                              if shift else ""))
                                   + ("" if args.policy == "uniform" else ", effective-action policy")
                                   + ("" if args.api == "raw" else
                                      f", Gymnasium vector-env step (next-step autoreset, action masks, "
                                      f"{args.obs_dtype} obs)"),
                       "boards_per_gpu": nb, "rows": R, "cols": C, "colours": k,
                       "specials": cl + co, "env_groups_per_gpu": env.groups, "phase_blocks": args.phase_blocks,
                       "policy": args.policy,
                       "api": args.api, "graph": bool(graph is not None),
                       "parallelism": f"dp{world} (independent env shards, no collective)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 6),
                         "traffic": traffic.get("hbm_bytes_per_launch") if traffic else None,
                         "traffic_bytes_per_env_step": traffic.get("hbm_bytes_per_env_step") if traffic else None,
                         "algorithmic_bytes_per_env_step": bpu, "device_ms_per_step": round(step_ms, 4),
                         "kernel_ms_per_launch": round(kern_ms, 4), "envs_per_launch": launch_envs,
                         "per_launch_gbs": round(per_launch_gbs, 2),
                         # what limits the path: integer work whose
                         # SALU / VALU issue and dependent chains (the redraw loop of
                         # generate_board) bind long before HBM bandwidth
                         "binding": "issue/latency (SALU + VALU issue, dependent per-board chains), not HBM",
                         "issue": issue},
            "cpu_baseline": cpu,
            "build": {k: (v[:16] if k in ("src", "so_sha256") else v) for k, v in build.items() if k != "path"},
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
