"""Reduce rocprofv3 SQ instruction-count passes (scripts/gpu_issue.sh) to
wave-instructions per env-step for bench.py's `roofline.issue`.

    python tools/issue.py gpurun_out/issue STEPS_PLUS_WARMUP > profiles/issue.json

Each `<run>` directory holds one `--pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES
...` pass of `bench.py <run's args> --steps S --warmup W --no-cpu-baseline`
(bench.run_args: a config, c4 = the c2 shard of 131 072 boards, `-eff` = the
effective-action policy), and `<run>.log` that run's bench line, whose build
hash, policy, boards and env groups are recorded with the counts (bench.py
attaches a profile only to a line of the same build and run shape).
Counted: every step_kernel dispatch and every reset_kernel / sampler dispatch
issued after the first step_kernel one (the deferred autoreset launches of the
512-cell / general kernels and the policy draw ahead of the general kernels
are part of a step); the initial reset() launch is not.  Env-steps = (S + W) x boards of the config (bench.CONFIGS).
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]

COUNTERS = ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVES", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_WAVE_CYCLES",
            "SQ_BUSY_CYCLES")


def per_dispatch(path):
    rows = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            d = int(r["Dispatch_Id"])
            names[d] = r["Kernel_Name"]
            rows[d][r["Counter_Name"]] += float(r["Counter_Value"])
    return names, rows


def main():
    import bench
    root, steps = sys.argv[1], int(sys.argv[2])
    out = {}
    for d in sorted(glob.glob(os.path.join(root, "c*"))):
        name = os.path.basename(d)                          # a bench.run_args name
        if not os.path.isdir(d):
            continue
        line = bench.last_bench_line(d + ".log")
        if line is None:
            continue
        names, rows = per_dispatch(d)
        order = sorted(names)
        first_step = next((i for i in order if "step_kernel" in names[i]), None)
        if first_step is None:
            continue
        tot = collections.defaultdict(float)
        n_step = n_reset = 0
        for i in order:
            nm = names[i]
            if "step_kernel" in nm:
                n_step += 1
            elif ("reset_kernel" in nm or "sample_effective_kernel" in nm) and i > first_step:
                n_reset += 1
            else:
                continue
            for c, v in rows[i].items():
                tot[c] += v
        boards = line["config"]["boards_per_gpu"]
        env_steps = steps * boards
        out[name] = {
            "valu_per_env_step": round(tot["SQ_INSTS_VALU"] / env_steps, 2),
            "salu_per_env_step": round(tot["SQ_INSTS_SALU"] / env_steps, 2),
            "lds_per_env_step": round(tot["SQ_INSTS_LDS"] / env_steps, 2),
            "smem_per_env_step": round(tot["SQ_INSTS_SMEM"] / env_steps, 2),
            "waves_per_env_step": round(tot["SQ_WAVES"] / env_steps, 4),
            "env_steps": env_steps,
            # the bench run these counts belong to (bench.py attaches them only to a line of the same build and
            # run shape)
            **bench.run_identity(line),
            "dispatches": {"step_kernel": n_step, "reset_or_sampler_kernel": n_reset},
            "source": (f"rocprofv3 --pmc {' '.join(COUNTERS)} --kernel-trace, bench.py {' '.join(bench.run_args(name))} "
                       f"(steps + warmup = {steps}); scripts/gpu_issue.sh, tools/issue.py"),
        }
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
