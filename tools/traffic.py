"""Reduce rocprofv3 FETCH_SIZE / WRITE_SIZE passes (scripts/gpu_traffic.sh) to
HBM bytes per step_kernel launch, averaged over every dispatch of the bench
(warm-up + timed: 1 in 30 is an autoreset launch, as in the timed region).

    python tools/traffic.py gpurun_out/traffic [STEPS_PLUS_WARMUP] > profiles/traffic.json

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch.  MI355X_MICROARCH.md
("HBM [CDNA4]"): gfx950 FETCH_SIZE counts half the bytes of coalesced reads,
so it is doubled; WRITE_SIZE is taken as is.
"""
import collections
import csv
import glob
import json
import os
import sys


def per_dispatch(path, counter, with_resets=False):
    """KiB per step_kernel dispatch; with_resets: also the reset_kernel and
    sampler dispatches after the first step_kernel one (deferred autoresets,
    the policy draw ahead of the general kernels)."""
    vals = collections.defaultdict(float)
    names = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            d = int(r["Dispatch_Id"])
            names[d] = r["Kernel_Name"]
            vals[d] += float(r["Counter_Value"])
    steps = sorted(d for d in vals if "step_kernel" in names[d])
    keep = set(steps)
    if with_resets and steps:
        keep |= {d for d in vals if ("reset_kernel" in names[d] or "sample_effective_kernel" in names[d])
                 and d > steps[0]}
    return [vals[d] for d in sorted(keep)]


def main():
    sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
    import bench
    root = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else None
    out = {}
    for d in sorted(glob.glob(os.path.join(root, "*_FETCH_SIZE"))):
        name = os.path.basename(d).split("_")[0]         # a bench.run_args name
        line = bench.last_bench_line(d + ".log")
        if line is None or not os.path.isdir(d):
            continue
        boards = line["config"]["boards_per_gpu"]
        f = per_dispatch(d, "FETCH_SIZE")
        w = per_dispatch(os.path.join(root, f"{name}_WRITE_SIZE"), "WRITE_SIZE")
        if not f or not w:
            continue
        fk = sum(f) / len(f)
        wk = sum(w) / len(w)
        out[name] = {
            "hbm_bytes_per_launch": round((2 * fk + wk) * 1024),
            "fetch_size_kib_raw": round(fk, 1),
            "write_size_kib": round(wk, 1),
            "dispatches": [len(f), len(w)],
            "hbm_bytes_per_env_step": (round((2 * sum(per_dispatch(d, "FETCH_SIZE", True))
                                               + sum(per_dispatch(os.path.join(root, f"{name}_WRITE_SIZE"),
                                                                  "WRITE_SIZE", True))) * 1024
                                              / (steps * boards), 1) if steps else None),
            "correction": "FETCH_SIZE x2 (gfx950 half-count, MI355X_MICROARCH.md HBM section); WRITE_SIZE as is",
            # the bench run these counts belong to (bench.py attaches them only to a line of the same build and
            # run shape)
            **bench.run_identity(line),
        }
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
