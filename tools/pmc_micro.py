"""Per-launch instruction counts of tools/microbench.py (diagnostics).

    rocprofv3 --pmc <SQ counters> --kernel-trace -d DIR -o run --output-format csv -- \\
        python3 tools/microbench.py --config c2
    python tools/pmc_micro.py DIR [DIR ...] --boards BOARDS [--eff-frac F]

microbench.py launches, in order: 60 steps of the bench's action stream (the
autoreset storm at steps 29 and 59, normal steps otherwise), then 20
quick-exit launches (every move ineffective), then 20 steps of the
effective-action policy ("policy": every env plays an effective move; the
general kernels' sampler kernel ahead of each is not counted).  Each step is one step_kernel
launch, plus, for the general / 512-cell kernels, a spill_kernel launch and a
reset_kernel launch masked by FL_RESET (the deferred autoreset).  This prints
the median count per env of each counter over the normal, storm and quick
step_kernel launches ("normal" / "storm" / "quick"), over the masked reset
launches of the storm steps ("reset_storm": the regeneration of every board)
and of the other steps ("reset_idle": no board to regenerate), and over the
spill launches ("spill"); and (normal - quick) / effective fraction as the
cost of one effective step when --eff-frac is given.
"""
import argparse
import collections
import csv
import glob
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--boards", type=int, required=True)
    ap.add_argument("--eff-frac", type=float, default=0.0)
    args = ap.parse_args()
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for d in args.dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                key = (d, int(r["Dispatch_Id"]))
                names[key] = r["Kernel_Name"]
                per[key][r["Counter_Name"]] += float(r["Counter_Value"])
    out = {}
    for d in args.dirs:
        keys = sorted(k for k in names if k[0] == d)
        steps = [k for k in keys if "step_kernel" in names[k]]
        cats = collections.defaultdict(list)
        for i, k in enumerate(steps):
            if i < 60:
                cats["storm" if i % 30 == 29 else "normal"].append(per[k])
            elif i < 80:
                cats["quick"].append(per[k])
            else:
                cats["policy"].append(per[k])
        # the masked reset / spill launches that follow step i (before step i + 1)
        first = steps[0][1] if steps else None
        si = -1
        for k in keys:
            if first is None or k[1] < first:
                continue                      # the initial reset() launch
            nm = names[k]
            if "step_kernel" in nm:
                si += 1
            elif si < 60 and "reset_kernel" in nm:
                cats["reset_storm" if si % 30 == 29 else "reset_idle"].append(per[k])
            elif si < 60 and "spill_kernel" in nm:
                cats["spill"].append(per[k])
        for c, rows in cats.items():
            if not rows:
                continue
            for cn in sorted(rows[0]):
                out.setdefault(c, {})[cn] = round(statistics.median(r[cn] for r in rows) / args.boards, 2)
    if args.eff_frac and "normal" in out and "quick" in out:
        out["effective_step"] = {cn: round((out["normal"][cn] - out["quick"][cn]) / args.eff_frac, 1)
                                 for cn in out["normal"] if cn in out["quick"]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
