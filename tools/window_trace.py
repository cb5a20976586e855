"""Timeline of the bench's timed window from a rocprofv3 --kernel-trace run.

    rocprofv3 --kernel-trace -d OUT -o run --output-format csv -- python3 bench.py --steps K --warmup W
    python tools/window_trace.py OUT K [GROUPS]

The timed window is the last K x GROUPS step_kernel launches (plus the reset /
spill launches between them).  Prints the window's span, each stream's busy
time, first start / last end relative to the window, and the long launches
(autoreset storms), to show where a short window loses against the steady
state.
"""
import csv
import glob
import os
import statistics
import sys


def main():
    root, K = sys.argv[1], int(sys.argv[2])
    G = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    rows = []
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if "tmg::" not in n:
                continue
            q = r.get("Stream_Id") or r.get("Queue_Id")
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), q, n.split("<")[0].replace("void ", "").replace("tmg::", "").strip()))
    rows.sort()
    steps = [i for i, r in enumerate(rows) if r[3] == "step_kernel"]
    first = steps[-K * G]
    win = rows[first:]
    t0 = min(r[0] for r in win)
    t1 = max(r[1] for r in win)
    span = (t1 - t0) / 1e3
    print(f"window: {len(win)} launches, span {span:.1f} us ({span / K:.1f} us per step)")
    durs = [(r[1] - r[0]) / 1e3 for r in win]
    med = statistics.median(durs)
    print(f"sum of launch durations {sum(durs):.1f} us (average concurrency {sum(durs) / span:.2f}), median launch {med:.1f} us")
    for q in sorted({r[2] for r in win}):
        rs = [r for r in win if r[2] == q]
        busy = sum(r[1] - r[0] for r in rs) / 1e3
        print(f"  stream {q}: {len(rs)} launches, busy {busy:.1f} us, first start +{(rs[0][0] - t0) / 1e3:.1f}, "
              f"last end +{(rs[-1][1] - t0) / 1e3:.1f} us, longest {max(r[1] - r[0] for r in rs) / 1e3:.1f} us")
    for r in win:
        d = (r[1] - r[0]) / 1e3
        if d > 3 * med:
            print(f"  long: {r[3]} stream {r[2]} +{(r[0] - t0) / 1e3:.1f} .. +{(r[1] - t0) / 1e3:.1f} us ({d:.1f} us)")


if __name__ == "__main__":
    main()
