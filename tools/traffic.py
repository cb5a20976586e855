"""Reduce rocprofv3 FETCH_SIZE / WRITE_SIZE passes (scripts/gpu_traffic.sh) to
HBM bytes per step_kernel launch, averaged over every dispatch of the bench
(warm-up + timed: 1 in 30 is an autoreset launch, as in the timed region).

    python tools/traffic.py gpurun_out/traffic > profiles/traffic.json

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


def per_dispatch(path, counter):
    vals = collections.defaultdict(float)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "step_kernel" not in r["Kernel_Name"] or r["Counter_Name"] != counter:
                continue
            vals[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return list(vals.values())


def main():
    root = sys.argv[1]
    out = {}
    for d in sorted(glob.glob(os.path.join(root, "*_FETCH_SIZE"))):
        cfg = os.path.basename(d).split("_")[0]
        f = per_dispatch(d, "FETCH_SIZE")
        w = per_dispatch(os.path.join(root, f"{cfg}_WRITE_SIZE"), "WRITE_SIZE")
        if not f or not w:
            continue
        fk = sum(f) / len(f)
        wk = sum(w) / len(w)
        out[cfg] = {
            "hbm_bytes_per_launch": round((2 * fk + wk) * 1024),
            "fetch_size_kib_raw": round(fk, 1),
            "write_size_kib": round(wk, 1),
            "dispatches": [len(f), len(w)],
            "correction": "FETCH_SIZE x2 (gfx950 half-count, MI355X_MICROARCH.md HBM section); WRITE_SIZE as is",
        }
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
