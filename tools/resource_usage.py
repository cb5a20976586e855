"""Per-kernel register / scratch / occupancy table of libtmg's translation
units, from the compiler's kernel-resource-usage remarks (diagnostics).

    python tools/resource_usage.py [EXTRA_HIPCC_FLAGS ...]     (TMG_TUS="4 5": those units only)
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "tile-match-gym_amd")
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-I../include", "-Icsrc", "-Wall",
         "-Wno-unused-function", "-Rpass-analysis=kernel-resource-usage", "--offload-device-only", "-c"]


def short(name):
    m = re.search(r"_ZN3tmg(\d+)(\w+?)I(.*)E(E?)v", name)
    if not m:
        return name[:60]
    base = m.group(2)[: int(m.group(1))]
    args = re.findall(r"L([ib])(\d+)E", m.group(3))
    return base + "<" + ",".join(("true" if v == "1" else "false") if t == "b" else v for t, v in args) + ">"


def main():
    extra = sys.argv[1:]
    rows = []
    tus = [int(t) for t in os.environ.get("TMG_TUS", "1 2 3 4 5 6 7").split()]
    with tempfile.TemporaryDirectory() as tmp:          # the translation units compile in parallel
        procs = [(tu, subprocess.Popen(["/opt/rocm/bin/hipcc", *FLAGS, *extra, f"-DTMG_TU={tu}", "-o",
                                        os.path.join(tmp, f"k{tu}.o"), "csrc/tmg_kernels.hip"], cwd=PKG,
                                       stderr=subprocess.PIPE, stdout=subprocess.DEVNULL, text=True))
                 for tu in tus]
        outs = [(tu, p.communicate()[1], p.returncode) for tu, p in procs]
    for tu, err, rc in outs:
        cur = None
        for line in err.splitlines():
            m = re.search(r"remark: Function Name: (\S+)", line)
            if m:
                cur = {"name": short(m.group(1)), "tu": tu}
                rows.append(cur)
                continue
            m = re.search(r"remark:\s+(VGPRs|AGPRs|TotalSGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                          r"SGPRs Spill|LDS Size \[bytes/block\]): (\d+)", line)
            if m and cur is not None:
                cur[m.group(1).replace("SGPRs Spill", "SGPRsSpill").split()[0]] = int(m.group(2))
        if rc:
            print(err[-3000:])
            sys.exit(1)
    print(f"{'kernel':44s} {'TU':>2s} {'VGPR':>4s} {'SGPR':>4s} {'scr':>4s} {'occ':>3s} {'sspill':>6s}")
    for r in rows:
        print(f"{r['name']:44s} {r['tu']:2d} {r.get('VGPRs', 0):4d} {r.get('TotalSGPRs', 0):4d} "
              f"{r.get('ScratchSize', 0):4d} {r.get('Occupancy', 0):3d} {r.get('SGPRsSpill', 0):6d}")


if __name__ == "__main__":
    main()
