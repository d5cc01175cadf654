"""Per-step kernel timeline from a rocprofv3 --kernel-trace CSV.

  python tools/timeline.py <dir with *kernel_trace.csv> [steps]

A step starts at a get_rays_kernel dispatch.  For the last `steps` steps it
prints each dispatch's start offset within the step, duration, and the idle
gap since the previous dispatch ended (any stream), then the step's busy /
idle totals, so launch gaps and host syncs on the critical path show up.
"""
import csv
import glob
import os
import sys


def short(n):
    n = n.split("(")[0]
    return n.replace("void ", "").replace("cn::", "")[:60]


def main():
    d = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    rows = []
    for fn in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if "get_rays_kernel" in r[2]]
    if len(starts) < steps + 1:
        print("not enough steps", len(starts))
        return
    for k in range(len(starts) - steps - 1, len(starts) - 1):
        a, b = starts[k], starts[k + 1]
        t0 = rows[a][0]
        busy_end = t0
        idle = 0
        print(f"--- step {k}: {(rows[b][0] - t0) / 1e3:.1f} us")
        for s, e, n in rows[a:b]:
            gap = max(0, s - busy_end)
            idle += gap
            busy_end = max(busy_end, e)
            print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:9.1f}  gap {gap / 1e3:7.1f}  {short(n)}")
        print(f"idle (no kernel running) {idle / 1e3:.1f} us")


if __name__ == "__main__":
    main()
