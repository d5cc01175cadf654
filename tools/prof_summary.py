"""Summarise rocprofv3 CSV output into profiles/ (kernel stats + HBM traffic).

  python tools/prof_summary.py <stats_dir> <fetch_dir> <write_dir> <tag>

HBM bytes per launch follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE and
WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half the bytes of wide
coalesced reads, so reads are doubled: hbm = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
"""
import csv
import glob
import json
import os
import sys

SHORT = {"chain_kernel<1, 3, 1, false, 8, true>": "fwd", "chain_kernel<1, 3, 1, true, 8, true>": "bwd",
         "dw_kernel<1>": "dw", "chain_kernel<0, 3, 1, false, 4, true>": "fwd",
         "chain_kernel<0, 3, 1, true, 4, true>": "bwd", "dw_kernel<0>": "dw"}


def short(name):
    for k, v in SHORT.items():
        if k in name:
            return v
    return None


def counters(d, counter):
    out = {}
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            if r["Counter_Name"] == counter:
                out.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in out.items()}


def main():
    stats_dir, fetch_dir, write_dir, tag = sys.argv[1:5]
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(repo, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = list(csv.DictReader(open(glob.glob(os.path.join(stats_dir, "**", "*kernel_stats.csv"), recursive=True)[0])))
    fetch, write = counters(fetch_dir, "FETCH_SIZE"), counters(write_dir, "WRITE_SIZE")
    lines = [f"# rocprofv3 --kernel-trace --stats ({tag})", "",
             "| kernel | calls | avg us | % time | FETCH_SIZE KiB | WRITE_SIZE KiB | HBM GB/launch (2F+W) | GB/s |",
             "|---|---|---|---|---|---|---|---|"]
    traffic = {}
    for r in stats:
        name = r["Name"]
        avg_ns = float(r["AverageNs"])
        f, w = fetch.get(name), write.get(name)
        hbm = (2 * f + w) * 1024 if f is not None and w is not None else None
        gbs = hbm / avg_ns if hbm else None
        lines.append(f"| `{name[:90]}` | {r['Calls']} | {avg_ns / 1e3:.1f} | {float(r['Percentage']):.2f} | "
                     f"{f if f is None else round(f)} | {w if w is None else round(w)} | "
                     f"{'' if hbm is None else round(hbm / 1e9, 3)} | {'' if gbs is None else round(gbs, 1)} |")
        s = short(name)
        if s and hbm:
            traffic[s] = {"hbm_bytes": int(hbm), "fetch_kib": f, "write_kib": w, "avg_ns": avg_ns,
                          "source": f"profiles/{tag}_kernels.md"}
    open(os.path.join(prof, f"{tag}_kernels.md"), "w").write("\n".join(lines) + "\n")
    # keyed by bench config (the profiled command is bench.py's default, C2)
    json.dump({"c2": traffic}, open(os.path.join(prof, "pmc_traffic.json"), "w"), indent=1)
    print("\n".join(lines[:16]))


if __name__ == "__main__":
    main()
