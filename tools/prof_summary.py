"""Summarise a tools/gpu_profile.sh run into profiles/ (kernel stats, HBM
traffic, MFMA utilisation).

  python tools/prof_summary.py <gpurun_out/TAG> <tag> [config]

Inputs (rocprofv3 CSV): stats/ (--kernel-trace --stats), mfma/ (SQ/GRBM
counters), fetch/ (FETCH_SIZE), write/ (WRITE_SIZE) -- separate passes.

HBM bytes per launch follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE and
WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half the bytes of wide
coalesced reads, so reads are doubled: hbm = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8
XCDs); effective clock = GRBM_GUI_ACTIVE / 8 / kernel time; MFMA FLOPs =
SQ_INSTS_VALU_MFMA_MOPS_* x 512.
"""
import csv
import glob
import json
import os
import re
import sys

N_SIMD = 1024      # 256 CUs x 4
N_XCD = 8


# chain-kernel precision template argument of the forward / backward chains
# of each plan (bf16x3f: the bf16x3 forward, the bf16 backward)
FWD_P = {"fp32": 0, "bf16": 1, "bf16x3": 2, "bf16x3f": 2}
BWD_P = {"fp32": 0, "bf16": 1, "bf16x3": 2, "bf16x3f": 1}


def short(name, prec):
    m = re.search(r"chain(?:16)?_kernel<(\d), \d, \d, (true|false), \d+, (\d)>", name)
    if m:
        kind = "bwd" if m.group(2) == "true" else "fwd"
        if int(m.group(1)) != (BWD_P if kind == "bwd" else FWD_P)[prec]:
            return None
        mode = int(m.group(3))       # 1 train, 3 train (hi planes only), 2 codes, 0 infer
        return kind if mode in (1, 3) else f"{kind}_codes" if mode == 2 else f"{kind}_infer"
    m = re.search(r"\bdw_kernel<(\d)>", name)
    if m and int(m.group(1)) == min(FWD_P[prec], 1):     # every bf16 plan stores bf16 planes: the bf16 dW pass
        return "dw"
    return None


def counters(d):
    """kernel -> counter -> mean per dispatch; '_ns' = mean dispatch duration of
    the PMC pass (counter collection serialises dispatches)."""
    out, dur = {}, {}
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            k = r["Kernel_Name"]
            out.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
            dur.setdefault(k, {})[r["Dispatch_Id"]] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    res = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in out.items()}
    for k, v in dur.items():
        res[k]["_ns"] = sum(v.values()) / len(v)
    return res


def main():
    src, tag = sys.argv[1:3]
    config = sys.argv[3] if len(sys.argv) > 3 else "c2"
    precision = sys.argv[4] if len(sys.argv) > 4 else ("fp32" if config == "c5" else "bf16")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(repo, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = list(csv.DictReader(open(glob.glob(os.path.join(src, "stats", "**", "*kernel_stats.csv"),
                                               recursive=True)[0])))
    mf, fe, wr = (counters(os.path.join(src, d)) for d in ("mfma", "fetch", "write"))
    lines = [f"# rocprofv3 summary ({tag}, bench config {config})", "",
             "Passes (separate runs of the same command): --kernel-trace --stats; --pmc SQ_WAVE_CYCLES "
             "SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 "
             "GRBM_GUI_ACTIVE GRBM_COUNT; --pmc FETCH_SIZE; --pmc WRITE_SIZE.  HBM = (2 FETCH_SIZE + WRITE_SIZE) KiB "
             "(gfx950 FETCH_SIZE halving); MFMA util = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMD x GRBM_GUI_ACTIVE / 8); "
             "clock = GRBM_GUI_ACTIVE / 8 / the PMC pass's own dispatch time (counter passes serialise dispatches, so the dX / dW overlap is absent there; profiled runs clock lower than unprofiled ones).", "",
             "| kernel | calls | avg us | % time | HBM GB/launch | GB/s | MFMA TFLOP/launch | avg us (PMC pass, serialised) | MFMA util | eff. clock GHz |",
             "|---|---|---|---|---|---|---|---|---|---|"]
    traffic = {}
    for r in stats:
        name = r["Name"]
        avg_ns = float(r["AverageNs"])
        f = fe.get(name, {}).get("FETCH_SIZE")
        w = wr.get(name, {}).get("WRITE_SIZE")
        c = mf.get(name, {})
        hbm = (2 * f + w) * 1024 if f is not None and w is not None else None
        gbs = hbm / avg_ns if hbm else None
        gui = c.get("GRBM_GUI_ACTIVE")
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES")
        mops = (c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16") or 0) + (c.get("SQ_INSTS_VALU_MFMA_MOPS_F32") or 0)
        util = busy / (N_SIMD * gui / N_XCD) if gui and busy is not None else None
        pmc_ns = c.get("_ns")
        clk = gui / N_XCD / pmc_ns if gui and pmc_ns else None
        tfl = mops * 512 / 1e12 if mops else None

        def fmt(x, nd):
            return "" if x is None else round(x, nd)
        lines.append(f"| `{name[:90]}` | {r['Calls']} | {avg_ns / 1e3:.1f} | {float(r['Percentage']):.2f} | "
                     f"{fmt(hbm and hbm / 1e9, 3)} | {fmt(gbs, 1)} | {fmt(tfl, 4)} | {fmt(pmc_ns and pmc_ns / 1e3, 1)} | "
                     f"{fmt(util, 3)} | {fmt(clk, 2)} |")
        s = short(name, precision)
        if s and hbm:
            traffic[s] = {"hbm_bytes": int(hbm), "fetch_kib": f, "write_kib": w, "avg_ns": avg_ns,
                          "mfma_util": util, "eff_clock_ghz": clk, "pmc_pass_avg_ns": pmc_ns, "mfma_flop": mops * 512 if mops else None,
                          "source": f"profiles/{tag}_kernels.md"}
    open(os.path.join(prof, f"{tag}_kernels.md"), "w").write("\n".join(lines) + "\n")
    path = os.path.join(prof, "pmc_traffic.json")
    allt = json.load(open(path)) if os.path.exists(path) else {}
    allt[config if precision == "bf16" or config == "c5" else f"{config}_{precision}"] = traffic
    json.dump(allt, open(path, "w"), indent=1)
    print("\n".join(lines[:18]))


if __name__ == "__main__":
    main()
