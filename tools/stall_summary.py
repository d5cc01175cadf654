"""Per-kernel stall / issue fractions from tools/gpu_stalls.sh's two PMC passes.

  python tools/stall_summary.py <pass1 dir> <pass2 dir>

SIMD-cycle fractions = counter / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs);
wave-cycle fractions = counter / SQ_WAVE_CYCLES (pass 1's, per kernel);
instruction counts are per wave (/ waves launched).
"""
import collections
import csv
import glob
import re
import sys

N_SIMD, N_XCD = 1024, 8


def load(d):
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"chain(?:16)?_kernel<(\d), \d, \d, (true|false), (\d+), (\d)>", r["Kernel_Name"])
            d = re.search(r"\bdw_kernel<(\d)>", r["Kernel_Name"])
            if m:
                k = f"chain<P{m.group(1)},{'bwd' if m.group(2) == 'true' else 'fwd'},{m.group(3)}w,mode{m.group(4)}>"
            elif d:
                k = f"dw_kernel<P{d.group(1)}>"
            else:
                continue
            out[k][r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"]), int(r["Grid_Size"]),
                                              int(r["Workgroup_Size"])))
    return out


def mean(v):
    return sum(x[1] for x in v) / len(v)


def main():
    a, b = load(sys.argv[1]), load(sys.argv[2])
    print("| kernel | MFMA busy (SIMD) | MFMA+VALU co-exec (SIMD) | VALU active (wave) | LDS active (wave) | "
          "MISC active (wave) | WAIT_ANY (wave) | WAIT_INST_ANY (wave) | WAIT_INST_LDS (wave) | ACTIVE_INST_ANY (wave) | "
          "LDS bank conflict (SIMD) | VALU / MFMA / LDS / SALU insts per wave |")
    print("|" + "---|" * 13)
    for k in sorted(a):
        c1, c2 = a[k], b.get(k, {})
        simd = N_SIMD * mean(c1["GRBM_GUI_ACTIVE"]) / N_XCD
        wave = mean(c1["SQ_WAVE_CYCLES"])
        g = c1["GRBM_GUI_ACTIVE"][0]
        waves = g[2] / 64
        f = lambda c, n, base: (mean(c[n]) / base) if n in c else float("nan")
        ins = lambda n: (mean(c2[n]) / waves) if n in c2 else float("nan")
        print(f"| `{k}` | {f(c1, 'SQ_VALU_MFMA_BUSY_CYCLES', simd):.3f} | {f(c1, 'SQ_VALU_MFMA_COEXEC_CYCLES', simd):.3f} | "
              f"{f(c1, 'SQ_ACTIVE_INST_VALU', wave):.3f} | {f(c2, 'SQ_ACTIVE_INST_LDS', wave):.3f} | "
              f"{f(c1, 'SQ_ACTIVE_INST_MISC', wave):.3f} | {f(c2, 'SQ_WAIT_ANY', wave):.3f} | "
              f"{f(c2, 'SQ_WAIT_INST_ANY', wave):.3f} | {f(c1, 'SQ_WAIT_INST_LDS', wave):.3f} | "
              f"{f(c2, 'SQ_ACTIVE_INST_ANY', wave):.3f} | {f(c1, 'SQ_LDS_BANK_CONFLICT', simd):.4f} | "
              f"{ins('SQ_INSTS_VALU'):.0f} / {ins('SQ_INSTS_MFMA'):.0f} / {ins('SQ_INSTS_LDS'):.0f} / {ins('SQ_INSTS_SALU'):.0f} |")


if __name__ == "__main__":
    main()
