"""ISA check for the chain kernels' counted LDS waits (tools/extract_isa.py
output): every MFMA's A operand must come straight from a ds_read_b128 (no
register copy in between) that an s_waitcnt lgkmcnt(n) between the read and
the MFMA has retired -- LDS reads return in order, so a read is retired when
at least n LDS operations were issued after it before the wait.  Used on
builds where the wait is the s_waitcnt builtin (the compiler does not know
the asm reads are pending).

  python tools/check_frag_waits.py <file.s>   -> exit 1 on a violation
"""
import re
import sys


def regs(tok):
    m = re.match(r"([va])\[(\d+):(\d+)\]", tok)
    if m:
        return {f"{m.group(1)}{i}" for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r"([va])(\d+)$", tok)
    return {tok} if m else set()


def main(path):
    ins = []
    for line in open(path):
        if re.match(r"\s+[a-z]", line):
            ins.append(line.split("//")[0].strip())
    bad = checked = 0
    for k, l in enumerate(ins):
        if not l.startswith("v_mfma"):
            continue
        ops = [o.strip() for o in l.split(None, 1)[1].split(",")]
        a = regs(ops[1])
        # last writer of the A registers
        j = k - 1
        while j >= 0:
            w = ins[j].split(None, 1)
            if len(w) == 2:
                dst = regs(w[1].split(",")[0].strip())
                if dst & a and not ins[j].startswith(("s_", "buffer_store", "global_store", "ds_write")):
                    break
            j -= 1
        if j < 0:
            continue           # an operand from before the kernel's first instruction: not a fragment
        if not ins[j].startswith("ds_read"):
            if ins[j].startswith("v_mfma"):
                continue
            print(f"MFMA {k}: A operand {ops[1]} last written by '{ins[j]}' (not an LDS read)")
            bad += 1
            continue
        checked += 1
        after = 0
        ok = False
        for x in range(j + 1, k):
            s = ins[x]
            if s.startswith("ds_"):
                after += 1
            m = re.match(r"s_waitcnt.*lgkmcnt\((\d+)\)", s)
            if m and after >= int(m.group(1)):
                ok = True
                break
        if not ok:
            print(f"MFMA {k}: fragment read at {j} ({ins[j]}) not retired by a wait before it")
            bad += 1
    print(f"{path}: {checked} fragment reads checked, {bad} violations")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
