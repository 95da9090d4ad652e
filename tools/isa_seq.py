"""Compact per-basic-block instruction sequence of one kernel in a hipcc --save-temps .s file.

    python tools/isa_seq.py FILE.s KERNEL_SUBSTRING [--min-mfma 1]

One line per basic block: its label, instruction counts by class and a run-length string
(M = MFMA, V = VALU, E = transcendental, A = accvgpr move, R = LDS read, W = LDS write,
G = global/buffer memory, B = s_barrier, w = s_waitcnt, S = other scalar), e.g.
"R4 M1 V5 M1 E2 ...".  Used to check how a kernel's MFMAs and softmax VALU interleave and where
register copies land.
"""
import re
import sys


def klass(op):
    if op.startswith("v_mfma"):
        return "M"
    if op.startswith("v_accvgpr"):
        return "A"
    if op in ("v_exp_f32", "v_log_f32", "v_rcp_f32", "v_rsq_f32", "v_sqrt_f32"):
        return "E"
    if op.startswith("ds_read") or op.startswith("ds_load"):
        return "R"
    if op.startswith("ds_"):
        return "W"
    if op.startswith(("global_", "buffer_", "scratch_", "flat_")):
        return "G"
    if op == "s_barrier":
        return "B"
    if op.startswith("s_waitcnt"):
        return "w"
    if op.startswith("v_"):
        return "V"
    if op.startswith("s_"):
        return "S"
    return None


def main():
    path, sub = sys.argv[1], sys.argv[2]
    min_mfma = int(sys.argv[sys.argv.index("--min-mfma") + 1]) if "--min-mfma" in sys.argv else 0
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*" + re.escape(sub) + r"\w*:", l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks, cur = [], ["entry", []]
    for l in lines[start + 1:end]:
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            blocks.append(cur)
            cur = [m.group(1), []]
            continue
        t = l.strip().split()
        if not t or t[0].startswith((";", ".")):
            continue
        c = klass(t[0])
        if c:
            cur[1].append(c)
    blocks.append(cur)
    for name, seq in blocks:
        if seq.count("M") < min_mfma:
            continue
        runs, prev, n = [], None, 0
        for c in seq + [None]:
            if c == prev:
                n += 1
                continue
            if prev is not None:
                runs.append(f"{prev}{n}")
            prev, n = c, 1
        counts = {k: seq.count(k) for k in "MVEARWGBwS" if seq.count(k)}
        print(f"{name} {counts}\n   {' '.join(runs)}")


if __name__ == "__main__":
    main()
