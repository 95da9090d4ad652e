"""Summarise rocprofv3 --kernel-trace --stats and --pmc CSVs per kernel (tools/gpu.sh, attention and GEMM
counter passes): python tools/pmc_table.py <stats.csv> <counter_collection.csv>... [--match REGEX]"""
import collections
import csv
import re
import sys


def short(name):
    m = re.search(r"(\w+(?:<[^()]*>)?)\(", name.replace("(anonymous namespace)::", ""))
    return m.group(1) if m else name[:60]


def main(argv):
    match = None
    if "--match" in argv:
        i = argv.index("--match")
        match, argv = argv[i + 1], argv[:i] + argv[i + 2:]
    stats, pmcs = argv[0], argv[1:]
    for r in csv.DictReader(open(stats)):
        if match and not re.search(match, r["Name"]):
            continue
        print(f"{short(r['Name']):55s} calls {r['Calls']:>5s} avg {float(r['AverageNs']) / 1e3:8.1f} us")
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in pmcs:
        for r in csv.DictReader(open(p)):
            if match and not re.search(match, r["Kernel_Name"]):
                continue
            k = short(r["Kernel_Name"])
            per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            for c in ("Arch_VGPR_Count", "Accum_VGPR_Count", "LDS_Block_Size", "Scratch_Size"):
                if r.get(c) not in (None, ""):
                    per[k][c] = [float(r[c])]
    for k, d in per.items():
        a = {c: sum(v) / len(v) for c, v in d.items()}
        out = {"vgpr": a.get("Arch_VGPR_Count"), "agpr": a.get("Accum_VGPR_Count"), "lds": a.get("LDS_Block_Size")}
        g = a.get("GRBM_GUI_ACTIVE")
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in a:
            out["mfma_busy"] = round(a["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / 8 * 1024), 3)
        if g and "SQ_LDS_IDX_ACTIVE" in a:
            out["lds_busy"] = round(a["SQ_LDS_IDX_ACTIVE"] / (g / 8 * 256), 3)
        if a.get("SQ_INSTS_MFMA"):
            out["valu_per_mfma"] = round(a.get("SQ_INSTS_VALU", 0) / a["SQ_INSTS_MFMA"], 2)
            out["lds_per_mfma"] = round(a.get("SQ_INSTS_LDS", 0) / a["SQ_INSTS_MFMA"], 2)
            out["salu_per_mfma"] = round(a.get("SQ_INSTS_SALU", 0) / a["SQ_INSTS_MFMA"], 2)
        wc = a.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY"):
                if c in a:
                    out[c.replace("SQ_", "").lower() + "_frac"] = round(a[c] / wc, 3)
        if "SQ_LDS_BANK_CONFLICT" in a:
            out["bank_conflict"] = a["SQ_LDS_BANK_CONFLICT"]
        print(k, out)


if __name__ == "__main__":
    main(sys.argv[1:])
