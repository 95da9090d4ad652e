"""Summarise a rocprofv3 run of bench.py into a markdown table for profiles/.

    python tools/prof_summary.py --trace gpurun_out/prof/r1_kernel_trace.csv(.gz) \
        --fetch gpurun_out/pmc1/fetch_counter_collection.csv --write gpurun_out/pmc2/write_counter_collection.csv \
        --steps 3 > profiles/round1_bench_kernels.md

Per kernel instance (template args + grid): launches, total / average duration, and for the GEMM
the algorithmic FLOP of the launch shape, TF/s, and the PMC HBM bytes per launch (FETCH_SIZE x 2,
the gfx950 correction of MI355X_MICROARCH.md §HBM, + WRITE_SIZE; both counters are in KiB).
"""
import argparse
import collections
import csv
import gzip


def rd(path):
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rt") as f:
        return list(csv.DictReader(f))


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(")[0] if "<" not in name else name.split(">")[0] + ">"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--steps", type=int, default=1)
    a = ap.parse_args()
    rows = rd(a.trace)
    groups = collections.defaultdict(list)
    for r in rows:
        threads = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        groups[(short(r["Kernel_Name"]), grid // max(threads, 1))].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    total = sum(sum(v) for v in groups.values())
    pmc = collections.defaultdict(lambda: [0.0, 0, 0.0, 0])
    for path, idx, mul in ((a.fetch, 0, 2.0), (a.write, 2, 1.0)):
        if not path:
            continue
        for r in rd(path):
            key = (short(r["Kernel_Name"]), int(r["Grid_Size"]) // max(int(r["Workgroup_Size"]), 1))
            pmc[key][idx] += float(r["Counter_Value"]) * 1024 * mul
            pmc[key][idx + 1] += 1
    print(f"Total kernel time {total / 1e6:.1f} ms over {a.steps} step(s) = {total / 1e6 / a.steps:.1f} ms/step\n")
    print("| kernel | workgroups | launches | total ms | share | avg us | HBM MB/launch (PMC) |")
    print("|---|---|---|---|---|---|---|")
    for k, v in sorted(groups.items(), key=lambda kv: -sum(kv[1]))[:40]:
        p = pmc.get(k)
        hbm = ""
        if p and p[1] and p[3]:
            hbm = f"{(p[0] / p[1] + p[2] / p[3]) / 1e6:.1f}"
        print(f"| `{k[0]}` | {k[1]} | {len(v)} | {sum(v) / 1e6:.1f} | {sum(v) / total * 100:.1f}% | "
              f"{sum(v) / len(v) / 1e3:.1f} | {hbm} |")
    # the bench line's roofline kernel is "every GEMM launch": its average, to set beside
    # roofline.avg_launch_ms (bench.py times one steady-state micro-batch per step with HIP events)
    g = [d for k, v in groups.items() if k[0].startswith("void gemm_") for d in v]
    if g:
        print(f"\nAll GEMM launches (`gemm_*` kernels): {len(g)} launches, {sum(g) / 1e6:.1f} ms, "
              f"average {sum(g) / len(g) / 1e3:.1f} us per launch, {sum(g) / total * 100:.1f}% of kernel time")


if __name__ == "__main__":
    main()
