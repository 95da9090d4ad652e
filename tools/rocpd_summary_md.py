"""rocpd2summary kernels CSV -> markdown table for profiles/ (per-step ms = total / --steps, the
number of train steps inside the profiled run, warmup included).

    rocpd2summary -i run_results.db -f csv -d out -o run   # -> out/run_kernels_summary.csv
    python tools/rocpd_summary_md.py out/run_kernels_summary.csv --steps 3 --title "..." > profiles/x.md
"""
import argparse
import csv


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(")[0] if "<" not in name else name.split(">")[0] + ">"


ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--steps", type=int, required=True)
ap.add_argument("--title", default="")
ap.add_argument("--top", type=int, default=40)
a = ap.parse_args()
rows = list(csv.DictReader(open(a.csv)))
tot = sum(float(r["Duration (Nsec)"]) for r in rows)
print(f"# {a.title}\n\nSource: rocprofv3 --kernel-trace --stats (rocpd database -> rocpd2summary CSV). "
      f"{a.steps} train steps in the profiled run; per-step ms = total / {a.steps}. "
      f"Sum of kernel time: {tot / 1e6 / a.steps:.1f} ms per step.\n")
print("| kernel | calls | ms / step | avg us | share |\n|---|---|---|---|---|")
for r in rows[:a.top]:
    d = float(r["Duration (Nsec)"])
    print(f"| `{short(r['Name'])}` | {r['Calls']} | {d / 1e6 / a.steps:.2f} | {float(r['Average (Nsec)']) / 1e3:.1f} | "
          f"{100 * d / tot:.1f}% |")
