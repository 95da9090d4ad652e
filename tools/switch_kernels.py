"""Which launches each switch form of tests/test_switch_forms_gpu.py changes: run the test's models
once per case (a warm-up first) with 0.2 s idle between cases, under
    rocprofv3 --kernel-trace --output-format csv -d DIR -o k -- python tools/switch_kernels.py
then `python tools/switch_kernels.py --trace DIR/k_kernel_trace.csv` splits the trace at the idle
gaps and prints, per case, the kernels it launched that its parent case (same shape, all but the
last override) did not and vice versa."""
import argparse
import collections
import csv
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run():
    import torch
    import test_switch_forms_gpu as T
    from picotron_amd import switches
    built = {name: T.build(name) for name in T.CONFIGS}
    for name, over in [("a", {})] + T.CASES:   # the first: warm-up (descriptor tables, first-launch attributes)
        torch.cuda.synchronize()
        time.sleep(0.2)
        with switches.override(**T.FORCE, **over):
            T.run(*built[name])
        print(name, over, flush=True)


def summarize(path):
    import test_switch_forms_gpu as T
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    segs, cur, last = [], [], None
    for r in rows:
        s = int(r["Start_Timestamp"])
        if last is not None and s - last > 100_000_000:   # 0.1 s idle: a case boundary
            segs.append(cur)
            cur = []
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        cur.append(n[:n.find("(")] if "(" in n else n)
        last = int(r["End_Timestamp"])
    segs.append(cur)
    # the cases are the last len(CASES) segments (before them: model construction and the warm-up)
    assert len(segs) >= len(T.CASES) + 1, (len(segs), len(T.CASES))
    cases, segs = [None] + T.CASES, segs[-len(T.CASES) - 1:]
    prev = {}
    for case, seg in zip(cases[1:], segs[1:]):
        c = collections.Counter(seg)
        name, over = case
        if not over:
            prev[name] = c
            print(f"{T.case_id(case)}: {sum(c.values())} launches")
            continue
        # against the nearest listed case with the same shape and a prefix of these overrides
        known = {T.case_id(cs): collections.Counter(sg) for cs, sg in zip(cases[1:], segs[1:])}
        items = list(over.items())
        for n in range(len(items) - 1, -1, -1):
            parent = dict(items[:n])
            if T.case_id((name, parent)) in known:
                break
        base = known[T.case_id((name, parent))]
        plus, minus = c - base, base - c
        print(f"{T.case_id(case)} vs {T.case_id((name, parent))}: {sum(c.values())} launches ({sum(base.values())})")
        for k, v in sorted(plus.items()):
            print(f"   + {v:3d} {k}")
        for k, v in sorted(minus.items()):
            print(f"   - {v:3d} {k}")
        if not plus and not minus:
            print("   (same kernels: the form changes a launch's grid / tile order / work split only)")


sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", default="")
    a = ap.parse_args()
    if a.trace:
        summarize(a.trace)
    else:
        run()
