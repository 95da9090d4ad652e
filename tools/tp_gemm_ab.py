"""TP-shard GEMM launch forms, timed on the GPU: for every GEMM a TP = 8 rank of SmolLM-1.7B runs
(T = 4096), the production call (kernels.py's choice) against the 128x128 k-substep tile (15)
unsplit and as 2 / 4 K-slices, and the simple 128x128 tile (2).  Informs kernels.fewtile_ksplit /
wgrad_ksplit.   python tools/tp_gemm_ab.py [--tp 8] [--reps 20]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotron_amd import kernels as K  # noqa: E402

T, H, I = 4096, 2048, 8192
BF = torch.bfloat16


def timed(fn, reps):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = None
    for _ in range(3):
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        best = ms if best is None else min(best, ms)
    return best * 1e3   # us


def r(*shape):
    return ((torch.rand(*shape, device="cuda") * 2 - 1) * 0.1).to(BF)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    tp = args.tp
    q, i2, o, i1 = 3 * H // tp, 2 * I // tp, H // tp, I // tp
    rows = []

    def report(name, flop, variants):
        res = {"shape": name, "gflop": round(flop / 1e9, 2)}
        for vn, fn in variants:
            try:
                us = timed(fn, args.reps)
                res[vn] = round(us, 1)
            except Exception as e:   # a form that does not tile this shape
                res[vn] = f"n/a ({type(e).__name__})"
        print(json.dumps(res), flush=True)
        rows.append(res)

    # forward projections: x [T, H] . W^T
    for name, n, kin in (("fwd.qkv", q, H), ("fwd.o", H, o), ("fwd.gate_up", i2, H), ("fwd.down", H, i1)):
        x, w = r(T, kin), r(n, kin)
        y = torch.empty(T, n, dtype=BF, device="cuda")
        v = [("prod", lambda: K.linear_fwd(x, [w])),
             ("t15", lambda: K.linear_fwd(x, [w], tile=15)),
             ("t13", lambda: K.linear_fwd(x, [w], tile=13) if n % 128 == 0 else None),
             ("t2", lambda: K.linear_fwd(x, [w], tile=2))]
        for s in (2, 4):
            if kin % (s * 64) == 0:
                v.append((f"t15ks{s}", lambda s=s: K._gemm_ksplit(x, x.stride(0), 1, [w], [kin], [0, n], 1, 0, y, T, n,
                                                                  kin, s, 15, K.EPI_BF16)))
        report(name, 2.0 * T * n * kin, v)
    # dX projections: dy [T, N] . W [N, Kin]
    for name, n, kin in (("dgrad.o", H, o), ("dgrad.qkv", q, H), ("dgrad.gate_up", i2, H), ("dgrad.down", H, i1)):
        dy, w = r(T, n), r(n, kin)
        dx = torch.empty(T, kin, dtype=BF, device="cuda")
        v = [("prod", lambda: K.linear_dgrad(dy, [w])),
             ("t15", lambda: K.linear_dgrad(dy, [w], tile=15)),
             ("t2", lambda: K.linear_dgrad(dy, [w], tile=2))]
        for s in (2, 4, 8):
            if n % (s * 64) == 0:
                v.append((f"t15ks{s}", lambda s=s: K._gemm_ksplit(dy, dy.stride(0), 1, [w], [kin], [0, n], 0, 1, dx, T,
                                                                  kin, n, s, 15, K.EPI_BF16)))
        report(name, 2.0 * T * n * kin, v)
    # weight gradients, as the layer groups them: q|k|v + o_proj in one launch, gate|up, down
    groups = {"wgrad.qkv+o": [(q, H), (H, o)], "wgrad.gate_up": [(i2, H)], "wgrad.down": [(H, i1)]}
    for name, shapes in groups.items():
        jobs = [(r(T, n), r(T, kin), [torch.zeros(n, kin, dtype=BF, device="cuda")]) for n, kin in shapes]
        flop = sum(2.0 * T * n * kin for n, kin in shapes)
        v = [("prod", lambda: K.linear_wgrad_grouped(jobs, epilogue=K.EPI_BF16)),
             ("t15", lambda: K.linear_wgrad_grouped(jobs, epilogue=K.EPI_BF16, tile=15)),
             ("t2", lambda: K.linear_wgrad_grouped(jobs, epilogue=K.EPI_BF16, tile=2))]
        for s in (2, 4):
            v.append((f"t15ks{s}", lambda s=s: K._wgrad_ksplit_run(jobs, K.EPI_BF16, s, tile=15)))
        report(name, flop, v)
    print(json.dumps({"summary": rows}))


if __name__ == "__main__":
    main()
