"""MLP-backward GEMM launches at SmolLM-1.7B shapes (T 4096, H 2048, I 8192), graph-timed, for A/B
of builds (--old lib.so[,lib2.so]: the same entry points from another build, rounds interleaved):
the down_proj dX with the SwiGLU backward epilogue, the down_proj dW (bf16 / f32 accumulate
sinks), both in one dual launch (each dispatch order), and the gate|up dX / dW (separate / dual).

    python tools/epi_bench.py [--reps 10] [--rounds 3] [--old tools/ab/old.so]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotron_amd import _C  # noqa: E402
from picotron_amd import kernels as K  # noqa: E402
from tools.attn_bench import graph_us  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--old", default="")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    T, H, I = 4096, 2048, 8192
    g = torch.Generator(device="cuda").manual_seed(0)

    def r(*s, scale=1.0):
        return (torch.randn(*s, device="cuda", generator=g) * scale).to(torch.bfloat16)
    dm, h2 = r(T, H), r(T, H)
    wd = r(H, I, scale=I ** -0.5)
    wg, wu = r(I, H, scale=H ** -0.5), r(I, H, scale=H ** -0.5)
    gu, hh, dgu = r(T, 2 * I), r(T, I), r(T, 2 * I)
    gb = torch.zeros(H, I, device="cuda", dtype=torch.bfloat16)
    gf = torch.zeros(H, I, device="cuda", dtype=torch.float32)
    gg, gu_ = torch.zeros(I, H, device="cuda", dtype=torch.bfloat16), torch.zeros(I, H, device="cuda", dtype=torch.bfloat16)
    gg32, gu32 = torch.zeros(I, H, device="cuda"), torch.zeros(I, H, device="cuda")
    flop = {"down": 2.0 * T * H * I, "gu": 2.0 * T * H * 2 * I}
    cases = {
        "swiglu_bwd": (lambda: K.linear_dgrad_swiglu(dm, wd, gu), flop["down"]),
        "wgrad_down_bf16acc": (lambda: K.linear_wgrad(dm, hh, [gb], epilogue=1), flop["down"]),
        "wgrad_down_f32acc": (lambda: K.linear_wgrad(dm, hh, [gf], epilogue=3), flop["down"]),
        "dual_down_o0": (lambda: K.linear_dgrad_dual(dm, [wd], [(dm, hh, [gb])], 1, gu=gu, order=0), 2 * flop["down"]),
        "dual_down_o1": (lambda: K.linear_dgrad_dual(dm, [wd], [(dm, hh, [gb])], 1, gu=gu, order=1), 2 * flop["down"]),
        "dual_down_f32_o1": (lambda: K.linear_dgrad_dual(dm, [wd], [(dm, hh, [gf])], 3, gu=gu, order=1), 2 * flop["down"]),
        "dgrad_gu": (lambda: K.linear_dgrad(dgu, [wg, wu]), flop["gu"]),
        "wgrad_gu_bf16acc": (lambda: K.linear_wgrad(dgu, h2, [gg, gu_], epilogue=1), flop["gu"]),
        "wgrad_gu_f32acc": (lambda: K.linear_wgrad(dgu, h2, [gg32, gu32], epilogue=3), flop["gu"]),
        "dual_gu_o1": (lambda: K.linear_dgrad_dual(dgu, [wg, wu], [(dgu, h2, [gg, gu_])], 1, order=1), 2 * flop["gu"]),
    }
    if a.only:
        cases = {k: v for k, v in cases.items() if k in a.only.split(",")}
    libs = {"new": _C.load_library()}
    for i, path in enumerate(x for x in a.old.split(",") if x):
        libs["old" if i == 0 else f"old{i}"] = _C.load_library(os.path.abspath(path), strict=False)
    med = {(n, c): [] for n in libs for c in cases}
    for rnd in range(a.rounds):
        order = list(libs.items())
        order = order[rnd % len(order):] + order[:rnd % len(order)]
        for name, lib in order:
            _C._lib = lib
            for c, (fn, fl) in cases.items():
                us = graph_us(fn, a.reps)
                med[(name, c)].append(us)
                print(json.dumps({"lib": f"{name}:r{rnd}", "case": c, "us": round(us, 1),
                                  "tflops": round(fl / us / 1e6, 1)}), flush=True)
    _C._lib = libs["new"]
    for (name, c), v in med.items():
        m = sorted(v)[len(v) // 2]
        print(json.dumps({"median": name, "case": c, "us": round(m, 1), "tflops": round(cases[c][1] / m / 1e6, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
