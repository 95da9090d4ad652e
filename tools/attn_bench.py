"""Attention microbenchmark at the decoder layer's shape (SmolLM-1.7B: B 4, S 1024, 32 heads, d 64,
causal), q/k/v as strided views of one fused [T, 3 H d] projection like the model.  Prints us and
TF/s (causal FLOP: fwd 2 GEMMs, bwd dK/dV kernel 4, dQ kernel 3, each 2 B h S^2 d / 2).

    python tools/attn_bench.py [--reps 20] [--B 4 --S 1024 --H 32 --D 64]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotron_amd import kernels as K  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--B", type=int, default=4)
    ap.add_argument("--S", type=int, default=1024)
    ap.add_argument("--H", type=int, default=32)
    ap.add_argument("--D", type=int, default=64)
    ap.add_argument("--lib", default="", help="load this libpicotron_hip.so instead (A/B runs)")
    a = ap.parse_args()
    if a.lib:
        K._C.load_library(os.path.abspath(a.lib))
    B, S, H, D = a.B, a.S, a.H, a.D
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(B, S, 3, H, D, device="cuda", generator=g).to(torch.bfloat16)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    do = torch.randn(B, S, H, D, device="cuda", generator=g).to(torch.bfloat16)
    scale = D ** -0.5
    o, lse = K.attn_fwd(q, k, v, scale, True)
    delta = K.attn_delta(do, o)
    unit = 2.0 * B * H * S * S * D / 2
    t_fwd = timeit(lambda: K.attn_fwd(q, k, v, scale, True, out=o, lse=lse), a.reps)
    t_delta = timeit(lambda: K.attn_delta(do, o), a.reps)
    t_bwd = timeit(lambda: K.attn_bwd(do, q, k, v, o, lse, scale, True, delta=delta), a.reps)
    print(json.dumps({"lib": a.lib or "in-tree", "B": B, "S": S, "H": H, "D": D,
                      "fwd_us": round(t_fwd, 1), "fwd_tflops": round(2 * unit / t_fwd / 1e6, 1),
                      "delta_us": round(t_delta, 1),
                      "bwd_us": round(t_bwd, 1), "bwd_tflops": round(5 * unit / t_bwd / 1e6, 1),
                      "bwd_kernel_flop_tflops": round(7 * unit / t_bwd / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
