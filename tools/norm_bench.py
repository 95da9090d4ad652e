"""RMSNorm fwd (+ fused residual) / bwd (+ fused residual grad, dweight sink) microbenchmark at the
decoder layer's shape (T 4096, H 2048): us per call and achieved HBM GB/s (algorithmic bytes).

    python tools/norm_bench.py [--rows 4096 --cols 2048] [--lib path/to/libpicotron_hip.so]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotron_amd import kernels as K  # noqa: E402


def timeit(fn, reps=50):
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
    ap.add_argument("--rows", type=int, default=4096)
    ap.add_argument("--cols", type=int, default=2048)
    ap.add_argument("--lib", default="")
    a = ap.parse_args()
    if a.lib:
        K._C.load_library(os.path.abspath(a.lib))
    R, C = a.rows, a.cols
    bf = torch.bfloat16
    x, r, dy, dres = (torch.randn(R, C, device="cuda").to(bf) for _ in range(4))
    w = torch.ones(C, device="cuda", dtype=bf)
    y, rstd, z = K.rmsnorm_fwd(x, w, 1e-5, 0, residual=r)
    grad = torch.zeros(C, device="cuda", dtype=bf)
    t_f = timeit(lambda: K.rmsnorm_fwd(x, w, 1e-5, 0, residual=r))
    t_b = timeit(lambda: K.rmsnorm_bwd(dy, z, w, rstd, 0, dres=dres, dw_out=grad, dw_sink=K.DW_ACC_BF16))
    n = R * C
    print(json.dumps({"lib": a.lib or "in-tree", "rows": R, "cols": C, "fwd_us": round(t_f, 1),
                      "fwd_GBps": round(8 * n / t_f / 1e3, 1), "bwd_us": round(t_b, 1),
                      "bwd_GBps": round(8 * n / t_b / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
