"""Does the GEMM's speed depend on cache state?  (in-situ dgrad GEMMs run at 0.70-0.80 of the
microbench's rate, the forward / wgrad ones at 0.92-0.99.)  Times one shape with operands drawn
from different distributions: uniform [-1, 1] (the microbench), N(0, 0.02) (initialised weights),
N(0, 1e-4) (gradient-like), zeros.  Run on the GPU box: python tools/gemm_data.py [shape] [tile]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.gemm_bench import SHAPES  # noqa: E402
from picotron_amd import kernels as K  # noqa: E402


def gen(kind, shape):
    if kind == "unif":
        return (torch.rand(*shape, device="cuda") * 2 - 1).to(torch.bfloat16)
    if kind == "w002":
        return (torch.randn(*shape, device="cuda") * 0.02).to(torch.bfloat16)
    if kind == "g1e-4":
        return (torch.randn(*shape, device="cuda") * 1e-4).to(torch.bfloat16)
    if kind == "zero":
        return torch.zeros(*shape, device="cuda", dtype=torch.bfloat16)
    if kind == "ones":
        return torch.ones(*shape, device="cuda", dtype=torch.bfloat16)
    raise ValueError(kind)


_SCRATCH = []


def time_it(A, ak, B, bk, C, M, N, Kd, tile, reps=20, cold=False):
    def call():
        K._gemm(A, A.stride(0), ak, [B], [B.stride(0)], [0, N], bk, 0, [C], [N], [0, M], M, N, Kd, K.EPI_BF16, tile)
    for _ in range(3):
        call()
    if cold:  # evict L2 / MALL before every launch, time each launch alone
        if not _SCRATCH:
            _SCRATCH.append(torch.empty(1 << 30, dtype=torch.uint8, device="cuda"))
        tot = 0.0
        for _ in range(reps):
            _SCRATCH[0].fill_(1)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            call()
            e1.record()
            torch.cuda.synchronize()
            tot += e0.elapsed_time(e1)
        return 2.0 * M * N * Kd / (tot / reps * 1e-3) / 1e12
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        call()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return 2.0 * M * N * Kd / (ms * 1e-3) / 1e12


def main():
    shapes = sys.argv[1].split(",") if len(sys.argv) > 1 else ["dgrad.gate_up", "fwd.down", "wgrad.down"]
    tile = int(sys.argv[2]) if len(sys.argv) > 2 else -1
    for name, M, N, Kd, ak, bk in SHAPES:
        if name not in shapes:
            continue
        ashape = (M, Kd) if ak else (Kd, M)
        bshape = (N, Kd) if bk else (Kd, N)
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        A, B = gen("unif", ashape), gen("unif", bshape)
        for cold in (False, True, False, True):
            tf = time_it(A, ak, B, bk, C, M, N, Kd, tile, cold=cold)
            print(f"{name:14s} {'cold' if cold else 'warm'} {tf:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
