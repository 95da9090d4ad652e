"""Per-round fixed cost of the phased GEMMs: one round of tiles (256 workgroups) at K = 1024 ... 16384,
graph-timed; the intercept of time vs K is the prologue + epilogue + dispatch cost of a tile.

    python tools/gemm_kscan.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotron_amd import kernels as K  # noqa: E402
from tools.attn_bench import graph_us  # noqa: E402


def main():
    dev = "cuda"
    for tile, (M, N) in ((12, (4096, 4096)), (13, (4096, 2048))):
        for ak, bk, epi in ((1, 1, 0), (1, 0, 0), (0, 0, 1)):
            pts = []
            for Kd in (1024, 2048, 4096, 8192, 16384):
                A = (torch.rand(M, Kd, device=dev) - 0.5).to(torch.bfloat16) if ak else (torch.rand(Kd, M, device=dev) - 0.5).to(torch.bfloat16)
                B = (torch.rand(N, Kd, device=dev) - 0.5).to(torch.bfloat16) if bk else (torch.rand(Kd, N, device=dev) - 0.5).to(torch.bfloat16)
                C = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
                fn = lambda: K._gemm(A, A.stride(0), ak, [B], [B.stride(0)], [0, N], bk, 0, [C], [N], [0, M], M, N, Kd, epi, tile)
                us = graph_us(fn, 10)
                pts.append((Kd, us))
            n = len(pts)
            mx = sum(k for k, _ in pts) / n
            my = sum(t for _, t in pts) / n
            slope = sum((k - mx) * (t - my) for k, t in pts) / sum((k - mx) ** 2 for k, _ in pts)
            icpt = my - slope * mx
            print(json.dumps({"tile": tile, "M": M, "N": N, "a_k": ak, "b_k": bk, "epi": epi,
                              "us": {k: round(t, 1) for k, t in pts}, "us_per_1k_K": round(slope * 1024, 2),
                              "intercept_us": round(icpt, 2),
                              "tflops_at_16k": round(2 * M * N * 16384 / pts[-1][1] / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
