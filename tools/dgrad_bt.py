"""dX GEMM layouts at the layer's N = 2048 shapes: B = W [K, N] N-contiguous (as stored, the dX
GEMM today) vs B = W^T [N, K] K-contiguous (a transposed weight copy), 256x128 4-phase kernel,
graph-timed.  python tools/dgrad_bt.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotron_amd import kernels as K  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from attn_bench import graph_us  # noqa: E402


def main():
    M, N = 4096, 2048
    for Kd in (2048, 6144, 16384, 49152):
        dy = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
        w = (torch.randn(Kd, N, device="cuda") * 0.02).to(torch.bfloat16)   # [K, N]: out x in
        wt = w.t().contiguous()                                             # [N, K]
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        c2 = torch.empty_like(c)
        f_nc = lambda: K._gemm(dy, Kd, 1, [w], [N], [0, N], 0, 0, [c], [N], [0, M], M, N, Kd, K.EPI_BF16, 13)
        f_kc = lambda: K._gemm(dy, Kd, 1, [wt], [Kd], [0, N], 1, 0, [c2], [N], [0, M], M, N, Kd, K.EPI_BF16, 13)
        t_tr = graph_us(lambda: wt.copy_(w.t()), 10)
        res = {"K": Kd}
        for rnd in range(2):
            res[f"nc_us_{rnd}"] = round(graph_us(f_nc, 10), 1)
            res[f"kc_us_{rnd}"] = round(graph_us(f_kc, 10), 1)
        res["transpose_copy_us"] = round(t_tr, 1)
        res["equal"] = bool(torch.equal(c, c2))
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
