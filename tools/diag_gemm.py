"""Diagnose GEMM operand layouts with exact structured data (A = I)."""
import sys, os, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotron_amd import kernels as K
dev = "cuda"
M = N = 64; Kd = 64
for tile in (3, 2):
    if tile == 2: M = N = 128; Kd = 128
    eye = torch.eye(M, Kd).to(torch.bfloat16).to(dev)
    kk = torch.arange(Kd).float().view(Kd, 1).expand(Kd, N).contiguous()
    nn = torch.arange(N).float().view(1, N).expand(Kd, N).contiguous()
    for name, B in (("k", kk), ("n", nn)):
        # NN: C = A . B with B stored [K][N] (W = B^T... linear_dgrad takes W [N_out=K][Kin=N])
        Bw = B.to(torch.bfloat16).to(dev)  # [K, N]
        C = K.linear_dgrad(eye, [Bw], tile=tile)
        exp = eye.float() @ B.to(dev)
        bad = (C.float() != exp)
        print(f"tile {tile} NN B={name}: wrong {bad.sum().item()}/{bad.numel()}")
        if bad.any():
            idx = bad.nonzero()[:6].tolist()
            for m, n in idx:
                print("   m,n", m, n, "got", C[m, n].item(), "exp", exp[m, n].item())
        # TN: dW = dY^T X with dY = I [T=K..] : C[n_out][kin] = sum_t dY[t][n_out] X[t][kin]
        dw = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        K.linear_wgrad(eye.t().contiguous()[:Kd, :M].contiguous(), Bw, [dw], tile=tile)
        exp2 = eye.t().contiguous()[:Kd, :M].float().t() @ B.to(dev)
        bad = (dw.float() != exp2)
        print(f"tile {tile} TN B={name}: wrong {bad.sum().item()}/{bad.numel()}")
        if bad.any():
            for m, n in bad.nonzero()[:6].tolist():
                print("   m,n", m, n, "got", dw[m, n].item(), "exp", exp2[m, n].item())
