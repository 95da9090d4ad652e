"""Diagnostic: per-step timeline of the dK/dV wave-pair kernel from a -DPT_STAMP build
(python -m picotron_amd.build --out tools/ab/diag_stamp.so -DPT_STAMP).  Workgroups 0-7 record, per
wave and step, s_memtime at the step's start and at its arrival at the end-of-step wait; printed:
per role the median work and wait cycles per step."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotron_amd import _C  # noqa: E402
from picotron_amd import kernels as K  # noqa: E402

STEPS = 136


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--B", type=int, default=1)
    ap.add_argument("--S", type=int, default=4096)
    ap.add_argument("--H", type=int, default=32)
    ap.add_argument("--D", type=int, default=128)
    a = ap.parse_args()
    _C.use_library(a.lib)
    B, S, H, D = a.B, a.S, a.H, a.D
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(B, S, 3, H, D, device="cuda", generator=g).to(torch.bfloat16)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    do = torch.randn(B, S, H, D, device="cuda", generator=g).to(torch.bfloat16)
    o, lse = K.attn_fwd(q, k, v, D ** -0.5, False)
    delta = K.attn_delta(do, o)
    acc = [torch.zeros(B, S, H, D, device="cuda") for _ in range(3)]
    st = torch.zeros(8, 8, STEPS, 2, dtype=torch.int64, device="cuda")
    os.environ["PICOTRON_ATTN_STAMPS"] = str(st.data_ptr())
    os.environ["PICOTRON_ATTN_SPLIT"] = "3"
    for _ in range(3):
        K.attn_bwd(do, q, k, v, o, lse, D ** -0.5, False, dq=acc[0], dk=acc[1], dv=acc[2], grad_f32=True, delta=delta)
    torch.cuda.synchronize()
    t = st.cpu()
    nsteps = S // 64 * 2 + 1
    for role, waves in (("score", range(0, 4)), ("accum", range(4, 8))):
        work, wait = [], []
        for wg in range(8):
            for w in waves:
                for j in range(1, min(nsteps, STEPS) - 1):
                    s0, arr, s1 = t[wg, w, j, 0].item(), t[wg, w, j, 1].item(), t[wg, w, j + 1, 0].item()
                    work.append(arr - s0)
                    wait.append(s1 - arr)
        work.sort(), wait.sort()
        med = lambda x: x[len(x) // 2]
        print(f"{role}: work median {med(work)} p90 {work[int(len(work) * .9)]}  wait median {med(wait)} "
              f"p90 {wait[int(len(wait) * .9)]} (cycles per step)")
    odd = [t[0, 0, j + 1, 0].item() - t[0, 0, j, 0].item() for j in range(1, nsteps - 2, 2)]
    even = [t[0, 0, j + 1, 0].item() - t[0, 0, j, 0].item() for j in range(2, nsteps - 2, 2)]
    odd.sort(), even.sort()
    print("step length wg0 wave0: odd (issue + wait) median", odd[len(odd) // 2], " even median", even[len(even) // 2])


if __name__ == "__main__":
    main()
