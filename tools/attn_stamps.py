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

STEPS = 72


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
    st = torch.zeros(8, 8, STEPS, 4, dtype=torch.int64, device="cuda")
    os.environ["PICOTRON_ATTN_STAMPS"] = str(st.data_ptr())
    os.environ["PICOTRON_ATTN_SPLIT"] = "3"
    for _ in range(3):
        K.attn_bwd(do, q, k, v, o, lse, D ** -0.5, False, dq=acc[0], dk=acc[1], dv=acc[2], grad_f32=True, delta=delta)
    torch.cuda.synchronize()
    t = st.cpu()
    nsteps = min(S // 64 * 2 + 1, STEPS)
    import statistics
    for role, waves in (("score", range(0, 4)), ("accum", range(4, 8))):
        ph = {"lds operands": [], "mfma": [], "rest of work": [], "barrier wait": []}
        for wg in range(8):
            for w in waves:
                for j in range(2, nsteps - 2):
                    s0, s1, s2, s3 = (t[wg, w, j, i].item() for i in range(4))
                    nxt = t[wg, w, j + 1, 0].item()
                    if s1 == 0 or s2 == 0:
                        continue
                    ph["lds operands"].append(s1 - s0)
                    ph["mfma"].append(s2 - s1)
                    ph["rest of work"].append(s3 - s2)
                    ph["barrier wait"].append(nxt - s3)
        print(role, {k: int(statistics.median(v)) for k, v in ph.items() if v}, "(median cycles per step)")
    steps = [t[0, 0, j + 1, 0].item() - t[0, 0, j, 0].item() for j in range(2, nsteps - 2)]
    print("step length wg0 wave0 median", int(statistics.median(steps)))


if __name__ == "__main__":
    main()
