"""RMSNorm fwd / fwd+residual / bwd (+ fused residual grad, f32 dweight sink) at the decoder layer's
shape (T 4096, H 2048): us per call from a HIP graph of `reps` back-to-back calls (no host gaps) and
the achieved HBM rate on algorithmic bytes (fwd 4 B/elem, fwd+res 8, bwd+dres 8).

    python tools/norm_bench.py [--rows 4096 --cols 2048] [--old lib.so]

--old: a library holding another build of the pt_rmsnorm_* entry points, timed in the same process.
bwd_split: the backward fed by a split-K dX's two f32 halves (pt_rmsnorm_bwd_splitk, 16 B/elem).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotron_amd import _C  # noqa: E402
from picotron_amd import kernels as K  # noqa: E402


def graph_us(fn, reps=20, rounds=3):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best.append(e0.elapsed_time(e1) / reps * 1e3)
    return min(best)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=4096)
    ap.add_argument("--cols", type=int, default=2048)
    ap.add_argument("--old", default="")
    a = ap.parse_args()
    R, C = a.rows, a.cols
    bf = torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(0)
    x, r, dy, dres = (torch.randn(R, C, device="cuda", generator=g).to(bf) for _ in range(4))
    w = (1 + 0.1 * torch.randn(C, device="cuda", generator=g)).to(bf)
    mg = torch.zeros(C, device="cuda", dtype=torch.float32)
    p0, p1 = (torch.randn(R, C, device="cuda", generator=g) for _ in range(2))
    n = R * C

    def measure(tag):
        y, rstd, z = K.rmsnorm_fwd(x, w, 1e-5, 0, residual=r)
        mg.zero_()
        dx, _ = K.rmsnorm_bwd(dy, z, w, rstd, 0, dres=dres, dw_out=mg, dw_sink=K.DW_ACC_F32)
        ref = (y.clone(), z.clone(), dx.clone(), mg.clone())
        t_f = graph_us(lambda: K.rmsnorm_fwd(x, w, 1e-5, 0))
        t_r = graph_us(lambda: K.rmsnorm_fwd(x, w, 1e-5, 0, residual=r))
        t_b = graph_us(lambda: K.rmsnorm_bwd(dy, z, w, rstd, 0, dres=dres, dw_out=mg, dw_sink=K.DW_ACC_F32))
        sp = K.SplitKParts(p0, p1)
        t_s = graph_us(lambda: K.rmsnorm_bwd(sp, z, w, rstd, 0, dres=dres, dw_out=mg, dw_sink=K.DW_ACC_F32))
        row = {"cfg": tag, "fwd_us": round(t_f, 2), "fwd_TBps": round(4 * n / t_f / 1e6, 2),
               "fwdres_us": round(t_r, 2), "fwdres_TBps": round(8 * n / t_r / 1e6, 2),
               "bwd_us": round(t_b, 2), "bwd_TBps": round(8 * n / t_b / 1e6, 2),
               "bwd_split_us": round(t_s, 2), "bwd_split_TBps": round(14 * n / t_s / 1e6, 2)}
        print(json.dumps(row), flush=True)
        return ref

    refs = {}
    libs = {"new": _C.load_library()}
    if a.old:
        libs["old"] = _C.load_library(os.path.abspath(a.old), strict=False)
    for rnd in range(3):
        for name, lib in (list(libs.items())[::-1] if rnd % 2 else libs.items()):
            _C._lib = lib
            refs[name] = measure(f"{name}:r{rnd}")
    _C._lib = libs["new"]
    if "old" in libs:
        o = refs["old"]
        for k, v in refs.items():
            d = [(p.float() - q.float()).abs().max().item() for p, q in zip(v, o)]
            print(json.dumps({"vs_old": k, "max_abs_diff_y_z_dx_dw": d}), flush=True)


if __name__ == "__main__":
    main()
