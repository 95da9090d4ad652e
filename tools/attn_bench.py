"""Attention microbenchmark at the decoder layer's shape (SmolLM-1.7B: B 4, S 1024, 32 heads, d 64,
causal), q/k/v as strided views of one fused [T, 3 H d] projection like the model.  Prints us per
call from a HIP graph of `reps` back-to-back calls (no host gaps between launches) and TF/s (causal
FLOP: fwd 2 GEMMs, bwd 5 = the algorithm's, bwd_kernel 7 = what the dK/dV (4) + dQ (3) kernels run;
each 2 B h S^2 d / 2).

    python tools/attn_bench.py [--reps 20] [--B 4 --S 1024 --H 32 --D 64] [--old lib.so]

--old: libraries (comma-separated) holding other builds of the pt_attn_* entry points, timed in the
same process (rounds interleaved, first one rotated) and compared element-wise with this build's outputs.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotron_amd import _C  # noqa: E402
from picotron_amd import kernels as K  # noqa: E402


def graph_us(fn, reps, rounds=3):
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
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--B", type=int, default=4)
    ap.add_argument("--S", type=int, default=1024)
    ap.add_argument("--H", type=int, default=32)
    ap.add_argument("--D", type=int, default=64)
    ap.add_argument("--old", default="")
    ap.add_argument("--model-path", action="store_true",
                    help="causal: time the backward as the layer calls it (delta inside, no precomputed delta)")
    ap.add_argument("--variant", default="",
                    help="NAME=V1,V2,...: time the new library once per value of this native variant "
                         "(pt_set_variant; e.g. attn_pair=1,0), compared like --old builds")
    ap.add_argument("--full", action="store_true",
                    help="the CP ring's visiting block: no causal mask, f32 dq/dk/dv accumulators (grad_f32)")
    ap.add_argument("--rounds", type=int, default=2, help="interleaved rounds; medians are printed at the end")
    a = ap.parse_args()
    B, S, H, D = a.B, a.S, a.H, a.D
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(B, S, 3, H, D, device="cuda", generator=g).to(torch.bfloat16)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    do = torch.randn(B, S, H, D, device="cuda", generator=g).to(torch.bfloat16)
    scale = D ** -0.5
    causal = not a.full
    unit = 2.0 * B * H * S * S * D / (2 if causal else 1)
    if a.full:
        acc = [torch.zeros(B, S, H, D, device="cuda") for _ in range(3)]
    libs = {"new": _C.load_library()}
    for i, path in enumerate(x for x in a.old.split(",") if x):   # comma-separated: old, old1, old2 ...
        libs["old" if i == 0 else f"old{i}"] = _C.load_library(os.path.abspath(path), strict=False)
    variants = {name: {} for name in libs}
    if a.variant:   # the new library once per value: arm "new" = the first value, "<var>=<v>" the others
        var, vals = a.variant.split("=")
        vals = [int(x) for x in vals.split(",")]
        variants["new"] = {var: vals[0]}
        for val in vals[1:]:
            libs[f"{var}={val}"] = libs["new"]
            variants[f"{var}={val}"] = {var: val}
    defaults = {}
    outs = {}
    split_ws = K._attn_split_ws
    med = {name: {"fwd": [], "bwd": []} for name in libs}
    for rnd in range(a.rounds):
        order = list(libs.items())
        order = order[rnd % len(order):] + order[:rnd % len(order)]   # rotate who goes first
        for name, lib in order:
            _C._lib = lib
            # builds from before the few-head split forms lack pt_attn_split_plan: the unsplit kernels
            K._attn_split_ws = split_ws if hasattr(lib, "pt_attn_split_plan") else (lambda *args: None)
            for var, val in variants[name].items():
                if var not in defaults:
                    defaults[var] = lib.pt_get_variant(var.encode())
                lib.pt_set_variant(var.encode(), int(val))
            o, lse = K.attn_fwd(q, k, v, scale, causal)
            delta = K.attn_delta(do, o)
            if a.full:
                for t in acc:
                    t.zero_()
                K.attn_bwd(do, q, k, v, o, lse, scale, False, dq=acc[0], dk=acc[1], dv=acc[2], grad_f32=True,
                           delta=delta)
                dq, dk, dv = acc

                def bwd():
                    K.attn_bwd(do, q, k, v, o, lse, scale, False, dq=acc[0], dk=acc[1], dv=acc[2], grad_f32=True,
                               delta=delta)
            else:
                dl = None if a.model_path else delta
                dq, dk, dv, _ = K.attn_bwd(do, q, k, v, o, lse, scale, True, delta=dl)

                def bwd():
                    K.attn_bwd(do, q, k, v, o, lse, scale, True, delta=dl)
            outs[name] = [t.clone() for t in (o, lse, dq, dk, dv)]
            t_fwd = graph_us(lambda: K.attn_fwd(q, k, v, scale, causal, out=o, lse=lse), a.reps)
            t_bwd = graph_us(bwd, a.reps)
            for var, val in defaults.items():
                lib.pt_set_variant(var.encode(), int(val))
            med[name]["fwd"].append(t_fwd)
            med[name]["bwd"].append(t_bwd)
            print(json.dumps({"lib": f"{name}:r{rnd}", "B": B, "S": S, "H": H, "D": D, "causal": causal,
                              "fwd_us": round(t_fwd, 1), "fwd_tflops": round(2 * unit / t_fwd / 1e6, 1),
                              "bwd_us": round(t_bwd, 1), "bwd_tflops": round(5 * unit / t_bwd / 1e6, 1),
                              "bwd_kernel_flop_tflops": round(7 * unit / t_bwd / 1e6, 1)}), flush=True)
    _C._lib = libs["new"]
    K._attn_split_ws = split_ws
    for name, m in med.items():
        f, b = sorted(m["fwd"])[len(m["fwd"]) // 2], sorted(m["bwd"])[len(m["bwd"]) // 2]
        print(json.dumps({"median": name, "fwd_us": round(f, 1), "bwd_us": round(b, 1)}), flush=True)
    for name in outs:
        if name == "new":
            continue
        rel = [((x.float() - y.float()).norm() / y.float().norm()).item() for x, y in zip(outs["new"], outs[name])]
        print(json.dumps({f"new_vs_{name}_rel_o_lse_dq_dk_dv": rel}), flush=True)


if __name__ == "__main__":
    main()
