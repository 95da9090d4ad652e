"""Multi-tensor AdamW over the SmolLM-1.7B parameter set (1.21 B bf16 parameters, the model's tensor
sizes): us per step (graph-timed) and HBM rate on 14 B per parameter; --old: another build's
pt_adamw_step_multi in the same process; --calib: beside it torch's fused AdamW on the same tensors and
the HBM rate of torch's copy (1 read : 1 write) and add (2 : 1) over the same bytes, which bracket
AdamW's 8 : 6 mix.  python tools/adamw_bench.py [--old lib.so] [--calib]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotron_amd import _C  # noqa: E402
from picotron_amd import kernels as K  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from attn_bench import graph_us  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--old", default="")
    ap.add_argument("--calib", action="store_true")
    a = ap.parse_args()
    H, I, V, L = 2048, 8192, 49152, 15
    shapes = [(V, H)] + [s for _ in range(L) for s in ((H,), (H, H), (H, H), (H, H), (H, H), (I, H), (I, H), (H, I), (H,))] + [(H,)]
    items = []
    n = 0
    for sh in shapes:
        p = torch.randn(*sh, device="cuda").to(torch.bfloat16)
        items.append((p, torch.randn_like(p) * 1e-3, torch.zeros_like(p), torch.zeros_like(p)))
        n += p.numel()
    args = (0.999 * 3e-4, 0.1, 0.999, 0.001, 0.03, 1e-8, 3e-4)
    libs = {"new": _C.load_library()}
    if a.old:
        libs["old"] = _C.load_library(os.path.abspath(a.old), strict=False)
    for rnd in range(2):
        for name, lib in libs.items():
            _C._lib = lib
            K._ADAM_DESC.clear() if hasattr(K, "_ADAM_DESC") else None
            us = graph_us(lambda: K.adamw_step_multi(items, *args), 3)
            print(json.dumps({"lib": f"{name}:r{rnd}", "params": n, "us": round(us, 1), "TBps": round(14 * n / us / 1e6, 2)}),
                  flush=True)
    if a.calib:
        calib(items, n, args)


def calib(items, n, args):
    ps, gs, ms, vs = (list(t) for t in zip(*items))
    lr, wd, b1, b2, eps = args[6], 0.1, 0.9, args[2], args[5]
    step = torch.tensor(3.0, device="cuda")
    us = graph_us(lambda: torch._fused_adamw_(ps, gs, ms, vs, [], [step] * len(ps), lr=lr, beta1=b1, beta2=b2,
                                              weight_decay=wd, eps=eps, amsgrad=False, maximize=False), 3)
    print(json.dumps({"lib": "torch._fused_adamw_", "params": n, "us": round(us, 1), "TBps": round(14 * n / us / 1e6, 2)}),
          flush=True)
    hot_cold(items, args)
    x = torch.empty(n, dtype=torch.bfloat16, device="cuda").normal_()
    y, z = torch.empty_like(x), torch.empty_like(x)
    us = graph_us(lambda: y.copy_(x), 3)
    print(json.dumps({"probe": "copy 1r:1w", "bytes": 4 * n, "us": round(us, 1), "TBps": round(4 * n / us / 1e6, 2)}), flush=True)
    us = graph_us(lambda: torch.add(x, y, out=z), 3)
    print(json.dumps({"probe": "add 2r:1w", "bytes": 6 * n, "us": round(us, 1), "TBps": round(6 * n / us / 1e6, 2)}), flush=True)
    us = graph_us(lambda: x.sum(), 3)
    print(json.dumps({"probe": "sum 1r", "bytes": 2 * n, "us": round(us, 1), "TBps": round(2 * n / us / 1e6, 2)}), flush=True)


def hot_cold(items, args):
    """One AdamW launch right after ~0.8 s of back-to-back bf16 GEMMs (the chip as the training step
    leaves it) vs after 0.5 s idle: the in-situ kernel table's launch is ~25 % slower than the graph loop."""
    import time
    fn = lambda: K.adamw_step_multi(items, *args)  # noqa: E731
    fn()
    torch.cuda.synchronize()
    A = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    C = torch.empty_like(A)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for rnd in range(3):
        for mode in ("idle", "hot"):
            torch.cuda.synchronize()
            if mode == "idle":
                time.sleep(0.5)
            else:
                for _ in range(900):
                    torch.mm(A, A, out=C)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            print(json.dumps({"adamw_after": mode, "round": rnd, "us": round(e0.elapsed_time(e1) * 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
