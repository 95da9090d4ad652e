"""Multi-tensor AdamW over the SmolLM-1.7B parameter set (1.21 B bf16 parameters, the model's tensor
sizes): us per step (graph-timed) and HBM rate on 14 B per parameter; --old: another build's
pt_adamw_step_multi in the same process.  python tools/adamw_bench.py [--old lib.so]"""
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


if __name__ == "__main__":
    main()
