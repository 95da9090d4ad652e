"""GEMM microbenchmark on the decoder layer's real shapes (SmolLM-1.7B, T = 4096 tokens).

For each (shape, layout) and each tile id that divides it: TF/s of pt_gemm (HIP events, 20 reps,
random operands), relative error against torch's fp32 matmul, and torch's own bf16 matmul
(hipBLASLt) for reference.  Run on the GPU box:  python tools/gemm_bench.py [--tiles 0,1,2,4,5]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotron_amd import kernels as K  # noqa: E402

T, H, I, V = 4096, 2048, 8192, 49152
SHAPES = [
    # name, M, N, K, a_kcontig, b_kcontig
    ("fwd.qkv", T, 3 * H, H, 1, 1), ("fwd.o", T, H, H, 1, 1), ("fwd.gate_up", T, 2 * I, H, 1, 1),
    ("fwd.down", T, H, I, 1, 1), ("fwd.lm_head", T, V, H, 1, 1),
    ("dgrad.o", T, H, H, 1, 0), ("dgrad.qkv", T, H, 3 * H, 1, 0), ("dgrad.gate_up", T, H, 2 * I, 1, 0),
    ("dgrad.down", T, I, H, 1, 0), ("dgrad.lm_head", T, H, V, 1, 0),
    ("wgrad.o", H, H, T, 0, 0), ("wgrad.qkv", 3 * H, H, T, 0, 0), ("wgrad.gate_up", 2 * I, H, T, 0, 0),
    ("wgrad.down", H, I, T, 0, 0), ("wgrad.lm_head", V, H, T, 0, 0),
]
def tp_shapes(tp):
    """The TP shard shapes of the same layer (ColumnParallel q|k|v, gate|up: N / tp; RowParallel o, down:
    K / tp) -- the TP=8 proxy's GEMMs."""
    q, i = 3 * H // tp, I // tp
    return [("tp.fwd.qkv", T, q, H, 1, 1), ("tp.fwd.o", T, H, H // tp, 1, 1), ("tp.fwd.gate_up", T, 2 * i, H, 1, 1),
            ("tp.fwd.down", T, H, i, 1, 1), ("tp.dgrad.o", T, H // tp, H, 1, 0), ("tp.dgrad.qkv", T, H, q, 1, 0),
            ("tp.dgrad.gate_up", T, H, 2 * i, 1, 0), ("tp.dgrad.down", T, i, H, 1, 0),
            ("tp.wgrad.o", H, H // tp, T, 0, 0), ("tp.wgrad.qkv", q, H, T, 0, 0), ("tp.wgrad.gate_up", 2 * i, H, T, 0, 0),
            ("tp.wgrad.down", H, i, T, 0, 0)]


TILES = {0: (256, 256), 1: (256, 128), 2: (128, 128), 3: (64, 64), 4: (256, 256), 5: (256, 128), 6: (256, 256), 7: (256, 128), 8: (256, 256), 9: (128, 128), 10: (256, 256), 11: (256, 256), 12: (256, 256), 13: (256, 128), 14: (256, 128), 15: (128, 128)}


def run(name, M, N, Kd, ak, bk, tile, reps=20):
    dev = "cuda"
    A = (torch.rand(M, Kd, device=dev) * 2 - 1).to(torch.bfloat16) if ak else \
        (torch.rand(Kd, M, device=dev) * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N, Kd, device=dev) * 2 - 1).to(torch.bfloat16) if bk else \
        (torch.rand(Kd, N, device=dev) * 2 - 1).to(torch.bfloat16)
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)

    def call():
        K._gemm(A, A.stride(0), ak, [B], [B.stride(0)], [0, N if True else Kd], bk, 0, [C], [N], [0, M], M, N, Kd,
                K.EPI_BF16, tile)
    call()
    torch.cuda.synchronize()
    ref = (A.float() if ak else A.float().t()) @ (B.float().t() if bk else B.float())
    err = ((C.float() - ref).norm() / ref.norm()).item()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        call()
    e0.record()
    for _ in range(reps):
        call()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return 2.0 * M * N * Kd / (ms * 1e-3) / 1e12, err, ms


def torch_ref(M, N, Kd, ak, bk, reps=20):
    a = (torch.rand(M, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(Kd, N, device="cuda") * 2 - 1).to(torch.bfloat16)
    for _ in range(3):
        torch.matmul(a, b)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        torch.matmul(a, b)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return 2.0 * M * N * Kd / (ms * 1e-3) / 1e12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="0,1,2,4,5")
    ap.add_argument("--only", default="")
    ap.add_argument("--lib", default="", help="load this libpicotron_hip.so instead (A/B runs)")
    ap.add_argument("--brief", action="store_true", help="one short line per shape")
    ap.add_argument("--tp", type=int, default=0, help="the TP shard shapes at this degree instead")
    args = ap.parse_args()
    global SHAPES
    if args.tp:
        SHAPES = tp_shapes(args.tp)
    if args.lib:
        K._C.use_library(os.path.abspath(args.lib))
    tiles = [int(t) for t in args.tiles.split(",")]
    out = []
    for name, M, N, Kd, ak, bk in SHAPES:
        if args.only and args.only not in name:
            continue
        row = {"shape": name, "M": M, "N": N, "K": Kd, "torch_tflops": round(torch_ref(M, N, Kd, ak, bk), 1),
               "auto_tile": K._C.lib().pt_gemm_pick_tile(M, N, None, 0, None, 0)}
        for t in tiles:
            bm, bn = TILES[t]
            if M % bm or N % bn:
                continue
            tf, err, ms = run(name, M, N, Kd, ak, bk, t)
            row[f"tile{t}"] = round(tf, 1)
            row[f"err{t}"] = float(f"{err:.2e}")
        if args.brief:
            print(name, " ".join(f"t{t}={row.get(f'tile{t}')}" for t in tiles), flush=True)
        else:
            print(json.dumps(row), flush=True)
        out.append(row)




def one(shape, tile, reps):
    """Launch a single (shape, tile) `reps` times -- for rocprofv3 --pmc passes."""
    if shape in ("swiglu_bwd", "swiglu_fwd"):   # the epilogue-fused MLP GEMMs at the layer's shape
        x = (torch.rand(T, H, device="cuda") * 2 - 1).to(torch.bfloat16)
        wd = (torch.rand(H, I, device="cuda") * 0.02).to(torch.bfloat16)
        wg = (torch.rand(I, H, device="cuda") * 0.02).to(torch.bfloat16)
        wu = (torch.rand(I, H, device="cuda") * 0.02).to(torch.bfloat16)
        gu, _ = K.linear_swiglu_fwd(x, wg, wu)
        fn = (lambda: K.linear_dgrad_swiglu(x, wd, gu)) if shape == "swiglu_bwd" else (lambda: K.linear_swiglu_fwd(x, wg, wu))
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(json.dumps({"shape": shape, "us": round(ms * 1e3, 1), "tflops": round(2.0 * T * 2 * I * H / ms / 1e9 / (2 if shape == "swiglu_bwd" else 1), 1)}))
        return
    for name, M, N, Kd, ak, bk in SHAPES:
        if name == shape:
            tf, err, ms = run(name, M, N, Kd, ak, bk, tile, reps=reps)
            print(json.dumps({"shape": name, "tile": tile, "tflops": round(tf, 1), "err": err}))


if __name__ == "__main__":
    if os.environ.get("PT_LIB"):   # A/B: load another build of the library (before any launch)
        K._C.use_library(os.path.abspath(os.environ["PT_LIB"]))
    if len(sys.argv) > 1 and sys.argv[1] == "one":
        one(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]) if len(sys.argv) > 4 else 5)
    else:
        main()
