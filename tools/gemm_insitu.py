"""In-situ GEMM rates: every pt_gemm launch of a short training run timed with HIP events, grouped
by problem, next to an immediate back-to-back replay of the same launch on the same tensors.

    python tools/gemm_insitu.py [--layers 3] [--grad-acc 4]

Tells apart "this kernel is slow on this shape" (replay slow too) from "the surroundings slow it
down" (cold operands, the producing kernel's dirty lines, clocks).
"""
import argparse
import collections
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--grad-acc", type=int, default=4)
    ap.add_argument("--replay", type=int, default=5)
    ap.add_argument("--variants", action="store_true", help="replay with cloned / random operands")
    args = ap.parse_args()
    os.environ.setdefault("FLASH_ATTEN", "1")
    os.environ["DEVICE"] = "cuda"
    os.environ.setdefault("LOCAL_RANK", "0")
    from picotron_amd import kernels as K
    from picotron_amd.model import Llama
    from picotron_amd.optim import AdamW
    from picotron_amd.process_group_manager import setup_process_group_manager
    from picotron_amd.train import SMOLLM_1_7B, SyntheticMicroBatchDataLoader, make_config, train_step

    setup_process_group_manager(tp_size=1, cp_size=1, pp_size=1, dp_size=1)
    torch.manual_seed(42)
    dev = torch.device("cuda", 0)
    cfg = make_config(SMOLLM_1_7B, 1024, num_hidden_layers=args.layers)
    with torch.device(dev):
        model = Llama(cfg)
    model.to(torch.bfloat16)
    opt = AdamW(model.parameters(), lr=3e-4)
    loader = SyntheticMicroBatchDataLoader(4, 1024, args.grad_acc, cfg.vocab_size, dev, seed=1234)

    orig = K._gemm
    recs = []
    on = [False]

    def timed(*a, **kw):
        if not on[0]:
            return orig(*a, **kw)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        orig(*a, **kw)
        e1.record()
        recs.append((e0, e1, a, kw))

    K._gemm = timed
    for step in range(2):
        on[0] = step == 1
        opt.zero_grad()
        train_step(model, loader, dev)
        opt.step()
    torch.cuda.synchronize()
    on[0] = False

    groups = collections.OrderedDict()
    for e0, e1, a, kw in recs:
        M, N, Kd, epi = a[11], a[12], a[13], a[14]
        key = (M, N, Kd, int(a[2]), int(a[6]), epi, len(a[3]))
        ms = e0.elapsed_time(e1)
        g = groups.setdefault(key, {"ms": [], "args": (a, kw)})
        g["ms"].append(ms)
    print(f"{'M':>6} {'N':>6} {'K':>6} ak bk epi nseg  n  insitu_TF  replay_TF", flush=True)
    for key, g in groups.items():
        M, N, Kd, ak, bk, epi, nseg = key
        fl = 2.0 * M * N * Kd
        ins = fl / (sum(g["ms"]) / len(g["ms"]) * 1e-3) / 1e12
        a, kw = g["args"]
        if True:   # (accumulating epilogues just accumulate again: values do not matter here)
            for _ in range(2):
                orig(*a, **kw)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.replay):
                orig(*a, **kw)
            e1.record()
            torch.cuda.synchronize()
            rep = fl / (e0.elapsed_time(e1) / args.replay * 1e-3) / 1e12
        print(f"{M:6d} {N:6d} {Kd:6d} {ak:2d} {bk:2d} {epi:3d} {nseg:4d} {len(g['ms']):3d} {ins:9.1f} {rep:9.1f}",
              flush=True)
        if args.variants and epi == K.EPI_BF16:
            # the same launch with operands replaced: fresh copies (placement) / fresh random values
            A, Bs = a[0], a[3]

            def rnd(t):
                return ((torch.rand(t.shape, device=t.device) * 2 - 1) * t.float().abs().max()).to(t.dtype)
            vs = {"cloneA": (A.clone(), Bs), "cloneB": (A, [b.clone() for b in Bs]),
                  "cloneAB": (A.clone(), [b.clone() for b in Bs]), "randAB": (rnd(A), [rnd(b) for b in Bs]),
                  "randA": (rnd(A), Bs), "randB": (A, [rnd(b) for b in Bs])}
            out = []
            for name, (A2, B2) in vs.items():
                a2 = (A2,) + a[1:3] + (B2,) + a[4:]
                for _ in range(2):
                    orig(*a2, **kw)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.replay):
                    orig(*a2, **kw)
                e1.record()
                torch.cuda.synchronize()
                out.append(f"{name}={fl / (e0.elapsed_time(e1) / args.replay * 1e-3) / 1e12:.0f}")
            print("      ", " ".join(out), f"A absmax {A.float().abs().max().item():.3g} "
                  f"zeros {(A == 0).float().mean().item():.3f}", flush=True)


if __name__ == "__main__":
    main()
