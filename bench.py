"""bench.py -- picotron's headline metric on MI355X: training tokens/s (and MFU) of SmolLM-1.7B.

Workload (BASELINE.json configs[1]): SmolLM-1.7B dims (H 2048, I 8192, 32 heads, d 64, V 49152) with
15 decoder layers, micro-batch 4 x seq 1024, grad_acc 32, bf16, random init, synthetic tokens.
One step = train.py:219-240 of the reference: zero_grad, 32 x (forward, fused cross-entropy,
backward), AdamW step (train.py:209's torch.optim.AdamW semantics, fused HIP kernel:
picotron_amd/optim.py) and, for N > 1, the DataParallelBucket
all-reduce of the gradients over RCCL (dp = N, weak scaling: per-GPU work fixed).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
        bench.py --gpus N --steps K --warmup W

Rank 0 prints ONE JSON line.  `value` is whole-job tokens/s (max wall time over ranks);
tokens/s/GPU and MFU (utils.py:42-48 formula, N counted once, 2.5 PF bf16 dense peak) ride along.
`roofline` is the MFMA GEMM (the dominant kernel), timed live with HIP events around every launch
in the timed region; `cpu_baseline` is the oracle (a plain-torch fp32 restatement of the reference
path, oracle/picotron_oracle.py) timed on this host's cores on a bounded sample.
"""
import argparse
import json
import os
import sys
import time
import types

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


# HBM bytes per GEMM launch from rocprofv3 PMC passes (tools/gpu_round.sh <tag> pmc, then
# tools/traffic_summary.py); read for the roofline's `traffic`
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "r01_gemm_traffic.json")


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def cpu_baseline(cfg, tokens):
    """The oracle's fwd+bwd of the full model over one [1, tokens] micro-batch on the host cores."""
    from oracle import picotron_oracle as O
    import torch.nn.functional as F
    c = dict(hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
             num_attention_heads=cfg.num_attention_heads, num_key_value_heads=cfg.num_key_value_heads,
             rms_norm_eps=cfg.rms_norm_eps, vocab_size=cfg.vocab_size, num_hidden_layers=cfg.num_hidden_layers)
    params = O.init_params(c, seed=42)
    for p in params.values():
        p.requires_grad_(True)
    d = cfg.hidden_size // cfg.num_attention_heads
    cos, sin = O.get_cos_sin(tokens, d, base=cfg.rope_theta)
    g = torch.Generator().manual_seed(1234)
    ids = torch.randint(0, cfg.vocab_size, (1, tokens + 1), generator=g)
    t0 = time.perf_counter()
    logits = O.llama_forward(ids[:, :-1], params, c, cos.float(), sin.float(), norm=O.rmsnorm_flash_semantics)
    loss = F.cross_entropy(logits.reshape(-1, cfg.vocab_size), ids[:, 1:].reshape(-1))
    loss.backward()
    dt = time.perf_counter() - t0
    return {"value": tokens / dt, "unit": "tokens/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"oracle fp32 fwd+bwd of the same {cfg.num_hidden_layers}-layer model on one [1, {tokens}] "
                      f"micro-batch ({dt:.1f} s)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--layers", type=int, default=15)
    ap.add_argument("--mbs", type=int, default=4)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--grad-acc", type=int, default=32)
    ap.add_argument("--cpu-tokens", type=int, default=1024, help="tokens in the cpu_baseline sample (0 = skip)")
    ap.add_argument("--no-probe", action="store_true", help="do not time GEMM launches with events")
    ap.add_argument("--dp-bucket", action="store_true",
                    help="N = 1 only: run the DP path anyway (DataParallelBucket, fp32 main_grad, bucket "
                         "all-reduce over a 1-rank RCCL group) -- the per-GPU cost of N > 1 minus the links")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("LOCAL_RANK", str(local_rank))
    os.environ.setdefault("FLASH_ATTEN", "1")
    os.environ["DEVICE"] = "cuda"
    torch.cuda.set_device(local_rank)
    device = torch.device("cuda", local_rank)
    force_dp = args.dp_bucket and world == 1
    if world > 1 or force_dp:
        if force_dp:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group(backend="nccl", init_method="env://", device_id=device)

    from picotron_amd import kernels as K
    from picotron_amd.data_parallel.data_parallel import DataParallelBucket
    from picotron_amd.model import Llama
    from picotron_amd.optim import AdamW
    from picotron_amd.process_group_manager import setup_process_group_manager
    from picotron_amd.train import (SMOLLM_1_7B, SyntheticMicroBatchDataLoader, count_params, flops_per_token,
                                    make_config, train_step, MI355X_BF16_DENSE_PEAK)

    setup_process_group_manager(tp_size=1, cp_size=1, pp_size=1, dp_size=world)
    torch.manual_seed(42)
    cfg = make_config(SMOLLM_1_7B, args.seq, num_hidden_layers=args.layers)
    t0 = time.time()
    with torch.device(device):
        model = Llama(cfg)
    model.to(torch.bfloat16)
    num_params = count_params(model)
    if world > 1 or force_dp:
        model = DataParallelBucket(model)
        model._force_grad_sync = force_dp
    optimizer = AdamW(model.parameters(), lr=3e-4)
    loader = SyntheticMicroBatchDataLoader(args.mbs, args.seq, args.grad_acc, cfg.vocab_size, device, seed=1234)
    log(f"rank {rank}/{world}: model {num_params / 1e9:.3f} B params built in {time.time() - t0:.1f} s")

    probe = None
    probe_mb = 1 if args.grad_acc > 1 else 0   # a steady-state micro-batch (grads accumulate)

    def sample(i):
        # GEMM timing events only around the launches of one micro-batch per step: an event pair
        # on all ~550 GEMM launches of a step costs ~5 % of the step on ROCm
        K._PROBE = probe if (probe is not None and i == probe_mb) else None

    def step():
        optimizer.zero_grad()
        loss = train_step(model, loader, device, on_microbatch=sample)
        optimizer.step()
        if hasattr(model, "reset"):
            model.reset()
        return loss

    for i in range(args.warmup):
        t = time.time()
        loss = step()
        log(f"warmup {i}: loss {loss:.4f} ({time.time() - t:.2f} s)")

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    losses = []
    probe = K.GemmProbe() if not args.no_probe else None
    for i in range(args.steps):
        losses.append(step())
        log(f"step {i}: loss {losses[-1]:.4f}")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    K._PROBE = None
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()

    tokens = world * args.grad_acc * args.mbs * args.seq * args.steps
    value = tokens / elapsed
    per_gpu = value / world
    fpt = flops_per_token(num_params, cfg)
    mfu = per_gpu * fpt / MI355X_BF16_DENSE_PEAK

    roofline = None
    if probe:
        s = probe.summary()
        achieved = s["avg_flop"] / (s["avg_ms"] * 1e-3) / 1e12
        traffic, tsrc = None, None
        if os.path.exists(TRAFFIC_FILE):   # PMC-measured HBM bytes per GEMM launch (offline passes)
            with open(TRAFFIC_FILE) as f:
                tj = json.load(f)
            traffic, tsrc = tj["gemm_avg_bytes_per_launch"], os.path.relpath(TRAFFIC_FILE, ROOT)
        roofline = {"bound": "mfma", "kernel": "gemm (all bf16 MFMA GEMM launches of micro-batch "
                    f"{probe_mb} of every timed step)", "achieved": achieved,
                    "peak": MI355X_BF16_DENSE_PEAK / 1e12, "unit": "TFLOP/s",
                    "frac": achieved / (MI355X_BF16_DENSE_PEAK / 1e12), "traffic": traffic,
                    "traffic_unit": "bytes per launch", "traffic_source": tsrc,
                    "algorithmic_bytes_per_launch": s["avg_alg_bytes"],
                    "launches": s["launches"], "avg_launch_ms": s["avg_ms"], "avg_launch_gflop": s["avg_flop"] / 1e9,
                    "gemm_share_of_step": s["total_ms"] * 1e-3 * args.grad_acc / elapsed}

    cpu = None
    if rank == 0 and world == 1 and args.cpu_tokens > 0:
        log("cpu baseline ...")
        cpu = cpu_baseline(cfg, args.cpu_tokens)

    if rank == 0:
        out = {"metric": "tokens/s/GPU and MFU, SmolLM-1.7B seq1024 at 1/2/4/8 MI355X", "value": value,
               "unit": "tokens/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
               "vs_baseline": None, "dtype": "bf16", "data": "synthetic (seeded random tokens, random init)",
               "tokens_per_s_per_gpu": per_gpu, "mfu": mfu, "flops_per_token": fpt, "num_params": num_params,
               "final_loss": losses[-1] if losses else None,
               "config": {"workload": "SmolLM-1.7B dims, 15 layers, train step (fwd+bwd+AdamW)",
                          "model": "SmolLM-1.7B", "layers": args.layers, "micro_batch": args.mbs,
                          "grad_acc": args.grad_acc, "global_batch": args.mbs * args.grad_acc * world,
                          "seq_len": args.seq, "parallelism": f"dp{world}" + ("-bucket" if force_dp else "")},
               "roofline": roofline, "cpu_baseline": cpu}
        print(json.dumps(out), flush=True)
    if world > 1 or force_dp:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
