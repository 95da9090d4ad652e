"""bench.py -- picotron's headline metric on MI355X: training tokens/s (and MFU) of SmolLM-1.7B.

Workload (BASELINE.json configs[1]): SmolLM-1.7B dims (H 2048, I 8192, 32 heads, d 64, V 49152) with
15 decoder layers, micro-batch 4 x seq 1024, grad_acc 32, bf16, random init, synthetic tokens.
One step = train.py:219-240 of the reference: zero_grad, 32 x (forward, fused cross-entropy,
backward), AdamW step (train.py:209's torch.optim.AdamW semantics, fused HIP kernel:
picotron_amd/optim.py) and, for N > 1, the DataParallelBucket
all-reduce of the gradients over RCCL (dp = N, weak scaling: per-GPU work fixed).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
        bench.py --gpus N --steps K --warmup W [--model llama2-7b] [--tp T] [--cp C] [--seq S]

The other BASELINE configs through the same step (process grid from
setup_process_group_manager(tp, cp, 1, N / (tp cp)), train.py:95-100; apply_tensor_parallel /
apply_context_parallel / DataParallelBucket in train.py's order):
    config 3  --tp 8                                  (SmolLM-1.7B TP=8 over xGMI, strong scaling)
    config 4  --model llama2-7b --tp 2 --pp 2 --gpus 8  (dp2 tp2 pp2, 1F1B: pipeline_parallel/pipeline_parallel.py)
    config 5  --model llama2-7b --cp 8 --seq 32768 --mbs 1   (ring attention at 32k)
One-GPU per-rank compute proxies (no collectives; what one rank of the multi-GPU run computes):
    --tp-proxy 8      the decoder stack + lm_head with TP=8 shard widths (q|k|v 3 x 256, I 1024)
    --cp-proxy 8      Llama-2-7B at 32k, CP=8: the ring's critical rank -- the zig-zag schedule (1 causal
                      + 7 half blocks per layer on every rank) and the reference's (the last rank: 1
                      causal + 7 full 4096 x 4096 d128 blocks) -- attention blocks and the layer's GEMMs

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


# HBM bytes per GEMM launch from rocprofv3 PMC passes (tools/gpu.sh counters: bench.py --grad-acc 2, then
# tools/traffic_summary.py); read for the roofline's `traffic`
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "r06", "gemm_traffic_r06pm.json")


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def _md5(path):
    import hashlib
    with open(path, "rb") as f:
        return hashlib.md5(f.read()).hexdigest()


def cpu_baseline(cfg, tokens):
    """The oracle's training step -- fwd + bwd of the full model and torch's AdamW over every
    parameter -- on one [1, tokens] micro-batch, on this host's cores (the reference's own path cannot
    run on the GPU box; the oracle restates it in plain torch)."""
    from oracle import picotron_oracle as O
    import torch.nn.functional as F
    c = dict(hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
             num_attention_heads=cfg.num_attention_heads, num_key_value_heads=cfg.num_key_value_heads,
             rms_norm_eps=cfg.rms_norm_eps, vocab_size=cfg.vocab_size, num_hidden_layers=cfg.num_hidden_layers)
    params = O.init_params(c, seed=42)
    for p in params.values():
        p.requires_grad_(True)
    opt = torch.optim.AdamW(list(params.values()), lr=3e-4)
    d = cfg.hidden_size // cfg.num_attention_heads
    cos, sin = O.get_cos_sin(tokens, d, base=cfg.rope_theta)
    g = torch.Generator().manual_seed(1234)
    ids = torch.randint(0, cfg.vocab_size, (1, tokens + 1), generator=g)

    def step(n):
        opt.zero_grad()
        logits = O.llama_forward(ids[:, :n], params, c, cos[:n].float(), sin[:n].float(), norm=O.rmsnorm_flash_semantics)
        F.cross_entropy(logits.reshape(-1, cfg.vocab_size), ids[:, 1:n + 1].reshape(-1)).backward()
        opt.step()
    step(min(tokens, 64))      # warm-up (thread pool, allocator, AdamW state) on a short sequence, untimed
    t0 = time.perf_counter()
    step(tokens)
    dt = time.perf_counter() - t0
    return {"value": tokens / dt, "unit": "tokens/s", "cores": torch.get_num_threads(), "nproc": os.cpu_count(),
            "kind": "port",
            "sample": f"oracle fp32 train step (fwd + bwd + torch AdamW) of the same {cfg.num_hidden_layers}-layer "
                      f"model on one [1, {tokens}] micro-batch after an untimed warm-up step ({dt:.1f} s, "
                      f"{torch.get_num_threads()} threads of {os.cpu_count()} host CPUs); the reference's own "
                      f"--use_cpu gloo path (config 1, 8 processes) runs ~113 tokens/s in the build container "
                      f"(BASELINE.md)"}


MODELS = {"smollm-1.7b": ("SmolLM-1.7B", "SMOLLM_1_7B", 15), "llama2-7b": ("Llama-2-7B", "LLAMA2_7B", 32)}


def _events_time(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


class OneRankTP:
    """A tp group of `world` ranks as one of its ranks sees it, with every collective a REAL RCCL
    launch on a ONE-rank group (functional.TPContext's interface): an all-gather moves this rank's
    rows through RCCL into its slot (the other ranks' slots are filled with copies of them on the
    compute stream, so values stay finite and deterministic), a reduce-scatter reduces this rank's
    share of the rows, an all-reduce the whole tensor -- on RCCL's stream, async where the layer
    issues them async, captured into a HIP graph with the rest.  What one rank of a tp group launches
    and waits on, minus the xGMI transfer time (bench.py --tp-proxy; tests/test_graph_gpu.py)."""

    _cls = None

    def __new__(cls, group, world, fill=True):
        """fill=False (the throughput proxy): the other ranks' slots keep whatever the buffer held --
        their values do not change any kernel's time, and the fill copies (~0.6 ms per SmolLM-1.7B
        micro-batch at TP = 8) are not work a real rank does."""
        if cls._cls is None:
            cls._cls = cls._make()
        t = cls._cls(group, world, 0)
        t.fill = fill
        return t

    @staticmethod
    def _make():
        from picotron_amd import functional as FN

        class _OneRankTP(FN.TPContext):
            def _nccl(self):
                return True

            def all_reduce(self, t, async_op=False):
                return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=async_op)

            def all_gather_rows_into(self, out, t, async_op=False):
                n = t.shape[0]
                t = t.contiguous()
                if self.fill:
                    rest = out[n:].view(self.world_size - 1, *t.shape)
                    rest.copy_(t.unsqueeze(0).expand_as(rest))
                return dist.all_gather_into_tensor(out[:n], t, group=self.group, async_op=async_op)

            def reduce_scatter_rows_into(self, out, t, async_op=False):
                return dist.reduce_scatter_tensor(out, t[:out.shape[0]].contiguous(), op=dist.ReduceOp.SUM,
                                                  group=self.group, async_op=async_op)

            def reduce_scatter_rows(self, t, async_op=False):
                out = torch.empty((t.shape[0] // self.world_size,) + tuple(t.shape[1:]), dtype=t.dtype,
                                  device=t.device)
                return out, self.reduce_scatter_rows_into(out, t, async_op)
        return _OneRankTP


def init_one_rank_group(device):
    """A one-rank RCCL process group on `device` (127.0.0.1 rendezvous) for the one-GPU proxies."""
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        dist.init_process_group(backend="nccl", init_method="env://", rank=0, world_size=1, device_id=device)
    return dist.group.WORLD


def tp_proxy(args, base, layers):
    """One TP rank's compute for a micro-batch: `layers` decoder layers with the shard widths
    (heads / tp, I / tp; the layer kernels read shards exactly like this inside the TP model) and the
    launch forms of a tp > 1 group -- the sequence-parallel layout in its chunks, each collective a
    real RCCL launch on a one-rank group (OneRankTP: no xGMI transfer time) -- the embedding lookup
    and the lm_head's vocab shard (ColumnParallel, V / tp) plus the cross-entropy -- on the vocab
    shard (functional.VocabParallelCEFunction, the shipped form) or, with PICOTRON_VP_CE=0, over the
    gathered vocabulary as the reference -- fwd + bwd, eager and (--graph 1, how the product TP path
    runs: train.GraphedTrainStep) replayed as one HIP graph.  Returns the JSON line."""
    import math
    from picotron_amd import functional as FN
    from picotron_amd import kernels as K
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.tensor_parallel import sequence_parallel as SPM
    from picotron_amd.train import MI355X_BF16_DENSE_PEAK, make_config
    pgm.setup_process_group_manager(1, 1, 1, 1)
    tp = args.tp_proxy
    cfg = make_config(base, args.seq, num_hidden_layers=layers)
    H, I, V = cfg.hidden_size, cfg.intermediate_size // tp, cfg.vocab_size
    nh, nkv, d = cfg.num_attention_heads // tp, cfg.num_key_value_heads // tp, cfg.hidden_size // cfg.num_attention_heads
    T = args.mbs * args.seq
    dev = torch.device("cuda")
    group = init_one_rank_group(dev)
    g = torch.Generator(device=dev).manual_seed(0)

    def u(o, i):
        return torch.nn.Parameter(((torch.rand(o, i, device=dev, generator=g) * 2 - 1) / math.sqrt(i)).to(torch.bfloat16))
    stack = [[torch.nn.Parameter(torch.ones(H, device=dev, dtype=torch.bfloat16)) for _ in range(2)] +
             [u(nh * d, H), u(nkv * d, H), u(nkv * d, H), u(H, nh * d), u(I, H), u(I, H), u(H, I)] for _ in range(layers)]
    emb = torch.nn.Parameter(torch.randn(V // tp, H, device=dev, generator=g).to(torch.bfloat16))
    head = u(V // tp, H)
    cos = torch.ones(args.seq, d, device=dev, dtype=torch.bfloat16)
    sin = torch.zeros(args.seq, d, device=dev, dtype=torch.bfloat16)
    ids = torch.randint(0, V // tp, (args.mbs, args.seq), device=dev, generator=g)
    tgt = torch.randint(0, V, (T,), device=dev, generator=g)

    class _GatherStandIn(torch.autograd.Function):
        """ColumnParallelLinear(gather_output=True)'s all-gather of the vocab shards (tp_communications.py:51-72)
        as one rank sees it: forward writes the [T, V] gathered logits (here tp copies of the shard),
        backward hands this rank its own column slice (no sum: the reference's backward is a split)."""

        @staticmethod
        def forward(ctx, shard):
            return torch.cat([shard] * tp, dim=1)

        @staticmethod
        def backward(ctx, g):
            return g[:, :g.shape[1] // tp]

    from picotron_amd.switches import S as SW
    # sequence parallelism (sequence_parallel.py) in the layout's chunks (0: not shardable)
    chunks = SPM.layout_chunks(args.mbs, args.seq, tp) if tp > 1 and SW.tp_sp != 0 else 0
    vp = tp > 1 and FN.vp_ce_shape_ok(T, V // tp, H)          # the lm_head's vocab-parallel CE

    def micro_batch():
        x = FN.embedding(ids, emb)
        if chunks:   # the entry: this rank's rows of the summed lookups (reduce-scatter)
            x = SPM.ReduceScatterToSequenceRegion.apply(x, chunks)
        else:
            FN.TPContext.current().all_reduce(x)
        for w in stack:
            x = FN.DecoderLayerFunction.apply(x, *w, cos, sin, cfg.rms_norm_eps, 0, nh, nkv, d, False, chunks)
        if chunks:   # the exit's all-gather before the final norm
            x = SPM.GatherFromSequenceRegion.apply(x, chunks)
        if vp:   # the vocab-parallel CE (functional.VocabParallelCEFunction): no logits gather
            lg, stats = FN.lm_head_shard(x.reshape(T, H), head)
            full = FN.vp_logits(lg, stats, 0, V, lambda: _GatherStandIn.apply(lg))
        else:
            lg = FN.linear(x.reshape(T, H), head)                  # this rank's vocab shard
            full = _GatherStandIn.apply(lg) if tp > 1 else lg       # stands in for the all-gather
        FN.cross_entropy(full, tgt).backward()
    # the layers see a tp group of `tp` ranks (one-rank RCCL collectives), so they take the TP
    # launch forms (dX and dW as separate launches around the dX reduce-scatter), not tp = 1's duals
    current = FN.TPContext.current
    FN.TPContext.current = staticmethod(lambda: OneRankTP(group, tp, fill=False))
    try:
        probe = K.GemmProbe()
        for _ in range(args.warmup + 1):
            micro_batch()
        torch.cuda.synchronize()
        # the backward reached every layer's weights (a stand-in off the autograd graph would cut it)
        assert all(p.grad is not None for w in stack for p in w) and emb.grad is not None, "proxy backward incomplete"
        t = t_eager = _events_time(micro_batch, args.steps)
        graph_note = None
        if args.graph:
            # the product TP path's launch mode (train.GraphedTrainStep): the micro-batch (fwd, CE,
            # bwd, the RCCL collectives) captured as one HIP graph and replayed
            try:
                side = torch.cuda.Stream()
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    micro_batch()
                torch.cuda.current_stream().wait_stream(side)
                from picotron_amd.train import quiesce_collectives
                quiesce_collectives(dev)
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    micro_batch()
                t = _events_time(graph.replay, args.steps)
            except Exception as e:   # a capture the stack refuses: report it, keep the eager timing
                graph_note = f"graph capture failed: {type(e).__name__}: {e}"[:300]
                torch.cuda.synchronize()
        with probe:
            micro_batch()
        s = probe.summary()
    finally:
        FN.TPContext.current = current
    fpt_rank = 6 * sum(p.numel() for w in stack for p in w) + 6 * head.numel() + 12 * layers * nh * d * args.seq
    ach = s["avg_flop"] / (s["avg_ms"] * 1e-3) / 1e12
    tok_gpu = T / t / tp          # tp ranks share these tokens
    dist.destroy_process_group()
    return {"metric": f"TP={tp} per-rank compute proxy (1 GPU, one-rank RCCL collectives: no xGMI transfer time)",
            "value": tok_gpu, "unit": "tokens/s/GPU (compute + collective launches, no link time)",
            "ms_per_microbatch": t * 1e3,
            "launch": "hip graph replay (as train.GraphedTrainStep runs the TP path)"
            if (args.graph and graph_note is None) else "eager",
            "eager_ms_per_microbatch": t_eager * 1e3, "eager_tokens_per_s_per_gpu": T / t_eager / tp,
            **({"graph_note": graph_note} if graph_note else {}),
            "mfu_upper_bound": tok_gpu * (fpt_rank * tp) / MI355X_BF16_DENSE_PEAK,
            "config": {"model": cfg_name(base), "layers": layers, "micro_batch": args.mbs, "seq_len": args.seq,
                       "shard": {"q|k|v": 3 * nh * d, "I": I, "heads": nh, "vocab": V // tp},
                       "sequence_parallel": bool(chunks), "sp_chunks": chunks, "vocab_parallel_ce": vp},
            "roofline": {"bound": "mfma", "kernel": "gemm (every GEMM launch of one eager micro-batch)", "achieved": ach,
                         "peak": MI355X_BF16_DENSE_PEAK / 1e12, "unit": "TFLOP/s",
                         "frac": ach / (MI355X_BF16_DENSE_PEAK / 1e12), "launches": s["launches"],
                         "gemm_share": s["total_ms"] * 1e-3 / t},
            "gemm_by_launch": {k: {"launches": v[0], "ms": v[1], "tflops": v[2]} for k, v in probe.by_label().items()}}


XGMI_LINK_GBPS = 153.0   # one MI355X xGMI link, per direction (7 links per GPU, full mesh)


def cp_proxy(args, base, layers):
    """The critical rank of a CP ring for one layer of Llama-2-7B at seq = C x S_local: the layer's
    GEMMs + its causal diagonal block (the fused layer at S_local) and the visiting blocks (forward
    with the LSE merge epilogue, backward from the global LSE, f32 dQ / dK / dV as the ring keeps
    them), fwd + bwd, timed on one GPU.  Schedules:
      reference  (context_parallel.py:30-45): the last rank computes C - 1 full S_local^2 blocks;
      zig-zag    (the shipped one, context_parallel.zigzag_enabled): every rank computes C - 1 half
                 blocks -- rank r: r of [S_local x S_local/2] (its queries x the first half of the
                 keys) and C - 1 - r of [S_local/2 x S_local] -- the slowest rank sets the pace.
    Communication is not run (one GPU); it is costed per layer from its bytes at XGMI_LINK_GBPS per
    link and direction, overlapped with the compute it can hide under:
      ring (the reference's transport): step s sends the K|V shard to the next rank while the
                 visiting block computes -- C - 1 sequential one-link hops forward; backward the K|V
                 hops plus C hops of the fp32 dK|dV accumulator (context_parallel.py:72-106);
      mesh (shipped with the zig-zag layout): the visiting K|V fetched from their owners on C - 1
                 links at once, first half-chunks under the diagonal block, the second halves a
                 'q1' block needs under the first blocks; backward the K|V shards (under the
                 diagonal block's backward) then the visiting queries / dO (bf16) and LSE / D (f32)
                 (under the dQ parts) -- each rank computes its own keys' dK / dV, so no gradient
                 partial travels;
      re-lay     the residual stream's zig-zag re-lay, twice per forward and twice per backward for
                 the whole stack (context_parallel.enable_zigzag_residual: on with the cp gradient
                 averaging of DataParallelBucket), amortised per layer."""
    import math
    from picotron_amd import functional as FN
    from picotron_amd import kernels as K
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.train import MI355X_BF16_DENSE_PEAK, make_config
    pgm.setup_process_group_manager(1, 1, 1, 1)
    C = args.cp_proxy
    cfg = make_config(base, args.seq, num_hidden_layers=layers)
    S = args.seq // C
    h = S // 2
    H, I = cfg.hidden_size, cfg.intermediate_size
    nh, nkv, d = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.hidden_size // cfg.num_attention_heads
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    B = args.mbs

    def r(*shape):
        return torch.randn(*shape, device=dev, generator=g).to(torch.bfloat16)

    def u(o, i):
        return torch.nn.Parameter(((torch.rand(o, i, device=dev, generator=g) * 2 - 1) / math.sqrt(i)).to(torch.bfloat16))
    w = [torch.nn.Parameter(torch.ones(H, device=dev, dtype=torch.bfloat16)) for _ in range(2)] + \
        [u(nh * d, H), u(nkv * d, H), u(nkv * d, H), u(H, nh * d), u(I, H), u(I, H), u(H, I)]
    cos = torch.ones(S, d, device=dev, dtype=torch.bfloat16)
    sin = torch.zeros(S, d, device=dev, dtype=torch.bfloat16)
    x = r(B, S, H).requires_grad_(True)
    q, k, v, do = r(B, S, nh, d), r(B, S, nkv, d), r(B, S, nkv, d), r(B, S, nh, d)
    sc = 1 / math.sqrt(d)
    acc = torch.zeros(B, S, nh, d, device=dev)
    lse = torch.zeros(B, nh, S, device=dev)
    o = r(B, S, nh, d)
    dq = torch.zeros(B, S, nh, d, device=dev)
    dk, dv = torch.zeros(B, S, nkv, d, device=dev), torch.zeros(B, S, nkv, d, device=dev)
    delta = K.attn_delta(do, o)

    def layer():
        FN.DecoderLayerFunction.apply(x, *w, cos, sin, cfg.rms_norm_eps, 0, nh, nkv, d).backward(r(B, S, H))
    fns = {
        "diag_fwd": lambda: K.attn_fwd(q, k, v, sc, True, out=acc, lse=lse, merge=True),
        "diag_bwd": lambda: K.attn_bwd(do, q, k, v, o, lse, sc, True, dq=dq, dk=dk, dv=dv, grad_f32=True, delta=delta),
        "full_fwd": lambda: K.attn_fwd(q, k, v, sc, False, out=acc, lse=lse, merge=True),
        "full_bwd": lambda: K.attn_bwd(do, q, k, v, o, lse, sc, False, dq=dq, dk=dk, dv=dv, grad_f32=True, delta=delta),
        # all S_local queries x the first half of the visiting keys
        "kv0_fwd": lambda: K.attn_fwd(q, k[:, :h], v[:, :h], sc, False, out=acc, lse=lse, merge=True),
        "kv0_bwd": lambda: K.attn_bwd(do, q, k[:, :h], v[:, :h], o, lse, sc, False, dq=dq, dk=dk[:, :h], dv=dv[:, :h],
                                      grad_f32=True, delta=delta),
        # the second half of the queries x all the visiting keys
        "q1_fwd": lambda: K.attn_fwd(q[:, h:], k, v, sc, False, out=acc[:, h:], lse=lse[:, :, h:], merge=True),
        "q1_bwd": lambda: K.attn_bwd(do[:, h:], q[:, h:], k, v, o[:, h:], lse[:, :, h:], sc, False, dq=dq[:, h:], dk=dk,
                                     dv=dv, grad_f32=True, delta=delta[:, :, h:]),
        # the mesh schedule's launches: a 'q1' forward as two quarters (second-half queries x one
        # half-chunk of keys), the backward halves as dQ-only / dK|dV-only parts
        "q1q_fwd": lambda: K.attn_fwd(q[:, h:], k[:, :h], v[:, :h], sc, False, out=acc[:, h:], lse=lse[:, :, h:],
                                      merge=True),
        "kv0_dq": lambda: K.attn_bwd_part(do, q, k[:, :h], v[:, :h], lse, delta, sc, False, dq=dq),
        "q1_dq": lambda: K.attn_bwd_part(do[:, h:], q[:, h:], k, v, lse[:, :, h:], delta[:, :, h:], sc, False,
                                         dq=dq[:, h:]),
        "kv0_dkdv": lambda: K.attn_bwd_part(do, q, k[:, :h], v[:, :h], lse, delta, sc, False, dk=dk[:, :h],
                                            dv=dv[:, :h]),
        "q1_dkdv": lambda: K.attn_bwd_part(do[:, h:], q[:, h:], k, v, lse[:, :, h:], delta[:, :, h:], sc, False,
                                           dk=dk, dv=dv),
    }
    t_layer = _events_time(layer, args.steps)
    t = {kname: _events_time(fn, args.steps * 4) for kname, fn in fns.items()}
    blk_flop = 4.0 * B * nh * S * S * d           # full block: QK^T + PV
    t_f, t_b = t["full_fwd"], t["full_bwd"]
    t_kv0, t_q1 = t["kv0_fwd"] + t["kv0_bwd"], t["q1_fwd"] + t["q1_bwd"]
    t_ref = t_layer + (C - 1) * (t_f + t_b)       # reference schedule: the last rank
    crit = max(range(C), key=lambda rk: rk * t_kv0 + (C - 1 - rk) * t_q1)
    t_zz = t_layer + crit * t_kv0 + (C - 1 - crit) * t_q1

    # ---- communication budget per layer (bytes per rank, link time, what stays exposed)
    bw = XGMI_LINK_GBPS * 1e9
    kv_b = B * S * 2 * nkv * d * 2               # one K|V shard, bf16
    dkv_b = 2 * kv_b                             # its fp32 dK|dV accumulator (the ring's)
    qdo_b = B * S * 2 * nh * d * 2 + B * nh * S * 2 * 4   # a rank's queries + dO (bf16), LSE + D (f32)
    relay_b = 4 * B * S * H * 2                  # re-lay of [B, S, H] bf16: entry + exit, fwd + bwd, per pass
    halves_f = [t["kv0_fwd"]] * crit + [t["q1_fwd"]] * (C - 1 - crit)
    halves_b = [t["kv0_bwd"]] * crit + [t["q1_bwd"]] * (C - 1 - crit)
    # ring: each step's transfer hides under that step's block
    ring_f = sum(max(kv_b / bw, tf) - tf for tf in halves_f)
    ring_b = sum(max((kv_b + dkv_b) / bw, tb) - tb for tb in halves_b) + dkv_b / bw   # + the last dK|dV hop
    # mesh (context_parallel.mesh_forward / mesh_backward), rank rk's own schedule: forward, batch A =
    # every peer's first half-chunk (hidden under the diagonal block), batch B = the second halves
    # of the peers j > rk, waited for after the 'kv0' blocks and the first 'q1' quarters; backward,
    # batch A = the K|V shards (under the diagonal block's backward), batch B = Q|dO|LSE|D (under the
    # dQ parts).  Per link the batches run back to back.
    def mesh_rank(rk):
        lo, hi = rk, C - 1 - rk                  # peers below / above
        c_f = lo * t["kv0_fwd"] + hi * 2 * t["q1q_fwd"]
        dq_parts = lo * t["kv0_dq"] + hi * t["q1_dq"]
        c_b = dq_parts + hi * t["kv0_dkdv"] + lo * t["q1_dkdv"]
        a_f = max(t["diag_fwd"], kv_b / 2 / bw)
        x_f = a_f - t["diag_fwd"]
        if hi:
            x_f += max(0.0, kv_b / bw - (a_f + lo * t["kv0_fwd"] + hi * t["q1q_fwd"]))
        a_b = max(t["diag_bwd"], kv_b / bw)
        x_b = a_b - t["diag_bwd"] + max(0.0, (kv_b + qdo_b) / bw - (a_b + dq_parts))
        return c_f + c_b, x_f, x_b
    crit_m = max(range(C), key=lambda rk: sum(mesh_rank(rk)))
    mesh_c, mesh_f, mesh_b = mesh_rank(crit_m)
    relay_t = relay_b / layers / (2 * bw)        # two peers, two links
    comm = {"link_GBps_per_direction": XGMI_LINK_GBPS, "kv_shard_bytes": kv_b, "dkv_f32_bytes": dkv_b,
            "ring": {"comm_bytes_per_layer": (C - 1) * kv_b + (C - 1) * kv_b + C * dkv_b,
                     "link_time_ms": ((C - 1) * kv_b * 2 + C * dkv_b) / bw * 1e3,
                     "exposed_ms": (ring_f + ring_b) * 1e3},
            # received by the critical rank; its busiest link
            "mesh": {"comm_bytes_per_layer": (C - 1) * (kv_b / 2 + kv_b + qdo_b) + (C - 1 - crit_m) * kv_b / 2,
                     "link_time_ms": ((kv_b if crit_m < C - 1 else kv_b / 2) + kv_b + qdo_b) / bw * 1e3,
                     "links": C - 1,
                     "exposed_ms": (mesh_f + mesh_b) * 1e3,
                     # the backward's receive buffers, all peers' at once (mesh_backward), vs the ring's two
                     "recv_buffer_bytes": (C - 1) * (kv_b + qdo_b), "ring_recv_buffer_bytes": 2 * (kv_b + dkv_b)},
            "relayout": {"comm_bytes_per_pass": relay_b, "per_layer_ms": relay_t * 1e3}}
    t_mesh = t_layer + mesh_c + mesh_f + mesh_b + relay_t
    t_ring_zz = t_zz + ring_f + ring_b + relay_t
    attn_compute = t["diag_fwd"] + t["diag_bwd"] + sum(halves_f) + sum(halves_b)
    layer_flop_model = 6 * (2 * H * nh * d + 2 * H * nkv * d + 3 * H * I) + 12 * H * args.seq   # per token
    tok_gpu = B * S / (t_zz * layers)             # each rank holds S tokens; the ring's pace = its slowest rank
    tok_mesh = B * S / (t_mesh * layers)
    return {"metric": f"CP={C} critical-rank proxy (1 GPU, compute measured; xGMI communication costed separately)",
            "value": tok_gpu, "unit": "tokens/s/GPU (compute-only, measured: zig-zag schedule's critical rank)",
            # modelled, not measured: the mesh transfers costed at XGMI_LINK_GBPS (an assumed per-link
            # rate) and overlapped as the schedule overlaps them
            "modelled_with_mesh_comm_tokens_per_s_per_gpu": tok_mesh,
            "comm_model": f"{XGMI_LINK_GBPS} GB/s per xGMI link and direction (assumed, not measured on this box)",
            "config": {"model": cfg_name(base), "layers": layers, "micro_batch": B, "seq_len": args.seq,
                       "S_local": S, "head_dim": d, "schedule": "zig-zag (load-balanced), full-mesh K|V exchange"},
            "compute_only_tokens_per_s_per_gpu": tok_gpu,
            "ring_transport_tokens_per_s_per_gpu": B * S / (t_ring_zz * layers),
            "layer_ms": t_layer * 1e3, "block_fwd_ms": t_f * 1e3, "block_bwd_ms": t_b * 1e3,
            "blocks_ms": {kname: v * 1e3 for kname, v in t.items()},
            "half_block_kv0_ms": t_kv0 * 1e3, "half_block_q1_ms": t_q1 * 1e3, "critical_rank": crit,
            "critical_rank_mesh": crit_m, "critical_rank_mesh_compute_ms": (t_layer + mesh_c) * 1e3,
            "critical_rank_layer_ms": t_zz * 1e3, "critical_rank_layer_ms_with_comm": {"mesh": t_mesh * 1e3,
                                                                                      "ring": t_ring_zz * 1e3},
            "reference_schedule_layer_ms": t_ref * 1e3,
            "reference_schedule_tokens_per_s_per_gpu": B * S / (t_ref * layers),
            "comm": comm,
            # link-bound: the layer's link time exceeds the attention compute it could hide under
            "bound": {"mesh": "link" if comm["mesh"]["link_time_ms"] * 1e-3 > attn_compute else "compute",
                      "ring": "link" if comm["ring"]["link_time_ms"] * 1e-3 > attn_compute else "compute",
                      "exposed_share_of_layer": {"mesh": (mesh_f + mesh_b + relay_t) / t_mesh,
                                                 "ring": (ring_f + ring_b + relay_t) / t_ring_zz}},
            "mfu_upper_bound": tok_gpu * layer_flop_model * layers / MI355X_BF16_DENSE_PEAK,
            "mfu_with_comm": tok_mesh * layer_flop_model * layers / MI355X_BF16_DENSE_PEAK,
            "roofline": {"bound": "mfma", "kernel": "attention block S_local x S_local d128 (fwd merge + bwd)",
                         "achieved": (blk_flop * 3.5) / (t_f + t_b) / 1e12, "peak": MI355X_BF16_DENSE_PEAK / 1e12,
                         "unit": "TFLOP/s", "frac": (blk_flop * 3.5) / (t_f + t_b) / MI355X_BF16_DENSE_PEAK,
                         "fwd_frac": blk_flop / t_f / MI355X_BF16_DENSE_PEAK,
                         "bwd_frac": blk_flop * 2.5 / t_b / MI355X_BF16_DENSE_PEAK,
                         "half_block_frac": (blk_flop / 2 * 3.5) / t_kv0 / MI355X_BF16_DENSE_PEAK}}


def pmc_kernel_key(label):
    """The rocprofv3 kernel (name + workgroup count, tools/traffic_summary.py's key) a GemmProbe
    label of a dual launch (kernels.linear_dgrad_dual) ran as: gemm_8ph_dual_kernel<AK0 = true,
    BKC0 = false, dX epilogue, false, false, dW epilogue> with one workgroup per 256x256 tile (the dX
    split-K halves, epilogue 2, count twice).  Other labels: the label itself."""
    import re
    m = re.fullmatch(r"dual dX (\d+)x(\d+)x(\d+) e(\d+) \+ dW ([\dx,]+) e(\d+)", label)
    if not m:
        return label
    T, N, _, e0, dws, e1 = m.groups()
    wg = (int(T) // 256) * (int(N) // 256) * (2 if e0 == "2" else 1)
    for dw in dws.split(","):
        nw, kin, _ = (int(v) for v in dw.split("x"))
        wg += (nw // 256) * (kin // 256)
    return f"void gemm_8ph_dual_kernel<true, false, {e0}, false, false, {e1}> [{wg} WG]"


def cfg_name(base):
    return {v[1]: v[0] for v in MODELS.values()}.get(base.get("_name"), "custom")


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_cmd(argv, nproc, port):
    """The torchrun command line `bench.py --gpus N` starts for N > 1 when it was not itself started
    by a launcher: one process per GPU on this node, env:// rendezvous on 127.0.0.1 -- the
    reference's launch (train.py:2 docstring, template/base_job.slurm:64: torchrun --nproc_per_node
    --nnodes ... train.py), with this script's own arguments passed through unchanged."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def launch_ranks(argv, nproc):
    """Run the N-rank job as a CHILD process (nothing in this process has touched the GPU: no exec)
    and forward rank 0's single JSON line to stdout; everything else goes to stderr.  Returns the
    child's exit code (non-zero also when no JSON line came back)."""
    import subprocess
    cmd = launcher_cmd(argv, nproc, _free_port())
    log("launching", nproc, "ranks:", " ".join(cmd))
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True)
    result = None
    for line in p.stdout:
        s = line.strip()
        if s.startswith("{") and '"metric"' in s and result is None:
            result = s
        else:
            sys.stderr.write(line)
    rc = p.wait()
    if result is not None:
        print(result, flush=True)
    if rc == 0 and result is None:
        log("the ranks exited without a result line")
        return 1
    return rc


def assemble_report(args, model, m, cfg, num_params, rank, world, result_out):
    """--assemble-only: every rank reports its grid coordinates (process_group_manager.py:13: view(dp,
    pp, cp, tp)), its shard (parameters held, pipeline layers, embedding / lm_head presence), the
    zig-zag residual flag and the bucket count; rank 0 checks the grid covers every coordinate once
    and that the ranks of one tp group hold equal shard sizes, then prints ONE JSON line."""
    inner = model.module if hasattr(model, "bucket_manager") else model
    names = [n for n, _ in inner.named_parameters()]
    me = {"rank": rank, "grid": [m.dp_rank, m.pp_rank, m.cp_rank, m.tp_rank],
          "params": sum(p.numel() for p in inner.parameters()),
          "layers": sorted({int(n.split(".")[1]) for n in names if n.startswith("decoder_layers.")}),
          "embedding": any(n.startswith("embedding.") for n in names),
          "lm_head": any(n.startswith("final_proj.") for n in names),
          "zigzag_residual": bool(getattr(inner, "_pt_zigzag_residual", False)),
          "buckets": len(model.bucket_manager.buckets) if hasattr(model, "bucket_manager") else 0}
    allr = [None] * world
    if world > 1:
        dist.all_gather_object(allr, me)
    else:
        allr = [me]
    if rank == 0:
        coords = {tuple(r["grid"]) for r in allr}
        dims = (m.dp_world_size, m.pp_world_size, m.cp_world_size, m.tp_world_size)
        assert len(coords) == world == dims[0] * dims[1] * dims[2] * dims[3], (coords, dims)
        by_stage = {}
        for r in allr:
            by_stage.setdefault(r["grid"][1], set()).add(r["params"])
        assert all(len(v) == 1 for v in by_stage.values()), by_stage   # same shard per stage, every dp/cp/tp
        layers = sorted({i for r in allr for i in r["layers"]})
        assert layers == list(range(cfg.num_hidden_layers)), layers
        par = "-".join(f"{k}{v}" for k, v in zip(("dp", "pp", "cp", "tp"), dims) if v > 1 or k == "dp")
        out = {"metric": "grid assembly (no step run)", "assembled": True, "ranks": world, "backend": "gloo",
               "config": {"model": MODELS[args.model][0], "layers": cfg.num_hidden_layers, "seq_len": args.seq,
                          "micro_batch": args.mbs, "parallelism": par},
               "model_params": num_params, "per_rank": allr}
        print(json.dumps(out), file=result_out, flush=True)
    if world > 1:
        dist.destroy_process_group()


def build_parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", choices=sorted(MODELS), default="smollm-1.7b")
    ap.add_argument("--layers", type=int, default=0, help="decoder layers (0 = the config's: 15 / 32)")
    ap.add_argument("--tp", type=int, default=1, help="tensor-parallel degree (N GPUs = dp x tp x cp)")
    ap.add_argument("--cp", type=int, default=1, help="context-parallel (ring attention) degree")
    ap.add_argument("--pp", type=int, default=1, help="pipeline-parallel degree (N GPUs = dp x tp x cp x pp)")
    ap.add_argument("--pp-engine", choices=["1f1b", "afab"], default="1f1b", help="pipeline schedule (train.py:222-225)")
    ap.add_argument("--tp-proxy", type=int, default=0, help="1 GPU: one TP rank's compute at this degree")
    ap.add_argument("--cp-proxy", type=int, default=0, help="1 GPU: the CP ring's critical rank at this degree")
    ap.add_argument("--graph", type=int, default=1, help="tp > 1 (and --tp-proxy): run each micro-batch as a "
                                                         "replayed HIP graph (train.GraphedTrainStep; 0: eager)")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="gloo: rehearse an N-rank grid with every rank on cuda:0 (one-GPU box); timing meaningless")
    ap.add_argument("--mbs", type=int, default=None,
                    help="micro-batch (default 4; 32 with --tp / --tp-proxy > 1, see resolve_batch)")
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--grad-acc", type=int, default=None,
                    help="micro-batches per step (default 32; 4 with the TP micro-batch default)")
    ap.add_argument("--cpu-tokens", type=int, default=1024, help="tokens in the cpu_baseline sample (0 = skip)")
    ap.add_argument("--no-probe", action="store_true", help="do not time GEMM launches with events")
    ap.add_argument("--bucket-mb", type=float, default=25, help="DataParallelBucket bucket_cap_mb (reference: 25)")
    ap.add_argument("--grad-type", choices=["fp32", "bf16"], default="fp32",
                    help="DataParallelBucket grad_type: fp32 main_grad (reference default) or bf16")
    ap.add_argument("--assemble-only", action="store_true",
                    help="build the process grid, model shards and wrappers on the CPU (gloo), report them, "
                         "run no step: rehearses an N-rank grid without a GPU")
    ap.add_argument("--dp-bucket", action="store_true",
                    help="N = 1 only: run the DP path anyway (DataParallelBucket, fp32 main_grad, bucket "
                         "all-reduce over a 1-rank RCCL group) -- the per-GPU cost of N > 1 minus the links")
    return ap


def resolve_batch(args):
    """Fill in --mbs / --grad-acc.  Defaults: mbs 4 x grad_acc 32 (BASELINE's config 2).  Pure tensor
    parallelism (--tp or --tp-proxy > 1 without cp / pp: config 3, which names no micro-batch) with
    neither given: mbs 32 x grad_acc 4 -- the same 128 sequences and the same gradient per step --
    because a TP = 8 rank's shard GEMMs starve at 4096 rows (64 k tokens/s/GPU of compute at mbs 4,
    101 k at mbs 32) and a micro-batch of 32 sequences runs the chunked layout in 4 chunks, 3/4 of
    its collectives under the other chunks' compute (sequence_parallel.CHUNK_MIN_ROWS; the
    measurements and the projection in profiles/r06/notes_r06.md)."""
    pure_tp = max(args.tp, args.tp_proxy) > 1 and args.cp == 1 and args.pp == 1
    if pure_tp and args.mbs is None and args.grad_acc is None:
        args.mbs, args.grad_acc = 32, 4
    if args.mbs is None:
        args.mbs = 4
    if args.grad_acc is None:
        args.grad_acc = 32
    return args


def main():
    args = resolve_batch(build_parser().parse_args())
    proxy = bool(args.tp_proxy or args.cp_proxy)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1 and not proxy:
        # `python bench.py --gpus N`: start the N ranks ourselves (before any GPU call in this process)
        sys.exit(launch_ranks(sys.argv[1:], args.gpus))
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus and not proxy:
        raise SystemExit(f"bench.py: WORLD_SIZE={os.environ['WORLD_SIZE']} from the launcher but --gpus "
                         f"{args.gpus}: refusing to report a run with a different GPU count")
    # stdout carries exactly ONE line, the JSON result: anything else written to fd 1 (RCCL prints
    # its version banner there when a communicator is created) is sent to stderr
    result_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("LOCAL_RANK", str(local_rank))
    os.environ.setdefault("FLASH_ATTEN", "1")
    os.environ["DEVICE"] = "cpu" if args.assemble_only else "cuda"
    if args.assemble_only and args.backend != "gloo":
        raise SystemExit("bench.py --assemble-only runs on the CPU: use --backend gloo")
    if args.backend == "gloo":
        local_rank = 0
        os.environ["LOCAL_RANK"] = "0"
    if args.assemble_only:
        device = torch.device("cpu")
    else:
        torch.cuda.set_device(local_rank)
        device = torch.device("cuda", local_rank)
    force_dp = args.dp_bucket and world == 1
    if world > 1 or force_dp:
        if force_dp:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if args.backend == "gloo":
            dist.init_process_group(backend="gloo", init_method="env://")
        else:
            dist.init_process_group(backend="nccl", init_method="env://", device_id=device)

    from picotron_amd import kernels as K
    from picotron_amd import train as TR
    from picotron_amd.context_parallel.context_parallel import apply_context_parallel
    from picotron_amd.data_parallel.data_parallel import DataParallelBucket
    from picotron_amd.model import Llama
    from picotron_amd.optim import AdamW
    from picotron_amd.process_group_manager import setup_process_group_manager
    from picotron_amd.tensor_parallel.tensor_parallel import apply_tensor_parallel
    from picotron_amd.train import (SyntheticMicroBatchDataLoader, count_params, flops_per_token, make_config,
                                    train_step, read_step_loss, MI355X_BF16_DENSE_PEAK)

    model_name, base_name, default_layers = MODELS[args.model]
    base = dict(getattr(TR, base_name), _name=base_name)
    layers = args.layers or default_layers
    if args.tp_proxy or args.cp_proxy:
        out = tp_proxy(args, base, layers) if args.tp_proxy else cp_proxy(args, base, layers)
        print(json.dumps(out), file=result_out, flush=True)
        return
    tp, cp, pp = args.tp, args.cp, args.pp
    if world % (tp * cp * pp):
        raise SystemExit(f"--gpus {world} is not a multiple of tp {tp} x cp {cp} x pp {pp}")
    dp = world // (tp * cp * pp)
    m = setup_process_group_manager(tp_size=tp, cp_size=cp, pp_size=pp, dp_size=dp)
    torch.manual_seed(42)
    cfg = make_config({k: v for k, v in base.items() if k != "_name"}, args.seq, num_hidden_layers=layers)
    t0 = time.time()
    with torch.device(device):
        model = Llama(cfg)            # train.py:174-186 order: build, TP swap, PP, CP, dtype, DP wrap
        if tp > 1:
            apply_tensor_parallel(model)
        num_params = count_params(model)   # the whole model (before a pipeline stage keeps its slice)
        if pp > 1:
            from picotron_amd.pipeline_parallel.pipeline_parallel import PipelineParallel
            model = PipelineParallel(model, cfg)
    apply_context_parallel(model)
    model.to(torch.bfloat16)
    if m.cp_dp_world_size > 1 or force_dp:
        model = DataParallelBucket(model, bucket_cap_mb=args.bucket_mb,
                                   grad_type=torch.bfloat16 if args.grad_type == "bf16" else torch.float32)
        model._force_grad_sync = force_dp
    if args.assemble_only:
        return assemble_report(args, model, m, cfg, num_params, rank, world, result_out)
    optimizer = AdamW(model.parameters(), lr=3e-4)
    loader = SyntheticMicroBatchDataLoader(args.mbs, args.seq, args.grad_acc, cfg.vocab_size, device, seed=1234,
                                           fresh=True)
    log(f"rank {rank}/{world}: model {num_params / 1e9:.3f} B params built in {time.time() - t0:.1f} s")

    probe = None
    # a steady-state micro-batch: the gradients accumulate (the ACC epilogues) and, with the weight-
    # gradient pairing of train_step, the pair (2, 3) completes in it (its K = 2 T weight gradients)
    probe_mb = 3 if args.grad_acc >= 4 else (1 if args.grad_acc > 1 else 0)

    def sample(i):
        # GEMM timing events only around the launches of one micro-batch per step: an event pair
        # on all ~550 GEMM launches of a step costs ~5 % of the step on ROCm
        K._PROBE = probe if (probe is not None and i == probe_mb) else None

    # tensor parallelism: the micro-batch replayed as one HIP graph (its RCCL collectives inside)
    graphed = None
    if args.graph and tp > 1 and args.backend == "nccl" and TR.GraphedTrainStep.supported(model):
        graphed = TR.GraphedTrainStep(model, loader, device)
    if pp > 1:
        from picotron_amd.pipeline_parallel import pipeline_parallel as PPE
        pp_step = PPE.train_step_pipeline_1f1b if args.pp_engine == "1f1b" else PPE.train_step_pipeline_afab
        shapes = (args.mbs, args.seq // cp, cfg.hidden_size)

    def step():
        if pp > 1:   # train.py:222-225 (the GEMM probe samples micro-batches of train_step only)
            optimizer.zero_grad()
            loss = pp_step(model, loader, shapes, device, torch.bfloat16)
            if hasattr(model, "reset"):
                model.reset()
            optimizer.step()
            return loss
        # train.py:220-225 with the host work of the step boundary moved under the GPU's: the optimizer
        # is enqueued behind the backward before the host reads the loss (train_step(read_loss=False)),
        # and the next step's zero_grad (set_to_none: drops the gradients, stream-ordered) runs while
        # the AdamW launch does -- same work, no GPU idle gap at the boundary
        if graphed is not None:
            loss = graphed(read_loss=False)
        else:
            loss = train_step(model, loader, device, on_microbatch=sample, read_loss=False)
        optimizer.step()
        if hasattr(model, "reset"):
            model.reset()
        optimizer.zero_grad()
        return read_step_loss(loss, device)

    optimizer.zero_grad()

    for i in range(args.warmup):
        t = time.time()
        loss = step()
        log(f"warmup {i}: loss {loss:.4f} ({time.time() - t:.2f} s)")

    # GEMM timing (HIP events on the launch stream, micro-batch `probe_mb` of a step): the first timed
    # step times every GEMM launch (the family average, and which launch kind dominates), the later
    # ones only the dominant kind's launches -- an event pair per launch idles the GPU a few us, ~1.3
    # ms for a micro-batch's whole family
    use_probe = not (args.no_probe or pp > 1 or graphed is not None)
    fam_probe, dom = None, None

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    losses = []
    dom_probe = None
    for i in range(args.steps):
        if use_probe and i == 0:
            probe = fam_probe = K.GemmProbe()
        elif use_probe and i == 1:
            labels = fam_probe.by_label() if fam_probe.records else {}
            dom = max(labels, key=lambda k: labels[k][1]) if labels else None
            probe = dom_probe = K.GemmProbe(only=dom) if dom else None
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

    tokens = dp * args.grad_acc * args.mbs * args.seq * args.steps    # tp / cp / pp ranks share their tokens
    if pp > 1 and losses:   # the loss lives on the last stage: report it from rank 0 too
        lt = torch.tensor([losses[-1]], dtype=torch.float64, device=device)
        dist.all_reduce(lt, op=dist.ReduceOp.SUM, group=m.pp_group)
        losses[-1] = lt.item()
    value = tokens / elapsed
    per_gpu = value / world
    fpt = flops_per_token(num_params, cfg)
    mfu = per_gpu * fpt / MI355X_BF16_DENSE_PEAK

    roofline = None
    probe = None
    if fam_probe is not None and fam_probe.records:
        fam = fam_probe
        s = fam.summary()
        fam_achieved = s["avg_flop"] / (s["avg_ms"] * 1e-3) / 1e12
        # the dominant kernel: the GEMM launch kind with the most time in the sampled micro-batch
        # (SmolLM-1.7B: the gate|up dX split-K halves + gate|up dW dual launch, ~24 % of the step);
        # its launches of every timed step
        if dom is None:
            labels = fam.by_label()
            dom = max(labels, key=lambda k: labels[k][1])
        d = fam.label_stats(dom)
        if dom_probe is not None and dom_probe.records:
            d2 = dom_probe.label_stats(dom)
            n = d["launches"] + d2["launches"]
            d = {"launches": n, "total_ms": d["total_ms"] + d2["total_ms"],
                 "avg_ms": (d["total_ms"] + d2["total_ms"]) / n,
                 "avg_flop": (d["avg_flop"] * d["launches"] + d2["avg_flop"] * d2["launches"]) / n,
                 "avg_alg_bytes": (d["avg_alg_bytes"] * d["launches"] + d2["avg_alg_bytes"] * d2["launches"]) / n}
        achieved = d["avg_flop"] / (d["avg_ms"] * 1e-3) / 1e12
        traffic, tsrc, tnote, pmc_key = None, None, "no PMC traffic file", pmc_kernel_key(dom)
        fam_traffic = None
        if os.path.exists(TRAFFIC_FILE):   # PMC-measured HBM bytes per launch (offline passes)
            with open(TRAFFIC_FILE) as f:
                tj = json.load(f)
            # only a measurement of THIS line's workload with THIS library build counts
            wl = {"model": model_name, "layers": layers, "micro_batch": args.mbs, "seq_len": args.seq,
                  "parallelism": f"dp{dp}" if tp * cp * pp == 1 and not force_dp else None}
            mine = _md5(K._C.LIB_PATH)
            if tj.get("workload") != wl:
                tnote = f"{os.path.relpath(TRAFFIC_FILE, ROOT)} measured another workload ({tj.get('workload')})"
            elif tj.get("library_md5") != mine:
                tnote = f"{os.path.relpath(TRAFFIC_FILE, ROOT)} measured another library build"
            elif pmc_key not in tj.get("kernels", {}):
                tnote = f"{os.path.relpath(TRAFFIC_FILE, ROOT)} has no entry {pmc_key!r}"
            else:
                traffic, tsrc, tnote = tj["kernels"][pmc_key]["avg_bytes"], os.path.relpath(TRAFFIC_FILE, ROOT), None
                fam_traffic = tj["gemm_avg_bytes_per_launch"]
        roofline = {"bound": "mfma", "kernel": f"{pmc_key} = {dom} (launches of micro-batch {probe_mb} of every "
                    "timed step)", "achieved": achieved,
                    "peak": MI355X_BF16_DENSE_PEAK / 1e12, "unit": "TFLOP/s",
                    "frac": achieved / (MI355X_BF16_DENSE_PEAK / 1e12), "traffic": traffic,
                    "traffic_unit": "bytes per launch", "traffic_source": tsrc, "traffic_note": tnote,
                    "algorithmic_bytes_per_launch": d["avg_alg_bytes"], "algorithmic_flop_per_launch": d["avg_flop"],
                    "launches": d["launches"], "avg_launch_ms": d["avg_ms"],
                    # of the GEMM time of the micro-batch the family was sampled in
                    "share_of_sampled_microbatch_gemm": fam.label_stats(dom)["total_ms"] / max(s["total_ms"], 1e-9),
                    # every bf16 MFMA GEMM launch of one micro-batch (rounds 1-5 reported this as the
                    # roofline), sampled in the last warm-up step
                    "gemm_family": {"sampled": "micro-batch %d of the first timed step" % probe_mb,
                                    "achieved": fam_achieved, "frac": fam_achieved / (MI355X_BF16_DENSE_PEAK / 1e12),
                                    "launches": s["launches"], "avg_launch_ms": s["avg_ms"],
                                    "avg_launch_gflop": s["avg_flop"] / 1e9,
                                    "algorithmic_bytes_per_launch": s["avg_alg_bytes"], "traffic": fam_traffic,
                                    "sampled_microbatch_gemm_ms": s["total_ms"],
                                    "by_launch_kind": {k: {"launches": v[0], "ms": v[1], "tflops": v[2]}
                                                       for k, v in fam.by_label().items()}}}

    cpu = None
    if rank == 0 and world == 1 and args.cpu_tokens > 0 and args.model == "smollm-1.7b":
        log("cpu baseline ...")
        cpu = cpu_baseline(cfg, args.cpu_tokens)

    if rank == 0:
        par = "-".join(f"{k}{v}" for k, v in (("dp", dp), ("tp", tp), ("cp", cp), ("pp", pp)) if v > 1 or k == "dp")
        if pp > 1:
            par += f"-{args.pp_engine}"
        out = {"metric": "tokens/s/GPU and MFU, SmolLM-1.7B seq1024 at 1/2/4/8 MI355X", "value": value,
               "unit": "tokens/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ranks": dist.get_world_size() if dist.is_initialized() else 1,
               "backend": dist.get_backend() if dist.is_initialized() else None,
               "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
               "scaling": "weak" if tp * cp * pp == 1 else "strong",
               "vs_baseline": None, "dtype": "bf16", "data": "synthetic (seeded uniform random tokens, a fresh batch every step; random init)",
               "tokens_per_s_per_gpu": per_gpu, "mfu": mfu, "flops_per_token": fpt, "num_params": num_params,
               "final_loss": losses[-1] if losses else None,
               "config": {"workload": f"{model_name} dims, {layers} layers, train step (fwd+bwd+AdamW)",
                          "model": model_name, "layers": layers, "micro_batch": args.mbs,
                          "grad_acc": args.grad_acc, "global_batch": args.mbs * args.grad_acc * dp,
                          "seq_len": args.seq, "parallelism": par + ("-bucket" if force_dp else ""),
                          "launch": "hip graph replay per micro-batch" if graphed is not None else "eager",
                          **({"bucket_mb": args.bucket_mb, "grad_type": args.grad_type}
                             if (m.cp_dp_world_size > 1 or force_dp) else {})},
               "roofline": roofline, "cpu_baseline": cpu}
        print(json.dumps(out), file=result_out, flush=True)
    if world > 1 or force_dp:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
