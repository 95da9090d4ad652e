"""Generate the golden vectors that pin the CPU oracle (oracle/picotron_oracle.py).

Run IN THE BUILD CONTAINER ONLY (the reference checkout is not on the GPU box):
    python tests/golden/make_golden.py  [--ref /root/reference]

It imports the reference's own modules from the read-only checkout and evaluates them on tiny
seeded inputs (CPU, FLASH_ATTEN=0, the reference's eager path).  flash_attn (requirements.txt:6)
is not installed, so its three import names are satisfied by empty placeholder modules -- only
FLASH_ATTEN=0 code runs.  Outputs are plain tensor dicts saved with torch.save and read back with
torch.load(weights_only=True).  No reference source is copied; only inputs/outputs are stored.
"""
import argparse
import math
import os
import sys
import types

import torch

OUT = os.path.dirname(os.path.abspath(__file__))


def _install_stubs():
    for name in ["flash_attn", "flash_attn.flash_attn_interface", "flash_attn.layers", "flash_attn.layers.rotary",
                 "flash_attn.ops", "flash_attn.ops.triton", "flash_attn.ops.triton.layer_norm"]:
        m = types.ModuleType(name)
        m.flash_attn_func = m.apply_rotary_emb = m.layer_norm_fn = None
        sys.modules[name] = m


def _fake_pgm(pgm_mod):
    pgm_mod.process_group_manager = types.SimpleNamespace(
        tp_world_size=1, tp_rank=0, cp_world_size=1, cp_rank=0, pp_world_size=1, pp_rank=0,
        dp_world_size=1, cp_dp_world_size=1, pp_is_first_stage=True, pp_is_last_stage=True)


# ---------------------------------------------------------------- multi-rank fixtures (gloo, CPU)
def _dist_worker(rank, world, port, ref, fn, out_dir):
    os.environ.update(DEVICE="cpu", LOCAL_RANK=str(rank), FLASH_ATTEN="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ref)
    _install_stubs()
    # the reference calls torch.cuda.synchronize() after every ring p2p (cp_comm.py:51); there is no
    # GPU here, and on CPU tensors gloo's wait() already completed the transfer (SURVEY.md §4 probe)
    torch.cuda.synchronize = lambda *a, **k: None
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = fn(rank, world)
        torch.save({k: (v.contiguous() if torch.is_tensor(v) else v) for k, v in res.items()},
                   os.path.join(out_dir, f"_part{rank}.pt"))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _run_dist(fn, world, ref, name):
    """Run fn(rank, world) -> dict on `world` gloo ranks; save {rank{r}.key: tensor} as <name>.pt."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    mp.spawn(_dist_worker, args=(world, port, ref, fn, OUT), nprocs=world, join=True)
    merged = {}
    for r in range(world):
        part = os.path.join(OUT, f"_part{r}.pt")
        for k, v in torch.load(part, weights_only=True).items():
            merged[f"rank{r}.{k}"] = v
        os.remove(part)
    torch.save(merged, os.path.join(OUT, f"{name}.pt"))


def g7_tensor_parallel(rank, world):
    """G7: the reference's own TP pin, tests/test_tensor_parallel.py:20-73, run on gloo/CPU at shapes
    the MFMA GEMM tiles (B 2, S 64, in 128, out 256; the test's own are 2 x 4 x 8 -> 16), bias=True,
    ColumnParallelLinear(gather_output=True) with and without async_all_reduce, RowParallelLinear,
    and VocabParallelEmbedding (tensor_parallel.py:191-270) -- all against a dense layer."""
    from picotron.process_group_manager import setup_process_group_manager
    from picotron.tensor_parallel.tensor_parallel import (ColumnParallelLinear, RowParallelLinear,
                                                          VocabParallelEmbedding)
    setup_process_group_manager(tp_size=world, cp_size=1, pp_size=1, dp_size=1)
    torch.manual_seed(42)
    B, S, IN, OUT_ = 2, 64, 128, 256
    res = {}
    for async_ar in (False, True):
        x = torch.randn(B, S, IN, requires_grad=True)
        xc = x.clone().detach().requires_grad_(True)
        xr = x.clone().chunk(world, dim=-1)[rank].detach().requires_grad_(True)
        col = ColumnParallelLinear(IN, OUT_, bias=True, gather_output=True, async_all_reduce=async_ar)
        row = RowParallelLinear(IN, OUT_, bias=True)
        dense = torch.nn.Linear(IN, OUT_, bias=True)
        col.weight = torch.nn.Parameter(dense.weight.chunk(world, dim=0)[rank])
        row.weight = torch.nn.Parameter(dense.weight.chunk(world, dim=1)[rank])
        col.bias = torch.nn.Parameter(dense.bias.chunk(world, dim=0)[rank])
        row.bias = torch.nn.Parameter(dense.bias)
        y, yc, yr = dense(x), col(xc), row(xr)
        y.backward(torch.ones_like(y))
        yc.backward(torch.ones_like(yc))
        yr.backward(torch.ones_like(yr))
        t = "async." if async_ar else ""
        res.update({t + "x": x.detach(), t + "dense_w": dense.weight.detach(), t + "dense_b": dense.bias.detach(),
                    t + "y_dense": y.detach(), t + "y_col": yc.detach(), t + "y_row": yr.detach(),
                    t + "dx_dense": x.grad, t + "dx_col": xc.grad, t + "dx_row": xr.grad,
                    t + "dw_col": col.weight.grad, t + "db_col": col.bias.grad,
                    t + "dw_row": row.weight.grad, t + "db_row": row.bias.grad,
                    t + "dw_dense": dense.weight.grad, t + "db_dense": dense.bias.grad})
    V, H = 512, 128
    emb = VocabParallelEmbedding(V, H)
    ids = torch.randint(0, V, (2, 64))
    ye = emb(ids)
    dye = torch.randn(ye.shape)
    ye.backward(dye)
    res.update(emb_ids=ids, emb_w=emb.weight.detach(), emb_y=ye.detach(), emb_dy=dye, emb_dw=emb.weight.grad,
               emb_lo=torch.tensor(emb.vocab_start_index), emb_hi=torch.tensor(emb.vocab_end_index))
    return res


G8_CFG = dict(hidden_size=128, intermediate_size=256, num_attention_heads=2, num_key_value_heads=2,
              rms_norm_eps=1e-5, max_position_embeddings=128, rope_theta=10000.0, vocab_size=256,
              num_hidden_layers=2)


def g8_data_parallel(rank, world):
    """G8: DataParallelBucket (data_parallel.py:62-170, bucket.py) at dp=2 over the reference's tiny
    Llama (FLASH_ATTEN=0, fp32): grad_acc 2, sync on the last micro-batch only (train.py:39-41), each
    rank its own tokens; the averaged p.grad (= main_grad after _post_backward) per rank."""
    import torch.nn.functional as F
    from picotron.process_group_manager import setup_process_group_manager
    setup_process_group_manager(tp_size=1, cp_size=1, pp_size=1, dp_size=world)
    from picotron import model as M
    from picotron.data_parallel.data_parallel import DataParallelBucket
    cfg = types.SimpleNamespace(**G8_CFG)
    torch.manual_seed(7)
    llama = M.Llama(cfg)
    for layer in llama.decoder_layers:
        layer.cos, layer.sin = layer.cos.float(), layer.sin.float()
    init = {n: p.detach().clone() for n, p in llama.named_parameters()}
    dp = DataParallelBucket(llama)
    g = torch.Generator().manual_seed(99)
    ids = torch.randint(0, cfg.vocab_size, (world, 2, 2, 129), generator=g)   # [dp, ga, mbs, seq+1]
    ga = 2
    for i in range(ga):
        dp.require_backward_grad_sync = (i == ga - 1)
        t = ids[rank, i]
        lo = dp(input_ids=t[:, :-1])
        loss = F.cross_entropy(lo.reshape(-1, cfg.vocab_size), t[:, 1:].reshape(-1)) / ga
        loss.backward()
    res = {"ids": ids}
    res.update({f"param.{n}": v for n, v in init.items()})
    res.update({f"grad.{n}": p.grad.detach().clone() for n, p in llama.named_parameters()})
    return res


G10M_CFG = dict(hidden_size=128, intermediate_size=256, num_attention_heads=2, num_key_value_heads=2,
                rms_norm_eps=1e-5, max_position_embeddings=256, rope_theta=10000.0, vocab_size=256,
                num_hidden_layers=2)
G10M_STEPS, G10M_GA, G10M_MBS, G10M_LR = 4, 2, 2, 1e-2


def _g10m_data():
    """[steps, dp 2, ga, mbs, seq + 1] tokens shared by every topology (seed 1234): the same batch
    every step, so the loss curve falls steeply (memorisation) and a 1 % bar separates real
    training from a broken update."""
    g = torch.Generator().manual_seed(1234)
    S = G10M_CFG["max_position_embeddings"]
    one = torch.randint(0, G10M_CFG["vocab_size"], (1, 2, G10M_GA, G10M_MBS, S + 1), generator=g)
    return one.expand(G10M_STEPS, -1, -1, -1, -1).contiguous()


def _g10m_shard(full, local, rank):
    if full.shape == local.shape:
        return full
    (d,) = [i for i, (a, b) in enumerate(zip(full.shape, local.shape)) if a != b]
    n = local.shape[d]
    return full.narrow(d, rank * n, n)


def g10m_multirank(rank, world, tp, cp, dp):
    """G10 multi-rank: train.py's loop (train_step 29-55, the step loop 232-249) run by the reference
    itself on gloo/CPU, fp32, FLASH_ATTEN=0, at tp / cp / dp = 2: G10M_STEPS AdamW steps (lr 1e-2,
    torch defaults), grad_acc 2, mbs 2, seq 256 (each cp rank its contiguous half, data.py:105-109);
    every topology starts from the SAME full weights (one tp=1 init, seed 7, sharded as
    apply_tensor_parallel shards).  DataParallelBucket wraps the model only when dp > 1, as
    train.py:194-195 does (so at cp 2 / dp 1 the two cp ranks' replicas train on their own
    gradients, the reference's behaviour).  Records the logged loss per step
    (average_loss_across_dp_cp_ranks, utils.py:93-98) and the full initial weights (rank 0)."""
    import torch.nn.functional as F
    import picotron.process_group_manager as pgm
    pgm.setup_process_group_manager(tp_size=tp, cp_size=cp, pp_size=1, dp_size=dp)
    m = pgm.process_group_manager
    from picotron import model as M
    from picotron.context_parallel.context_parallel import apply_context_parallel
    from picotron.data_parallel.data_parallel import DataParallelBucket
    from picotron.tensor_parallel.tensor_parallel import apply_tensor_parallel
    from picotron.utils import average_loss_across_dp_cp_ranks
    cfg = types.SimpleNamespace(**G10M_CFG)
    torch.manual_seed(7)
    model = M.Llama(cfg)
    full = {n: p.detach().clone() for n, p in model.named_parameters()}
    if tp > 1:
        model = apply_tensor_parallel(model)
    if cp > 1:
        model = apply_context_parallel(model)
    for layer in model.decoder_layers:
        layer.cos, layer.sin = layer.cos.float(), layer.sin.float()
    with torch.no_grad():
        for n, p in model.named_parameters():
            p.copy_(_g10m_shard(full[n], p, m.tp_rank))
    if dp > 1:
        model = DataParallelBucket(model)
    opt = torch.optim.AdamW(model.parameters(), lr=G10M_LR)
    ids = _g10m_data()
    S, V = G10M_CFG["max_position_embeddings"], G10M_CFG["vocab_size"]
    sl = slice(m.cp_rank * S // cp, (m.cp_rank + 1) * S // cp)
    losses = []
    for step in range(G10M_STEPS):
        opt.zero_grad()
        acc = 0.0
        for i in range(G10M_GA):
            if m.cp_dp_world_size > 1:
                model.require_backward_grad_sync = (i == G10M_GA - 1)
            t = ids[step, m.dp_rank, i]
            x, y = t[:, :-1][:, sl].contiguous(), t[:, 1:][:, sl].contiguous()
            out = model(input_ids=x)
            loss = F.cross_entropy(out.reshape(-1, V), y.reshape(-1), reduction="mean") / G10M_GA
            loss.backward()
            acc += loss.item()
        losses.append(average_loss_across_dp_cp_ranks(acc, "cpu"))
        opt.step()
        if hasattr(model, "reset"):
            model.reset()
    res = {"losses": torch.tensor(losses, dtype=torch.float64)}
    if rank == 0:
        res.update({f"param.{n}": v for n, v in full.items()})
    return res


def g10m_pipeline(rank, world, engine):
    """G10m at pp = world (BASELINE config 4's composition): the reference's PipelineParallel stages
    (pipeline_parallel.py:8-75) trained by its own 1F1B / AFAB step (:77-214) on gloo/CPU, fp32,
    FLASH_ATTEN=0, from the same full weights (seed 7) re-applied after the stage re-draws its
    parameters, the G10m batch every step, G10M_STEPS AdamW steps at lr 1e-2.  Records the last
    stage's logged loss per step (the engine's loss: each micro-batch's mean CE, not divided by
    grad_acc) and the full initial weights (rank 0)."""
    import picotron.process_group_manager as pgm
    pgm.setup_process_group_manager(tp_size=1, cp_size=1, pp_size=world, dp_size=1)
    m = pgm.process_group_manager
    from picotron import model as M
    from picotron.pipeline_parallel import pipeline_parallel as PP
    cfg = types.SimpleNamespace(**G10M_CFG)
    torch.manual_seed(7)
    full_model = M.Llama(cfg)
    full = {n: p.detach().clone() for n, p in full_model.named_parameters()}
    model = PP.PipelineParallel(full_model, cfg)
    for layer in model.decoder_layers.values():
        layer.cos, layer.sin = layer.cos.float(), layer.sin.float()
    with torch.no_grad():
        for n, p in model.named_parameters():
            p.copy_(full[n])
    opt = torch.optim.AdamW(model.parameters(), lr=G10M_LR)
    ids = _g10m_data()
    S = G10M_CFG["max_position_embeddings"]
    step_fn = PP.train_step_pipeline_1f1b if engine == "1f1b" else PP.train_step_pipeline_afab

    class Loader:
        grad_acc_steps = G10M_GA

        def __init__(self, step):
            self.step, self.i = step, 0

        def __next__(self):
            t = ids[self.step, 0, self.i]
            self.i += 1
            return {"input_ids": t[:, :-1], "target_ids": t[:, 1:],
                    "position_ids": torch.arange(S).expand(G10M_MBS, S), "hidden_states": None}
    losses = []
    for step in range(G10M_STEPS):
        opt.zero_grad()
        loss = step_fn(model, Loader(step), (G10M_MBS, S, G10M_CFG["hidden_size"]), "cpu", torch.float32)
        losses.append(loss if m.pp_is_last_stage else 0.0)
        opt.step()
    res = {"losses": torch.tensor(losses, dtype=torch.float64)}
    if rank == 0:
        res.update({f"param.{n}": v for n, v in full.items()})
    return res


# ---------------------------------------------------------------- G12: BASELINE configs 1 / 4's grid
# dp2 tp2 pp2 1F1B on 8 gloo processes -- the reference's README CPU command (README.md:43) at
# config 1's shape: 5 layers, mbs 4, seq 128, grad_acc 2.  Two model sizes:
#   "tiny":    G10m's dims (H 128), 6 AdamW steps at lr 1e-2 (a steep, sensitive curve);
#   "smollm":  SmolLM-1.7B's own dims (H 2048, I 8192, 32 heads, V 49152), 4 steps at lr 1e-4, in the
#              reference's GPU training precision (bf16 model and AdamW states, train.py:76,190): at
#              lr 1e-4 an update is about one bf16 ulp of these weights, so the precision, not the
#              implementation, would set a bf16-vs-fp32 gap (G11's reason for its bf16 curves).
# The weights are not stored: every full parameter is drawn by `g12_full_param` from a generator
# seeded by the parameter's name, so both sides materialise the same full model (then shard it as
# apply_tensor_parallel shards and keep their pipeline stage's slice) without a 2 GB fixture.
G12_CFGS = {
    "tiny": dict(G10M_CFG, num_hidden_layers=5, max_position_embeddings=128),
    "smollm": dict(hidden_size=2048, intermediate_size=8192, num_attention_heads=32, num_key_value_heads=32,
                   rms_norm_eps=1e-5, max_position_embeddings=128, rope_theta=10000.0, vocab_size=49152,
                   num_hidden_layers=5),
}
# "smollm_f32": the same run at config 1's literal precision (the README's --use_cpu path trains in
# fp32) -- G12f32_smollm, which records the bf16-vs-fp32 gap as G11f32_* does for G11
G12_CFGS["smollm_f32"] = G12_CFGS["smollm"]
G12_RUN = {"tiny": dict(steps=6, lr=1e-2, dtype="f32"), "smollm": dict(steps=4, lr=1e-4, dtype="bf16"),
           "smollm_f32": dict(steps=4, lr=1e-4, dtype="f32")}
G12_NAMES = {"tiny": "G12_tiny", "smollm": "G12_smollm", "smollm_f32": "G12f32_smollm"}
G12_GA, G12_MBS = 2, 4


def g12_full_param(name, shape):
    """Deterministic full (unsharded) parameter `name` of G12's model: norms ones
    (model.py:48-49,78-79), linears U(+-1/sqrt(fan_in)) (model.py:110-118,173-181), the embedding
    N(0, 1) (model.py:221-222) -- the reference's init distributions, each from torch.Generator
    seeded with crc32(name) instead of the global RNG order (which changes with TP / PP)."""
    import zlib
    g = torch.Generator().manual_seed(zlib.crc32(name.encode()))
    if name.endswith("norm.weight"):
        return torch.ones(shape)
    if name.startswith("embedding"):
        return torch.randn(shape, generator=g)
    b = 1.0 / math.sqrt(shape[1])
    return torch.rand(shape, generator=g) * (2 * b) - b


def g12_tokens(V, S, dp=2):
    """[dp, ga, mbs, S + 1] tokens (seed 1234), the same batch every step."""
    g = torch.Generator().manual_seed(1234)
    return torch.randint(0, V, (dp, G12_GA, G12_MBS, S + 1), generator=g)


def g12_grid(rank, world, size):
    """G12: the reference's own train.py composition for configs 1 / 4 (train.py:174-195: Llama ->
    apply_tensor_parallel -> PipelineParallel -> weights -> DataParallelBucket) trained by its
    train_step_pipeline_1f1b (pipeline_parallel.py:124-214) on 8 gloo CPU processes at
    dp2 tp2 pp2, fp32 (tiny) or bf16 (smollm), FLASH_ATTEN=0, AdamW (torch defaults); records the logged loss of every step
    (train.py:228: average_loss_across_dp_cp_ranks of the last stage's loss) on every rank."""
    import picotron.process_group_manager as pgm
    torch.set_num_threads(1)
    pgm.setup_process_group_manager(tp_size=2, cp_size=1, pp_size=2, dp_size=2)
    m = pgm.process_group_manager
    from picotron import model as M
    from picotron.data_parallel.data_parallel import DataParallelBucket
    from picotron.pipeline_parallel import pipeline_parallel as PP
    from picotron.tensor_parallel.tensor_parallel import apply_tensor_parallel
    from picotron.utils import average_loss_across_dp_cp_ranks
    c = G12_CFGS[size]
    dtype = torch.bfloat16 if G12_RUN[size]["dtype"] == "bf16" else torch.float32
    cfg = types.SimpleNamespace(**c)
    torch.manual_seed(7)
    model = PP.PipelineParallel(apply_tensor_parallel(M.Llama(cfg)), cfg)
    for layer in model.decoder_layers.values():
        layer.cos, layer.sin = layer.cos.to(dtype), layer.sin.to(dtype)
    with torch.no_grad():
        for n, p in model.named_parameters():
            full = g12_full_param(n, _g12_full_shape(n, p, c))
            p.copy_(_g10m_shard(full, p, m.tp_rank))
    model = DataParallelBucket(model.to(dtype))   # train.py:190, 194-195
    opt = torch.optim.AdamW(model.parameters(), lr=G12_RUN[size]["lr"])
    S, V = c["max_position_embeddings"], c["vocab_size"]
    ids = g12_tokens(V, S)

    class Loader:
        grad_acc_steps, micro_batch_size, seq_length_per_gpu = G12_GA, G12_MBS, S

        def __init__(self):
            self.i = 0

        def __next__(self):
            t = ids[m.dp_rank, self.i]
            self.i += 1
            return {"input_ids": t[:, :-1], "target_ids": t[:, 1:],
                    "position_ids": torch.arange(S).expand(G12_MBS, S), "hidden_states": None}
    losses = []
    for _ in range(G12_RUN[size]["steps"]):
        opt.zero_grad()
        loss = PP.train_step_pipeline_1f1b(model, Loader(), (G12_MBS, S, c["hidden_size"]), "cpu", dtype)
        losses.append(average_loss_across_dp_cp_ranks(loss, "cpu"))
        opt.step()
        model.reset()
    return {"losses": torch.tensor(losses, dtype=torch.float64),
            "grid": torch.tensor([m.dp_rank, m.pp_rank, m.cp_rank, m.tp_rank])}


def _g12_full_shape(name, p, c):
    """The unsharded shape of parameter `name` (TP shards dim 0 of column / vocab, dim 1 of row)."""
    H, I, V = c["hidden_size"], c["intermediate_size"], c["vocab_size"]
    d = H // c["num_attention_heads"]
    kv = c["num_key_value_heads"] * d
    tail = name.split(".")[-2]
    return {"q_proj": (H, H), "k_proj": (kv, H), "v_proj": (kv, H), "out_proj": (H, H), "gate_proj": (I, H),
            "up_proj": (I, H), "down_proj": (H, I), "embedding": (V, H), "final_proj": (V, H)}.get(tail, tuple(p.shape))


def g12_all(ref, sizes=("tiny", "smollm", "smollm_f32")):
    import functools
    for size in sizes:
        _run_dist(functools.partial(g12_grid, size=size), 8, ref, G12_NAMES[size])


G11_STEPS, G11_GA, G11_MBS, G11_LR = 50, 2, 2, 1e-3


def _g11_data(seq=None):
    """[steps, dp 2, ga, mbs, seq + 1] uint8 tokens (seed 2468): a FRESH batch every step, drawn from
    a fixed sparse bigram process (each token has 4 successors with probabilities .55 / .25 / .15 /
    .05, about 1.1 nats of entropy) -- learnable structure, so the 50-step loss falls from ln 256 =
    5.5 towards ~1.1 like a real run instead of memorising one batch."""
    g = torch.Generator().manual_seed(2468)
    V, S = G10M_CFG["vocab_size"], seq or G10M_CFG["max_position_embeddings"]
    succ = torch.randint(0, V, (V, 4), generator=g)
    n = G11_STEPS * 2 * G11_GA * G11_MBS
    choice = torch.multinomial(torch.tensor([0.55, 0.25, 0.15, 0.05]).expand(n, 4), S, replacement=True,
                               generator=g)
    seq = torch.empty(n, S + 1, dtype=torch.long)
    seq[:, 0] = torch.randint(0, V, (n,), generator=g)
    for t in range(S):
        seq[:, t + 1] = succ[seq[:, t], choice[:, t]]
    return seq.view(G11_STEPS, 2, G11_GA, G11_MBS, S + 1).to(torch.uint8)


def g11_curve(rank, world, tp, cp, dp, dtype=torch.bfloat16, seq=None, avg=False):
    """G11: north_star's "loss curve within 1 % over 50 steps", pinned by the reference itself:
    train.py's loop (train_step 29-55, the step loop 219-240) on gloo/CPU, FLASH_ATTEN=0, in the
    reference's GPU training precision (train.py:76,190: the model and so AdamW's states in bf16,
    cos/sin in bf16 as get_cos_sin makes them; G11f32_*: the same run in fp32), for
    G11_STEPS AdamW steps (lr G11_LR, torch defaults), grad_acc 2, mbs 2, seq 256, a fresh bigram
    batch every step (_g11_data), at 1 rank and at tp / cp / dp = 2.  Same model and initial weights
    as G10m (one tp=1 init, seed 7, sharded as apply_tensor_parallel shards); DataParallelBucket only
    for dp > 1 (train.py:194-195).  Records the logged loss per step (utils.py:93-98) and the
    token stream (rank 0; the initial weights are G10m's: rank0.param.* of G10m_tp2.pt)."""
    import torch.nn.functional as F
    import picotron.process_group_manager as pgm
    pgm.setup_process_group_manager(tp_size=tp, cp_size=cp, pp_size=1, dp_size=dp)
    m = pgm.process_group_manager
    from picotron import model as M
    from picotron.context_parallel.context_parallel import apply_context_parallel
    from picotron.data_parallel.data_parallel import DataParallelBucket
    from picotron.tensor_parallel.tensor_parallel import apply_tensor_parallel
    from picotron.utils import average_loss_across_dp_cp_ranks
    cfg = types.SimpleNamespace(**dict(G10M_CFG, max_position_embeddings=seq or G10M_CFG["max_position_embeddings"]))
    torch.set_num_threads(max(1, 8 // world))
    torch.manual_seed(7)
    model = M.Llama(cfg)
    full = {n: p.detach().clone() for n, p in model.named_parameters()}
    if tp > 1:
        model = apply_tensor_parallel(model)
    if cp > 1:
        model = apply_context_parallel(model)
    for layer in model.decoder_layers:
        layer.cos, layer.sin = layer.cos.to(dtype), layer.sin.to(dtype)
    with torch.no_grad():
        for n, p in model.named_parameters():
            p.copy_(_g10m_shard(full[n], p, m.tp_rank))
    model = model.to(dtype)            # train.py:190
    if dp > 1 or avg:                  # avg: the reference's own DataParallelBucket over cp_dp at dp 1
        model = DataParallelBucket(model)
    opt = torch.optim.AdamW(model.parameters(), lr=G11_LR)
    ids = _g11_data(seq)
    S, V = cfg.max_position_embeddings, G10M_CFG["vocab_size"]
    sl = slice(m.cp_rank * S // cp, (m.cp_rank + 1) * S // cp)
    losses = []
    for step in range(G11_STEPS):
        opt.zero_grad()
        acc = 0.0
        for i in range(G11_GA):
            if m.cp_dp_world_size > 1:
                model.require_backward_grad_sync = (i == G11_GA - 1)
            t = ids[step, m.dp_rank, i].long()
            x, y = t[:, :-1][:, sl].contiguous(), t[:, 1:][:, sl].contiguous()
            out = model(input_ids=x)
            loss = F.cross_entropy(out.reshape(-1, V), y.reshape(-1), reduction="mean") / G11_GA
            loss.backward()
            acc += loss.item()
        losses.append(average_loss_across_dp_cp_ranks(acc, "cpu") if world > 1 else acc)
        opt.step()
        if hasattr(model, "reset"):
            model.reset()
    res = {"losses": torch.tensor(losses, dtype=torch.float64)}
    if rank == 0:
        res["ids"] = ids
    return res


def g10m_pp_all(ref):
    import functools
    _run_dist(functools.partial(g10m_pipeline, engine="1f1b"), 2, ref, "G10m_pp2")
    _run_dist(functools.partial(g10m_pipeline, engine="afab"), 2, ref, "G10m_pp2afab")


def g11_all(ref, dtypes=("bf16", "f32")):
    import functools
    # cp2 at seq 512: 256 tokens per rank, the shard length from which the build runs its zig-zag
    # (load-balanced) ring with the zig-zag residual layout -- that schedule against the reference
    _run_dist(functools.partial(g11_curve, tp=1, cp=2, dp=1, dtype=torch.bfloat16, seq=512), 2, ref, "G11_cp2s512")
    # ... and with the cp ranks' gradients averaged (the reference's DataParallelBucket over cp_dp_group,
    # which its train.py applies only for dp > 1): the build then keeps its residual stream zig-zag
    _run_dist(functools.partial(g11_curve, tp=1, cp=2, dp=1, dtype=torch.bfloat16, seq=512, avg=True), 2, ref,
              "G11_cp2s512avg")
    for tag in dtypes:
        dt = torch.bfloat16 if tag == "bf16" else torch.float32
        for name, (tp, cp, dp) in (("1", (1, 1, 1)), ("tp2", (2, 1, 1)), ("cp2", (1, 2, 1)), ("dp2", (1, 1, 2))):
            _run_dist(functools.partial(g11_curve, tp=tp, cp=cp, dp=dp, dtype=dt), tp * cp * dp, ref,
                      f"G11_{name}" if tag == "bf16" else f"G11f32_{name}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", choices=["G11", "G11bf16", "G11s512", "G10m_pp", "G12", "G12f32"],
                    help="regenerate only these fixtures")
    args = ap.parse_args()
    if args.only == "G11s512":
        import functools
        _run_dist(functools.partial(g11_curve, tp=1, cp=2, dp=1, dtype=torch.bfloat16, seq=512), 2, args.ref,
                  "G11_cp2s512")
        _run_dist(functools.partial(g11_curve, tp=1, cp=2, dp=1, dtype=torch.bfloat16, seq=512, avg=True), 2,
                  args.ref, "G11_cp2s512avg")
        print("wrote G11_cp2s512, G11_cp2s512avg")
        return
    if args.only == "G12":
        g12_all(args.ref)
        print("wrote G12 fixtures")
        return
    if args.only == "G12f32":
        g12_all(args.ref, ("smollm_f32",))
        print("wrote G12f32_smollm")
        return
    if args.only == "G10m_pp":
        g10m_pp_all(args.ref)
        print("wrote G10m_pp fixtures")
        return
    if args.only:
        g11_all(args.ref, ("bf16",) if args.only == "G11bf16" else ("bf16", "f32"))
        print("wrote G11 fixtures")
        return
    os.environ.update(DEVICE="cpu", LOCAL_RANK="0", FLASH_ATTEN="0")
    sys.path.insert(0, args.ref)
    _install_stubs()
    import picotron.process_group_manager as pgm
    _fake_pgm(pgm)
    from picotron import model as M
    from picotron.context_parallel import context_parallel as CP

    g = torch.Generator().manual_seed(1234)
    gold = {}

    # G1: LlamaRMSNorm fwd/bwd (fp32 and bf16)
    for dt in (torch.float32, torch.bfloat16):
        tag = "f32" if dt == torch.float32 else "bf16"
        x = torch.randn(6, 64, generator=g).to(dt).requires_grad_(True)
        norm = M.LlamaRMSNorm(64, eps=1e-5)
        with torch.no_grad():
            norm.weight.copy_(1 + 0.1 * torch.randn(64, generator=g))
        norm = norm.to(dt)
        y = norm(x)
        dy = torch.randn(y.shape, generator=g).to(dt)
        y.backward(dy)
        gold[f"G1_{tag}"] = dict(x=x.detach(), w=norm.weight.detach(), eps=torch.tensor(1e-5), y=y.detach(), dy=dy,
                                 dx=x.grad.detach(), dw=norm.weight.grad.detach())

    # G2: get_cos_sin + apply_rotary_pos_emb fwd/bwd, [B, H, S, D]
    cos, sin = M.get_cos_sin(16, 32, base=10000.0)
    x = torch.randn(2, 3, 16, 32, generator=g, requires_grad=True)
    y = M.apply_rotary_pos_emb(x, cos.float(), sin.float())
    dy = torch.randn(y.shape, generator=g)
    y.backward(dy)
    gold["G2"] = dict(cos=cos, sin=sin, x=x.detach(), y=y.detach(), dy=dy, dx=x.grad.detach(), base=torch.tensor(1e4))
    cos5, sin5 = M.get_cos_sin(64, 128, base=500000.0)
    gold["G2_tables"] = dict(cos_16_32=cos, sin_16_32=sin, cos_64_128_default=cos5, sin_64_128_default=sin5)

    # tiny config shared by G3/G5/G6
    cfg = types.SimpleNamespace(hidden_size=64, intermediate_size=128, num_attention_heads=4, num_key_value_heads=2,
                                rms_norm_eps=1e-5, max_position_embeddings=16, rope_theta=10000.0, vocab_size=96,
                                num_hidden_layers=2)
    torch.manual_seed(42)

    # G3: Attention fwd/bwd (SDPA path, GQA 4/2)
    att = M.Attention(cfg, layer_idx=0)
    cos, sin = M.get_cos_sin(16, 16, base=10000.0)
    x = torch.randn(2, 16, 64, generator=g, requires_grad=True)
    y = att(x, cos.float(), sin.float())
    dy = torch.randn(y.shape, generator=g)
    y.backward(dy)
    gold["G3"] = dict(x=x.detach(), y=y.detach(), dy=dy, dx=x.grad.detach(), cos=cos, sin=sin,
                      **{f"{n}": p.detach() for n, p in att.named_parameters()},
                      **{f"grad.{n}": p.grad.detach() for n, p in att.named_parameters()})

    # G4: ring pure functions (fp32 and bf16 -- bf16 keeps the reference's bf16 LSE)
    for dt in (torch.float32, torch.bfloat16):
        tag = "f32" if dt == torch.float32 else "bf16"
        q, k, v = (torch.randn(1, 2, 8, 16, generator=g).to(dt) for _ in range(3))
        sc = 1 / math.sqrt(16)
        o_c, l_c = CP.ring_attention_forward(q, k, v, sc, True)
        o_f, l_f = CP.ring_attention_forward(q, k, v, sc, False)
        out, lse = CP.update_out_and_lse(None, None, o_c, l_c)
        out, lse = CP.update_out_and_lse(out, lse, o_f, l_f)
        dO = torch.randn(q.shape, generator=g).to(dt)
        dq, dk, dv = CP.ring_attention_backward(dO, q, k, v, out.to(dt), lse.squeeze(-1), sc, True)
        gold[f"G4_{tag}"] = dict(q=q, k=k, v=v, o_causal=o_c, lse_causal=l_c, o_full=o_f, lse_full=l_f,
                                 merged_out=out, merged_lse=lse, dO=dO, dq=dq, dk=dk, dv=dv)

    # G4b: one ring step of rank 1 at a shape the flash kernels tile ([1, 2, 128, 64]): the causal
    # diagonal block, then the full block of rank 0's K/V, merged by update_out_and_lse -- in bf16
    # (the reference's bf16 LSE) and in f32 from the SAME bf16-representable inputs
    g4 = torch.Generator().manual_seed(4242)   # its own stream: the later fixtures stay as they were
    base = [torch.randn(1, 2, 128, 64, generator=g4).to(torch.bfloat16) for _ in range(5)]
    for dt in (torch.float32, torch.bfloat16):
        tag = "f32" if dt == torch.float32 else "bf16"
        q1, k0, v0, k1, v1 = (t.to(dt) for t in base)
        sc = 1 / math.sqrt(64)
        o_c, l_c = CP.ring_attention_forward(q1, k1, v1, sc, True)
        o_f, l_f = CP.ring_attention_forward(q1, k0, v0, sc, False)
        out, lse = CP.update_out_and_lse(None, None, o_c, l_c)
        out, lse = CP.update_out_and_lse(out, lse, o_f, l_f)
        gold[f"G4b_{tag}"] = dict(q1=q1, k0=k0, v0=v0, k1=k1, v1=v1, out=out, lse=lse)

    # G5: MLP fwd/bwd
    mlp = M.MLP(cfg)
    x = torch.randn(2, 5, 64, generator=g, requires_grad=True)
    y = mlp(x)
    dy = torch.randn(y.shape, generator=g)
    y.backward(dy)
    gold["G5"] = dict(x=x.detach(), y=y.detach(), dy=dy, dx=x.grad.detach(),
                      **{n: p.detach() for n, p in mlp.named_parameters()},
                      **{f"grad.{n}": p.grad.detach() for n, p in mlp.named_parameters()})

    # G6: DecoderLayer fwd/bwd
    layer = M.DecoderLayer(cfg, layer_idx=0)
    x = torch.randn(2, 16, 64, generator=g, requires_grad=True)
    layer.cos, layer.sin = layer.cos.float(), layer.sin.float()
    y = layer(x)
    dy = torch.randn(y.shape, generator=g)
    y.backward(dy)
    gold["G6"] = dict(x=x.detach(), y=y.detach(), dy=dy, dx=x.grad.detach(), cos=layer.cos, sin=layer.sin,
                      **{n: p.detach() for n, p in layer.named_parameters()},
                      **{f"grad.{n}": p.grad.detach() for n, p in layer.named_parameters()})

    # G9: cross entropy on bf16 logits / grad_acc (train.py:46-49)
    logits = torch.randn(2, 8, 96, generator=g).to(torch.bfloat16).requires_grad_(True)
    tgt = torch.randint(0, 96, (2, 8), generator=g)
    loss = torch.nn.functional.cross_entropy(logits.view(16, -1), tgt.reshape(-1), reduction="mean") / 4
    loss.backward()
    gold["G9"] = dict(logits=logits.detach(), targets=tgt, loss=loss.detach(), dlogits=logits.grad.detach(),
                      grad_acc=torch.tensor(4))

    # G10: tiny Llama forward + CE loss (single rank), weights from the reference's own init
    torch.manual_seed(7)
    llama = M.Llama(cfg)
    for layer in llama.decoder_layers:
        layer.cos, layer.sin = layer.cos.float(), layer.sin.float()
    ids = torch.randint(0, 96, (2, 17), generator=g)
    logits = llama(ids[:, :-1])
    loss = torch.nn.functional.cross_entropy(logits.reshape(-1, 96), ids[:, 1:].reshape(-1))
    loss.backward()
    gold["G10"] = dict(ids=ids, logits=logits.detach(), loss=loss.detach(),
                       **{f"param.{n}": p.detach() for n, p in llama.named_parameters()},
                       **{f"grad.{n}": p.grad.detach() for n, p in llama.named_parameters()})

    for name, d in gold.items():
        torch.save({k: (v.contiguous() if torch.is_tensor(v) else v) for k, v in d.items()},
                   os.path.join(OUT, f"{name}.pt"))
    _run_dist(g7_tensor_parallel, 2, args.ref, "G7")
    _run_dist(g8_data_parallel, 2, args.ref, "G8")
    import functools
    for name, (tp, cp, dp) in (("G10m_tp2", (2, 1, 1)), ("G10m_cp2", (1, 2, 1)), ("G10m_dp2", (1, 1, 2))):
        _run_dist(functools.partial(g10m_multirank, tp=tp, cp=cp, dp=dp), 2, args.ref, name)
    g10m_pp_all(args.ref)
    g11_all(args.ref)
    g12_all(args.ref)
    print("wrote", sorted(gold) + ["G7", "G8", "G10m_tp2", "G10m_cp2", "G10m_dp2", "G10m_pp2*", "G11_*", "G11f32_*",
                                   "G12_*"])


if __name__ == "__main__":
    main()
