"""The reference-pinned multi-rank fixtures on the GPU path (HIP kernels through the C ABI, two ranks
on cuda:0 over gloo -- tests/_dist.py):

  * G7 -- the reference's own TP test (tests/test_tensor_parallel.py:42-73): ColumnParallelLinear
    (gather_output=True, bias, with and without async_all_reduce), RowParallelLinear (bias) and
    VocabParallelEmbedding forward AND backward through the MFMA GEMM / embedding kernels against
    the reference's dense-layer outputs and gradients;
  * G8 -- DataParallelBucket's averaged gradients (data_parallel.py:62-170) at dp=2, grad_acc 2, plus
    the same contract through DataParallelNaive and through a bf16 bucket (grad_type knob);
  * G10m -- the reference's own multi-rank training loss curves (train.py's loop) at tp2, cp2, dp2.

Tolerance: norm-relative 2e-2 (north_star's bf16 tolerance) against the fp32 fixtures, stated per
assertion; bit-exact where the reference asserts equality (Column-gathered == dense, both on the
same GEMM).  The fixtures are generated from the reference by tests/golden/make_golden.py."""
import os
import types

import pytest
import torch

from tests import _dist

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
TOL = 2e-2
BF = torch.bfloat16


def _rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def _tp_modules(rank, world):
    os.environ["FLASH_ATTEN"] = "1"
    torch.cuda.set_device(0)
    from picotron_amd import functional as FN
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.tensor_parallel.tensor_parallel import (ColumnParallelLinear, RowParallelLinear,
                                                               VocabParallelEmbedding)
    pgm.setup_process_group_manager(tp_size=world, cp_size=1, pp_size=1, dp_size=1)
    g = torch.load(os.path.join(GOLD, "G7.pt"), weights_only=True)
    P = f"rank{rank}."
    dev = torch.device("cuda", 0)
    for t, async_ar in (("", False), ("async.", True)):
        x = g[P + t + "x"].to(dev, BF)
        w, b = g[P + t + "dense_w"].to(dev, BF), g[P + t + "dense_b"].to(dev, BF)
        out_f, in_f = w.shape
        with torch.device(dev):
            col = ColumnParallelLinear(in_f, out_f, bias=True, gather_output=True, async_all_reduce=async_ar)
            row = RowParallelLinear(in_f, out_f, bias=True)
        col.weight = torch.nn.Parameter(w.chunk(world, dim=0)[rank].contiguous())
        col.bias = torch.nn.Parameter(b.chunk(world, dim=0)[rank].contiguous())
        row.weight = torch.nn.Parameter(w.chunk(world, dim=1)[rank].contiguous())
        row.bias = torch.nn.Parameter(b.clone())
        xc = x.clone().requires_grad_(True)
        xr = x.chunk(world, dim=-1)[rank].contiguous().requires_grad_(True)
        yc, yr = col(xc), row(xr)
        # test_tensor_parallel.py:54: the gathered Column output IS the dense output (same GEMM)
        dense = FN.linear(x, w) + b
        assert torch.equal(yc, dense), "column-gathered != dense on the HIP GEMM"
        assert _rel(yc, g[P + t + "y_dense"]) < TOL
        assert _rel(yr, g[P + t + "y_dense"]) < TOL
        yc.backward(torch.ones_like(yc))
        yr.backward(torch.ones_like(yr))
        assert _rel(xc.grad, g[P + t + "dx_dense"]) < TOL
        assert _rel(xr.grad, g[P + t + "dx_dense"].chunk(world, dim=-1)[rank]) < TOL
        assert _rel(col.weight.grad, g[P + t + "dw_dense"].chunk(world, dim=0)[rank]) < TOL
        assert _rel(row.weight.grad, g[P + t + "dw_dense"].chunk(world, dim=1)[rank]) < TOL
        assert _rel(col.bias.grad, g[P + t + "db_dense"].chunk(world, dim=0)[rank]) < TOL
        assert _rel(row.bias.grad, g[P + t + "db_dense"]) < TOL
    V, H = 512, 128
    with torch.device(dev):
        emb = VocabParallelEmbedding(V, H)
    assert (emb.vocab_start_index, emb.vocab_end_index) == (int(g[P + "emb_lo"]), int(g[P + "emb_hi"]))
    with torch.no_grad():
        emb.weight.copy_(g[P + "emb_w"])
    emb.to(BF)
    ye = emb(g[P + "emb_ids"].to(dev))
    assert _rel(ye, g[P + "emb_y"]) < TOL
    ye.backward(g[P + "emb_dy"].to(dev, BF))
    assert _rel(emb.weight.grad, g[P + "emb_dw"]) < TOL


def test_tp_modules_match_reference_g7():
    _dist.run(_tp_modules, 2, device="cuda")


def _dp_g8(rank, world, wrapper, grad_type, pair=False):
    os.environ["FLASH_ATTEN"] = "0"   # the fixture is the reference's eager path (LlamaRMSNorm)
    torch.cuda.set_device(0)
    import torch.nn.functional as F
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.data_parallel.data_parallel import DataParallelBucket, DataParallelNaive
    from picotron_amd.model import Llama
    sys_cfg = dict(hidden_size=128, intermediate_size=256, num_attention_heads=2, num_key_value_heads=2,
                   rms_norm_eps=1e-5, max_position_embeddings=128, rope_theta=10000.0, vocab_size=256,
                   num_hidden_layers=2)
    pgm.setup_process_group_manager(tp_size=1, cp_size=1, pp_size=1, dp_size=world)
    g = torch.load(os.path.join(GOLD, "G8.pt"), weights_only=True)
    dev = torch.device("cuda", 0)
    with torch.device(dev):
        model = Llama(types.SimpleNamespace(**sys_cfg))
    model.to(BF)
    with torch.no_grad():
        for n, p in model.named_parameters():
            p.copy_(g[f"rank{rank}.param.{n}"])
    if wrapper == "bucket":
        dp = DataParallelBucket(model, grad_type=grad_type)
    else:
        dp = DataParallelNaive(model)
    ids = g[f"rank{rank}.ids"]
    ga = ids.shape[1]
    from picotron_amd import functional as FN
    from picotron_amd.train import pairing_phase
    for i in range(ga):
        dp.require_backward_grad_sync = (i == ga - 1)
        t = ids[rank, i].to(dev)
        lo = dp(input_ids=t[:, :-1])
        loss = F.cross_entropy(lo.reshape(-1, 256), t[:, 1:].reshape(-1)) / ga   # HipLogits -> HIP CE
        if pair:   # train_step's weight-gradient pairing: micro-batch 0 defers, 1 launches K = 2 T
            FN.wgrad_pairing(pairing_phase(i, ga))
        loss.backward()
    FN.wgrad_pairing(None)
    assert not FN.WgradPairing.pending
    torch.cuda.synchronize()
    tol = TOL if grad_type == torch.float32 else 3e-2
    for n, p in model.named_parameters():
        assert p.grad is not None, n
        assert _rel(p.grad, g[f"rank{rank}.grad.{n}"]) < tol, (n, _rel(p.grad, g[f"rank{rank}.grad.{n}"]))


@pytest.mark.parametrize("wrapper,grad_type,pair", [("bucket", torch.float32, False), ("bucket", torch.bfloat16, False),
                                                    ("naive", torch.float32, False), ("bucket", torch.float32, True),
                                                    ("bucket", torch.bfloat16, True)])
def test_data_parallel_matches_reference_g8(wrapper, grad_type, pair):
    """pair: the two micro-batches' weight gradients as one K = 2 T launch each (train_step's
    default, functional.WgradPairing) into the fp32 / bf16 main_grad buckets."""
    _dist.run(_dp_g8, 2, wrapper, grad_type, pair, device="cuda")


def _train_curve(rank, world, tp, cp, dp, out_q, kind="G10m", seq=256, avg=False, pair=False, chunks=0):
    """train.py's loop (train_step 29-55, steps 219-240) on the GPU path at the given tp / cp / dp from
    the fixtures' full initial weights (G10m's): the reference's wrapping rule (DataParallelBucket only
    for dp > 1, train.py:194-195), picotron_amd's fused AdamW, HipLogits -> HIP CE, the logged loss
    averaged over cp_dp (utils.py:93-98).  kind G10m: 4 steps on one batch, lr 1e-2; G11: 50 steps,
    a fresh bigram batch per step (the fixture's token stream), lr 1e-3.  chunks > 0: the
    sequence-parallel layout forced to that many chunks (tp > 1)."""
    os.environ["FLASH_ATTEN"] = "0"   # the fixture is the reference's eager path (LlamaRMSNorm, SDPA)
    torch.cuda.set_device(0)
    import torch.distributed as dist
    import torch.nn.functional as F
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.context_parallel.context_parallel import apply_context_parallel
    from picotron_amd.data_parallel.data_parallel import DataParallelBucket
    from picotron_amd.model import Llama
    from picotron_amd.optim import AdamW
    from picotron_amd.tensor_parallel.tensor_parallel import apply_tensor_parallel
    cfg = dict(hidden_size=128, intermediate_size=256, num_attention_heads=2, num_key_value_heads=2,
               rms_norm_eps=1e-5, max_position_embeddings=seq, rope_theta=10000.0, vocab_size=256,
               num_hidden_layers=2)
    tag = {(2, 1, 1): "tp2", (1, 2, 1): "cp2", (1, 1, 2): "dp2", (1, 1, 1): "1"}[(tp, cp, dp)]
    tag += ("" if seq == 256 else f"s{seq}") + ("avg" if avg else "")
    g = torch.load(os.path.join(GOLD, f"{kind}_{tag}.pt"), weights_only=True)
    init = g if kind == "G10m" else torch.load(os.path.join(GOLD, "G10m_tp2.pt"), weights_only=True)
    m = pgm.setup_process_group_manager(tp_size=tp, cp_size=cp, pp_size=1, dp_size=dp)
    if seq == 512:
        from picotron_amd.context_parallel.context_parallel import zigzag_enabled
        assert zigzag_enabled(seq // cp, True)
    dev = torch.device("cuda", 0)
    with torch.device(dev):
        model = Llama(types.SimpleNamespace(**cfg))
        if tp > 1:
            apply_tensor_parallel(model)
    apply_context_parallel(model)
    model.to(BF)
    with torch.no_grad():
        for n, p in model.named_parameters():
            full = init[f"rank0.param.{n}"]
            if full.shape != p.shape:   # Column / Vocab: dim 0, Row: dim 1 (tensor_parallel.py:76-152)
                (d,) = [i for i, (x, y) in enumerate(zip(full.shape, p.shape)) if x != y]
                full = full.narrow(d, m.tp_rank * p.shape[d], p.shape[d])
            p.copy_(full)
    if dp > 1 or avg:
        model = DataParallelBucket(model)
    if seq == 512:   # cp2, 256 tokens per rank: the zig-zag schedule; the residual stream stays
        # zig-zag exactly when the cp ranks' gradients are averaged (enable_zigzag_residual)
        inner = model.module if isinstance(model, DataParallelBucket) else model
        assert getattr(inner, "_pt_zigzag_residual", False) == avg
    S, V = cfg["max_position_embeddings"], cfg["vocab_size"]
    if kind == "G10m":
        lr = 1e-2
        gen = torch.Generator().manual_seed(1234)   # make_golden._g10m_data: the same batch every step
        one = torch.randint(0, V, (1, 2, 2, 2, S + 1), generator=gen)
        ids = one.expand(g["rank0.losses"].numel(), -1, -1, -1, -1)
    else:
        lr, ids = 1e-3, g["rank0.ids"].long()           # make_golden._g11_data
    opt = AdamW(model.parameters(), lr=lr)
    sl = slice(m.cp_rank * S // cp, (m.cp_rank + 1) * S // cp)
    losses = []
    from picotron_amd import switches
    force = switches.override(tp_sp_chunks=chunks)
    force.__enter__()
    seen_c = set()
    if chunks:
        from picotron_amd import functional as FN_
        from picotron_amd.tensor_parallel import sequence_parallel as SPM
        assert SPM.layout_chunks(ids.shape[-2], S // cp, tp) == chunks
        orig_gc = FN_.TPContext.gather_chunk

        def gc(self, full, shard, c, j, async_op=False):
            seen_c.add(c)
            return orig_gc(self, full, shard, c, j, async_op)
        FN_.TPContext.gather_chunk = gc
    for step in range(g["rank0.losses"].numel()):
        opt.zero_grad()
        acc = 0.0
        for i in range(2):
            if m.cp_dp_world_size > 1:
                model.require_backward_grad_sync = (i == 1)
            t = ids[step, m.dp_rank, i]
            x, y = t[:, :-1][:, sl].contiguous().to(dev), t[:, 1:][:, sl].contiguous().to(dev)
            out = model(input_ids=x)
            loss = F.cross_entropy(out.reshape(-1, V), y.reshape(-1), reduction="mean") / 2
            if pair:   # train_step's weight-gradient pairing (functional.WgradPairing)
                from picotron_amd import functional as FN
                from picotron_amd.train import pairing_phase
                FN.wgrad_pairing(pairing_phase(i, 2))
            loss.backward()
            if pair:
                FN.wgrad_pairing(None)
            acc += loss.item()
        if world > 1:
            red = torch.tensor([acc], dtype=torch.float32)
            dist.all_reduce(red, group=m.cp_dp_group)
            acc = red.item() / m.cp_dp_world_size
        losses.append(acc)
        opt.step()
        if hasattr(model, "reset"):
            model.reset()
    force.__exit__(None, None, None)
    if chunks:
        FN_.TPContext.gather_chunk = orig_gc
        assert seen_c == {chunks}, seen_c   # every sharded collective ran in the forced layout
    ref = g["rank0.losses"].tolist()
    if rank == 0:
        out_q.put((tag + (f"c{chunks}" if chunks else ""), losses, ref))
    for k, (a, b) in enumerate(zip(losses, ref)):
        assert abs(a - b) <= 0.01 * abs(b), (tag, k, losses, ref)   # north_star: within 1 %


@pytest.mark.parametrize("tp,cp,dp", [(2, 1, 1), (1, 2, 1), (1, 1, 2)])
def test_multirank_loss_curve_matches_reference_g10m(tp, cp, dp):
    """G10 at tp2 / cp2 / dp2: the reference's own 4-step loss curve (fp32, gloo,
    same batch every step, lr 1e-2: 5.7 -> 3.0 / 2.2 / 3.8) reproduced by the bf16 HIP path within
    1 % per step (north_star's loss-curve bar; measured <= 0.4 %, gpurun_out/r02r_g10m.log), bf16
    weights and Adam states against the reference's fp32.  cp2 falls fastest in both: the
    reference's train.py does not average gradients over cp ranks when dp = 1."""
    import torch.multiprocessing as mp
    q = mp.get_context("spawn").SimpleQueue()
    _dist.run(_train_curve, 2, tp, cp, dp, q, "G10m", device="cuda")
    tag, losses, ref = q.get()
    print(tag, [round(x, 4) for x in losses], [round(x, 4) for x in ref])


@pytest.mark.parametrize("tp,cp,dp,seq,avg,pair,chunks", [
    (1, 1, 1, 256, False, False, 0), (2, 1, 1, 256, False, False, 0), (2, 1, 1, 256, False, False, 2),
    (1, 2, 1, 256, False, False, 0), (1, 1, 2, 256, False, False, 0),
    (1, 2, 1, 512, False, False, 0), (1, 2, 1, 512, True, False, 0),
    (1, 1, 1, 256, False, True, 0), (1, 1, 2, 256, False, True, 0)])
def test_50_step_loss_curve_matches_reference_g11(tp, cp, dp, seq, avg, pair, chunks):
    """north_star: "the loss curve within 1 % over 50 steps", against the REFERENCE's own curves
    (G11, make_golden.g11_curve: train.py's loop run by the reference on gloo/CPU in its GPU training
    precision -- bf16 model and AdamW states, train.py:76,190 -- 50 AdamW steps at lr 1e-3, a fresh
    bigram batch per step, 5.7 -> 1.9): the HIP path at 1 rank and at tp2 / cp2 / dp2 within 1 % at
    every step.  (Against the reference's fp32 run, G11f32_*, bf16 training of either code base
    ends 4 % higher: precision, not the implementation -- the fixtures' own test pins that gap.)
    seq 512 at cp2: 256 tokens per rank, where the build runs the zig-zag schedule, K|V over the
    mesh, pinned to the reference's own ring -- as train.py runs it at dp 1 (G11_cp2s512: no gradient
    averaging, each cp rank steps on its own chunk's gradient; the build re-lays inside each
    attention call) and with the reference's DataParallelBucket averaging the cp ranks
    (G11_cp2s512avg; the build keeps the whole residual stream zig-zag).  pair: the step's two
    micro-batches' weight gradients as one K = 2 T launch each (train_step's default at tp 1).
    chunks 2 at tp2: the sequence-parallel layer in two token chunks, each with its own collectives."""
    import torch.multiprocessing as mp
    q = mp.get_context("spawn").SimpleQueue()
    _dist.run(_train_curve, tp * cp * dp, tp, cp, dp, q, "G11", seq, avg, pair, chunks, device="cuda")
    tag, losses, ref = q.get()
    print(tag, "max rel dev", max(abs(a - b) / b for a, b in zip(losses, ref)), "last", losses[-1], "ref", ref[-1])


def _pp_curve(rank, world, engine, out_q):
    """G10m_pp2 on the GPU path: picotron_amd's PipelineParallel stages of the HIP Llama (eager
    FLASH_ATTEN=0 path, as the fixture) trained by its 1F1B / AFAB step over p2p, fused AdamW,
    HipLogits -> HIP CE in the engine's F.cross_entropy(logits.transpose(1, 2)) form; the last
    stage's logged loss per step."""
    os.environ["FLASH_ATTEN"] = "0"
    torch.cuda.set_device(0)
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.model import Llama
    from picotron_amd.optim import AdamW
    from picotron_amd.pipeline_parallel import pipeline_parallel as PPE
    cfg = dict(hidden_size=128, intermediate_size=256, num_attention_heads=2, num_key_value_heads=2,
               rms_norm_eps=1e-5, max_position_embeddings=256, rope_theta=10000.0, vocab_size=256,
               num_hidden_layers=2)
    g = torch.load(os.path.join(GOLD, "G10m_pp2.pt" if engine == "1f1b" else "G10m_pp2afab.pt"), weights_only=True)
    m = pgm.setup_process_group_manager(tp_size=1, cp_size=1, pp_size=world, dp_size=1)
    dev = torch.device("cuda", 0)
    ns = types.SimpleNamespace(**cfg)
    with torch.device(dev):
        model = PPE.PipelineParallel(Llama(ns), ns)
    model.to(BF)
    with torch.no_grad():
        for n, p in model.named_parameters():
            p.copy_(g[f"rank0.param.{n}"])
    S, V = cfg["max_position_embeddings"], cfg["vocab_size"]
    gen = torch.Generator().manual_seed(1234)   # make_golden._g10m_data: the same batch every step
    ids = torch.randint(0, V, (1, 2, 2, 2, S + 1), generator=gen)[0, 0].to(dev)

    class Loader:
        grad_acc_steps = 2

        def __init__(self):
            self.i = 0

        def __next__(self):
            t = ids[self.i]
            self.i += 1
            return {"input_ids": t[:, :-1], "target_ids": t[:, 1:], "position_ids": torch.arange(S, device=dev).expand(2, S),
                    "hidden_states": None}
    step = PPE.train_step_pipeline_1f1b if engine == "1f1b" else PPE.train_step_pipeline_afab
    opt = AdamW(model.parameters(), lr=1e-2)
    losses = []
    for _ in range(g["rank1.losses"].numel()):
        opt.zero_grad()
        losses.append(step(model, Loader(), (2, S, cfg["hidden_size"]), dev, BF))
        opt.step()
    if m.pp_is_last_stage:
        ref = g["rank1.losses"].tolist()
        out_q.put((engine, losses, ref))
        for k, (a, b) in enumerate(zip(losses, ref)):
            assert abs(a - b) <= 0.01 * abs(b), (engine, k, losses, ref)   # north_star: within 1 %


@pytest.mark.parametrize("engine", ["1f1b", "afab"])
def test_pipeline_loss_curve_matches_reference_g10m_pp2(engine):
    """BASELINE config 4's pipeline composition against the reference's own run of it (G10m_pp2:
    its PipelineParallel + 1F1B / AFAB at pp 2, fp32 on gloo/CPU, 5.71 -> 3.04): the HIP path through
    picotron_amd's engine within 1 % at every step."""
    import torch.multiprocessing as mp
    q = mp.get_context("spawn").SimpleQueue()
    _dist.run(_pp_curve, 2, engine, q, device="cuda")
    tag, losses, ref = q.get()
    print(tag, [round(x, 4) for x in losses], [round(x, 4) for x in ref])


def _grid_curve(rank, world, size, out_q):
    """G12 on the GPU path -- BASELINE configs 1 / 4's composition: train.py:174-195's order (Llama ->
    apply_tensor_parallel -> PipelineParallel -> weights -> bf16 -> DataParallelBucket, fp32 main_grad)
    of picotron_amd over the HIP kernels (eager FLASH_ATTEN=0 path, as the fixture), dp2 tp2 pp2 on 8
    gloo ranks sharing cuda:0, trained by the package's 1F1B step from G12's deterministic full
    weights; the logged loss (the last stage's, averaged over cp_dp: utils.py:93-98) per step."""
    os.environ["FLASH_ATTEN"] = "0"
    torch.cuda.set_device(0)
    import torch.distributed as dist
    from tests import _g12
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.data_parallel.data_parallel import DataParallelBucket
    from picotron_amd.model import Llama
    from picotron_amd.optim import AdamW
    from picotron_amd.pipeline_parallel import pipeline_parallel as PPE
    from picotron_amd.tensor_parallel.tensor_parallel import apply_tensor_parallel
    torch.set_num_threads(2)
    c = _g12.CFGS[size]
    m = pgm.setup_process_group_manager(tp_size=2, cp_size=1, pp_size=2, dp_size=2)
    g = torch.load(os.path.join(GOLD, f"G12_{size}.pt"), weights_only=True)
    assert g[f"rank{rank}.grid"].tolist() == [m.dp_rank, m.pp_rank, m.cp_rank, m.tp_rank]
    dev = torch.device("cuda", 0)
    ns = types.SimpleNamespace(**c)
    with torch.device(dev):
        model = Llama(ns)
        apply_tensor_parallel(model)
        model = PPE.PipelineParallel(model, ns)
    model.to(BF)
    with torch.no_grad():
        for n, p in model.named_parameters():
            full = _g12.full_param(n, _g12.full_shape(n, p, c))
            if full.shape != p.shape:   # Column / Vocab: dim 0, Row: dim 1 (tensor_parallel.py:76-152)
                (d,) = [i for i, (x, y) in enumerate(zip(full.shape, p.shape)) if x != y]
                full = full.narrow(d, m.tp_rank * p.shape[d], p.shape[d])
            p.copy_(full)
            del full
    model = DataParallelBucket(model)
    S, V = c["max_position_embeddings"], c["vocab_size"]
    ids = _g12.tokens(V, S)[m.dp_rank].to(dev)
    pos = torch.arange(S, device=dev).expand(_g12.MBS, S)

    class Loader:
        grad_acc_steps, micro_batch_size, seq_length_per_gpu = _g12.GA, _g12.MBS, S

        def __init__(self):
            self.i = 0

        def __next__(self):
            t = ids[self.i]
            self.i += 1
            return {"input_ids": t[:, :-1], "target_ids": t[:, 1:], "position_ids": pos, "hidden_states": None}
    opt = AdamW(model.parameters(), lr=_g12.RUN[size]["lr"])
    losses = []
    for _ in range(_g12.RUN[size]["steps"]):
        opt.zero_grad()
        loss = PPE.train_step_pipeline_1f1b(model, Loader(), (_g12.MBS, S, c["hidden_size"]), dev, BF)
        red = torch.tensor([loss], dtype=torch.float32)
        if m.pp_is_last_stage:
            dist.all_reduce(red, group=m.cp_dp_group)
            red /= m.cp_dp_world_size
        losses.append(red.item())
        opt.step()
        model.reset()
    ref = g[f"rank{rank}.losses"].tolist()
    if rank == world - 1:
        out_q.put((size, losses, ref))
    for k, (a, b) in enumerate(zip(losses, ref)):
        assert abs(a - b) <= 0.01 * abs(b), (size, rank, k, losses, ref)   # north_star: within 1 %
    if size == "smollm" and m.pp_is_last_stage:
        # config 1's literal fp32 (G12f32_smollm): the bf16 HIP curve sits below it by the reference's
        # own bf16-vs-fp32 gap (0.9 / 2.2 / 3.6 %, test_oracle_golden.py) -- within 1 % of that gap
        f32 = torch.load(os.path.join(GOLD, "G12f32_smollm.pt"), weights_only=True)[f"rank{rank}.losses"].tolist()
        for k, (a, b, c) in enumerate(zip(losses, ref, f32)):
            assert abs((c - a) / c - (c - b) / c) <= 0.01, ("G12f32 gap", k, losses, ref, f32)


@pytest.mark.parametrize("size", ["tiny", "smollm"])
def test_dp2_tp2_pp2_1f1b_loss_curve_matches_reference_g12(size):
    """BASELINE configs 1 and 4's dp2 tp2 pp2 1F1B grid against the reference's own run of it (G12:
    its train.py composition on 8 gloo CPU processes; tiny = G10m dims, 5 layers, fp32, 6 steps at
    lr 1e-2, 5.69 -> 2.24; smollm = SmolLM-1.7B dims, 5 layers -- config 1 itself -- in the
    reference's bf16 training precision, 4 steps at lr 1e-4, 10.97 -> 7.67): the bf16 HIP path through picotron_amd's TP modules, pipeline engine and
    DataParallelBucket on 8 gloo ranks sharing cuda:0, within 1 % at every step."""
    import torch.multiprocessing as mp
    q = mp.get_context("spawn").SimpleQueue()
    _dist.run(_grid_curve, 8, size, q, device="cuda")
    tag, losses, ref = q.get()
    print(tag, [round(x, 4) for x in losses], [round(x, 4) for x in ref])
