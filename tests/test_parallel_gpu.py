"""TP and CP through the HIP kernels with two ranks: the fused decoder layers, VocabParallelEmbedding,
the gathered lm_head, the fused CE and (CP) the ring-attention schedule over the flash kernels with
the LSE merge in their epilogue, checked against the oracle on the full, unsharded model.

Both ranks drive cuda:0 of the one-GPU box and talk over gloo, which stages the CUDA tensors of the
collectives through host memory (tests/_dist.py): the kernels, shards, f/g collectives
(tensor_parallel.py:116-189, tp_comm.py:19-49) and ring schedule (context_parallel.py:17-110) are
the product path; only the transport differs from RCCL over xGMI.  Sequence 256 so that each CP
rank holds 128 tokens (the flash kernels tile the sequence in 128-row blocks).  Tolerance: norm-relative 2e-2
(north_star's bf16 tolerance) on the fp32 oracle evaluated from the same bf16 weights."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.nn.functional as F

from tests import _dist

pytestmark = pytest.mark.gpu
TOL = 2e-2
CFG = dict(hidden_size=256, intermediate_size=512, num_attention_heads=4, num_key_value_heads=2, vocab_size=512,
           rms_norm_eps=1e-5, rope_theta=10000.0, num_hidden_layers=2, max_position_embeddings=256)


def _rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def _shard(full, local, rank):
    """The rank's block of a master tensor: the one dim where the shapes differ is split evenly
    (Column: dim 0, Row: dim 1, VocabParallelEmbedding: dim 0 -- tensor_parallel.py:76-82,111-117,147-152)."""
    if full.shape == local.shape:
        return full
    (d,) = [i for i, (a, b) in enumerate(zip(full.shape, local.shape)) if a != b]
    n = local.shape[d]
    return full.narrow(d, rank * n, n)


def _setup(tp, cp, seq=256, cfg_over=None, batch=2):
    import types
    os.environ["FLASH_ATTEN"] = "1"
    torch.cuda.set_device(0)
    from oracle import picotron_oracle as O
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.context_parallel.context_parallel import apply_context_parallel
    from picotron_amd.model import Llama
    from picotron_amd.tensor_parallel.tensor_parallel import apply_tensor_parallel
    m = pgm.setup_process_group_manager(tp_size=tp, cp_size=cp, pp_size=1, dp_size=1)
    base = dict(CFG, **(cfg_over or {}))
    c = dict(base, max_position_embeddings=seq)
    cfg = types.SimpleNamespace(**c)
    full = {k: v.to(torch.bfloat16) for k, v in O.init_params(dict(base), seed=7).items()}
    with torch.device("cuda"):
        model = Llama(cfg)
        if tp > 1:
            apply_tensor_parallel(model)
    apply_context_parallel(model)
    assert os.environ["CONTEXT_PARALLEL"] == ("1" if cp > 1 else "0")
    model.to(torch.bfloat16)
    names = dict(model.named_parameters())
    assert sorted(names) == sorted(full), (sorted(names), sorted(full))
    with torch.no_grad():
        for n, p in names.items():
            p.copy_(_shard(full[n], p, m.tp_rank))
    g = torch.Generator().manual_seed(11)
    ids = torch.randint(0, base["vocab_size"], (batch, seq + 1), generator=g)
    # the oracle on the full model, fp32 from the same bf16 weights
    pf = {k: v.float().requires_grad_(True) for k, v in full.items()}
    cos, sin = O.get_cos_sin(seq, base["hidden_size"] // base["num_attention_heads"], base=CFG["rope_theta"])
    lo = O.llama_forward(ids[:, :-1], pf, dict(base), cos.float(), sin.float(), norm=O.rmsnorm_flash_semantics)
    loss_r = F.cross_entropy(lo.reshape(-1, base["vocab_size"]), ids[:, 1:].reshape(-1))
    loss_r.backward()
    return m, model, names, pf, ids, lo, loss_r


def _llama(rank, world, tp, cp, seq=256, zigzag=False, residual=1, mesh=1, production_thresholds=False, sp=1,
           cfg_over=None, chunks=2, batch=2):
    from picotron_amd import switches
    # conftest.py zeroes the RoPE / SwiGLU fusion tile thresholds for the small test shapes;
    # production_thresholds restores the shipped ones (96 / 192 / 0), under which these TP-shard
    # widths take the split (GEMM + separate rope / swiglu kernel) paths
    thr = dict(rope_fuse_min_tiles=96, swiglu_fuse_min_tiles=192, swiglu_bwd_min_tiles=0) \
        if production_thresholds else {}
    with switches.override(zigzag_residual=residual, ring_mesh=mesh, tp_sp=sp, tp_sp_chunks=chunks, **thr):
        _llama_body(rank, world, tp, cp, seq, zigzag, residual, cfg_over, batch)


def _llama_body(rank, world, tp, cp, seq, zigzag, residual, cfg_over=None, batch=2):
    from picotron_amd import functional as FN
    from picotron_amd import switches
    from picotron_amd.context_parallel import context_parallel as CP
    m, model, names, pf, ids, lo, loss_r = _setup(tp, cp, seq, cfg_over, batch)
    B = batch
    V = dict(CFG, **(cfg_over or {}))["vocab_size"]
    # sequence parallelism (tensor_parallel/sequence_parallel.py): on at tp > 1 without cp, by default
    sp_on = tp > 1 and cp == 1 and switches.S.tp_sp != 0
    assert all(layer.tp_sequence_parallel == sp_on for layer in model.decoder_layers)
    gathers = []
    orig_ag = FN.TPContext.all_gather_rows_into

    def counted_ag(self, out, t, async_op=False):
        gathers.append(tuple(t.shape))
        return orig_ag(self, out, t, async_op)
    FN.TPContext.all_gather_rows_into = counted_ag
    if residual:   # what the data-parallel wrappers do at cp > 1 (the grads are checked summed over cp)
        CP.enable_zigzag_residual(model)
    s = seq // cp
    assert CP.zigzag_enabled(s, True) == zigzag   # which ring schedule this case exercises
    sl = slice(m.cp_rank * s, (m.cp_rank + 1) * s)                # data.py:105-109: contiguous chunks
    x, t = ids[:, :-1][:, sl].contiguous(), ids[:, 1:][:, sl].contiguous()
    calls = []
    orig = CP.zigzag_exchange

    def counted(*a, **k):
        calls.append(a[2])
        return orig(*a, **k)
    CP.zigzag_exchange = counted
    try:
        logits = model(x.cuda())
        n_fwd = len(calls)
        n_ag_fwd = len(gathers)
        assert logits.shape == (B, s, V)             # final_proj gathers its vocab shards
        loss = FN.cross_entropy(logits.view(-1, V), t.reshape(-1).cuda())
        loss.backward()
        torch.cuda.synchronize()
    finally:
        CP.zigzag_exchange = orig
        FN.TPContext.all_gather_rows_into = orig_ag
    L, H = CFG["num_hidden_layers"], dict(CFG, **(cfg_over or {}))["hidden_size"]
    # the vocab-parallel CE (functional.VocabParallelCEFunction): one gather of 16 B per row at tp > 1
    vp = [g for g in gathers if g == (B * s, 4)]
    vp_on = tp > 1 and FN.vp_ce_shape_ok(B * s, V // tp, H)   # V 512 at tp 8: V / tp = 64 does not tile
    assert vp_on == (tp > 1 and (V // tp) % 128 == 0 and (B * s) % 256 == 0 and H % 64 == 0 and switches.S.vp_ce != 0)
    assert len(vp) == (1 if vp_on else 0), gathers
    gathers = [g for g in gathers if g != (B * s, 4)]
    if sp_on:   # per layer and chunk 2 gathers each way, plus the exit (forward) / the entry (backward)
        from picotron_amd.tensor_parallel import sequence_parallel as SPM
        c = SPM.layout_chunks(B, s, tp)
        assert c == (min(B, switches.S.tp_sp_chunks) if switches.S.tp_sp_chunks > 0 else 1), c
        assert n_ag_fwd == c * (2 * L + 1) and len(gathers) == c * (4 * L + 2), gathers
        assert all(g == (B * s // (tp * c), H) for g in gathers), gathers   # every gather is of T / (tp c) rows
    else:
        assert not gathers
    if zigzag and residual:
        # the residual stream is re-laid once on entry and once on exit (and its gradient twice),
        # not per layer
        assert n_fwd == 2 and len(calls) == 4, calls
    elif zigzag:
        # the standalone layers: q|K|V in and o out per layer, one combined exchange each way back
        assert n_fwd == 2 * CFG["num_hidden_layers"] and len(calls) == 4 * CFG["num_hidden_layers"], calls
    else:
        assert not calls
    assert _rel(logits, lo[:, sl]) < TOL
    lsum = loss.detach().float().cpu().view(1)
    if cp > 1:
        dist.all_reduce(lsum, group=m.cp_group)
    assert abs(lsum.item() / cp - loss_r.item()) < TOL * abs(loss_r.item())
    # each CP rank holds the grad of its chunk's mean loss; their cp_dp average (bucket.py) is the
    # grad of the full-sequence mean loss.  TP ranks hold their shard's grad.
    for n, p in names.items():
        assert p.grad is not None, n
        g = p.grad.detach().float().cpu()
        if cp > 1:
            dist.all_reduce(g, group=m.cp_group)
        assert _rel(g / cp, _shard(pf[n].grad, p, m.tp_rank)) < TOL, n


def test_tensor_parallel_llama_tp2():
    _dist.run(_llama, 2, 2, 1, device="cuda")


def test_tensor_parallel_llama_tp2_production_thresholds():
    """tp2 with the shipped fusion thresholds: the split RoPE / SwiGLU paths of narrow TP shards."""
    _dist.run(_llama, 2, 2, 1, 256, False, 1, 1, True, device="cuda")


def test_tensor_parallel_llama_tp2_one_chunk():
    """tp2 with the sequence-parallel layout in one chunk (PICOTRON_TP_SP_CHUNKS=1: rank r holds rows
    [r T/tp, (r+1) T/tp), every collective of a block in one piece)."""
    _dist.run(_llama, 2, 2, 1, 256, False, 1, 1, False, 1, None, 1, device="cuda")


def test_tensor_parallel_llama_tp8_four_chunks():
    """tp8 in the layout bench.py's config-3 default runs (mbs 32: 4 chunks): batch 4, each sequence a
    chunk, 32 token rows per rank and chunk -- every chunk's collectives its own -- against the oracle."""
    over = dict(hidden_size=512, intermediate_size=1024, num_attention_heads=8, num_key_value_heads=8)
    _dist.run(_llama, 8, 8, 1, 256, False, 1, 1, False, 1, over, 4, 4, device="cuda")


@pytest.mark.parametrize("tp", [1, 2])
def test_llama_off_grid_widths(tp):
    """An intermediate (344 per rank) and a vocabulary (1000; 500 per rank at tp2) off the GEMM tiles'
    64-element grid -- as Llama-2-7B's shards at tp 8 (1376, 4000) -- run on the padded projections
    (kernels._linear_*_padded) with the separate SwiGLU / cross-entropy kernels: the full model's
    logits, loss and every gradient against the oracle."""
    over = dict(intermediate_size=344 * tp, vocab_size=1000)
    _dist.run(_llama, tp, tp, 1, 256, False, 1, 1, False, 1, over, device="cuda")


@pytest.mark.parametrize("tp", [1, 2])
def test_llama_off_block_sequence(tp):
    """seq 200: off the attention kernels' 128-row query blocks (padded attention) and, with T = 400
    token rows, off the GEMM tiles' 64-grid (padded projections); at tp2 the sequence-parallel layout
    in 2 chunks of 100 rows per rank -- the full model against the oracle."""
    _dist.run(_llama, tp, tp, 1, 200, False, 1, 1, False, 1, None, device="cuda")


@pytest.mark.parametrize("tp", [1, 2])
def test_llama_head_dim_60(tp):
    """head_dim 60 (hidden 240, 4 heads; create_config.py's own example gives SmolLM-360M 16 heads of
    60): every head zero-padded to the kernels' 64 in its two rotary halves (functional.
    _attention_core_*_padded), the projections off the 64-grid padded too -- the full model against
    the oracle."""
    over = dict(hidden_size=240, num_attention_heads=4, num_key_value_heads=2)
    _dist.run(_llama, tp, tp, 1, 256, False, 1, 1, False, 1, over, device="cuda")


def test_tensor_parallel_llama_tp2_replicated_stream():
    """tp2 without sequence parallelism (PICOTRON_TP_SP=0): the reference's replicated residual
    stream and row-parallel all-reduces."""
    _dist.run(_llama, 2, 2, 1, 256, False, 1, 1, False, 0, device="cuda")


@pytest.mark.parametrize("sp", [1, 0])
def test_tensor_parallel_llama_tp4(sp):
    """tp4 (4 q / 4 kv heads: one head of each per rank) against the oracle on the full model, with
    the residual stream sharded by token rows (128 of the 512 per rank) and without."""
    _dist.run(_llama, 4, 4, 1, 256, False, 1, 1, False, sp, dict(num_key_value_heads=4), device="cuda")


def test_tensor_parallel_llama_tp8():
    """config 3's TP degree: 8 ranks (gloo on cuda:0), one q head and one kv head each, the residual
    stream sharded 64 token rows per rank, against the oracle on the full model."""
    over = dict(hidden_size=512, intermediate_size=1024, num_attention_heads=8, num_key_value_heads=8)
    _dist.run(_llama, 8, 8, 1, 256, False, 1, 1, False, 1, over, device="cuda")


def test_tensor_parallel_llama_tp8_vocab_parallel_ce():
    """config 3's shipped lm_head path at world 8: V 2048 (V / 8 = 256 columns per rank tile the
    lm_head GEMM's CE statistics), so the vocab-parallel cross-entropy runs (asserted in the body:
    one 16-B-per-row gather) with sequence parallelism on -- loss, logits and every gradient against
    the oracle on the full model."""
    over = dict(hidden_size=512, intermediate_size=1024, num_attention_heads=8, num_key_value_heads=8,
                vocab_size=2048)
    _dist.run(_llama, 8, 8, 1, 256, False, 1, 1, False, 1, over, device="cuda")


def test_context_parallel_llama_cp8():
    """config 5's CP degree: 8 ranks (gloo on cuda:0), seq 2048 = 256 tokens per rank -- the zig-zag
    schedule on the full mesh with the resident zig-zag residual -- against the oracle on the whole
    sequence."""
    _dist.run(_llama, 8, 1, 8, 2048, True, 1, 1, device="cuda")


def test_context_parallel_llama_cp2():
    _dist.run(_llama, 2, 1, 2, device="cuda")


def test_tp2_cp2_llama():
    _dist.run(_llama, 4, 2, 2, device="cuda")


@pytest.mark.parametrize("tp,cp,seq,residual,mesh", [(1, 2, 512, 1, 1), (1, 4, 1024, 1, 1), (2, 2, 512, 1, 1),
                                                    (1, 4, 1024, 0, 1), (1, 4, 1024, 1, 0)])
def test_zigzag_ring_llama(tp, cp, seq, residual, mesh):
    """The load-balanced (zig-zag) causal schedule (S_local = 256: its half shards tile the kernels):
    full Llama forward + backward at cp2 / cp4 / tp2.cp2 against the oracle on the whole sequence,
    the reference's contiguous token chunks in and out -- with the residual stream kept in the
    zig-zag layout (the default: two re-lays per pass) or re-laid per layer, and the K|V / dK|dV
    exchanged over the full mesh (default) or round the ring."""
    _dist.run(_llama, tp * cp, tp, cp, seq, True, residual, mesh, device="cuda")


def _llama_ring_plain(rank, world, tp, cp, seq):
    from picotron_amd import switches
    with switches.override(ring_zigzag=0):
        _llama(rank, world, tp, cp, seq, False, 1, 1)


def test_ring_zigzag_off_llama():
    """PICOTRON_RING_ZIGZAG=0 at a shape the zig-zag schedule tiles (cp2, S_local 256): the
    reference's contiguous-chunk ring (context_parallel.py:130-155 of the reference), no re-lays,
    against the oracle on the whole sequence."""
    _dist.run(_llama_ring_plain, 2, 1, 2, 512, device="cuda")


def _ring_api(rank, world):
    """ring_attention (context_parallel.py:14-15, RingAttentionFunc [B, H, S, D], GQA-expanded k/v
    as model.py:142-143 passes them) with the zig-zag schedule: out and dq / dk / dv of this rank's
    contiguous chunk against the oracle's full causal attention (fp32 from the same bf16 inputs)."""
    import math
    torch.cuda.set_device(0)
    from oracle import picotron_oracle as O
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.context_parallel import context_parallel as CP
    pgm.setup_process_group_manager(tp_size=1, cp_size=world, pp_size=1, dp_size=1)
    B, H, S, D = 1, 4, 256, 128
    g = torch.Generator().manual_seed(5)
    q, k, v, do = (torch.randn(B, H, world * S, D, generator=g).to(torch.bfloat16) for _ in range(4))
    sl = slice(rank * S, (rank + 1) * S)
    assert CP.zigzag_enabled(S, True)
    ql, kl, vl = (t[:, :, sl].cuda().requires_grad_(True) for t in (q, k, v))
    out = CP.ring_attention(ql, kl, vl, 1 / math.sqrt(D), True)
    out.backward(do[:, :, sl].cuda())
    qr, kr, vr = (t.float().requires_grad_(True) for t in (q, k, v))
    o_ref, _ = O.attention_lse(qr, kr, vr, 1 / math.sqrt(D), True)
    o_ref.backward(do.float())
    assert out.dtype == torch.bfloat16 and out.shape == ql.shape
    assert _rel(out, o_ref[:, :, sl]) < TOL
    for got, ref in ((ql.grad, qr.grad), (kl.grad, kr.grad), (vl.grad, vr.grad)):
        assert _rel(got, ref[:, :, sl]) < TOL


@pytest.mark.parametrize("world", [2, 4])
def test_ring_attention_api_zigzag(world):
    _dist.run(_ring_api, world, device="cuda")


def _dp_llama(rank, world, tp):
    """DataParallelBucket (data_parallel.py:93-165, bucket.py): fp32 main_grad written by the fused
    wgrad epilogues, grad_acc 2, bucket all-reduce on the last micro-batch; each DP rank sees its
    own tokens.  p.grad must be the average over ranks of the oracle's grads (x tp shards)."""
    import types
    os.environ["FLASH_ATTEN"] = "1"
    torch.cuda.set_device(0)
    from oracle import picotron_oracle as O
    from picotron_amd import functional as FN
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.context_parallel.context_parallel import apply_context_parallel
    from picotron_amd.data_parallel.data_parallel import DataParallelBucket
    from picotron_amd.model import Llama
    from picotron_amd.tensor_parallel.tensor_parallel import apply_tensor_parallel
    dp = world // tp
    m = pgm.setup_process_group_manager(tp_size=tp, cp_size=1, pp_size=1, dp_size=dp)
    cfg = types.SimpleNamespace(**CFG)
    full = {k: v.to(torch.bfloat16) for k, v in O.init_params(dict(CFG), seed=9).items()}
    with torch.device("cuda"):
        model = Llama(cfg)
        if tp > 1:
            apply_tensor_parallel(model)
    apply_context_parallel(model)
    model.to(torch.bfloat16)
    names = dict(model.named_parameters())
    with torch.no_grad():
        for n, p in names.items():
            p.copy_(_shard(full[n], p, m.tp_rank))
    ddp = DataParallelBucket(model)
    ga, S, V = 2, CFG["max_position_embeddings"], CFG["vocab_size"]
    g = torch.Generator().manual_seed(21)
    ids = torch.randint(0, V, (dp, ga, 2, S + 1), generator=g)     # [dp, ga, mbs, seq + 1]
    for i in range(ga):
        ddp.require_backward_grad_sync = (i == ga - 1)
        t = ids[m.dp_rank, i]
        lo = ddp(t[:, :-1].cuda())
        (FN.cross_entropy(lo.view(-1, V), t[:, 1:].reshape(-1).cuda()) / ga).backward()
    torch.cuda.synchronize()
    pf = {k: v.float().requires_grad_(True) for k, v in full.items()}
    cos, sin = O.get_cos_sin(S, 64, base=CFG["rope_theta"])
    for r in range(dp):
        for i in range(ga):
            t = ids[r, i]
            lo = O.llama_forward(t[:, :-1], pf, dict(CFG), cos.float(), sin.float(), norm=O.rmsnorm_flash_semantics)
            (F.cross_entropy(lo.reshape(-1, V), t[:, 1:].reshape(-1)) / (ga * dp)).backward()
    for n, p in names.items():
        assert p.grad is not None and p.grad.dtype == torch.bfloat16, n
        assert _rel(p.grad, _shard(pf[n].grad, p, m.tp_rank)) < TOL, n


def test_data_parallel_bucket_dp2():
    _dist.run(_dp_llama, 2, 1, device="cuda")


def test_data_parallel_bucket_dp2_tp2():
    _dist.run(_dp_llama, 4, 2, device="cuda")


# --------------------------------------------------------------------------- pipeline parallel
def _pp_llama(rank, world, kind):
    """BASELINE config 4's pipeline composition on the HIP path: PipelineParallel stages of the HIP
    Llama (embedding / decoder layers / final_norm + lm_head as the reference splits them) driven by
    the 1F1B or AFAB step over p2p; the lm_head's HipLogits meet F.cross_entropy(logits.transpose(1, 2))
    (pipeline_parallel.py:103,153), i.e. the HIP cross-entropy.  Against the oracle on the full model:
    the last stage's logging loss and every stage's gradients (summed over the micro-batches: the
    engine's loss is each micro-batch's mean, not divided by grad_acc)."""
    import types
    os.environ["FLASH_ATTEN"] = "1"
    torch.cuda.set_device(0)
    from oracle import picotron_oracle as O
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.model import Llama
    from picotron_amd.pipeline_parallel.pipeline_parallel import (PipelineParallel, train_step_pipeline_1f1b,
                                                                  train_step_pipeline_afab)
    from picotron_amd.train import SyntheticMicroBatchDataLoader
    m = pgm.setup_process_group_manager(tp_size=1, cp_size=1, pp_size=world, dp_size=1)
    seq, mbs, ga = 256, 2, 3
    cfg = types.SimpleNamespace(**dict(CFG, num_hidden_layers=3, max_position_embeddings=seq))
    full = {k: v.to(torch.bfloat16) for k, v in O.init_params(dict(CFG, num_hidden_layers=3), seed=7).items()}
    with torch.device("cuda"):
        model = PipelineParallel(Llama(cfg), cfg)
    model.to(torch.bfloat16)
    names = dict(model.named_parameters())
    assert set(names) <= set(full)
    with torch.no_grad():
        for n, p in names.items():
            p.copy_(full[n])
    loader = SyntheticMicroBatchDataLoader(mbs, seq, ga, CFG["vocab_size"], torch.device("cuda"), seed=1234)
    step = train_step_pipeline_1f1b if kind == "1f1b" else train_step_pipeline_afab
    loss = step(model, loader, (mbs, seq, CFG["hidden_size"]), torch.device("cuda"), torch.bfloat16)
    torch.cuda.synchronize()
    pf = {k: v.float().requires_grad_(True) for k, v in full.items()}
    cos, sin = O.get_cos_sin(seq, 64, base=CFG["rope_theta"])
    losses = []
    for i in range(ga):
        x, t = loader._inputs[i].cpu(), loader._targets[i].cpu()
        lo = O.llama_forward(x, pf, dict(CFG, num_hidden_layers=3), cos.float(), sin.float(),
                             norm=O.rmsnorm_flash_semantics)
        li = F.cross_entropy(lo.transpose(1, 2), t)
        li.backward()
        losses.append(li.item())
    if m.pp_is_last_stage:
        ref = sum(losses) / ga
        assert abs(loss - ref) < TOL * abs(ref), (loss, ref)
    for n, p in names.items():
        assert p.grad is not None, n
        assert _rel(p.grad, pf[n].grad) < TOL, n


@pytest.mark.parametrize("kind,world", [("1f1b", 2), ("afab", 2), ("1f1b", 3)])
def test_pipeline_parallel_llama(kind, world):
    _dist.run(_pp_llama, world, kind, device="cuda")


def _dp_overlap(rank, world):
    """Row f3: the bucket all-reduces are issued DURING the last micro-batch's backward, not after
    it (bucket.py:25-31: a bucket syncs once all its parameters reported ready; data_parallel.py:
    122-165).  The fused kernels report a weight ready as soon as its wgrad GEMM is enqueued, so
    with the backward running layers last-to-first, the buckets of layer L sync while layers
    L - 1 .. 0 still compute.  Host-side order of decoder-layer backward calls ('L') and bucket
    all-reduce issues ('B') over the last micro-batch: some 'B' precede the last 'L', every layer's
    buckets sync right after that layer's backward, and only the embedding's comes last."""
    import types
    os.environ["FLASH_ATTEN"] = "1"
    torch.cuda.set_device(0)
    from picotron_amd import functional as FN
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.data_parallel import bucket as BK
    from picotron_amd.data_parallel.data_parallel import DataParallelBucket
    from picotron_amd.model import Llama
    pgm.setup_process_group_manager(tp_size=1, cp_size=1, pp_size=1, dp_size=world)
    cfg = types.SimpleNamespace(**dict(CFG, num_hidden_layers=4))
    with torch.device("cuda"):
        model = Llama(cfg)
    model.to(torch.bfloat16)
    # 0.25 MiB fp32 buckets: every layer's weights span several buckets
    ddp = DataParallelBucket(model, bucket_cap_mb=0.25)
    events = []
    orig_bwd, orig_sync = FN.DecoderLayerFunction.backward, BK.Bucket.sync_gradient

    def bwd(ctx, *g):
        out = orig_bwd(ctx, *g)
        events.append("L")
        return out

    def sync(self):
        events.append(("B", self))
        return orig_sync(self)
    FN.DecoderLayerFunction.backward = staticmethod(bwd)
    BK.Bucket.sync_gradient = sync
    try:
        g = torch.Generator().manual_seed(rank)
        for i in range(2):
            ddp.require_backward_grad_sync = i == 1
            events.clear()
            ids = torch.randint(0, CFG["vocab_size"], (2, CFG["max_position_embeddings"] + 1), generator=g).cuda()
            lo = ddp(input_ids=ids[:, :-1])
            loss = FN.cross_entropy(lo.reshape(-1, CFG["vocab_size"]), ids[:, 1:].reshape(-1)) / 2
            loss.backward()
    finally:
        FN.DecoderLayerFunction.backward, BK.Bucket.sync_gradient = orig_bwd, orig_sync
    torch.cuda.synchronize()
    kinds = ["L" if e == "L" else "B" for e in events]
    assert kinds.count("L") == 4 and kinds.count("B") == len(ddp.bucket_manager.buckets), kinds
    last_l = max(i for i, k in enumerate(kinds) if k == "L")
    assert kinds.index("B") < kinds.index("L"), kinds          # the lm_head's buckets before any layer
    assert sum(k == "B" for k in kinds[:last_l]) >= len(kinds) // 2, kinds   # most overlap the backward
    emb = ddp.bucket_manager.buckets[ddp.bucket_manager.params_to_bucket_location[model.embedding.weight][2]]
    assert events[-1][1] is emb                               # only the embedding's bucket waits to the end
    if rank == 0:
        print("dp bucket issue order:", "".join(kinds))


def test_dp_bucket_allreduce_overlaps_last_backward():
    _dist.run(_dp_overlap, 2, device="cuda")


def _vp_ce(rank, world):
    """The TP lm_head's F.cross_entropy on the vocab shards (functional.VocabParallelCEFunction, no
    logits all-gather) against the reference's gathered logits (vp_ce = 0) and the fp32 loss: the
    reference's two call forms, reductions, ignore_index rows, and a stand-in read by another op."""
    from picotron_amd import functional as FN
    from picotron_amd import process_group_manager as pgm
    from picotron_amd import switches
    from picotron_amd.tensor_parallel.tensor_parallel import ColumnParallelLinear
    torch.cuda.set_device(0)
    m = pgm.setup_process_group_manager(tp_size=world, cp_size=1, pp_size=1, dp_size=1)
    B, S, H, V = 2, 256, 128, 512 * world      # V / world = 256: the vocab shards tile the CE statistics
    g = torch.Generator().manual_seed(5)
    w_full = (torch.randn(V, H, generator=g) * 0.05).to(torch.bfloat16)
    x_full = torch.randn(B, S, H, generator=g).to(torch.bfloat16)
    tgt = torch.randint(0, V, (B, S), generator=g)
    tgt[0, :7] = -100                                   # ignore_index rows
    lin = ColumnParallelLinear(H, V, bias=False, gather_output=True).cuda().to(torch.bfloat16)
    lin._pt_lm_head = True
    with torch.no_grad():
        lin.weight.copy_(w_full.narrow(0, m.tp_rank * (V // world), V // world))
    ref_loss = F.cross_entropy(x_full.float().reshape(-1, H) @ w_full.float().t(), tgt.reshape(-1))
    res = {}
    # the reference's two call forms and, through the same views, permute / contiguous spellings of
    # them; 'seqmajor' reorders the rows (sequence-major) with matching targets -- not a form the shard
    # rows can serve in order, so the stand-in gathers the logits and runs on them
    forms = ("rows", "bvs", "permute", "contig", "seqmajor")
    for vp in (1, 0):
        for form in forms:
            for red in ("mean", "sum", "none"):
                if form in ("permute", "contig", "seqmajor") and red != "mean":
                    continue
                with switches.override(vp_ce=vp):
                    x = x_full.cuda().requires_grad_(True)
                    lin.weight.grad = None
                    logits = lin(x)
                    assert FN._is_vp(logits) == bool(vp) and logits.shape == (B, S, V)
                    if form == "rows":
                        loss = F.cross_entropy(logits.view(-1, V), tgt.reshape(-1).cuda(), reduction=red)
                    elif form == "bvs":
                        loss = F.cross_entropy(logits.transpose(1, 2), tgt.cuda(), reduction=red)
                    elif form == "permute":
                        loss = F.cross_entropy(logits.permute(0, 2, 1), tgt.cuda(), reduction=red)
                    elif form == "contig":
                        loss = F.cross_entropy(logits.contiguous().view(-1, V), tgt.reshape(-1).cuda(), reduction=red)
                    else:
                        loss = F.cross_entropy(logits.transpose(0, 1).reshape(-1, V), tgt.t().reshape(-1).cuda(),
                                               reduction=red)
                    if vp:   # the shard path ran (no gather) exactly where the rows are in order
                        assert (logits._pt_vp.full is not None) == (form == "seqmajor"), form
                    (loss.float().sum() if red == "none" else loss.float()).backward()
                    torch.cuda.synchronize()
                    res[(vp, form, red)] = (loss.detach().float().cpu(), x.grad.float().cpu(),
                                            lin.weight.grad.float().cpu())
    for key, (l1, gx1, gw1) in res.items():
        l0, gx0, gw0 = res[(0,) + key[1:]]
        assert _rel(l1, l0) < 1e-2 and _rel(gx1, gx0) < 1e-2 and _rel(gw1, gw0) < 1e-2, key
    assert abs(res[(1, "rows", "mean")][0].item() - ref_loss.item()) < TOL * abs(ref_loss.item())
    # another op on the stand-in gathers the logits (as GatherFromModelParallelRegion) and runs on them
    with switches.override(vp_ce=1):
        logits = lin(x_full.cuda())
        full = (x_full.float().reshape(-1, H) @ w_full.float().t()).view(B, S, V)
        assert _rel(logits.float(), full) < 1e-2 and _rel(logits.view(-1, V)[3], full.view(-1, V)[3]) < 1e-2


@pytest.mark.parametrize("world", [2, 8])
def test_vocab_parallel_cross_entropy(world):
    _dist.run(_vp_ce, world, device="cuda")
