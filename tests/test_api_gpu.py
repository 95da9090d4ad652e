"""The reference API surface around the hot path on the GPU (HIP kernels through the C ABI):

  * update_out_and_lse (context_parallel.py:157-187) on the HIP merge kernel vs the reference's own
    outputs (G4, fp32 and the bf16-LSE behaviour);
  * ring_attention_backward (context_parallel.py:130-155) as a pure function vs the oracle;
  * F.cross_entropy as the reference's callers write it -- on the lm_head's output (HipLogits) and in
    the pipeline engine's [B, V, S] transpose form (pipeline_parallel.py:103,153) -- on the HIP
    kernel, and a target outside the vocabulary surfacing as an error (torch's device assert);
  * the lm_head after init_model_with_materialized_weights swaps in a torch nn.Linear
    (checkpoint.py:89-91): still the MFMA GEMM, same logits;
  * frozen (requires_grad=False) weights get no gradient from the fused kernels (autograd semantics).
Tolerances are stated per assertion."""
import math
import os
import types

import pytest
import torch
import torch.nn.functional as F

from oracle import picotron_oracle as O
from picotron_amd import switches

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
BF = torch.bfloat16


def rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


@pytest.fixture(autouse=True)
def _env(monkeypatch):
    monkeypatch.setenv("DEVICE", "cuda")
    monkeypatch.setenv("LOCAL_RANK", "0")
    monkeypatch.setenv("CONTEXT_PARALLEL", "0")
    monkeypatch.setenv("FLASH_ATTEN", "1")
    from picotron_amd import process_group_manager as pgm
    pgm.setup_process_group_manager(1, 1, 1, 1)


@pytest.mark.parametrize("tag", ["f32", "bf16"])
def test_update_out_and_lse_matches_reference_g4(tag):
    from picotron_amd.context_parallel.context_parallel import update_out_and_lse
    g = torch.load(os.path.join(GOLD, f"G4_{tag}.pt"), weights_only=True)
    dev = torch.device("cuda")
    out, lse = update_out_and_lse(None, None, g["o_causal"].to(dev), g["lse_causal"].to(dev))
    assert out.dtype == torch.float32 and lse.dtype == g["lse_causal"].dtype and lse.shape[-1] == 1
    out, lse = update_out_and_lse(out, lse, g["o_full"].to(dev), g["lse_full"].to(dev))
    assert lse.dtype == g["merged_lse"].dtype and lse.shape == g["merged_lse"].shape
    if tag == "f32":
        torch.testing.assert_close(out.cpu(), g["merged_out"], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(lse.cpu(), g["merged_lse"], rtol=1e-6, atol=1e-6)
    else:
        # the bf16 LSE path rounds op by op as torch's bf16 ops do: the reference's values to within
        # one bf16 ulp (the f32 transcendental may differ in its last bit before the rounding)
        ulp = g["merged_lse"].float().abs() * 2 ** -7
        assert ((lse.cpu().float() - g["merged_lse"].float()).abs() <= ulp + 1e-6).all()
        assert rel(out, g["merged_out"]) < 1e-2
    # slice_ form: merge rows [0, 4) of the sequence in place
    o2, l2 = update_out_and_lse(None, None, g["o_causal"].to(dev), g["lse_causal"].to(dev))
    sl = (slice(None), slice(None), slice(0, 4))
    o2, l2 = update_out_and_lse(o2, l2, g["o_full"][sl].to(dev), g["lse_full"][sl].to(dev), slice_=sl)
    assert rel(o2[sl], out[sl]) < 1e-6 and torch.equal(l2[sl].cpu(), lse[sl].cpu())


def test_fused_merge_ring_step_vs_reference_g4b():
    """Rank 1's ring step (causal diagonal block, then the full block from rank 0) with the merge
    fused into the attention kernel (f32 running LSE), against the reference's own two-stage result
    (G4b: ring_attention_forward + update_out_and_lse) computed in f32 and in bf16.  The reference's
    bf16 path keeps the running LSE in bf16; ours keeps it in f32, so the bar is: no further from the
    f32 result than the reference's bf16 result is, and within 2e-2 (relative L2) of the latter."""
    g32 = torch.load(os.path.join(GOLD, "G4b_f32.pt"), weights_only=True)
    g16 = torch.load(os.path.join(GOLD, "G4b_bf16.pt"), weights_only=True)
    K = __import__("picotron_amd.kernels", fromlist=["attn_fwd"])
    tok = lambda t: t.cuda().transpose(1, 2)          # [B, H, S, D] -> [B, S, H, D] view
    q1, k0, v0, k1, v1 = (tok(g16[n]) for n in ("q1", "k0", "v0", "k1", "v1"))
    B, S, H, D = q1.shape
    acc = torch.zeros(B, S, H, D, dtype=torch.float32, device="cuda")
    lse = torch.full((B, H, S), -math.inf, dtype=torch.float32, device="cuda")
    sc = 1 / math.sqrt(D)
    K.attn_fwd(q1, k1, v1, sc, True, out=acc, lse=lse, merge=True)
    K.attn_fwd(q1, k0, v0, sc, False, out=acc, lse=lse, merge=True)
    out = acc.transpose(1, 2).cpu()
    err_ours, err_ref = rel(out, g32["out"]), rel(g16["out"], g32["out"])
    assert err_ours <= err_ref + 1e-4, (err_ours, err_ref)
    assert rel(out, g16["out"]) < 2e-2
    torch.testing.assert_close(lse.cpu(), g32["lse"].squeeze(-1), rtol=1e-4, atol=1e-4)


def test_ring_attention_backward_pure_function():
    from picotron_amd.context_parallel import context_parallel as CP
    B, H, S, D = 2, 4, 256, 64
    sc = 1 / math.sqrt(D)
    g = torch.Generator().manual_seed(3)
    q, k, v, do = (torch.randn(B, H, S, D, generator=g).to(BF) for _ in range(4))
    for causal in (True, False):
        o, lse = O.attention_lse(q.float(), k.float(), v.float(), sc, causal)
        dq, dk, dv = CP.ring_attention_backward(do.cuda(), q.cuda(), k.cuda(), v.cuda(), o.to(BF).cuda(),
                                                lse.cuda(), sc, causal)
        rq, rk, rv = O.ring_attention_backward(do.float(), q.float(), k.float(), v.float(), o.to(BF).float(), lse,
                                               sc, causal)
        assert rel(dq, rq) < 2e-2 and rel(dk, rk) < 2e-2 and rel(dv, rv) < 2e-2


def _tiny_llama(layers=1):
    from picotron_amd.model import Llama
    cfg = types.SimpleNamespace(hidden_size=256, intermediate_size=512, num_attention_heads=4, num_key_value_heads=2,
                                vocab_size=512, rms_norm_eps=1e-5, rope_theta=10000.0, num_hidden_layers=layers,
                                max_position_embeddings=128)
    torch.manual_seed(0)
    with torch.device("cuda"):
        m = Llama(cfg)
    return m.to(BF), cfg


def test_reference_call_sites_take_the_hip_cross_entropy():
    """train.py:49 and pipeline_parallel.py:103 call torch's F.cross_entropy on the model output;
    the output is HipLogits, so both forms run csrc/cross_entropy.hip -- same loss and gradient as
    torch's kernel on the same bf16 logits (rel 1e-2 / 2e-2)."""
    from picotron_amd import functional as FN
    model, cfg = _tiny_llama()
    ids = torch.randint(0, cfg.vocab_size, (2, 129), generator=torch.Generator().manual_seed(4)).cuda()
    logits = model(ids[:, :-1])
    assert isinstance(logits, FN.HipLogits) and isinstance(logits.view(-1, cfg.vocab_size), FN.HipLogits)
    calls = []
    orig = FN.cross_entropy

    def spy(*a, **k):
        calls.append(a[0].shape)
        return orig(*a, **k)
    FN.cross_entropy = spy
    try:
        l1 = F.cross_entropy(logits.view(-1, cfg.vocab_size), ids[:, 1:].reshape(-1), reduction="mean")
        l2 = F.cross_entropy(logits.transpose(1, 2), ids[:, 1:], reduction="mean")
    finally:
        FN.cross_entropy = orig
    assert len(calls) == 2 and type(l1) is torch.Tensor
    plain = logits.detach().as_subclass(torch.Tensor).float().requires_grad_(True)
    ref = F.cross_entropy(plain.view(-1, cfg.vocab_size), ids[:, 1:].reshape(-1))
    assert abs(l1.float().item() - ref.item()) < 1e-2 * abs(ref.item())
    assert abs(l2.float().item() - ref.item()) < 1e-2 * abs(ref.item())
    # the transpose form's gradient flows back through the views
    lg = logits.detach().as_subclass(torch.Tensor).clone().requires_grad_(True)
    FN.cross_entropy(lg.transpose(1, 2), ids[:, 1:]).backward()
    ref.backward()
    assert rel(lg.grad, plain.grad) < 2e-2


def test_cross_entropy_bad_target_is_an_error():
    """A target outside [0, V) (not ignore_index): no out-of-bounds read, a NaN loss, and the device
    status word raises at the next check (train_step checks after its per-step host read)."""
    from picotron_amd import functional as FN
    from picotron_amd import kernels as K
    from picotron_amd._C import HipKernelError
    K.device_status(torch.device("cuda"))   # clear
    lg = torch.randn(16, 1000, device="cuda").to(BF).requires_grad_(True)
    tgt = torch.randint(0, 1000, (16,), device="cuda")
    tgt[5] = 1000
    loss = FN.cross_entropy(lg, tgt)
    assert math.isnan(loss.float().item())
    with pytest.raises(HipKernelError, match="outside"):
        K.check_device_status(torch.device("cuda"))
    K.check_device_status(torch.device("cuda"))   # cleared by the read
    tgt[5] = -7
    FN.cross_entropy(lg, tgt).backward()
    assert torch.isnan(lg.grad[5].float()).all() and not torch.isnan(lg.grad[4].float()).any()
    with pytest.raises(HipKernelError):
        K.check_device_status(torch.device("cuda"))


def test_cross_entropy_bad_target_raises_at_next_call_without_check():
    """The drop-in path (the reference's train.py) never calls check_device_status: the status word's
    pinned mirror makes the next cross_entropy call raise once the bad call's copy has landed."""
    from picotron_amd import functional as FN
    from picotron_amd import kernels as K
    from picotron_amd._C import HipKernelError
    K.device_status(torch.device("cuda"))
    lg = torch.randn(16, 1000, device="cuda").to(BF)
    tgt = torch.randint(0, 1000, (16,), device="cuda")
    bad = tgt.clone()
    bad[2] = 4000
    assert math.isnan(FN.cross_entropy(lg, bad).float().item())   # .item(): the host syncs, as train.py's print
    with pytest.raises(HipKernelError, match="outside"):
        FN.cross_entropy(lg, tgt)
    assert not math.isnan(FN.cross_entropy(lg, tgt).float().item())   # reported once, then cleared
    K.check_device_status(torch.device("cuda"))


def test_lm_head_swapped_for_torch_linear_stays_on_hip_gemm():
    """checkpoint.py:89-91 replaces final_proj by a torch nn.Linear; Llama.forward still runs it on
    the MFMA GEMM (bit-identical logits to the build's own Linear with the same weight)."""
    from picotron_amd import functional as FN
    model, cfg = _tiny_llama()
    ids = torch.randint(0, cfg.vocab_size, (2, 128), generator=torch.Generator().manual_seed(5)).cuda()
    before = model(ids).detach().clone()
    w = model.final_proj.weight.detach().clone()
    model.final_proj = torch.nn.Linear(cfg.hidden_size, cfg.vocab_size, bias=False, device="cuda", dtype=BF)
    with torch.no_grad():
        model.final_proj.weight.copy_(w)
    calls = []
    orig = FN.lm_head_linear
    FN.lm_head_linear = lambda *a, **k: (calls.append(a[1].shape), orig(*a, **k))[1]
    try:
        after = model(ids)
    finally:
        FN.lm_head_linear = orig
    assert calls == [w.shape] and isinstance(after, FN.HipLogits)
    assert torch.equal(after.detach().as_subclass(torch.Tensor), before.as_subclass(torch.Tensor))


def _pipeline_stage_forward(model, final_norm, final_proj, input_ids):
    """PipelineParallel.forward (pipeline_parallel.py:53-63) of a single (first and last) stage,
    restated: embedding -> decoder layers (position_ids keyword) -> final_norm -> final_proj called
    DIRECTLY (not through model.py:270 / Llama.forward)."""
    x = model.embedding(input_ids)
    for layer in model.decoder_layers:
        x = layer(x, position_ids=None)
    x = final_norm(x)
    return final_proj(x)


def test_pipeline_engine_lm_head_and_ce_stay_on_hip():
    """checkpoint.py:89-90 installs a torch nn.Linear final_proj on the PipelineParallel wrapper and
    pipeline_parallel.py:63 calls it directly; then F.cross_entropy(output.transpose(1, 2), target)
    (pipeline_parallel.py:103,153).  The final norm's HipHidden output routes nn.Linear's F.linear
    to the HIP lm_head GEMM: HipLogits bit-identical to Llama.forward's, the CE on the HIP kernel
    (with the GEMM's statistics), and gradients equal to the Llama.forward path's."""
    from picotron_amd import functional as FN
    model, cfg = _tiny_llama(layers=2)
    ids = torch.randint(0, cfg.vocab_size, (2, 129), generator=torch.Generator().manual_seed(6)).cuda()
    inp, tgt = ids[:, :-1], ids[:, 1:]
    ref_logits = model(inp)
    FN.cross_entropy(ref_logits.transpose(1, 2), tgt).backward()
    ref_grads = {n: p.grad.detach().clone() for n, p in model.named_parameters()}
    model.zero_grad(set_to_none=True)

    lin = torch.nn.Linear(cfg.hidden_size, cfg.vocab_size, bias=False, device="cuda", dtype=BF)
    with torch.no_grad():
        lin.weight.copy_(model.final_proj.weight)
    gemm_calls, ce_calls = [], []
    orig_lm, orig_ce, orig_take = FN.lm_head_linear, FN.cross_entropy, FN._take_ce_stats
    took = []
    FN.lm_head_linear = lambda *a, **k: (gemm_calls.append(a[1].shape), orig_lm(*a, **k))[1]
    FN.cross_entropy = lambda *a, **k: (ce_calls.append(a[0].shape), orig_ce(*a, **k))[1]
    FN._take_ce_stats = lambda lg: (lambda s: (took.append(s is not None), s)[1])(orig_take(lg))
    try:
        out = _pipeline_stage_forward(model, model.final_norm, lin, inp)
        loss = F.cross_entropy(out.transpose(1, 2), tgt)
        loss.backward()
    finally:
        FN.lm_head_linear, FN.cross_entropy, FN._take_ce_stats = orig_lm, orig_ce, orig_take
    assert isinstance(out, FN.HipLogits) and gemm_calls == [lin.weight.shape]
    assert len(ce_calls) == 1 and took == [True]
    assert torch.equal(out.detach().as_subclass(torch.Tensor), ref_logits.detach().as_subclass(torch.Tensor))
    assert torch.equal(lin.weight.grad, ref_grads["final_proj.weight"])
    for n, p in model.named_parameters():
        if n != "final_proj.weight":
            assert torch.equal(p.grad, ref_grads[n]), n


def test_cross_entropy_reductions_match_torch():
    """Consumers of the logits other than train.py:49 (eval scripts): reduction 'sum' / 'none' run the
    HIP kernel and match torch on the same bf16 logits (loss rel 1e-2, gradient rel 2e-2, ignored
    rows 0); class weights / label smoothing are torch's own op."""
    from picotron_amd import functional as FN
    model, cfg = _tiny_llama()
    ids = torch.randint(0, cfg.vocab_size, (2, 129), generator=torch.Generator().manual_seed(7)).cuda()
    tgt = ids[:, 1:].clone()
    tgt[0, :5] = -100
    logits = model(ids[:, :-1]).detach()
    for red in ("sum", "none"):
        lg = logits.as_subclass(torch.Tensor).clone().requires_grad_(True)
        ref_in = lg.detach().float().requires_grad_(True)
        for form in ("rows", "bvs"):
            lg.grad, ref_in.grad = None, None
            hip_in = FN.as_logits(lg)
            if form == "rows":
                out = F.cross_entropy(hip_in.view(-1, cfg.vocab_size), tgt.reshape(-1), reduction=red)
                ref = F.cross_entropy(ref_in.view(-1, cfg.vocab_size), tgt.reshape(-1), reduction=red)
            else:
                out = F.cross_entropy(hip_in.transpose(1, 2), tgt, reduction=red)
                ref = F.cross_entropy(ref_in.transpose(1, 2), tgt, reduction=red)
            assert out.shape == ref.shape and out.dtype == BF
            assert rel(out, ref) < 1e-2, (red, form)
            if red == "none":
                assert (out.reshape(-1)[tgt.reshape(-1) == -100] == 0).all()
            g = torch.rand_like(ref)
            out.backward(g.to(BF))
            ref.backward(g)
            assert rel(lg.grad, ref_in.grad) < 2e-2, (red, form)
    ls = F.cross_entropy(FN.as_logits(logits).view(-1, cfg.vocab_size), tgt.reshape(-1), label_smoothing=0.1)
    ref = F.cross_entropy(logits.as_subclass(torch.Tensor).view(-1, cfg.vocab_size), tgt.reshape(-1),
                          label_smoothing=0.1)
    assert torch.equal(ls, ref)


def test_frozen_weights_get_no_gradient():
    from picotron_amd import functional as FN
    model, cfg = _tiny_llama()
    frozen = [model.decoder_layers[0].attention.k_proj.weight, model.decoder_layers[0].mlp.up_proj.weight,
              model.decoder_layers[0].input_layernorm.weight, model.embedding.weight]
    for p in frozen:
        p.requires_grad_(False)
    ids = torch.randint(0, cfg.vocab_size, (2, 129), generator=torch.Generator().manual_seed(6)).cuda()
    FN.cross_entropy(model(ids[:, :-1]).view(-1, cfg.vocab_size), ids[:, 1:].reshape(-1)).backward()
    for p in frozen:
        assert p.grad is None
    for n, p in model.named_parameters():
        if p.requires_grad:
            assert p.grad is not None and torch.isfinite(p.grad.float()).all(), n


def test_lm_head_ce_statistics_epilogue():
    """pt_gemm_ce_stats: the logits are bit-identical to the plain lm_head GEMM on the same tile, and
    each row's (max, sum exp(x - max)) per 256- (8-phase) or 128-column (4-phase) tile equals torch's
    on the stored bf16 logits (max exact, sum rel 1e-5)."""
    from picotron_amd import kernels as K
    g = torch.Generator(device="cuda").manual_seed(11)
    for T, H, V in ((512, 256, 1536), (256, 128, 640)):   # block 256 / block 128
        x = (torch.randn(T, H, device="cuda", generator=g)).to(BF)
        w = (torch.randn(V, H, device="cuda", generator=g) * 0.2).to(BF)
        y, stats = K.linear_ce_stats(x, w)
        block = K.ce_stats_block(T, V)
        assert stats.shape == (V // block, T, 2)
        assert torch.equal(y, K.linear_fwd(x, [w], tile=12 if block == 256 else 13))
        blk = y.float().view(T, V // block, block).transpose(0, 1)
        m = blk.amax(-1)
        se = torch.exp(blk - m[..., None]).sum(-1)
        torch.testing.assert_close(stats[..., 0], m, rtol=0, atol=0)
        torch.testing.assert_close(stats[..., 1], se, rtol=1e-5, atol=1e-6)


def test_cross_entropy_from_lm_head_statistics():
    """Llama forward + F.cross_entropy with the lm_head's statistics (PICOTRON_CE_STATS=1, default)
    against the streaming CE kernel (=0): loss within 1e-6 relative, every gradient within 1e-3;
    the statistics are used only for the unmodified logits they were computed from."""
    from picotron_amd import functional as FN
    from picotron_amd import kernels as K
    ids = torch.randint(0, 512, (2, 129), generator=torch.Generator().manual_seed(8)).cuda()
    res = {}
    for flag in ("1", "0"):
        with switches.override(ce_stats=int(flag)):
            model, cfg = _tiny_llama()
            used = []
            orig = K.cross_entropy_loss_lse_stats
            K.cross_entropy_loss_lse_stats = lambda *a, **k: (used.append(1), orig(*a, **k))[1]
            try:
                loss = F.cross_entropy(model(ids[:, :-1]).view(-1, cfg.vocab_size), ids[:, 1:].reshape(-1))
            finally:
                K.cross_entropy_loss_lse_stats = orig
            loss.backward()
            res[flag] = (loss.float().item(), {n: p.grad.float().clone() for n, p in model.named_parameters()}, used)
    assert res["1"][2] == [1] and res["0"][2] == []
    assert abs(res["1"][0] - res["0"][0]) <= 1e-6 * abs(res["0"][0])
    for n, gr in res["0"][1].items():
        assert rel(res["1"][1][n], gr) < 1e-3, n
    # logits changed in place after the GEMM: the statistics no longer describe them -> streaming path
    model, cfg = _tiny_llama()
    used = []
    orig = K.cross_entropy_loss_lse_stats
    K.cross_entropy_loss_lse_stats = lambda *a, **k: (used.append(1), orig(*a, **k))[1]
    try:
        with torch.no_grad():
            logits = model(ids[:, :-1])
            logits.mul_(0.5)
            l_mod = F.cross_entropy(logits.view(-1, cfg.vocab_size), ids[:, 1:].reshape(-1))
    finally:
        K.cross_entropy_loss_lse_stats = orig
    plain = logits.detach().as_subclass(torch.Tensor).float()
    ref = F.cross_entropy(plain.view(-1, cfg.vocab_size), ids[:, 1:].reshape(-1))
    assert used == [] and abs(l_mod.float().item() - ref.item()) < 1e-2 * abs(ref.item())


def test_cross_entropy_stats_bad_target():
    from picotron_amd import functional as FN
    from picotron_amd import kernels as K
    from picotron_amd._C import HipKernelError
    K.device_status(torch.device("cuda"))
    x = torch.randn(256, 128, device="cuda").to(BF)
    w = (torch.randn(1024, 128, device="cuda") * 0.1).to(BF)
    y = FN.LMHeadFunction.apply(x, w, False)
    tgt = torch.randint(0, 1024, (256,), device="cuda")
    tgt[3] = 5000
    loss = FN.cross_entropy(y, tgt)
    assert math.isnan(loss.float().item())
    with pytest.raises(HipKernelError, match="outside"):
        K.check_device_status(torch.device("cuda"))
