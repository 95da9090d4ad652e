"""Model-level parity on the GPU: the fused decoder layer / attention / MLP / Llama / cross-entropy
of picotron_amd (HIP kernels through the C ABI) against the CPU oracle (oracle/picotron_oracle.py,
a plain-torch restatement of the reference path pinned to the reference's own outputs) evaluated in
fp32 on the same bf16 weights and inputs.  Tolerance: norm-relative 2e-2 (north_star's bf16
tolerance), stated per assertion."""
import math
import types

import pytest
import torch
import torch.nn.functional as F

from oracle import picotron_oracle as O

pytestmark = pytest.mark.gpu
BF = torch.bfloat16
TOL = 2e-2


def rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def cfg_tiny(layers=2, H=256, I=512, nh=4, nkv=2, V=512, S=128):
    return types.SimpleNamespace(hidden_size=H, intermediate_size=I, num_attention_heads=nh, num_key_value_heads=nkv,
                                 vocab_size=V, rms_norm_eps=1e-5, rope_theta=10000.0, num_hidden_layers=layers,
                                 max_position_embeddings=S)


@pytest.fixture(autouse=True)
def _env(monkeypatch):
    monkeypatch.setenv("DEVICE", "cuda")
    monkeypatch.setenv("LOCAL_RANK", "0")
    monkeypatch.setenv("CONTEXT_PARALLEL", "0")
    from picotron_amd import process_group_manager as pgm
    pgm.setup_process_group_manager(1, 1, 1, 1)
    torch.manual_seed(0)


def _params_f32(module, prefix=""):
    return {prefix + k: v.detach().float().cpu().requires_grad_(True) for k, v in module.named_parameters()}


@pytest.mark.parametrize("flash,nkv,d", [("1", 2, 64), ("0", 4, 64), ("1", 2, 128)])
def test_decoder_layer_matches_oracle(monkeypatch, flash, nkv, d):
    monkeypatch.setenv("FLASH_ATTEN", flash)
    from picotron_amd.model import DecoderLayer
    nh = 4
    cfg = cfg_tiny(H=nh * d, I=512, nh=nh, nkv=nkv, S=256)
    with torch.device("cuda"):
        layer = DecoderLayer(cfg, 0)
    layer.to(BF)
    for n in (layer.input_layernorm, layer.post_attention_layernorm):   # non-trivial norm weights
        with torch.no_grad():
            n.weight.copy_(1 + 0.1 * torch.randn_like(n.weight))
    x = torch.randn(2, 256, nh * d).to(BF)
    dy = torch.randn(2, 256, nh * d).to(BF)
    xg = x.cuda().requires_grad_(True)
    y = layer(xg)
    y.backward(dy.cuda())
    p = _params_f32(layer)
    xr = x.float().requires_grad_(True)
    cos, sin = O.get_cos_sin(256, d, base=10000.0)
    norm = O.rmsnorm_flash_semantics if flash == "1" else O.rmsnorm_llama
    yr = O.decoder_layer(xr, p, cos.float(), sin.float(), nh, nkv, 1e-5, norm=norm)
    yr.backward(dy.float())
    assert rel(y, yr) < TOL
    assert rel(xg.grad, xr.grad) < TOL
    for n, q in layer.named_parameters():
        assert rel(q.grad, p[n].grad) < TOL, n


def test_attention_and_mlp_modules(monkeypatch):
    monkeypatch.setenv("FLASH_ATTEN", "1")
    from picotron_amd.model import MLP, Attention, get_cos_sin
    cfg = cfg_tiny(H=256, nh=4, nkv=2, S=128)
    with torch.device("cuda"):
        att, mlp = Attention(cfg, 0), MLP(cfg)
    att.to(BF), mlp.to(BF)
    cos, sin = get_cos_sin(128, 64, base=10000.0)
    x = torch.randn(2, 128, 256).to(BF)
    dy = torch.randn(2, 128, 256).to(BF)
    for mod, fwd in ((att, lambda m, t: m(t, cos, sin)), (mlp, lambda m, t: m(t))):
        xg = x.cuda().requires_grad_(True)
        y = fwd(mod, xg)
        y.backward(dy.cuda())
        p = _params_f32(mod)
        xr = x.float().requires_grad_(True)
        if mod is att:
            yr = O.attention(xr, p["q_proj.weight"], p["k_proj.weight"], p["v_proj.weight"], p["out_proj.weight"],
                             cos.float().cpu(), sin.float().cpu(), 4, 2)
        else:
            yr = O.mlp(xr, p["gate_proj.weight"], p["up_proj.weight"], p["down_proj.weight"])
        yr.backward(dy.float())
        assert rel(y, yr) < TOL
        assert rel(xg.grad, xr.grad) < TOL
        for n, q in mod.named_parameters():
            assert rel(q.grad, p[n].grad) < TOL, n


def test_llama_loss_and_grads_match_oracle(monkeypatch):
    monkeypatch.setenv("FLASH_ATTEN", "1")
    from picotron_amd import functional as FN
    from picotron_amd.model import Llama
    cfg = cfg_tiny(layers=2)
    with torch.device("cuda"):
        model = Llama(cfg)
    model.to(BF)
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(0, cfg.vocab_size, (2, 129), generator=g)
    ga = 4
    logits = model(ids[:, :-1].cuda())
    loss = FN.cross_entropy(logits.view(-1, cfg.vocab_size), ids[:, 1:].reshape(-1).cuda()) / ga
    loss.backward()
    p = _params_f32(model)
    cos, sin = O.get_cos_sin(128, 64, base=10000.0)
    lr = O.llama_forward(ids[:, :-1], p, dict(vars(cfg)), cos.float(), sin.float(), norm=O.rmsnorm_flash_semantics)
    loss_r = F.cross_entropy(lr.reshape(-1, cfg.vocab_size), ids[:, 1:].reshape(-1)) / ga
    loss_r.backward()
    assert loss.dtype == BF                       # F.cross_entropy on bf16 logits returns bf16
    assert abs(loss.float().item() - loss_r.item()) < TOL * abs(loss_r.item())
    assert rel(logits, lr) < TOL
    for n, q in model.named_parameters():
        assert rel(q.grad, p[n].grad) < TOL, n


def test_grad_accumulation_bf16_sinks(monkeypatch):
    """Two micro-batches accumulate into bf16 param.grad through the GEMM epilogue (the DP=1 path
    of train.py: autograd accumulates bf16 grads across grad_acc, SURVEY §8c caveat 2)."""
    monkeypatch.setenv("FLASH_ATTEN", "1")
    from picotron_amd import functional as FN
    from picotron_amd.model import Llama
    cfg = cfg_tiny(layers=1)
    with torch.device("cuda"):
        model = Llama(cfg)
    model.to(BF)
    g = torch.Generator().manual_seed(2)
    ids = [torch.randint(0, cfg.vocab_size, (2, 129), generator=g) for _ in range(2)]
    for t in ids:
        lo = model(t[:, :-1].cuda())
        (FN.cross_entropy(lo.view(-1, cfg.vocab_size), t[:, 1:].reshape(-1).cuda()) / 2).backward()
    acc = {n: q.grad.float().cpu().clone() for n, q in model.named_parameters()}
    ref = {}
    for t in ids:
        model.zero_grad(set_to_none=True)
        lo = model(t[:, :-1].cuda())
        (FN.cross_entropy(lo.view(-1, cfg.vocab_size), t[:, 1:].reshape(-1).cuda()) / 2).backward()
        for n, q in model.named_parameters():
            ref[n] = ref.get(n, 0) + q.grad.float().cpu()
    for n in acc:
        assert rel(acc[n], ref[n]) < 1e-2, n


def test_cross_entropy_function_matches_torch():
    from picotron_amd import functional as FN
    T, V = 256, 49152
    logits = (2 * torch.randn(T, V)).to(BF)
    tgt = torch.randint(0, V, (T,))
    tgt[3] = -100
    lg = logits.cuda().requires_grad_(True)
    loss = FN.cross_entropy(lg, tgt.cuda()) / 32
    loss.backward()
    lr = logits.float().requires_grad_(True)
    loss_r = F.cross_entropy(lr, tgt) / 32
    loss_r.backward()
    assert abs(loss.float().item() - loss_r.item()) < 1e-2 * abs(loss_r.item())
    assert rel(lg.grad, lr.grad) < TOL
    assert lg.grad[3].float().abs().max().item() == 0.0


@pytest.mark.parametrize("reduction", ["mean", "sum", "none"])
def test_cross_entropy_vocab_off_8_columns(reduction):
    """A vocabulary off the CE kernels' 8-column grid (GPT-2's 50257): the logits padded with -inf
    columns (nothing added to any row's softmax), the gradient's padded columns dropped -- loss and
    dlogits against torch, with an ignored row."""
    from picotron_amd import functional as FN
    T, V = 128, 50257
    logits = (2 * torch.randn(T, V)).to(BF)
    tgt = torch.randint(0, V, (T,))
    tgt[7] = -100
    lg = logits.cuda().requires_grad_(True)
    out = FN.cross_entropy(lg, tgt.cuda(), reduction=reduction)
    lr = logits.float().requires_grad_(True)
    ref = F.cross_entropy(lr, tgt, reduction=reduction)
    g = torch.randn(ref.shape) if reduction == "none" else torch.tensor(0.25)
    out.backward(g.to(out.dtype).cuda())
    ref.backward(g)
    assert rel(out.float(), ref) < 1e-2
    assert lg.grad.shape == (T, V) and rel(lg.grad, lr.grad) < TOL


def test_llama_vocab_off_8_columns(monkeypatch):
    """The full model at vocab 1001: the lm_head GEMM padded (off the 64-grid), the CE padded (off
    the 8-column grid) -- loss and every gradient against the oracle."""
    monkeypatch.setenv("FLASH_ATTEN", "1")
    from picotron_amd import functional as FN
    from picotron_amd.model import Llama
    cfg = cfg_tiny(layers=1, V=1001)
    with torch.device("cuda"):
        model = Llama(cfg)
    model.to(BF)
    g = torch.Generator().manual_seed(4)
    ids = torch.randint(0, cfg.vocab_size, (2, 129), generator=g)
    logits = model(ids[:, :-1].cuda())
    loss = FN.cross_entropy(logits.view(-1, cfg.vocab_size), ids[:, 1:].reshape(-1).cuda())
    loss.backward()
    p = _params_f32(model)
    cos, sin = O.get_cos_sin(128, 64, base=10000.0)
    lr = O.llama_forward(ids[:, :-1], p, dict(vars(cfg)), cos.float(), sin.float(), norm=O.rmsnorm_flash_semantics)
    loss_r = F.cross_entropy(lr.reshape(-1, cfg.vocab_size), ids[:, 1:].reshape(-1))
    loss_r.backward()
    assert abs(loss.float().item() - loss_r.item()) < TOL * abs(loss_r.item())
    for n, q in model.named_parameters():
        assert rel(q.grad, p[n].grad) < TOL, n


def test_residual_epilogue_exact():
    """GEMM residual epilogue == bf16(residual + bf16(x W^T)) bit for bit (torch's bf16 add)."""
    from picotron_amd import kernels as K
    x = torch.randn(256, 512).to(BF).cuda()
    w = (torch.randn(256, 512) / 16).to(BF).cuda()
    r = torch.randn(256, 256).to(BF).cuda()
    y = K.linear_fwd(x, [w])
    yr = K.linear_fwd(x, [w], residual=r)
    assert torch.equal(yr, (r.float() + y.float()).to(BF))


def test_flash_attention_api_and_ring_pure_functions():
    """model.flash_attention and the ring's per-block functions (reference [B,H,S,D] API)."""
    from picotron_amd.context_parallel import context_parallel as CP
    from picotron_amd.model import flash_attention
    B, H, S, D = 2, 4, 256, 64
    q, k, v = (torch.randn(B, H, S, D).to(BF) for _ in range(3))
    o = flash_attention(q.cuda(), k.cuda(), v.cuda(), causal=True)
    o_ref = O.sdpa_causal(q.float(), k.float(), v.float(), True).transpose(1, 2)
    assert rel(o, o_ref) < TOL
    sc = 1 / math.sqrt(D)
    for causal in (True, False):
        ob, lb = CP.ring_attention_forward(q.cuda(), k.cuda(), v.cuda(), sc, causal)
        orf, lrf = O.attention_lse(q.float(), k.float(), v.float(), sc, causal)
        assert rel(ob, orf) < TOL and rel(lb, lrf) < 1e-3


def test_data_parallel_bucket_fused_sinks_world1(monkeypatch):
    """DataParallelBucket over the fused model (fp32 main_grad written by the wgrad epilogue,
    grad_acc 2, world 1 on gloo): p.grad equals the plain bf16-accumulated gradients."""
    import socket
    import torch.distributed as dist
    monkeypatch.setenv("FLASH_ATTEN", "1")
    from picotron_amd import functional as FN
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.data_parallel.data_parallel import DataParallelBucket
    from picotron_amd.model import Llama
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        pgm.setup_process_group_manager(1, 1, 1, 1)
        cfg = cfg_tiny(layers=1)
        torch.manual_seed(3)
        with torch.device("cuda"):
            model = Llama(cfg)
        model.to(BF)
        ref_state = {k: v.clone() for k, v in model.state_dict().items()}
        g = torch.Generator().manual_seed(5)
        ids = [torch.randint(0, cfg.vocab_size, (2, 129), generator=g) for _ in range(2)]
        # reference: bf16 autograd accumulation (DP = 1 semantics)
        for t in ids:
            lo = model(t[:, :-1].cuda())
            (FN.cross_entropy(lo.view(-1, cfg.vocab_size), t[:, 1:].reshape(-1).cuda()) / 2).backward()
        want = {n: p.grad.float().clone() for n, p in model.named_parameters()}
        model.zero_grad(set_to_none=True)
        model.load_state_dict(ref_state)
        dp = DataParallelBucket(model)
        for i, t in enumerate(ids):
            dp.require_backward_grad_sync = (i == 1)
            lo = dp(t[:, :-1].cuda())
            (FN.cross_entropy(lo.view(-1, cfg.vocab_size), t[:, 1:].reshape(-1).cuda()) / 2).backward()
        for n, p in model.named_parameters():
            assert p.grad is not None and p.grad.dtype == BF, n
            assert rel(p.grad, want[n]) < 1e-2, n
    finally:
        dist.destroy_process_group()
        pgm.setup_process_group_manager(1, 1, 1, 1)


def test_loss_curve_50_steps_matches_oracle(monkeypatch):
    """north_star: "the loss curve within 1% over 50 steps".  The GPU path (bf16 weights, fused
    HIP layers, fused CE, bf16 grad accumulation over grad_acc, fused HIP AdamW) is trained with
    train_step (train.py:29-55) for 50 steps; the oracle runs the reference's own GPU numerics on the
    CPU from the same initial weights and tokens: bf16 parameters, grads and Adam states
    (model.to(bfloat16), train.py:170), each micro-batch's forward/backward in fp32 from those bf16
    weights, grads rounded to bf16 and accumulated in bf16 (autograd's .grad accumulation), and
    torch.optim.AdamW (train.py:209) stepping the bf16 tensors.  The loader repeats the same two
    micro-batches every step, so the curve falls (the model memorises them) and 1% is a real bar."""
    monkeypatch.setenv("FLASH_ATTEN", "1")
    from picotron_amd.model import Llama
    from picotron_amd.optim import AdamW
    from picotron_amd.train import SyntheticMicroBatchDataLoader, train_step
    cfg = cfg_tiny(layers=2)
    dev = torch.device("cuda")
    with torch.device(dev):
        model = Llama(cfg)
    model.to(BF)
    lr, steps, ga = 3e-4, 50, 2
    opt = AdamW(model.parameters(), lr=lr)
    loader = SyntheticMicroBatchDataLoader(2, 128, ga, cfg.vocab_size, dev, seed=1234)

    ref = {k: v.detach().cpu().clone() for k, v in model.named_parameters()}   # bf16 leaves
    ropt = torch.optim.AdamW(list(ref.values()), lr=lr, foreach=False)
    cos, sin = O.get_cos_sin(128, 64, base=10000.0)
    c = dict(vars(cfg))
    inputs, targets = loader._inputs.cpu(), loader._targets.cpu()

    def ref_step():
        for p in ref.values():
            p.grad = None
        total = 0.0
        for i in range(ga):
            pf = {k: v.float().requires_grad_(True) for k, v in ref.items()}
            lo = O.llama_forward(inputs[i], pf, c, cos.float(), sin.float(), norm=O.rmsnorm_flash_semantics)
            loss = F.cross_entropy(lo.reshape(-1, cfg.vocab_size), targets[i].reshape(-1)) / ga
            loss.backward()
            total += loss.item()
            for k, p in ref.items():
                g = pf[k].grad.to(BF)
                p.grad = g if p.grad is None else (p.grad + g)
        ropt.step()
        return total

    ours, theirs = [], []
    for _ in range(steps):
        opt.zero_grad()
        ours.append(train_step(model, loader, dev))
        opt.step()
        theirs.append(ref_step())
    dev_rel = [abs(a - b) / abs(b) for a, b in zip(ours, theirs)]
    assert theirs[-1] < theirs[0] - 0.5, theirs          # the curve actually moves
    assert max(dev_rel) < 1e-2, (max(dev_rel), ours[::10], theirs[::10])


def test_cross_entropy_edge_cases_match_torch():
    """F.cross_entropy's edge cases through the autograd pair: every target ignored (mean = nan,
    grads 0, as torch), a single row, and a vocabulary that is not a multiple of the 256-thread
    row stride (ragged last chunk)."""
    from picotron_amd import functional as FN
    for T, V, ignore_all in ((8, 96, True), (1, 49152, False), (16, 1000, False)):
        logits = (2 * torch.randn(T, V)).to(BF)
        tgt = torch.full((T,), -100) if ignore_all else torch.randint(0, V, (T,))
        lg = logits.cuda().requires_grad_(True)
        loss = FN.cross_entropy(lg, tgt.cuda())
        loss.backward()
        lr = logits.float().requires_grad_(True)
        loss_r = F.cross_entropy(lr, tgt)
        loss_r.backward()
        if ignore_all:
            assert math.isnan(loss.float().item()) and math.isnan(loss_r.item())
            assert lg.grad.float().abs().max().item() == 0.0 and lr.grad.abs().max().item() == 0.0
        else:
            assert abs(loss.float().item() - loss_r.item()) < 1e-2 * abs(loss_r.item())
            assert rel(lg.grad, lr.grad) < TOL


def test_unsupported_shapes_fail_loudly():
    """Shapes outside what the kernels and the host padding cover raise HipKernelError / ValueError /
    RuntimeError -- never a silent fallback: a non-causal block off the 128-row query blocks (only
    causal self-attention is padded), a head dim the kernel entry points do not take (the model's
    attention pads even dims below 128; the kernels themselves take 64 / 128), a head dim above 128."""
    from picotron_amd import kernels as K
    from picotron_amd._C import HipKernelError
    from picotron_amd.model import flash_attention
    q = torch.randn(1, 100, 2, 64, device="cuda").to(BF)
    with pytest.raises((HipKernelError, ValueError)):
        K.attn_fwd(q, q, q, 0.125, False)
    K.attn_fwd(q, q, q, 0.125, True)   # causal: zero-padded to 128 rows (test_kernels_gpu's off-block test)
    q = torch.randn(1, 128, 2, 32, device="cuda").to(BF)
    with pytest.raises((HipKernelError, ValueError)):
        K.attn_fwd(q, q, q, 0.125, True)
    q = torch.randn(1, 2, 128, 160, device="cuda").to(BF)
    with pytest.raises((HipKernelError, ValueError, RuntimeError)):
        flash_attention(q, q, q, True)
