"""Parity at the BASELINE configs' real shapes (BASELINE.json configs 2-5), HIP path vs the CPU oracle
(fp32, from the same bf16 weights and inputs).  Tolerance: norm-relative 2e-2 (north_star's bf16
tolerance) for the activations, the input gradient and every weight gradient.

  * SmolLM-1.7B decoder layer, mbs 4 x seq 1024 (H 2048, I 8192, 32 heads of 64) -- config 2's
    every GEMM shape: the paired SwiGLU tile at N 16384, the RoPE q|k|v GEMM at N 6144, dX at K 16384;
  * Llama-2-7B decoder layer (H 4096, I 11008, 32 heads of 128; d 128 takes the separate RoPE
    kernel), mbs 2 x seq 1024 -- configs 4 and 5's layer;
  * the per-rank GEMM shapes of TP: Llama-2-7B at TP 2 (q|k|v 3 x 2048, I 5504 -- not a multiple of
    256, so the SwiGLU backward runs as its own kernel) and SmolLM-1.7B at TP 8 (q|k|v 3 x 256,
    4 heads, I 1024), as one rank's shard of the layer (the math of each rank's partial layer);
  * the CP = 8 ring block of config 5: S_local 4096, d 128 -- the diagonal (causal) and one
    off-diagonal (full) block merged in the forward kernel's epilogue, and both blocks' backward from
    the global O / LSE (context_parallel.py:19-155), against O.attention_lse /
    O.ring_attention_backward.
"""
import math

import pytest
import torch

from oracle import picotron_oracle as O
from picotron_amd import switches

pytestmark = pytest.mark.gpu
TOL = 2e-2
BF = torch.bfloat16


def rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


NAMES = ["input_layernorm.weight", "post_attention_layernorm.weight", "attention.q_proj.weight",
         "attention.k_proj.weight", "attention.v_proj.weight", "attention.out_proj.weight",
         "mlp.gate_proj.weight", "mlp.up_proj.weight", "mlp.down_proj.weight"]


def _weights(H, I, nh, nkv, d, seed):
    """bf16 weights with the reference's init distributions (model.py:110-120,173-182) and
    non-trivial norm weights, in the reference's state_dict naming."""
    g = torch.Generator().manual_seed(seed)

    def u(o, i):
        return ((torch.rand(o, i, generator=g) * 2 - 1) / math.sqrt(i)).to(BF)
    return {"input_layernorm.weight": (1 + 0.1 * torch.randn(H, generator=g)).to(BF),
            "post_attention_layernorm.weight": (1 + 0.1 * torch.randn(H, generator=g)).to(BF),
            "attention.q_proj.weight": u(nh * d, H), "attention.k_proj.weight": u(nkv * d, H),
            "attention.v_proj.weight": u(nkv * d, H), "attention.out_proj.weight": u(H, nh * d),
            "mlp.gate_proj.weight": u(I, H), "mlp.up_proj.weight": u(I, H), "mlp.down_proj.weight": u(H, I)}


def _layer_grads(B, S, H, I, nh, nkv, d, seed=0):
    """(y, dx, every weight grad) of one DecoderLayerFunction fwd + bwd at these dims (GPU)."""
    from picotron_amd import functional as FN
    from picotron_amd import process_group_manager as pgm
    pgm.setup_process_group_manager(1, 1, 1, 1)
    w = _weights(H, I, nh, nkv, d, seed)
    dev = torch.device("cuda")
    params = {k: torch.nn.Parameter(v.to(dev)) for k, v in w.items()}
    cos, sin = O.get_cos_sin(S, d, base=10000.0)
    g = torch.Generator().manual_seed(seed + 1)
    x = torch.randn(B, S, H, generator=g).to(BF).to(dev).requires_grad_(True)
    dy = torch.randn(B, S, H, generator=g).to(BF).to(dev)
    y = FN.DecoderLayerFunction.apply(x, *[params[n] for n in NAMES], cos.to(dev), sin.to(dev), 1e-5, 0, nh, nkv, d)
    y.backward(dy)
    torch.cuda.synchronize()
    return [y.detach(), x.grad] + [params[n].grad for n in NAMES]


def test_smollm_layer_norm_from_splitk_halves_is_bit_identical(monkeypatch):
    """At config 2's shape the gate|up dX is split-K (K 16384): its two f32 halves go straight into
    the post-attention norm backward (pt_rmsnorm_bwd_splitk) -- every output bit-identical to the
    sum pass + plain norm backward (PICOTRON_NORM_SPLITK=0).  The q|k|v dX stays one GEMM here
    (PICOTRON_DUAL_QKV=0; its split form is the next test)."""
    monkeypatch.setattr(switches.S, "dual_qkv", 0)
    outs = []
    for v in ("0", "1"):
        monkeypatch.setattr(switches.S, "norm_splitk", int(v))
        outs.append(_layer_grads(B=4, S=1024, H=2048, I=8192, nh=32, nkv=32, d=64, seed=11))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_smollm_layer_qkv_dx_split_beside_dw(monkeypatch):
    """tp = 1: the q|k|v dX as two split-K halves (summed by the input norm's backward) in one launch
    with the q|k|v and o_proj dW.  The dW tiles run the same 8-phase kernel over the same K order as
    the grouped dW launch: those gradients, the forward and everything upstream of the q|k|v dX are
    bit-identical; dX and the input norm's weight gradient differ only by the f32 split-K order
    (norm-relative 1e-3 here, far inside the 2e-2 tolerance)."""
    outs = []
    for v in ("0", "1"):
        monkeypatch.setattr(switches.S, "dual_qkv", int(v))
        outs.append(_layer_grads(B=4, S=1024, H=2048, I=8192, nh=32, nkv=32, d=64, seed=11))
    (y0, dx0, *g0), (y1, dx1, *g1) = outs
    assert torch.equal(y0, y1)
    for n, a, b in zip(NAMES, g0, g1):
        if n == "input_layernorm.weight":
            assert rel(b, a) < 1e-3, n
        else:
            assert torch.equal(a, b), n
    assert rel(dx1, dx0) < 1e-3


def test_smollm_layer_gate_up_dx_unsplit_beside_dw(monkeypatch):
    """gu_splitk = 0: the gate|up dX runs unsplit (bf16, 128 tiles) beside the gate|up dW in the
    dual launch (dX tiles first on every XCD) and the post-attention norm reads it directly.  The dW
    tiles and the forward are bit-identical to the split form; dX, the norm's weight gradient and
    everything below them differ only by the f32 split-K order."""
    outs = []
    for v in (1, 0):
        monkeypatch.setattr(switches.S, "gu_splitk", v)
        outs.append(_layer_grads(B=4, S=1024, H=2048, I=8192, nh=32, nkv=32, d=64, seed=13))
    (y0, dx0, *g0), (y1, dx1, *g1) = outs
    assert torch.equal(y0, y1)
    for n, a, b in zip(NAMES, g0, g1):
        if n in ("mlp.gate_proj.weight", "mlp.up_proj.weight", "mlp.down_proj.weight"):
            assert torch.equal(a, b), n
        else:
            assert rel(b, a) < 5e-3, n
    assert rel(dx1, dx0) < 5e-3


def _layer_parity(B, S, H, I, nh, nkv, d, seed=0, main_grad=False):
    """One decoder layer (model.py:204-209) fwd + bwd through functional.DecoderLayerFunction (the
    node model.DecoderLayer runs) at these dims vs the oracle.  main_grad: every weight carries an
    f32 `main_grad` as DataParallelBucket gives it (data_parallel.py:122-144), so each wgrad
    epilogue (the dual down_proj dX + dW launch included) accumulates in f32."""
    from picotron_amd import functional as FN
    from picotron_amd import process_group_manager as pgm
    pgm.setup_process_group_manager(1, 1, 1, 1)
    w = _weights(H, I, nh, nkv, d, seed)
    dev = torch.device("cuda")
    params = {k: torch.nn.Parameter(v.to(dev)) for k, v in w.items()}
    if main_grad:
        for p in params.values():
            p.main_grad = torch.zeros(p.shape, dtype=torch.float32, device=dev)
    cos, sin = O.get_cos_sin(S, d, base=10000.0)
    g = torch.Generator().manual_seed(seed + 1)
    x = torch.randn(B, S, H, generator=g).to(BF)
    dy = torch.randn(B, S, H, generator=g).to(BF)
    xg = x.to(dev).requires_grad_(True)
    y = FN.DecoderLayerFunction.apply(xg, *[params[n] for n in NAMES], cos.to(dev), sin.to(dev), 1e-5, 0, nh, nkv, d)
    y.backward(dy.to(dev))
    torch.cuda.synchronize()
    pr = {k: v.float().requires_grad_(True) for k, v in w.items()}
    xr = x.float().requires_grad_(True)
    yr = O.decoder_layer(xr, pr, cos.float(), sin.float(), nh, nkv, 1e-5, norm=O.rmsnorm_flash_semantics)
    yr.backward(dy.float())
    errs = {"y": rel(y, yr), "dx": rel(xg.grad, xr.grad)}
    for n in NAMES:
        errs["d" + n] = rel(params[n].main_grad if main_grad else params[n].grad, pr[n].grad)
    bad = {k: v for k, v in errs.items() if not v < TOL}
    assert not bad, (bad, errs)


def test_smollm_1_7b_layer_mbs4_seq1024():
    _layer_parity(B=4, S=1024, H=2048, I=8192, nh=32, nkv=32, d=64)


def test_smollm_1_7b_layer_f32_main_grad():
    _layer_parity(B=4, S=1024, H=2048, I=8192, nh=32, nkv=32, d=64, seed=7, main_grad=True)


def test_llama2_7b_layer_seq1024():
    _layer_parity(B=2, S=1024, H=4096, I=11008, nh=32, nkv=32, d=128)


def test_llama2_7b_tp2_shard_layer():
    _layer_parity(B=2, S=1024, H=4096, I=11008 // 2, nh=16, nkv=16, d=128, seed=3)


def test_smollm_1_7b_tp8_shard_layer():
    _layer_parity(B=4, S=1024, H=2048, I=8192 // 8, nh=4, nkv=4, d=64, seed=5)


def test_llama2_13b_layer():
    """Llama-2-13B's layer dims (H 5120: the wide-row RMSNorm kernels; I 13824, 40 heads of 128) at
    mbs 1 x seq 512."""
    _layer_parity(B=1, S=512, H=5120, I=13824, nh=40, nkv=40, d=128, seed=13)


def test_llama2_7b_tp8_shard_layer():
    """Llama-2-7B at TP 8: 4 heads of 128 and an intermediate shard of 1376, off the GEMM tiles'
    64-grid -- the gate|up / down projections on the padded GEMMs (kernels._linear_*_padded)."""
    _layer_parity(B=2, S=1024, H=4096, I=11008 // 8, nh=4, nkv=4, d=128, seed=11)


def test_cp8_ring_block_s4096_d128():
    """Rank 1 of a ring at S_local 4096, d 128 (Llama-2-7B CP = 8 at 32k, one head group): step 0 is
    the causal diagonal block, step 1 the full block of rank 0's K/V, merged into the running f32
    output / LSE by the forward kernel's epilogue; the backward of each block from the global O /
    LSE accumulates dQ and this step's dK / dV in f32."""
    from picotron_amd import kernels as K
    B, H, S, D = 1, 8, 4096, 128
    sc = 1 / math.sqrt(D)
    g = torch.Generator().manual_seed(17)
    q1, k0, v0, k1, v1, do = (torch.randn(B, S, H, D, generator=g).to(BF) for _ in range(6))
    dev = torch.device("cuda")
    qd, k0d, v0d, k1d, v1d, dod = (t.to(dev) for t in (q1, k0, v0, k1, v1, do))
    acc = torch.zeros(B, S, H, D, dtype=torch.float32, device=dev)
    lse = torch.full((B, H, S), float("-inf"), dtype=torch.float32, device=dev)
    K.attn_fwd(qd, k1d, v1d, sc, True, out=acc, lse=lse, merge=True)
    K.attn_fwd(qd, k0d, v0d, sc, False, out=acc, lse=lse, merge=True)
    o = acc.to(BF)
    delta = K.attn_delta(dod, o)
    dq = torch.zeros(B, S, H, D, dtype=torch.float32, device=dev)
    dk1, dv1, dk0, dv0 = (torch.zeros(B, S, H, D, dtype=torch.float32, device=dev) for _ in range(4))
    K.attn_bwd(dod, qd, k1d, v1d, o, lse, sc, True, dq=dq, dk=dk1, dv=dv1, grad_f32=True, delta=delta)
    K.attn_bwd(dod, qd, k0d, v0d, o, lse, sc, False, dq=dq, dk=dk0, dv=dv0, grad_f32=True, delta=delta)
    torch.cuda.synchronize()

    def bhsd(t):
        return t.float().transpose(1, 2).contiguous()
    Q, K0, V0, K1, V1, dO = (bhsd(t) for t in (q1, k0, v0, k1, v1, do))
    Or, Lr = torch.empty_like(Q), torch.empty(B, H, S)
    dQr, dK0r, dV0r, dK1r, dV1r = (torch.empty_like(Q) for _ in range(5))
    for h0 in range(0, H, 4):   # head chunks bound the oracle's [S, S] score matrices
        hs = slice(h0, h0 + 4)
        o_c, l_c = O.attention_lse(Q[:, hs], K1[:, hs], V1[:, hs], sc, True)
        o_f, l_f = O.attention_lse(Q[:, hs], K0[:, hs], V0[:, hs], sc, False)
        L = torch.logaddexp(l_c, l_f)
        Oh = o_c * torch.exp(l_c - L).unsqueeze(-1) + o_f * torch.exp(l_f - L).unsqueeze(-1)
        Or[:, hs], Lr[:, hs] = Oh, L
        Ob = Oh.to(BF).float()   # the backward sees the bf16 output, as the kernels do
        a = O.ring_attention_backward(dO[:, hs], Q[:, hs], K1[:, hs], V1[:, hs], Ob, L, sc, True)
        b = O.ring_attention_backward(dO[:, hs], Q[:, hs], K0[:, hs], V0[:, hs], Ob, L, sc, False)
        dQr[:, hs], dK1r[:, hs], dV1r[:, hs] = a[0] + b[0], a[1], a[2]
        dK0r[:, hs], dV0r[:, hs] = b[1], b[2]
    errs = {"out": rel(acc.transpose(1, 2), Or), "lse": rel(lse, Lr), "dq": rel(dq.transpose(1, 2), dQr),
            "dk_diag": rel(dk1.transpose(1, 2), dK1r), "dv_diag": rel(dv1.transpose(1, 2), dV1r),
            "dk_off": rel(dk0.transpose(1, 2), dK0r), "dv_off": rel(dv0.transpose(1, 2), dV0r)}
    bad = {k: v for k, v in errs.items() if not v < TOL}
    assert not bad, (bad, errs)
    assert errs["lse"] < 1e-3, errs
