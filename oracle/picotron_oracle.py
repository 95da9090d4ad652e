"""CPU oracle: a restatement of picotron's decoder-layer hot path in plain PyTorch (fp32 by default).

TEST INFRASTRUCTURE ONLY.  Nothing in picotron_amd/ imports this module; only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg use it -- as the checker / baseline,
never as the thing measured or shipped.

Parity status: PINNED.  Every function below is checked against golden vectors produced by
importing the reference itself in the build container (tests/golden/make_golden.py ->
tests/golden/*.pt, test tests/test_oracle_golden.py).  The reference's GPU kernels live in
flash-attn 2.5.0 (requirements.txt:6), which is not installed here; its semantics are restated
from the reference's own equivalent eager path (FLASH_ATTEN=0): see each function.

All paths below are relative to the reference checkout (okoge-kaz/picotron @ 2025-03-02).
Layout conventions follow the reference: attention tensors are [B, H, S, D].
"""
import math

import torch
import torch.nn.functional as F


# ------------------------------------------------------------------ rotary tables / RoPE
def get_cos_sin(seq_length, head_dim, base=500000.0, dtype=torch.bfloat16):
    """picotron/model.py:21-31: inverse frequencies on CPU in fp32, position*theta in fp32,
    cos/sin cast to the table dtype (bf16 by default, DTYPE is never set) and repeated (1, 2)."""
    assert head_dim % 2 == 0
    exps = torch.arange(0, head_dim, 2, dtype=torch.int64).float() / head_dim
    inv_freq = 1.0 / (base ** exps)
    pos = torch.arange(seq_length).float().unsqueeze(1)
    ang = pos * inv_freq.float()
    return ang.cos().to(dtype).repeat(1, 2), ang.sin().to(dtype).repeat(1, 2)


def apply_rotary_pos_emb(x, cos, sin):
    """picotron/model.py:12-19 (eager, [B, H, S, D]): x*cos + rotate_half(x)*sin."""
    half = x.shape[-1] // 2
    rot = torch.cat([-x[..., half:], x[..., :half]], dim=-1)
    return x * cos + rot * sin


def rotary_flash_semantics(x, cos, sin):
    """flash-attn apply_rotary_emb(x, cos[:, :d/2], sin[:, :d/2], interleaved=False) as called at
    picotron/model.py:136-137: the rotation evaluated in fp32 and rounded once to x's dtype."""
    xf, c, s = x.float(), cos.float(), sin.float()
    half = x.shape[-1] // 2
    x1, x2 = xf[..., :half], xf[..., half:]
    c1, s1 = c[..., :half], s[..., :half]
    return torch.cat([x1 * c1 - x2 * s1, x2 * c1 + x1 * s1], dim=-1).to(x.dtype)


# ------------------------------------------------------------------------------ RMSNorm
def rmsnorm_llama(x, weight, eps):
    """picotron/model.py:81-86 LlamaRMSNorm: fp32 statistics, round to the input dtype, then * w."""
    dt = x.dtype
    xf = x.float()
    var = xf.pow(2).mean(-1, keepdim=True)
    return weight * (xf * torch.rsqrt(var + eps)).to(dt)


def rmsnorm_flash_semantics(x, weight, eps):
    """flash-attn layer_norm_fn(is_rms_norm=True) as called by TritonRMSNorm (model.py:51-65):
    y = x * rstd * w evaluated in fp32, rounded once to the input dtype."""
    xf = x.float()
    rstd = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (xf * rstd * weight.float()).to(x.dtype)


# ---------------------------------------------------------------------------- attention
def sdpa_causal(q, k, v, causal=True, scale=None):
    """picotron/model.py:157 F.scaled_dot_product_attention(q, k, v, is_causal) restated:
    softmax(q k^T * scale + mask) v over [B, H, S, D]."""
    d = q.shape[-1]
    scale = 1.0 / math.sqrt(d) if scale is None else scale
    s = torch.matmul(q.float(), k.float().transpose(-2, -1)) * scale
    if causal:
        sq, sk = s.shape[-2], s.shape[-1]
        mask = torch.ones(sq, sk, dtype=torch.bool).triu(1)
        s = s.masked_fill(mask, float("-inf"))
    p = torch.softmax(s, dim=-1)
    return torch.matmul(p, v.float()).to(q.dtype)


def attention_lse(q, k, v, scale, causal):
    """Block attention returning (O, LSE) in fp32: the quantities ring_attention_forward
    (context_parallel.py:112-128) computes; LSE = log(sum(exp(S))) with S = q k^T * scale."""
    s = torch.matmul(q.float(), k.float().transpose(-2, -1)) * scale
    if causal:
        n = s.shape[-1]
        s = s.masked_fill(torch.ones(n, n, dtype=torch.bool).triu(1), float("-inf"))
    m = s.amax(-1, keepdim=True)
    e = torch.exp(s - m)
    z = e.sum(-1, keepdim=True)
    return torch.matmul(e / z, v.float()), (torch.log(z) + m).squeeze(-1)


def ring_attention_forward(q, k, v, sm_scale, is_causal):
    """context_parallel.py:112-128, in the input dtype (so a bf16 block returns a bf16 LSE,
    which is the reference's behaviour noted in SURVEY §8c caveat 1)."""
    b, h, n, d = q.shape
    s = torch.matmul(q, k.transpose(-2, -1)) * sm_scale
    if is_causal:
        s = s.masked_fill(torch.ones(n, n, dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    mx = s.max(dim=-1, keepdim=True)[0]
    e = torch.exp(s - mx)
    z = e.sum(dim=-1, keepdim=True)
    return torch.matmul(e / z, v), (torch.log(z) + mx).squeeze(-1)


def ring_attention_backward(dO, Q, K, V, O, lse, sm_scale, is_causal):
    """context_parallel.py:130-155: recompute P from the global LSE; FA2 decomposition."""
    n = Q.shape[-2]
    s = torch.matmul(Q, K.transpose(-2, -1)) * sm_scale
    mask = torch.ones(n, n, dtype=torch.bool, device=Q.device).triu(1) if is_causal else None
    if is_causal:
        s = s.masked_fill(mask, float("-inf"))
    p = torch.exp(s - lse.unsqueeze(-1))
    dV = torch.matmul(p.transpose(-2, -1), dO)
    dP = torch.matmul(dO, V.transpose(-2, -1))
    D = (dO * O).sum(-1, keepdim=True)
    dS = p * (dP - D)
    if is_causal:
        dS = dS.masked_fill(mask, 0)
    return torch.matmul(dS, K) * sm_scale, torch.matmul(dS.transpose(-2, -1), Q) * sm_scale, dV


def update_out_and_lse(out, lse, block_out, block_lse):
    """context_parallel.py:157-187: out is accumulated in fp32; lse keeps the block's dtype
    on the first call.  out <- out - sigmoid(blse - lse) (out - bout); lse <- lse - logsigmoid(lse - blse)."""
    block_out = block_out.to(torch.float32)
    block_lse = block_lse.unsqueeze(-1)
    if out is None:
        return block_out, block_lse
    out = out - torch.sigmoid(block_lse - lse) * (out - block_out)
    lse = lse - F.logsigmoid(lse - block_lse)
    return out, lse


def ring_attention_simulated(q_shards, k_shards, v_shards, sm_scale, is_causal):
    """RingAttentionFunc.forward (context_parallel.py:19-51) for all ranks at once, without a
    process group: rank r at step s holds the K/V shard of rank (r - s) mod W."""
    W = len(q_shards)
    outs = []
    for r in range(W):
        out = lse = None
        for step in range(W):
            src = (r - step) % W
            if not is_causal or step <= r:
                bo, bl = ring_attention_forward(q_shards[r], k_shards[src], v_shards[src], sm_scale,
                                                is_causal and step == 0)
                out, lse = update_out_and_lse(out, lse, bo, bl)
        outs.append((out.to(q_shards[r].dtype), lse.squeeze(-1)))
    return outs


# -------------------------------------------------------------------------- layer pieces
def linear(x, w):
    """F.linear without bias (model.py:124-126,161,186; tensor_parallel.py:186)."""
    return torch.matmul(x, w.t())


def mlp(x, w_gate, w_up, w_down):
    """picotron/model.py:184-186: down(silu(gate(x)) * up(x))."""
    return linear(F.silu(linear(x, w_gate)) * linear(x, w_up), w_down)


def attention(x, wq, wk, wv, wo, cos, sin, n_heads, n_kv_heads):
    """picotron/model.py:122-162 (FLASH_ATTEN=0 path, no CP): q/k/v projections, RoPE, GQA
    repeat_interleave (:142-143), causal SDPA, output projection.  x is [B, S, H]."""
    b, s, hdim = x.shape
    d = wq.shape[0] // n_heads
    q = linear(x, wq).view(b, s, n_heads, d).transpose(1, 2)
    k = linear(x, wk).view(b, s, n_kv_heads, d).transpose(1, 2)
    v = linear(x, wv).view(b, s, n_kv_heads, d).transpose(1, 2)
    q = apply_rotary_pos_emb(q, cos, sin)
    k = apply_rotary_pos_emb(k, cos, sin)
    rep = n_heads // n_kv_heads
    k = k.repeat_interleave(rep, dim=1)
    v = v.repeat_interleave(rep, dim=1)
    o = sdpa_causal(q, k, v, causal=(q.shape[2] == k.shape[2]))
    return linear(o.transpose(1, 2).reshape(b, s, n_heads * d), wo)


def decoder_layer(x, p, cos, sin, n_heads, n_kv_heads, eps, norm=rmsnorm_llama):
    """picotron/model.py:204-209: x + Attn(norm1(x)); then x + MLP(norm2(x)).  p: dict of weights
    named as the reference's state_dict (input_layernorm, attention.{q,k,v,out}_proj, mlp.*)."""
    h = norm(x, p["input_layernorm.weight"], eps)
    x = x + attention(h, p["attention.q_proj.weight"], p["attention.k_proj.weight"], p["attention.v_proj.weight"],
                      p["attention.out_proj.weight"], cos, sin, n_heads, n_kv_heads)
    h = norm(x, p["post_attention_layernorm.weight"], eps)
    return x + mlp(h, p["mlp.gate_proj.weight"], p["mlp.up_proj.weight"], p["mlp.down_proj.weight"])


def cross_entropy(logits, targets, grad_acc_steps=1):
    """train.py:46-49: F.cross_entropy(logits.view(-1, V), targets.view(-1), 'mean') / grad_acc."""
    return F.cross_entropy(logits.reshape(-1, logits.shape[-1]).float(), targets.reshape(-1)) / grad_acc_steps


def llama_forward(input_ids, params, cfg, cos, sin, norm=rmsnorm_llama):
    """picotron/model.py:265-272 for a param dict in the reference's state_dict naming."""
    x = F.embedding(input_ids, params["embedding.weight"])
    for i in range(cfg["num_hidden_layers"]):
        lp = {k[len(f"decoder_layers.{i}."):]: v for k, v in params.items() if k.startswith(f"decoder_layers.{i}.")}
        x = decoder_layer(x, lp, cos, sin, cfg["num_attention_heads"], cfg["num_key_value_heads"],
                          cfg["rms_norm_eps"], norm)
    x = norm(x, params["final_norm.weight"], cfg["rms_norm_eps"])
    return linear(x, params["final_proj.weight"])


def init_params(cfg, seed=42, dtype=torch.float32):
    """Deterministic random weights with the reference's init distributions (model.py:110-120,
    173-182, 221-222; RMSNorm weights = 1; nn.Linear default for final_proj), single-rank order."""
    g = torch.Generator().manual_seed(seed)
    H, I, V = cfg["hidden_size"], cfg["intermediate_size"], cfg["vocab_size"]
    nh, nkv = cfg["num_attention_heads"], cfg["num_key_value_heads"]
    d = H // nh

    def u(o, i):
        b = math.sqrt(1.0 / i)
        return (torch.rand(o, i, generator=g) * 2 - 1) * b

    p = {"embedding.weight": torch.randn(V, H, generator=g)}
    for l in range(cfg["num_hidden_layers"]):
        pre = f"decoder_layers.{l}."
        p[pre + "input_layernorm.weight"] = torch.ones(H)
        p[pre + "post_attention_layernorm.weight"] = torch.ones(H)
        p[pre + "attention.q_proj.weight"] = u(nh * d, H)
        p[pre + "attention.k_proj.weight"] = u(nkv * d, H)
        p[pre + "attention.v_proj.weight"] = u(nkv * d, H)
        p[pre + "attention.out_proj.weight"] = u(H, H)
        p[pre + "mlp.up_proj.weight"] = u(I, H)
        p[pre + "mlp.gate_proj.weight"] = u(I, H)
        p[pre + "mlp.down_proj.weight"] = u(H, I)
    p["final_norm.weight"] = torch.ones(H)
    p["final_proj.weight"] = u(V, H)
    return {k: v.to(dtype) for k, v in p.items()}
