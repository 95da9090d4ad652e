"""Context parallelism = ring attention over the cp group, on the gfx950 flash-attention kernels.

Mirrors picotron/context_parallel/context_parallel.py (okoge-kaz/picotron @ 2025-03-02):
  apply_context_parallel (:10-12), ring_attention (:14-15), RingAttentionFunc (:17-110),
  ring_attention_forward / ring_attention_backward (:112-155), update_rope_for_context_parallel
  (:189-195).  The schedule is the reference's: at step s rank r holds the K/V shard of rank r-s;
  causal blocks with s > r are skipped and only s = 0 is causally masked; the backward recomputes
  each block from the global out/LSE and passes dK/dV (fp32) around the ring with one extra hop.

What differs (MI355X-first):
  * every block is the flash kernel -- no [S/cp, S/cp] score matrix is materialised;
  * update_out_and_lse (:157-187) is fused into the forward kernel's epilogue (merge mode): the
    running output stays fp32 and the running LSE is fp32 (the reference keeps it in the input
    dtype, SURVEY.md §8c caveat 1);
  * the K|V shard travels as ONE contiguous [T, 2*kv*d] buffer per step (the reference sends k and
    v separately), and the host never synchronises the device between steps;
  * the token-major entry points (ring_attention_tokens*) read q/k/v straight out of the fused
    projection output, with grouped-query heads indexed, not repeat_interleave'd (model.py:142-143).
"""
import math
import os

import torch

from .. import kernels as K
from .. import process_group_manager as pgm
from .cp_communications import ContextCommunicate


def apply_context_parallel(model):
    os.environ["CONTEXT_PARALLEL"] = "1" if pgm.current().cp_world_size > 1 else "0"
    return model


def update_rope_for_context_parallel(cos, sin):
    seq_len, _ = cos.size()
    m = pgm.current()
    cp_rank, cp_world_size = m.cp_rank, m.cp_world_size
    assert seq_len % cp_world_size == 0, (
        f"Input sequence length ({seq_len}) must be divisible by cp_world_size ({cp_world_size})")
    size_per_partition = seq_len // cp_world_size
    start_idx, end_idx = cp_rank * size_per_partition, (cp_rank + 1) * size_per_partition
    return cos[start_idx:end_idx], sin[start_idx:end_idx]


class HipBlocks:
    """Per-block attention on the HIP kernels (the only implementation the package ships)."""

    @staticmethod
    def fwd(q, k, v, scale, causal, acc, lse):
        K.attn_fwd(q, k, v, scale, causal, out=acc, lse=lse, merge=True)

    @staticmethod
    def delta(do, o):
        return K.attn_delta(do, o)

    @staticmethod
    def bwd(do, q, k, v, o, lse, delta, scale, causal, dq, dk, dv):
        K.attn_bwd(do, q, k, v, o, lse, scale, causal, dq=dq, dk=dk, dv=dv, grad_f32=True, delta=delta)


def _kv_views(kv, B, S, nkv, d):
    w = nkv * d
    return kv[:, :w].view(B, S, nkv, d), kv[:, w:].view(B, S, nkv, d)


def ring_forward(q, kv, nkv, scale, is_causal, blocks=HipBlocks, comm=None):
    """RingAttentionFunc.forward (context_parallel.py:19-51) on token-major shards.
    q [B, S, nh, d] (any strides, d contiguous); kv [B*S, 2*nkv*d] contiguous (this rank's K|V).
    Returns (out_f32 [B, S, nh, d], lse f32 [B, nh, S])."""
    comm = comm or ContextCommunicate("comm")
    B, S, nh, d = q.shape
    acc = torch.zeros(B, S, nh, d, dtype=torch.float32, device=q.device)
    lse = torch.full((B, nh, S), float("-inf"), dtype=torch.float32, device=q.device)
    cur = kv
    for step in range(comm.world_size):
        nxt = None
        if step + 1 != comm.world_size:
            nxt = comm.send_recv(cur)
            comm.commit()
        if not is_causal or step <= comm.rank:
            k, v = _kv_views(cur, B, S, nkv, d)
            blocks.fwd(q, k, v, scale, is_causal and step == 0, acc, lse)
        if step + 1 != comm.world_size:
            comm.wait()
            cur = nxt
    return acc, lse


def ring_backward(do, q, kv, o, lse, nkv, scale, is_causal, blocks=HipBlocks, kv_comm=None, d_kv_comm=None):
    """RingAttentionFunc.backward (context_parallel.py:53-110).  Returns (dq f32 [B,S,nh,d],
    dkv f32 [B*S, 2*nkv*d]) for this rank's own shards."""
    kv_comm = kv_comm or ContextCommunicate("kv_comm")
    d_kv_comm = d_kv_comm or ContextCommunicate("d_kv_comm")
    B, S, nh, d = q.shape
    delta = blocks.delta(do, o)
    dq = torch.zeros(B, S, nh, d, dtype=torch.float32, device=q.device)
    cur = kv
    dkv = next_dkv = None
    W, r = kv_comm.world_size, kv_comm.rank
    for step in range(W):
        nxt = None
        if step + 1 != W:
            nxt = kv_comm.send_recv(cur)
            kv_comm.commit()
        if step == 0:
            dkv = torch.zeros(kv.shape, dtype=torch.float32, device=kv.device)
        else:  # the partial dK|dV of shard r-step, accumulated by the ranks before us
            d_kv_comm.wait()
            dkv = next_dkv
        if step <= r or not is_causal:
            k, v = _kv_views(cur, B, S, nkv, d)
            dk, dv = _kv_views(dkv, B, S, nkv, d)
            blocks.bwd(do, q, k, v, o, lse, delta, scale, is_causal and step == 0, dq, dk, dv)
        if step + 1 != W:
            kv_comm.wait()
            cur = nxt
        next_dkv = d_kv_comm.send_recv(dkv)
        d_kv_comm.commit()
    d_kv_comm.wait()
    return dq, next_dkv


# ---- token-major entry points used by the fused decoder layer (functional.py) ----------------
def ring_attention_tokens(qkv, sh, scale, is_causal):
    """q|k|v from the fused projection [T, q|k|v] -> (o bf16 [B,S,nh,d], lse f32)."""
    kv = qkv[:, sh.wq:].contiguous()
    acc, lse = ring_forward(sh.q(qkv), kv, sh.nkv, scale, is_causal)
    return acc.to(torch.bfloat16), lse


def ring_attention_tokens_bwd(do, qkv, o, lse, sh, scale, is_causal, dqkv):
    kv = qkv[:, sh.wq:].contiguous()
    dq, dkv = ring_backward(do, sh.q(qkv), kv, o, lse, sh.nkv, scale, is_causal)
    dqkv[:, :sh.wq].copy_(dq.view(sh.T, sh.wq))
    dqkv[:, sh.wq:].copy_(dkv)


# ---- the reference's [B, H, S, D] API -------------------------------------------------------
class RingAttentionFunc(torch.autograd.Function):
    """context_parallel.py:17-110 on [B, H, S, D] q/k/v (k/v already head-expanded by the caller,
    as model.py:142-143 does).  Saves q, k, v, out, lse as the reference does (:48)."""

    @staticmethod
    def forward(ctx, q, k, v, sm_scale, is_causal):
        B, H, S, D = q.shape
        qt = q.transpose(1, 2)
        kv = torch.cat([k.transpose(1, 2).reshape(B * S, -1), v.transpose(1, 2).reshape(B * S, -1)], dim=1)
        acc, lse = ring_forward(qt, kv.contiguous(), k.shape[1], sm_scale, is_causal)
        out = acc.to(q.dtype)                         # [B, S, H, D]
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.sm_scale, ctx.is_causal = sm_scale, is_causal
        return out.transpose(1, 2)

    @staticmethod
    def backward(ctx, dout, *args):
        q, k, v, out, lse = ctx.saved_tensors
        B, H, S, D = q.shape
        Hk = k.shape[1]
        kv = torch.cat([k.transpose(1, 2).reshape(B * S, -1), v.transpose(1, 2).reshape(B * S, -1)], dim=1)
        do = dout.transpose(1, 2)
        if do.stride(-1) != 1:
            do = do.contiguous()
        dq, dkv = ring_backward(do, q.transpose(1, 2), kv.contiguous(), out, lse, Hk, ctx.sm_scale, ctx.is_causal)
        w = Hk * D
        dk = dkv[:, :w].view(B, S, Hk, D).transpose(1, 2).to(k.dtype)
        dv = dkv[:, w:].view(B, S, Hk, D).transpose(1, 2).to(v.dtype)
        return dq.transpose(1, 2).to(q.dtype), dk, dv, None, None


def ring_attention(q, k, v, sm_scale, is_causal):
    return RingAttentionFunc.apply(q, k, v, sm_scale, is_causal)


def ring_attention_forward(q, k, v, sm_scale, is_causal):
    """context_parallel.py:112-128: one block, [B, H, S, D] -> (O in q's dtype, LSE f32 [B, H, S])."""
    o, lse = K.attn_fwd(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), sm_scale, is_causal)
    return o.transpose(1, 2), lse


def update_out_and_lse(out, lse, block_out, block_lse, slice_=None):
    """context_parallel.py:157-187, same signature and contract: block_out -> fp32, block_lse
    unsqueezed to [..., 1]; the first call (out None) returns them; later calls merge
        out <- out - sigmoid(block_lse - lse) * (out - block_out)
        lse <- lse - logsigmoid(lse - block_lse)
    on the HIP merge kernel (pt_lse_merge), with lse kept in the block LSE's dtype (bf16 in a bf16
    ring, rounded op by op as torch does).  Returns new tensors; with slice_ the merge writes
    out[slice_] / lse[slice_] in place, as the reference does."""
    block_out = block_out.to(torch.float32)
    block_lse = block_lse.unsqueeze(dim=-1)
    if out is None:
        if slice_ is not None:
            raise RuntimeError("first update_out_and_lse should not pass slice_ args")
        return block_out, block_lse
    if slice_ is not None:
        o_new, l_new = K.lse_merge(out[slice_], block_out, lse[slice_], block_lse)   # the block is the slice's
        out[slice_], lse[slice_] = o_new, l_new
        return out, lse
    return K.lse_merge(out, block_out, lse, block_lse)


def ring_attention_backward(dO, Q, K_, V, O, softmax_lse, sm_scale, is_causal):
    """context_parallel.py:130-155: one block's (dQ, dK, dV) from the global O / LSE, [B, H, S, D]."""
    do = dO.transpose(1, 2)
    if do.stride(-1) != 1:
        do = do.contiguous()
    o = O.transpose(1, 2)
    if o.stride(-1) != 1:
        o = o.contiguous()
    dq, dk, dv, _ = K.attn_bwd(do, Q.transpose(1, 2), K_.transpose(1, 2), V.transpose(1, 2), o,
                               softmax_lse.float().contiguous(), sm_scale, is_causal)
    return dq.transpose(1, 2), dk.transpose(1, 2), dv.transpose(1, 2)
