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
    projection output, with grouped-query heads indexed, not repeat_interleave'd (model.py:142-143);
  * load-balanced causal ring (zig-zag): the reference's schedule gives rank r r + 1 blocks
    (:30-45), so the last rank sets the pace with C blocks while rank 0 does 1.  Inside
    RingAttentionFunc / ring_attention_tokens the shards are re-laid (one batched p2p exchange,
    zigzag_exchange) so rank r holds global half-chunks r and 2C - 1 - r; then every step after the
    causal diagonal is exactly half a block on every rank -- (all my queries x the first half of
    the visiting keys) when they come from a lower rank, (my second-half queries x all the visiting
    keys) otherwise -- and the outputs / gradients are re-laid back.  The external contract (rank r
    holds tokens [r S, (r + 1) S), data.py:105-109, update_rope_for_context_parallel) is unchanged.
    PICOTRON_RING_ZIGZAG=0 runs the reference's schedule instead (A/B only);
  * the residual stream stays in the zig-zag layout across the whole decoder stack wherever the
    gradients are averaged over the cp group (enable_zigzag_residual, called by the data-parallel
    wrappers): every op outside attention is token-local, so the embedding's output is re-laid once
    on entry and the final norm's input once on exit (ZigzagRelayout, gradients the inverse way),
    and the decoder layers run on zig-zag shards with zig-zag RoPE tables -- two exchanges of
    [B, S, H] per forward instead of three (q, K|V, o) per layer (PICOTRON_ZIGZAG_RESIDUAL=0: the
    per-layer re-lay, A/B only);
  * with the zig-zag layout the K|V shards do not travel round a ring: MI355X's xGMI is a full mesh
    (7 point-to-point links per GPU), so each rank fetches every other rank's K|V straight from its
    owner in ONE batched p2p (C - 1 transfers on C - 1 distinct links at once, overlapped with the
    causal diagonal block), and in the backward sends each visiting shard's fp32 dK|dV partial
    straight back to its owner, which sums them -- one link-time of K|V per pass instead of C - 1
    sequential ring hops (PICOTRON_RING_MESH=0: the ring, A/B only).
"""
import math
import os

import torch
import torch.distributed as dist

from .. import kernels as K
from .. import process_group_manager as pgm
from ..switches import S as SW
from .cp_communications import ContextCommunicate, zigzag_exchange


def apply_context_parallel(model):
    """context_parallel.py:10-12: sets CONTEXT_PARALLEL (read by every attention call)."""
    os.environ["CONTEXT_PARALLEL"] = "1" if pgm.current().cp_world_size > 1 else "0"
    return model


def enable_zigzag_residual(model):
    """Keep the residual stream of `model` (a Llama or a pipeline stage) in the zig-zag layout
    across its decoder stack at cp > 1: the decoder layers run on zig-zag shards (with their
    positions' RoPE tables), the embedding module's output is re-laid into the layout and the final
    norm's input back out of it -- forward hooks, so any container (Llama.forward, either
    PipelineParallel) calls the modules unchanged and the logits stay the rank's contiguous tokens.
    Whether a batch uses the layout is decided per call from its local sequence length
    (zigzag_enabled), identically at the entry, in every layer and at the exit.

    The layout moves which tokens' weight-gradient contributions each cp rank holds (the sum over
    the cp group is unchanged), so it is enabled by the gradient averaging over cp_dp_group --
    DataParallelBucket / DataParallelNaive call this -- and not by apply_context_parallel: the
    reference's train.py wraps a data-parallel module only for dp > 1 (train.py:194-195), and at
    cp > 1 / dp = 1 each cp rank then steps on its own chunk's gradient, which the per-layer re-lay
    inside the ring reproduces exactly.  Returns True when enabled."""
    if pgm.current().cp_world_size == 1 or SW.zigzag_residual == 0 or getattr(model, "_pt_zigzag_residual", False):
        return getattr(model, "_pt_zigzag_residual", False)
    from ..model import DecoderLayer
    for name, mod in model.named_modules():
        leaf = name.rsplit(".", 1)[-1]
        if isinstance(mod, DecoderLayer):
            mod.cp_zigzag_residual = True   # its tables are built per local length (DecoderLayer._tables)
        elif leaf == "embedding" and not isinstance(mod, torch.nn.Identity):
            mod.register_forward_hook(_zz_entry_hook)
        elif leaf == "final_norm" and not isinstance(mod, torch.nn.Identity):
            mod.register_forward_pre_hook(_zz_exit_hook)
    model._pt_zigzag_residual = True
    return True


class ZigzagRelayout(torch.autograd.Function):
    """The residual stream between the reference's contiguous split and the zig-zag split, x
    [B, S, ...] (sequence on dim 1); the gradient goes the inverse way."""

    @staticmethod
    def forward(ctx, x, to_zigzag):
        ctx.to_zigzag = to_zigzag
        (y,) = zigzag_exchange([x], [1], to_zigzag)
        return y

    @staticmethod
    def backward(ctx, g):
        (dx,) = zigzag_exchange([g.contiguous()], [1], not ctx.to_zigzag)
        return dx, None


def _zz_entry_hook(module, inputs, output):
    if output.dim() == 3 and zigzag_enabled(output.shape[1], True):
        return ZigzagRelayout.apply(output, True)
    return output


def _zz_exit_hook(module, args):
    x = args[0]
    if x.dim() == 3 and zigzag_enabled(x.shape[1], True):
        return (ZigzagRelayout.apply(x, False),) + tuple(args[1:])
    return None


def zigzag_rope_tables(max_positions, head_dim, base, S=None):
    """The RoPE rows of this rank's zig-zag shard of local length S (default max_positions / C).

    The reference rotates rank c's contiguous chunk with rows [c P, c P + S) of get_cos_sin(max_positions),
    P = max_positions / C (update_rope_for_context_parallel's slice, of which Attention.forward uses
    the first S rows: model.py:134-135, context_parallel.py:189-195).  Zig-zag half-chunk c (S / 2
    tokens) is rank c // 2's half c % 2, so its rows are (c // 2) P + (c % 2) S / 2 + i; the shard
    holds half-chunks r and 2C - 1 - r.  With max_positions == C S that is just c S / 2 + i; for
    max_positions > C S the rows follow the reference's (non-contiguous) positions exactly."""
    from ..model import get_cos_sin
    m = pgm.current()
    C, r = m.cp_world_size, m.cp_rank
    P = max_positions // C
    S = P if S is None else S
    if S % 2 or S > P:
        raise ValueError(f"zigzag_rope_tables: local sequence {S} must be even and <= max_positions / cp = {P}")
    cos, sin = get_cos_sin(max_positions, head_dim=head_dim, base=base)
    h = S // 2
    idx = torch.cat([torch.arange(h) + (c // 2) * P + (c % 2) * h for c in (r, 2 * C - 1 - r)])
    return cos[idx], sin[idx]


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

    align = 128   # the kernels tile query / key blocks of 128 rows (a zig-zag half must be a multiple)

    @staticmethod
    def fwd(q, k, v, scale, causal, acc, lse):
        K.attn_fwd(q, k, v, scale, causal, out=acc, lse=lse, merge=True)

    @staticmethod
    def delta(do, o):
        return K.attn_delta(do, o)

    @staticmethod
    def bwd(do, q, k, v, o, lse, delta, scale, causal, dq, dk, dv):
        K.attn_bwd(do, q, k, v, o, lse, scale, causal, dq=dq, dk=dk, dv=dv, grad_f32=True, delta=delta)

    @staticmethod
    def bwd_dq(do, q, k, v, lse, delta, scale, causal, dq):
        K.attn_bwd_part(do, q, k, v, lse, delta, scale, causal, dq=dq)

    @staticmethod
    def bwd_dkdv(do, q, k, v, lse, delta, scale, causal, dk, dv):
        K.attn_bwd_part(do, q, k, v, lse, delta, scale, causal, dk=dk, dv=dv)


def _kv_views(kv, B, S, nkv, d):
    w = nkv * d
    return kv[:, :w].view(B, S, nkv, d), kv[:, w:].view(B, S, nkv, d)


def zigzag_enabled(S, is_causal, blocks=HipBlocks):
    """The load-balanced layout applies to a causal ring of C > 1 whose half shards tile."""
    C = pgm.current().cp_world_size
    return (is_causal and C > 1 and S % (2 * getattr(blocks, "align", 1)) == 0
            and SW.ring_zigzag != 0)


def _zz_kind(step, rank, world):
    """Zig-zag ring, step > 0: the visiting K|V shard is rank j = rank - step's (half-chunks j and
    2C - 1 - j).  j < rank: all my queries see its first half, none its second ('kv0');
    j > rank: only my second half (2C - 1 - rank) sees it, all of it ('q1')."""
    return "kv0" if (rank - step) % world < rank else "q1"


def ring_forward(q, kv, nkv, scale, is_causal, blocks=HipBlocks, comm=None, zigzag=False):
    """RingAttentionFunc.forward (context_parallel.py:19-51) on token-major shards.
    q [B, S, nh, d] (any strides, d contiguous); kv [B*S, 2*nkv*d] contiguous (this rank's K|V).
    zigzag: q / kv are in the zig-zag layout (zigzag_exchange) and the balanced schedule runs.
    Returns (out_f32 [B, S, nh, d], lse f32 [B, nh, S])."""
    if zigzag and comm is None and SW.ring_mesh != 0:
        return mesh_forward(q, kv, nkv, scale, blocks)
    comm = comm or ContextCommunicate("comm")
    B, S, nh, d = q.shape
    acc = torch.zeros(B, S, nh, d, dtype=torch.float32, device=q.device)
    lse = torch.full((B, nh, S), float("-inf"), dtype=torch.float32, device=q.device)
    cur = kv
    h = S // 2
    for step in range(comm.world_size):
        nxt = None
        if step + 1 != comm.world_size:
            nxt = comm.send_recv(cur)
            comm.commit()
        k, v = _kv_views(cur, B, S, nkv, d)
        if zigzag and step > 0:
            if _zz_kind(step, comm.rank, comm.world_size) == "kv0":
                blocks.fwd(q, k[:, :h], v[:, :h], scale, False, acc, lse)
            else:
                blocks.fwd(q[:, h:], k, v, scale, False, acc[:, h:], lse[:, :, h:])
        elif zigzag or not is_causal or step <= comm.rank:
            blocks.fwd(q, k, v, scale, is_causal and step == 0, acc, lse)
        if step + 1 != comm.world_size:
            comm.wait()
            cur = nxt
    return acc, lse


def ring_backward(do, q, kv, o, lse, nkv, scale, is_causal, blocks=HipBlocks, kv_comm=None, d_kv_comm=None,
                  zigzag=False):
    """RingAttentionFunc.backward (context_parallel.py:53-110).  Returns (dq f32 [B,S,nh,d],
    dkv f32 [B*S, 2*nkv*d]) for this rank's own shards (zigzag: all in the zig-zag layout)."""
    if zigzag and kv_comm is None and SW.ring_mesh != 0:
        return mesh_backward(do, q, kv, o, lse, nkv, scale, blocks)
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
        k, v = _kv_views(cur, B, S, nkv, d)
        dk, dv = _kv_views(dkv, B, S, nkv, d)
        h = S // 2
        if zigzag and step > 0:
            if _zz_kind(step, r, W) == "kv0":
                blocks.bwd(do, q, k[:, :h], v[:, :h], o, lse, delta, scale, False, dq, dk[:, :h], dv[:, :h])
            else:
                blocks.bwd(do[:, h:], q[:, h:], k, v, o[:, h:], lse[:, :, h:], delta[:, :, h:], scale, False,
                           dq[:, h:], dk, dv)
        elif zigzag or step <= r or not is_causal:
            blocks.bwd(do, q, k, v, o, lse, delta, scale, is_causal and step == 0, dq, dk, dv)
        if step + 1 != W:
            kv_comm.wait()
            cur = nxt
        next_dkv = d_kv_comm.send_recv(dkv)
        d_kv_comm.commit()
    d_kv_comm.wait()
    return dq, next_dkv


# ---- the full-mesh schedule (zig-zag layout) -------------------------------------------------
def _p2p(ops, group):
    """Post one batched isend/irecv (one RCCL group: the transfers to / from different peers run
    concurrently on their own xGMI links).  gloo (the one-GPU tests) is not stream-ordered: the
    host synchronises before the sends and after the receives, as ContextCommunicate does."""
    sync = dist.get_backend(group) != "nccl" and torch.cuda.is_available()
    if sync:
        torch.cuda.synchronize()
    return dist.batch_isend_irecv(ops), sync


def _p2p_wait(pending):
    reqs, sync = pending
    for req in reqs:
        req.wait()
    if sync:
        torch.cuda.synchronize()


def _mesh_ops(sends, recvs, group, ids):
    """P2P ops of one batch: sends = [(tensor, rank)], recvs = [(tensor, rank)]."""
    return ([dist.P2POp(dist.isend, t, ids[j], group=group) for t, j in sends]
            + [dist.P2POp(dist.irecv, t, ids[j], group=group) for t, j in recvs])


def _halves(kv, B, S):
    """kv [B*S, 2w] -> its first / second half-chunk token rows, each [B*h, 2w] contiguous."""
    h, w2 = S // 2, kv.shape[1]
    kv3 = kv.view(B, S, w2)
    return kv3[:, :h].contiguous().view(B * h, w2), kv3[:, h:].contiguous().view(B * h, w2)


def mesh_forward(q, kv, nkv, scale, blocks=HipBlocks):
    """The zig-zag causal forward on the mesh: the diagonal block (local causal mask over this
    rank's two half-chunks) runs while the visiting K|V arrive; then each visiting shard j is half a
    block -- j < r: all my queries x its first half ('kv0'), j > r: my second half x all of it
    ('q1') -- merged into the running (out, LSE) by the kernel epilogue.  The fetch is two batched
    p2ps, every peer's first half-chunk (all C - 1 links, half a shard each: hidden under the
    diagonal block), then the second halves of the peers j > r only (the 'q1' peers), which arrive
    while my second half x their first halves computes -- a 'q1' block runs as those two quarters."""
    m = pgm.current()
    C, r, ids, group = m.cp_world_size, m.cp_rank, m.cp_group_ids, m.cp_group
    B, S, nh, d = q.shape
    h = S // 2
    acc = torch.zeros(B, S, nh, d, dtype=torch.float32, device=q.device)
    lse = torch.full((B, nh, S), float("-inf"), dtype=torch.float32, device=q.device)
    first, second = _halves(kv, B, S)
    peers = [j for j in range(C) if j != r]
    f = {j: torch.empty_like(first) for j in peers}
    s = {j: torch.empty_like(second) for j in peers if j > r}
    pend_a = _p2p(_mesh_ops([(first, j) for j in peers], [(f[j], j) for j in peers], group, ids), group)
    ops_b = _mesh_ops([(second, j) for j in peers if j < r], [(s[j], j) for j in s], group, ids)
    pend_b = _p2p(ops_b, group) if ops_b else None
    k, v = _kv_views(kv, B, S, nkv, d)
    blocks.fwd(q, k, v, scale, True, acc, lse)
    _p2p_wait(pend_a)
    for j in peers:
        k, v = _kv_views(f[j], B, h, nkv, d)
        if j < r:
            blocks.fwd(q, k, v, scale, False, acc, lse)
        else:
            blocks.fwd(q[:, h:], k, v, scale, False, acc[:, h:], lse[:, :, h:])
    if pend_b is not None:
        _p2p_wait(pend_b)
    for j in s:
        k, v = _kv_views(s[j], B, h, nkv, d)
        blocks.fwd(q[:, h:], k, v, scale, False, acc[:, h:], lse[:, :, h:])
    return acc, lse


def mesh_backward(do, q, kv, o, lse, nkv, scale, blocks=HipBlocks):
    """The zig-zag causal backward on the mesh, with no gradient partial on the wire: every rank
    fetches, besides the visiting K|V shards (for its own queries' dQ), the visiting ranks' queries,
    dO, LSE and D = rowsum(dO * O) -- 64 MiB + 0.5 MiB per peer at Llama-2-7B CP8, half of an fp32
    dK|dV partial -- and computes its own keys' dK / dV against them (the FA2 split of the backward:
    dQ over the visiting keys, dK / dV over the visiting queries).  Two batched p2ps on all C - 1
    links: the K|V shards (under the diagonal block's backward), then Q|dO|LSE|D (under the dQ
    blocks).  Visiting block kinds as the forward's: for my queries, shard j < r is 'kv0' (all my
    queries x its first half), j > r 'q1' (my second half x all of it); for my keys, rank j > r sees
    them as 'kv0' (all its queries x my first half), j < r as 'q1' (its second-half queries x all my
    keys).  Returns (dq f32 [B,S,nh,d], dkv f32 [B*S, 2 w]) for this rank's shards."""
    m = pgm.current()
    C, r, ids, group = m.cp_world_size, m.cp_rank, m.cp_group_ids, m.cp_group
    B, S, nh, d = q.shape
    h = S // 2
    delta = blocks.delta(do, o)
    dq = torch.zeros(B, S, nh, d, dtype=torch.float32, device=q.device)
    dkv = torch.zeros(kv.shape, dtype=torch.float32, device=kv.device)
    # what the peers need from me: K|V (their dQ), my queries and dO (bf16) and LSE | D (f32) (their
    # dK/dV) -- all of them for a lower rank (it sees my keys as 'kv0': all my queries), only my
    # second half-chunk's for a higher one (it sees them as 'q1')
    qdo = torch.cat([q.reshape(B, S, nh * d), do.reshape(B, S, nh * d)], dim=2).contiguous()
    ld = torch.stack([lse, delta], dim=2).contiguous()            # [B, nh, 2, S]
    qdo_hi, ld_hi = qdo[:, h:].contiguous(), ld[..., h:].contiguous()
    peers = [j for j in range(C) if j != r]
    kvs = {j: torch.empty_like(kv) for j in peers}
    qdos = {j: torch.empty_like(qdo if j > r else qdo_hi) for j in peers}
    lds = {j: torch.empty_like(ld if j > r else ld_hi) for j in peers}
    pend_kv = _p2p(_mesh_ops([(kv, j) for j in peers], [(kvs[j], j) for j in peers], group, ids), group)
    pend_q = _p2p(_mesh_ops([(t, j) for j in peers for t in ((qdo, ld) if j < r else (qdo_hi, ld_hi))],
                            [(t[j], j) for j in peers for t in (qdos, lds)], group, ids), group)
    k, v = _kv_views(kv, B, S, nkv, d)
    dk, dv = _kv_views(dkv, B, S, nkv, d)
    blocks.bwd(do, q, k, v, o, lse, delta, scale, True, dq, dk, dv)
    _p2p_wait(pend_kv)
    for j in peers:
        kj, vj = _kv_views(kvs[j], B, S, nkv, d)
        if j < r:    # my queries x its first half
            blocks.bwd_dq(do, q, kj[:, :h], vj[:, :h], lse, delta, scale, False, dq)
        else:        # my second half x all of it
            blocks.bwd_dq(do[:, h:], q[:, h:], kj, vj, lse[:, :, h:], delta[:, :, h:], scale, False, dq[:, h:])
    kvs = kj = vj = None   # the visiting K|V shards are done with: release them before the dK|dV parts
    _p2p_wait(pend_q)
    for j in peers:
        n = qdos[j].shape[1]   # S (j > r: all its queries) or h (j < r: its second half only)
        qj = qdos[j][:, :, :nh * d].view(B, n, nh, d)
        doj = qdos[j][:, :, nh * d:].view(B, n, nh, d)
        lsej, dj = lds[j][:, :, 0], lds[j][:, :, 1]
        if j > r:    # all its queries x my first half
            blocks.bwd_dkdv(doj, qj, k[:, :h], v[:, :h], lsej, dj, scale, False, dk[:, :h], dv[:, :h])
        else:        # its second-half queries x all my keys
            blocks.bwd_dkdv(doj, qj, k, v, lsej, dj, scale, False, dk, dv)
    return dq, dkv


# ---- token-major entry points used by the fused decoder layer (functional.py) ----------------
def ring_attention_tokens(qkv, sh, scale, is_causal, resident=False):
    """q|k|v from the fused projection [T, q|k|v] -> (o bf16 [B,S,nh,d], lse f32 [B,nh,S]).
    resident: qkv is already in the zig-zag layout (the decoder stack's residual stream is, see
    apply_context_parallel) and so is o; otherwise, with the zig-zag schedule, q and K|V are re-laid
    here and o re-laid back (the LSE stays in the zig-zag layout: only the ring backward reads it)."""
    B, S, T = sh.B, sh.S, sh.T
    if resident:
        acc, lse = ring_forward(sh.q(qkv), qkv[:, sh.wq:].contiguous(), sh.nkv, scale, is_causal, zigzag=True)
        return acc.to(torch.bfloat16), lse
    if zigzag_enabled(S, is_causal):
        qz, kvz = zigzag_exchange([sh.q(qkv), qkv[:, sh.wq:].view(B, S, 2 * sh.wkv)], [1, 1], True)
        acc, lse = ring_forward(qz, kvz.view(T, 2 * sh.wkv), sh.nkv, scale, is_causal, zigzag=True)
        (o,) = zigzag_exchange([acc.to(torch.bfloat16)], [1], False)
        return o, lse
    kv = qkv[:, sh.wq:].contiguous()
    acc, lse = ring_forward(sh.q(qkv), kv, sh.nkv, scale, is_causal)
    return acc.to(torch.bfloat16), lse


def ring_attention_tokens_bwd(do, qkv, o, lse, sh, scale, is_causal, dqkv, resident=False):
    B, S, T = sh.B, sh.S, sh.T
    if resident:
        dq, dkv = ring_backward(do, sh.q(qkv), qkv[:, sh.wq:].contiguous(), o, lse, sh.nkv, scale, is_causal,
                                zigzag=True)
    elif zigzag_enabled(S, is_causal):
        # the standalone layer (contiguous residual): q / K|V / o / dO re-laid in one exchange
        qz, kvz, oz, doz = zigzag_exchange([sh.q(qkv), qkv[:, sh.wq:].view(B, S, 2 * sh.wkv), o, do],
                                           [1, 1, 1, 1], True)
        dq, dkv = ring_backward(doz, qz, kvz.view(T, 2 * sh.wkv), oz, lse, sh.nkv, scale, is_causal, zigzag=True)
        # rounded to bf16 before the way back (the same single rounding as the copy below)
        dq, dkv = zigzag_exchange([dq.to(torch.bfloat16), dkv.to(torch.bfloat16).view(B, S, 2 * sh.wkv)], [1, 1],
                                  False)
    else:
        kv = qkv[:, sh.wq:].contiguous()
        dq, dkv = ring_backward(do, sh.q(qkv), kv, o, lse, sh.nkv, scale, is_causal)
    dqkv[:, :sh.wq].copy_(dq.view(T, sh.wq))
    dqkv[:, sh.wq:].copy_(dkv.view(T, 2 * sh.wkv))


# ---- the reference's [B, H, S, D] API -------------------------------------------------------
class RingAttentionFunc(torch.autograd.Function):
    """context_parallel.py:17-110 on [B, H, S, D] q/k/v (k/v already head-expanded by the caller,
    as model.py:142-143 does).  Saves q, k, v, out, lse as the reference does (:48)."""

    @staticmethod
    def forward(ctx, q, k, v, sm_scale, is_causal):
        B, H, S, D = q.shape
        Hk = k.shape[1]
        qt = q.transpose(1, 2)
        kv = torch.cat([k.transpose(1, 2).reshape(B * S, -1), v.transpose(1, 2).reshape(B * S, -1)], dim=1)
        zz = zigzag_enabled(S, is_causal)
        if zz:   # the balanced schedule on re-laid shards; q / K|V / out / LSE kept in that layout
            qt, kv = zigzag_exchange([qt, kv.view(B, S, 2 * Hk * D)], [1, 1], True)
            kv = kv.view(B * S, 2 * Hk * D)
        acc, lse = ring_forward(qt, kv.contiguous(), Hk, sm_scale, is_causal, zigzag=zz)
        out = acc.to(q.dtype)                         # [B, S, H, D]
        ctx.save_for_backward(qt if zz else q, kv if zz else k, v, out, lse)
        ctx.sm_scale, ctx.is_causal, ctx.zz, ctx.shape = sm_scale, is_causal, zz, (B, H, S, D, Hk)
        if zz:
            (out,) = zigzag_exchange([out], [1], False)
        return out.transpose(1, 2)

    @staticmethod
    def backward(ctx, dout, *args):
        a, b_, v, out, lse = ctx.saved_tensors
        B, H, S, D, Hk = ctx.shape
        do = dout.transpose(1, 2)
        if do.stride(-1) != 1:
            do = do.contiguous()
        if ctx.zz:
            qt, kv = a, b_
            (do,) = zigzag_exchange([do], [1], True)
        else:
            qt = a.transpose(1, 2)
            kv = torch.cat([b_.transpose(1, 2).reshape(B * S, -1), v.transpose(1, 2).reshape(B * S, -1)], dim=1)
        dq, dkv = ring_backward(do, qt, kv.contiguous(), out, lse, Hk, ctx.sm_scale, ctx.is_causal, zigzag=ctx.zz)
        dtype = v.dtype
        dq, dkv = dq.to(dtype), dkv.to(dtype).view(B, S, 2 * Hk * D)
        if ctx.zz:
            dq, dkv = zigzag_exchange([dq, dkv], [1, 1], False)
        w = Hk * D
        dk = dkv[:, :, :w].reshape(B, S, Hk, D).transpose(1, 2)
        dv = dkv[:, :, w:].reshape(B, S, Hk, D).transpose(1, 2)
        return dq.transpose(1, 2), dk, dv, None, None


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
