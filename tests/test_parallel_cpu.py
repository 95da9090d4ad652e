"""CPU (gloo, world_size 2-4) tests of the parallel host logic: the process grid, the TP f/g
collectives, the DP gradient buckets (both the autograd-hook path and the fused-kernel sink path)
and the ring-attention schedule (forward merge, backward dK/dV ring).

The ring schedule runs with an oracle-backed block implementation injected by the test (the
package's only implementation is the HIP kernel): the schedule, the p2p pattern and the merge
algebra are what is under test, against full causal attention over the concatenated sequence."""
import math

import pytest
import torch
import torch.distributed as dist

from tests import _dist


# ----------------------------------------------------------------------------- process grid
def _grid(rank, world):
    from picotron_amd import process_group_manager as pgm
    m = pgm.setup_process_group_manager(tp_size=2, cp_size=1, pp_size=1, dp_size=2)
    # grid = arange(4).view(dp=2, pp=1, cp=1, tp=2): TP innermost (process_group_manager.py:13)
    assert (m.dp_rank, m.tp_rank) == (rank // 2, rank % 2)
    assert m.tp_group_ids == [rank - rank % 2, rank - rank % 2 + 1]
    assert m.dp_group_ids == [rank % 2, rank % 2 + 2]
    assert m.cp_dp_world_size == 2 and m.tp_world_size == 2
    t = torch.tensor([float(rank)])
    dist.all_reduce(t, group=m.tp_group)
    assert t.item() == sum(m.tp_group_ids)
    t = torch.tensor([float(rank)])
    dist.all_reduce(t, group=m.cp_dp_group)
    assert t.item() == sum(m.dp_group_ids)


def test_process_grid_dp2_tp2():
    _dist.run(_grid, 4)


# ----------------------------------------------------------------------------- TP f / g
def _tp_comms(rank, world):
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.tensor_parallel.tp_communications import (CopyToModelParallelRegion,
                                                                GatherFromModelParallelRegion,
                                                                ReduceFromModelParallelRegion)
    pgm.setup_process_group_manager(tp_size=world, cp_size=1, pp_size=1, dp_size=1)
    x = torch.full((2, 3), float(rank + 1), requires_grad=True)
    y = CopyToModelParallelRegion.apply(x)            # identity fwd, all-reduce bwd
    assert torch.equal(y, x)
    y.backward(torch.ones(2, 3))
    assert torch.equal(x.grad, torch.full((2, 3), float(world)))
    x2 = torch.full((2, 3), float(rank + 1), requires_grad=True)
    z = ReduceFromModelParallelRegion.apply(x2 * 1)   # all-reduce fwd, identity bwd
    assert torch.equal(z, torch.full((2, 3), float(sum(range(1, world + 1)))))
    z.backward(torch.ones(2, 3))
    assert torch.equal(x2.grad, torch.ones(2, 3))
    x3 = torch.full((2, 2), float(rank), requires_grad=True)
    g = GatherFromModelParallelRegion.apply(x3 * 1)   # all-gather along the last dim, split bwd
    assert g.shape == (2, 2 * world) and torch.equal(g[:, 2 * rank:2 * rank + 2], x3.detach())
    g.backward(torch.arange(2 * 2 * world, dtype=torch.float32).view(2, 2 * world))
    assert torch.equal(x3.grad, torch.arange(2 * 2 * world, dtype=torch.float32).view(2, 2 * world)[:, 2 * rank:2 * rank + 2])


def test_tp_collectives_world2():
    _dist.run(_tp_comms, 2)


# ----------------------------------------------------------------------------- DP buckets
class _FusedSinkLinear(torch.autograd.Function):
    """A stand-in for the fused kernels' gradient path: writes dW straight into the parameter's
    sink (main_grad when DataParallelBucket owns it) and returns None, like functional.wgrad."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return x @ w.t()

    @staticmethod
    def backward(ctx, dy):
        from picotron_amd import functional as FN
        x, w = ctx.saved_tensors
        g = dy.t() @ x
        if getattr(w, "main_grad", None) is not None:
            w.main_grad.add_(g)
        elif w.grad is None:
            w.grad = g
        else:
            w.grad.add_(g)
        FN._grad_ready(w)
        return dy @ w, None


class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        g = torch.Generator().manual_seed(0)
        self.emb = torch.nn.Parameter(torch.randn(16, 8, generator=g))       # autograd-hook path
        self.w1 = torch.nn.Parameter(torch.randn(8, 8, generator=g) / 3)     # fused-sink path
        self.w2 = torch.nn.Parameter(torch.randn(4, 8, generator=g) / 3)

    def forward(self, ids):
        h = torch.nn.functional.embedding(ids, self.emb)
        return _FusedSinkLinear.apply(torch.tanh(_FusedSinkLinear.apply(h, self.w1)), self.w2)


def _dp_bucket(rank, world, bucket_mb):
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.data_parallel.data_parallel import DataParallelBucket
    pgm.setup_process_group_manager(tp_size=1, cp_size=1, pp_size=1, dp_size=world)
    model = DataParallelBucket(_Net(), bucket_cap_mb=bucket_mb)
    ref = _Net()
    ga = 3
    grads = {n: torch.zeros_like(p) for n, p in ref.named_parameters()}
    for i in range(ga):
        g = torch.Generator().manual_seed(100 * i + rank)
        ids = torch.randint(0, 16, (5,), generator=g)
        model.require_backward_grad_sync = (i == ga - 1)
        (model(ids).square().mean() / ga).backward()
        ref.zero_grad()
        (ref(ids).square().mean() / ga).backward()
        for n, p in ref.named_parameters():
            grads[n] += p.grad
    for n, p in model.module.named_parameters():
        want = grads[n].clone()
        dist.all_reduce(want)
        want /= world
        torch.testing.assert_close(p.grad, want, rtol=1e-5, atol=1e-6)
    model.reset()
    for p in model.module.parameters():
        assert p.main_grad.abs().sum().item() == 0.0


@pytest.mark.parametrize("bucket_mb", [25, 0.0002])   # one bucket / one bucket per parameter
def test_dp_bucket_grad_average(bucket_mb):
    _dist.run(_dp_bucket, 2, bucket_mb)


def test_bucket_assignment_matches_reference_rule():
    """bucket.py:84-129: greedy in parameters() order; a parameter that does not fit opens a new
    bucket; an oversized parameter gets a bucket of its own."""
    import os
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    from picotron_amd.data_parallel import bucket as B

    class PG:  # world-size-1 stand-in: only dist.get_world_size(group) is consulted
        pass
    orig = dist.get_world_size
    dist.get_world_size = lambda group=None: 1
    try:
        ps = [torch.nn.Parameter(torch.zeros(n)) for n in (3, 4, 10, 2, 2, 1)]
        bm = B.BucketManager(ps, PG(), bucket_size=8)
        locs = [bm.params_to_bucket_location[p] for p in ps]
        assert locs == [(0, 3, 0), (3, 7, 0), (0, 10, 1), (0, 2, 2), (2, 4, 2), (4, 5, 2)]
        assert bm.bucket_sizes == [7, 10, 5]
        assert ps[1].main_grad.data_ptr() == bm.grad_data_list[0][3:].data_ptr()
    finally:
        dist.get_world_size = orig


# ----------------------------------------------------------------------------- ring attention
class OracleBlocks:
    """Per-block attention restated from the oracle (fp32), with the same accumulation contract as
    the HIP kernels: fwd merges into (acc f32 [B,S,nh,d], lse f32 [B,nh,S]); bwd accumulates."""

    @staticmethod
    def _expand(t, nh):
        tt = t.float().transpose(1, 2)
        return tt.repeat_interleave(nh // tt.shape[1], dim=1)

    @staticmethod
    def fwd(q, k, v, scale, causal, acc, lse):
        from oracle import picotron_oracle as O
        nh = q.shape[2]
        o, l = O.attention_lse(q.float().transpose(1, 2), OracleBlocks._expand(k, nh), OracleBlocks._expand(v, nh),
                               scale, causal)
        new = torch.logaddexp(lse, l)
        w_old = torch.exp(lse - new).nan_to_num(0.0)
        w_blk = torch.exp(l - new)
        acc.mul_(w_old.transpose(1, 2).unsqueeze(-1)).add_(o.transpose(1, 2) * w_blk.transpose(1, 2).unsqueeze(-1))
        lse.copy_(new)

    @staticmethod
    def delta(do, o):
        return (do.float() * o.float()).sum(-1).transpose(1, 2).contiguous()

    @staticmethod
    def bwd(do, q, k, v, o, lse, delta, scale, causal, dq, dk, dv):
        from oracle import picotron_oracle as O
        nh, nkv = q.shape[2], k.shape[2]
        dq_, dk_, dv_ = O.ring_attention_backward(do.float().transpose(1, 2), q.float().transpose(1, 2),
                                                  OracleBlocks._expand(k, nh), OracleBlocks._expand(v, nh),
                                                  o.float().transpose(1, 2), lse, scale, causal)
        B, Sk, _, d = k.shape
        dq += dq_.transpose(1, 2)
        dk += dk_.view(B, nkv, nh // nkv, Sk, d).sum(2).transpose(1, 2)
        dv += dv_.view(B, nkv, nh // nkv, Sk, d).sum(2).transpose(1, 2)


def _oracle_bwd_dq(do, q, k, v, lse, delta, scale, causal, dq):
    """dQ only: the oracle block backward with the given LSE (delta is implied by the oracle)."""
    _oracle_part(do, q, k, v, lse, delta, scale, causal, dq, None, None)


def _oracle_bwd_dkdv(do, q, k, v, lse, delta, scale, causal, dk, dv):
    _oracle_part(do, q, k, v, lse, delta, scale, causal, None, dk, dv)


def _oracle_part(do, q, k, v, lse, delta, scale, causal, dq, dk, dv):
    """One block's gradients from the rows' LSE and D = rowsum(dO * O) (FA2: dS = P (dP - D)), the
    contract of pt_attn_bwd_part: no O needed."""
    nh, nkv = q.shape[2], k.shape[2]
    qq = q.float().transpose(1, 2)
    kk, vv = OracleBlocks._expand(k, nh), OracleBlocks._expand(v, nh)
    dd = do.float().transpose(1, 2)
    s_ = qq @ kk.transpose(-1, -2) * scale
    if causal:
        Sq, Sk = s_.shape[-2], s_.shape[-1]
        s_ = s_.masked_fill(torch.ones(Sq, Sk, dtype=torch.bool).triu(1), float("-inf"))
    p_ = torch.exp(s_ - lse.unsqueeze(-1))
    dp = dd @ vv.transpose(-1, -2)
    ds = p_ * (dp - delta.unsqueeze(-1))
    B, Sk, _, d = k.shape
    if dq is not None:
        dq += (ds @ kk * scale).transpose(1, 2)
    if dk is not None:
        dk += (ds.transpose(-1, -2) @ qq * scale).view(B, nkv, nh // nkv, Sk, d).sum(2).transpose(1, 2)
        dv += (p_.transpose(-1, -2) @ dd).view(B, nkv, nh // nkv, Sk, d).sum(2).transpose(1, 2)


OracleBlocks.bwd_dq = staticmethod(_oracle_bwd_dq)
OracleBlocks.bwd_dkdv = staticmethod(_oracle_bwd_dkdv)


def _ring(rank, world, nh, nkv):
    from oracle import picotron_oracle as O
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.context_parallel import context_parallel as CP
    pgm.setup_process_group_manager(tp_size=1, cp_size=world, pp_size=1, dp_size=1)
    B, S, d = 2, 8, 16
    g = torch.Generator().manual_seed(7)
    q = torch.randn(B, world * S, nh, d, generator=g)
    k = torch.randn(B, world * S, nkv, d, generator=g)
    v = torch.randn(B, world * S, nkv, d, generator=g)
    do = torch.randn(B, world * S, nh, d, generator=g)
    sl = slice(rank * S, (rank + 1) * S)
    scale = 1 / math.sqrt(d)
    kv = torch.cat([k[:, sl].reshape(B * S, -1), v[:, sl].reshape(B * S, -1)], dim=1).contiguous()
    acc, lse = CP.ring_forward(q[:, sl], kv, nkv, scale, True, blocks=OracleBlocks)
    # reference: full causal attention over the whole sequence
    qr = q.transpose(1, 2).requires_grad_(True)
    kr = k.transpose(1, 2).repeat_interleave(nh // nkv, 1).detach().requires_grad_(True)
    vr = v.transpose(1, 2).repeat_interleave(nh // nkv, 1).detach().requires_grad_(True)
    o_ref, lse_ref = O.attention_lse(qr, kr, vr, scale, True)
    torch.testing.assert_close(acc, o_ref.transpose(1, 2)[:, sl].detach(), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(lse, lse_ref[:, :, sl].detach(), rtol=1e-5, atol=1e-5)
    (o_ref * do.transpose(1, 2)).sum().backward()
    dq, dkv = CP.ring_backward(do[:, sl], q[:, sl], kv, acc, lse, nkv, scale, True, blocks=OracleBlocks)
    torch.testing.assert_close(dq, qr.grad.transpose(1, 2)[:, sl], rtol=1e-4, atol=1e-5)
    dk_ref = kr.grad.view(B, nkv, nh // nkv, world * S, d).sum(2).transpose(1, 2)[:, sl]
    dv_ref = vr.grad.view(B, nkv, nh // nkv, world * S, d).sum(2).transpose(1, 2)[:, sl]
    w = nkv * d
    torch.testing.assert_close(dkv[:, :w].view(B, S, nkv, d), dk_ref, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(dkv[:, w:].view(B, S, nkv, d), dv_ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("world,nh,nkv", [(2, 2, 2), (4, 4, 2)])
def test_ring_attention_schedule_matches_full_attention(world, nh, nkv):
    _dist.run(_ring, world, nh, nkv)


class CountingBlocks(OracleBlocks):
    """OracleBlocks that also record the causal work (visible query-key pairs) of every call."""
    work = []

    @staticmethod
    def fwd(q, k, v, scale, causal, acc, lse):
        Sq, Sk = q.shape[1], k.shape[1]
        CountingBlocks.work.append(Sq * (Sq + 1) // 2 if causal else Sq * Sk)
        OracleBlocks.fwd(q, k, v, scale, causal, acc, lse)


def _ring_zigzag(rank, world, nh, nkv, mesh):
    """The load-balanced (zig-zag) schedule: shards re-laid by zigzag_exchange, the balanced
    schedule -- over the full mesh (mesh=1: K|V half-chunks and, in the backward, the peers'
    Q|dO|LSE|D fetched from their owners; no gradient travels) or round the ring (mesh=0) --
    outputs / gradients re-laid back: equal to full
    causal attention over the whole sequence on the reference's contiguous chunks, and every rank
    does the same causal work (the reference's schedule: rank r does r + 1 blocks)."""
    from picotron_amd import switches
    with switches.override(ring_mesh=mesh):
        _ring_zigzag_body(rank, world, nh, nkv)


def _ring_zigzag_body(rank, world, nh, nkv):
    from oracle import picotron_oracle as O
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.context_parallel import context_parallel as CP
    from picotron_amd.context_parallel.cp_communications import zigzag_exchange
    pgm.setup_process_group_manager(tp_size=1, cp_size=world, pp_size=1, dp_size=1)
    B, S, d = 2, 8, 16
    g = torch.Generator().manual_seed(7)
    q = torch.randn(B, world * S, nh, d, generator=g)
    k = torch.randn(B, world * S, nkv, d, generator=g)
    v = torch.randn(B, world * S, nkv, d, generator=g)
    do = torch.randn(B, world * S, nh, d, generator=g)
    sl = slice(rank * S, (rank + 1) * S)
    scale = 1 / math.sqrt(d)
    kv = torch.cat([k[:, sl].reshape(B, S, -1), v[:, sl].reshape(B, S, -1)], dim=2)
    # the exchange is a permutation: there and back is the identity
    back = zigzag_exchange(zigzag_exchange([q[:, sl], kv], [1, 1], True), [1, 1], False)
    assert torch.equal(back[0], q[:, sl]) and torch.equal(back[1], kv)
    qz, kvz = zigzag_exchange([q[:, sl], kv], [1, 1], True)
    # rank r holds global half-chunks r and 2 world - 1 - r
    h = S // 2
    assert torch.equal(qz[:, :h], q[:, rank * h:(rank + 1) * h])
    assert torch.equal(qz[:, h:], q[:, (2 * world - 1 - rank) * h:(2 * world - rank) * h])
    kvz = kvz.reshape(B * S, -1)
    CountingBlocks.work = []
    acc, lse = CP.ring_forward(qz, kvz, nkv, scale, True, blocks=CountingBlocks, zigzag=True)
    work = torch.tensor([float(sum(CountingBlocks.work))])
    allw = [torch.zeros(1) for _ in range(world)]
    dist.all_gather(allw, work)
    assert len({w.item() for w in allw}) == 1, allw         # balanced
    assert work.item() == S * (S + 1) // 2 + (world - 1) * S * S // 2
    (o,) = zigzag_exchange([acc], [1], False)
    (lse_c,) = zigzag_exchange([lse], [2], False)
    qr = q.transpose(1, 2).requires_grad_(True)
    kr = k.transpose(1, 2).repeat_interleave(nh // nkv, 1).detach().requires_grad_(True)
    vr = v.transpose(1, 2).repeat_interleave(nh // nkv, 1).detach().requires_grad_(True)
    o_ref, lse_ref = O.attention_lse(qr, kr, vr, scale, True)
    torch.testing.assert_close(o, o_ref.transpose(1, 2)[:, sl].detach(), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(lse_c, lse_ref[:, :, sl].detach(), rtol=1e-5, atol=1e-5)
    (o_ref * do.transpose(1, 2)).sum().backward()
    (doz,) = zigzag_exchange([do[:, sl]], [1], True)
    dq, dkv = CP.ring_backward(doz, qz, kvz, acc, lse, nkv, scale, True, blocks=OracleBlocks, zigzag=True)
    dq, dkv = zigzag_exchange([dq, dkv.view(B, S, -1)], [1, 1], False)
    torch.testing.assert_close(dq, qr.grad.transpose(1, 2)[:, sl], rtol=1e-4, atol=1e-5)
    dk_ref = kr.grad.view(B, nkv, nh // nkv, world * S, d).sum(2).transpose(1, 2)[:, sl]
    dv_ref = vr.grad.view(B, nkv, nh // nkv, world * S, d).sum(2).transpose(1, 2)[:, sl]
    w = nkv * d
    torch.testing.assert_close(dkv[:, :, :w].reshape(B, S, nkv, d), dk_ref, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(dkv[:, :, w:].reshape(B, S, nkv, d), dv_ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("mesh", [1, 0])
@pytest.mark.parametrize("world,nh,nkv", [(2, 2, 2), (3, 2, 1), (4, 4, 2)])
def test_zigzag_ring_is_balanced_and_exact(world, nh, nkv, mesh):
    _dist.run(_ring_zigzag, world, nh, nkv, mesh)


def _zz_residual(rank, world):
    """The zig-zag residual stream's pieces (context_parallel.enable_zigzag_residual): the re-lay is
    a permutation whose backward is the inverse permutation of the gradient, and the zig-zag RoPE
    tables are get_cos_sin's rows at the positions of the rank's zig-zag shard."""
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.context_parallel import context_parallel as CP
    from picotron_amd.model import get_cos_sin
    pgm.setup_process_group_manager(tp_size=1, cp_size=world, pp_size=1, dp_size=1)
    B, S, H = 2, 8, 3
    full = torch.arange(B * world * S * H, dtype=torch.float32).view(B, world * S, H)
    x = full[:, rank * S:(rank + 1) * S].clone().requires_grad_(True)
    y = CP.ZigzagRelayout.apply(x, True)
    h = S // 2
    pos = list(range(rank * h, (rank + 1) * h)) + list(range((2 * world - 1 - rank) * h, (2 * world - rank) * h))
    assert torch.equal(y.detach(), full[:, pos])
    g = torch.randn(y.shape, generator=torch.Generator().manual_seed(rank))
    y.backward(g)
    # the gradient of sum(y * g) w.r.t. the contiguous shard: g laid back
    (gb,) = CP.zigzag_exchange([g], [1], False)
    assert torch.equal(x.grad, gb)
    z = CP.ZigzagRelayout.apply(y.detach(), False)
    assert torch.equal(z, x.detach())
    cos, sin = CP.zigzag_rope_tables(world * S, 16, 10000.0)
    cf, sf = get_cos_sin(world * S, 16, base=10000.0)
    assert torch.equal(cos, cf[pos]) and torch.equal(sin, sf[pos])
    # max_position_embeddings > C * S: the reference rotates rank c's chunk with rows [c P, c P + S)
    # of the max_pos table (P = max_pos / C; update_rope_for_context_parallel, then the first S rows)
    maxp = 3 * world * S
    P = maxp // world
    cos, sin = CP.zigzag_rope_tables(maxp, 16, 10000.0, S=S)
    cf, sf = get_cos_sin(maxp, 16, base=10000.0)
    rows = [(g // S) * P + g % S for g in pos]
    assert torch.equal(cos, cf[rows]) and torch.equal(sin, sf[rows])
    # and a DecoderLayer on the zig-zag shard takes exactly those rows (keyed by its local length)
    from picotron_amd.model import DecoderLayer
    from picotron_amd.train import make_config
    cfg = make_config(dict(hidden_size=32, intermediate_size=64, num_attention_heads=2, num_key_value_heads=2,
                           vocab_size=64, rms_norm_eps=1e-5, rope_theta=10000.0), S, num_hidden_layers=1)
    cfg.max_position_embeddings = maxp
    layer = DecoderLayer(cfg, 0)
    layer.cp_zigzag_residual = True
    zc, zs = layer._tables(torch.device("cpu"), S)
    assert torch.equal(zc, cf[rows].to(torch.bfloat16)) and torch.equal(zs, sf[rows].to(torch.bfloat16))
    with pytest.raises(ValueError):
        CP.zigzag_rope_tables(world * S, 16, 10000.0, S=2 * S)   # longer than the rank's reference slice


@pytest.mark.parametrize("world", [2, 4])
def test_zigzag_residual_relayout_and_tables(world):
    _dist.run(_zz_residual, world)


# ----------------------------------------------------------------------------- PP p2p
def _pp_p2p(rank, world):
    """pp_communications.py:8-45 semantics on a pp=world pipeline: None at the pipeline ends, the
    received tensor equal to the peer's sent one (requires_grad, given shape / dtype), and the
    batched bidirectional exchange of the 1F1B steady state (pipeline_parallel.py:150-190)."""
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.pipeline_parallel import pp_communications as PC
    m = pgm.setup_process_group_manager(tp_size=1, cp_size=1, pp_size=world, dp_size=1)
    assert m.pp_rank == rank
    shape, dt = (2, 3, 4), torch.float32
    act = torch.full(shape, float(rank + 1))
    # forward: recv from the previous stage, send to the next one
    got = PC.pipeline_communicate("recv_forward", "cpu", dt, shapes=shape) if rank % 2 else None
    if rank % 2 == 0:
        assert PC.pipeline_communicate("send_forward", "cpu", dt, tensor=act) is None
        got = PC.pipeline_communicate("recv_forward", "cpu", dt, shapes=shape)
    else:
        PC.pipeline_communicate("send_forward", "cpu", dt, tensor=act)
    if rank == 0:
        assert got is None
    else:
        assert got.requires_grad and got.shape == shape and torch.equal(got.detach(), torch.full(shape, float(rank)))
    # backward: recv from the next stage, send to the previous one
    grad = torch.full(shape, -float(rank + 1))
    if rank % 2 == 0:
        gb = PC.pipeline_communicate("recv_backward", "cpu", dt, shapes=shape)
        PC.pipeline_communicate("send_backward", "cpu", dt, tensor=grad)
    else:
        PC.pipeline_communicate("send_backward", "cpu", dt, tensor=grad)
        gb = PC.pipeline_communicate("recv_backward", "cpu", dt, shapes=shape)
    if rank == world - 1:
        assert gb is None
    else:
        assert torch.equal(gb.detach(), torch.full(shape, -float(rank + 2)))
    # 1F1B steady state between stages 0 and 1: one batched isend + irecv each way
    if rank == 0:
        r = PC.bidirectional_pipeline_communicate("send_fwd_recv_bwd", act, shape, "cpu", dt)
        assert torch.equal(r.detach(), torch.full(shape, -2.0))
    elif rank == 1:
        r = PC.bidirectional_pipeline_communicate("send_bwd_recv_fwd", grad, shape, "cpu", dt)
        assert torch.equal(r.detach(), torch.full(shape, 1.0))
    if rank == world - 1:
        assert PC.bidirectional_pipeline_communicate("send_fwd_recv_bwd", act, shape, "cpu", dt) is None
    if rank == 0:
        assert PC.bidirectional_pipeline_communicate("send_bwd_recv_fwd", grad, shape, "cpu", dt) is None


@pytest.mark.parametrize("world", [2, 3])
def test_pp_p2p(world):
    _dist.run(_pp_p2p, world)


# ------------------------------------------------------------------------ pipeline engine
def _ref_order_1f1b(pp, rank, n):
    """The reference's 1F1B action order (pipeline_parallel.py:139-214), restated: warmup forwards,
    then (F, B) pairs, then the remaining backwards."""
    w = min(pp - rank - 1, n)
    out = [("F", i) for i in range(w)]
    for k in range(n - w):
        out += [("F", w + k), ("B", k)]
    return out + [("B", n - w + j) for j in range(w)]


@pytest.mark.parametrize("pp,n", [(2, 1), (2, 4), (3, 2), (4, 8), (4, 3)])
def test_pipeline_schedule_order_and_transfers(pp, n):
    """Every stage runs each micro-batch forward once and backward once, in the reference's 1F1B
    order; and replaying all stages' transfers (plain sends / receives, and the paired exchanges
    that the steady state batches) through blocking point-to-point channels terminates -- no stage
    waits on a transfer its neighbour never makes (the deadlock the pairing avoids)."""
    from picotron_amd.pipeline_parallel.pipeline_parallel import pipeline_schedule
    scheds = [pipeline_schedule("1f1b", pp, r, n) for r in range(pp)]
    for r, s in enumerate(scheds):
        assert [(op, i) for op, i, _, _ in s] == _ref_order_1f1b(pp, r, n)
    afab = pipeline_schedule("afab", pp, 0, n)
    assert [(op, i) for op, i, _, _ in afab] == [("F", i) for i in range(n)] + [("B", i) for i in range(n)]
    # expand every stage's actions into primitive transfer events in execution order
    ev = []
    for r, s in enumerate(scheds):
        e = []
        for op, i, recv, send in s:
            if recv == "fwd" and r > 0:
                e.append(("recv", r - 1, "act"))
            if recv == "bwd" and r < pp - 1:
                e.append(("recv", r + 1, "grad"))
            if send == "fwd" and r < pp - 1:
                e.append(("send", r + 1, "act"))
            if send == "bwd" and r > 0:
                e.append(("send", r - 1, "grad"))
            if send == "fwd+bwd" and r < pp - 1:
                e.append(("xchg", r + 1, "act", "grad"))
            if send == "bwd+fwd" and r > 0:
                e.append(("xchg", r - 1, "grad", "act"))
        ev.append(e)
    # rendezvous semantics: a send meets the peer's recv (or the peer's exchange that receives it);
    # an exchange completes when the peer posts the complementary exchange or a matching plain op
    pos = [0] * pp
    sent = {}       # (src, dst, kind) -> count delivered and not yet consumed
    progress = True
    while progress:
        progress = False
        for r in range(pp):
            while pos[r] < len(ev[r]):
                e = ev[r][pos[r]]
                if e[0] == "send":                       # buffered send (the batch_isend_irecv post)
                    sent[(r, e[1], e[2])] = sent.get((r, e[1], e[2]), 0) + 1
                elif e[0] == "recv":
                    key = (e[1], r, e[2])
                    if not sent.get(key):
                        break
                    sent[key] -= 1
                else:                                    # exchange: post the send, then wait for the recv
                    _, peer, out_kind, in_kind = e[:4]
                    if len(e) == 4:
                        sent[(r, peer, out_kind)] = sent.get((r, peer, out_kind), 0) + 1
                        ev[r][pos[r]] = e + ("posted",)
                    key = (peer, r, in_kind)
                    if not sent.get(key):
                        break
                    sent[key] -= 1
                pos[r] += 1
                progress = True
    assert pos == [len(e) for e in ev], f"stuck at {pos} of {[len(e) for e in ev]}"
    assert not any(sent.values())


class _TinyLayer(torch.nn.Module):
    """A decoder-layer stand-in with the submodules PipelineParallel.reset_parameters walks."""

    def __init__(self, h):
        super().__init__()
        self.input_layernorm = torch.nn.LayerNorm(h)
        self.attention = torch.nn.Linear(h, h)
        self.post_attention_layernorm = torch.nn.LayerNorm(h)
        self.mlp = torch.nn.Linear(h, h)

    def forward(self, x, position_ids=None):
        x = x + self.attention(self.input_layernorm(x))
        return x + torch.tanh(self.mlp(self.post_attention_layernorm(x)))


class _TinyModel(torch.nn.Module):
    def __init__(self, v, h, layers):
        super().__init__()
        self.embedding = torch.nn.Embedding(v, h)
        self.decoder_layers = torch.nn.ModuleList([_TinyLayer(h) for _ in range(layers)])
        self.final_norm = torch.nn.LayerNorm(h)
        self.final_proj = torch.nn.Linear(h, v)


def _pp_engine(rank, world, kind, dp):
    import types
    import torch.nn.functional as F
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.data_parallel.data_parallel import DataParallelBucket
    from picotron_amd.pipeline_parallel.pipeline_parallel import (PipelineParallel, train_step_pipeline_1f1b,
                                                                  train_step_pipeline_afab)
    pp = world // dp
    m = pgm.setup_process_group_manager(tp_size=1, cp_size=1, pp_size=pp, dp_size=dp)
    V, H, L, mbs, S, ga = 32, 16, 5, 2, 8, 4
    torch.manual_seed(0)
    full = _TinyModel(V, H, L)
    ref = {k: v.detach().clone() for k, v in full.state_dict().items()}
    stage = PipelineParallel(full, types.SimpleNamespace(num_hidden_layers=L))   # re-draws its parameters
    with torch.no_grad():
        for n, p in stage.named_parameters():
            p.copy_(ref[n])
    model = DataParallelBucket(stage) if dp > 1 else stage   # train.py:194-195
    g = torch.Generator().manual_seed(3)
    toks = torch.randint(0, V, (dp, ga, mbs, S + 1), generator=g)

    class Loader:
        grad_acc_steps = ga

        def __init__(self):
            self.i = 0

        def __next__(self):
            t = toks[m.dp_rank, self.i]
            self.i += 1
            return {"input_ids": t[:, :-1], "target_ids": t[:, 1:], "position_ids": torch.arange(S).expand(mbs, S),
                    "hidden_states": None}
    step = train_step_pipeline_1f1b if kind == "1f1b" else train_step_pipeline_afab
    loss = step(model, Loader(), (mbs, S, H), torch.device("cpu"), torch.float32)
    # single-process reference: the same micro-batches through the unsplit model (mean CE per
    # micro-batch, not divided by grad_acc -- pipeline_parallel.py:103,153), dp ranks averaged
    torch.manual_seed(0)
    whole = _TinyModel(V, H, L)
    whole.load_state_dict(ref)
    losses = []
    for r in range(dp):
        for i in range(ga):
            t = toks[r, i]
            x = whole.embedding(t[:, :-1])
            for lay in whole.decoder_layers:
                x = lay(x)
            out = whole.final_proj(whole.final_norm(x))
            lo = F.cross_entropy(out.transpose(1, 2), t[:, 1:])
            (lo / dp).backward()
            if r == m.dp_rank:
                losses.append(lo.item())
    if m.pp_is_last_stage:
        assert abs(loss - sum(losses) / ga) < 1e-5
    else:
        assert loss == 0.0
    wref = dict(whole.named_parameters())
    for n, p in stage.named_parameters():
        assert torch.allclose(p.grad, wref[n].grad, rtol=1e-4, atol=1e-5), n


@pytest.mark.parametrize("kind,world,dp", [("1f1b", 2, 1), ("afab", 2, 1), ("1f1b", 3, 1), ("1f1b", 4, 2)])
def test_pipeline_engine_matches_unsplit_model(kind, world, dp):
    """PipelineParallel + the 1F1B / AFAB steps over gloo (pp 2-3, and pp2 x dp2 under
    DataParallelBucket, whose all-reduce only the stage's last backward triggers): the last stage's logging loss is the mean micro-batch loss and every
    stage's gradients equal the unsplit model's on the same micro-batches."""
    _dist.run(_pp_engine, world, kind, dp)


# ----------------------------------------------------------------------------- TP sequence parallel
def _sp_host(rank, world):
    """tensor_parallel/sequence_parallel.py's host pieces over gloo: the row all-gather /
    reduce-scatter of TPContext, the entry / exit regions (values and gradients) and the hooks,
    against the unsharded computation."""
    from picotron_amd import functional as FN
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.tensor_parallel import sequence_parallel as SPM
    m = pgm.setup_process_group_manager(tp_size=world, cp_size=1, pp_size=1, dp_size=1)
    tp = FN.TPContext.current()
    assert tp.world_size == world and tp.rank == m.tp_rank
    B, S, H = 2, 4 * world, 3
    n = B * S // world
    full = torch.arange(B * S * H, dtype=torch.float32).view(B * S, H)
    # all-gather of token rows / reduce-scatter of partial sums
    mine = full[rank * n:(rank + 1) * n]
    assert torch.equal(tp.all_gather_rows(mine), full)
    part = full * (rank + 1)
    red, h = tp.reduce_scatter_rows(part.clone())
    assert h is None and torch.equal(red, (full * sum(range(1, world + 1)))[rank * n:(rank + 1) * n])
    # entry / exit regions: values and gradients
    x = full.view(B, S, H).clone().requires_grad_(True)
    shard = SPM.ScatterToSequenceRegion.apply(x)
    assert shard.shape == (B, S // world, H) and torch.equal(shard.reshape(n, H), mine)
    y = SPM.GatherFromSequenceRegion.apply(shard * 2)
    assert torch.equal(y, 2 * full.view(B, S, H))
    g = torch.randn(B, S, H, generator=torch.Generator().manual_seed(3))   # replicated upstream gradient
    y.backward(g)
    assert torch.equal(x.grad, 2 * g)   # each rank's rows came back, all-gathered
    # the hooks: an embedding / final_norm pair around a token-local body; a length that does not
    # divide by tp stays unsharded

    class Toy(torch.nn.Module):
        def __init__(self):
            super().__init__()
            torch.manual_seed(0)   # the same (replicated) weights on every rank
            self.embedding = torch.nn.Linear(H, H)
            self.final_norm = torch.nn.Linear(H, H)

        def forward(self, t):
            z = self.embedding(t)
            self.seen = z.shape
            return self.final_norm(z * 3)
    toy = Toy()
    ref = toy(full.view(B, S, H))
    assert SPM.sp_supported() and SPM.enable_sequence_parallel(toy)
    out = toy(full.view(B, S, H))
    assert toy.seen == (B, S // world, H) and torch.allclose(out, ref)
    out.sum().backward()
    ref_toy = Toy()
    ref_toy(full.view(B, S, H)).sum().backward()
    for (n, p), q in zip(toy.named_parameters(), ref_toy.parameters()):
        assert torch.allclose(p.grad, q.grad), n
    toy(torch.randn(B, S + 1, H))
    assert toy.seen == (B, S + 1, H) and toy._pt_sp_state.local_len == 0
    # a forward that raised between the entry and the exit: the next model forward starts unsharded
    toy._pt_sp_state.local_len = S // world
    toy(torch.randn(B, S + 1, H))
    assert toy._pt_sp_state.local_len == 0
    # the chunked layout (c = 2 chunks of one sequence each): rank r holds rows [r n, (r+1) n) of
    # every chunk; the per-chunk collectives, the entry reduce-scatter and the exit gather
    c, n2 = 2, B * S // (2 * world)
    mine2 = torch.cat([full[j * B * S // c + rank * n2: j * B * S // c + (rank + 1) * n2] for j in range(c)])
    from picotron_amd import switches
    with switches.override(tp_sp_chunks=2):
        assert SPM.layout_chunks(B, S, world) == 2 and SPM.layout_chunks(B, S + 1, world) == 0
        assert SPM.layout_chunks(1, S, world) == 1 and SPM.layout_chunks(3, S, world) == 1
    # auto: chunks of >= 8192 rows, at most 8 (mbs 4 / 8 x seq 1024: one chunk; 16: two; 32: four)
    assert SPM.layout_chunks(B, S, world) == 1 and SPM.layout_chunks(4, 1024, 8) == 1
    assert SPM.layout_chunks(8, 1024, 8) == 1 and SPM.layout_chunks(16, 1024, 8) == 2
    assert SPM.layout_chunks(32, 1024, 8) == 4 and SPM.layout_chunks(128, 1024, 8) == 8
    assert SPM.layout_chunks(12, 1024, 8) == 1
    assert torch.equal(SPM.shard_rows(full, tp, c), mine2)
    assert torch.equal(SPM.gather_rows(mine2, tp, c), full)
    out = torch.empty_like(full)
    for j in range(c):
        assert tp.gather_chunk(out, mine2, c, j, async_op=True) is None   # gloo: synchronous
    assert torch.equal(out, full)
    shard = torch.empty_like(mine2)
    for j in range(c):
        tp.scatter_chunk(shard, (full * (rank + 1))[j * B * S // c:(j + 1) * B * S // c], c, j)
    assert torch.equal(shard, mine2 * sum(range(1, world + 1)))
    xp = (full * (rank + 1)).view(B, S, H).requires_grad_(True)     # this rank's partial lookups
    sh2 = SPM.ReduceScatterToSequenceRegion.apply(xp, c)
    assert torch.equal(sh2.reshape(-1, H), mine2 * sum(range(1, world + 1)))
    y2 = SPM.GatherFromSequenceRegion.apply(sh2 * 2, c)
    assert torch.equal(y2, 2 * full.view(B, S, H) * sum(range(1, world + 1)))
    y2.backward(g)
    assert torch.equal(xp.grad, 2 * g)
    x3 = full.view(B, S, H).clone().requires_grad_(True)
    sh3 = SPM.ScatterToSequenceRegion.apply(x3, c)
    assert torch.equal(sh3.reshape(-1, H), mine2)
    SPM.GatherFromSequenceRegion.apply(sh3, c).backward(g)
    assert torch.equal(x3.grad, g)


@pytest.mark.parametrize("world", [2, 4])
def test_sequence_parallel_host_logic(world):
    _dist.run(_sp_host, world)
