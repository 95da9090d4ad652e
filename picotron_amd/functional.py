"""Autograd functions of the decoder-layer hot path, composed from the gfx950 kernels.

Each Function mirrors the saved-tensor contract of the reference op it replaces and launches only
HIP kernels from csrc/ (through kernels.py); collectives go through torch.distributed (RCCL).
There is no eager/CPU fallback: without the HIP library every forward raises.

Reference (okoge-kaz/picotron @ 2025-03-02, paths relative to the checkout):
  * DecoderLayer.forward             picotron/model.py:204-209
  * Attention.forward                picotron/model.py:122-162
  * MLP.forward                      picotron/model.py:184-186
  * TritonRMSNorm / LlamaRMSNorm     picotron/model.py:39-86
  * Column/Row TP linears            picotron/tensor_parallel/tensor_parallel.py:116-123,184-189
  * f / g conjugate TP collectives   picotron/tensor_parallel/tp_communications.py:19-49,74-101
  * F.cross_entropy / grad_acc       train.py:46-49

Layout: activations are token-major 2-D [T = B*S, features] bf16 buffers.  The fused projection
outputs ([T, q|k|v], [T, gate|up]) are consumed in place by strided kernels; nothing is transposed.

Weight gradients are written straight into the gradient buffer by the wgrad GEMM epilogue
(`_wgrad_target`): bf16 `param.grad` accumulation when there is no data parallelism (what autograd
does for the reference at DP=1) or fp32 `param.main_grad` when DataParallelBucket owns the
gradients (data_parallel.py:122-144).  The Functions therefore return None for weight inputs and
notify the gradient owner through `param._pt_grad_ready`.
"""
import math
import os
import weakref

import torch
import torch.distributed as dist

from . import kernels as K
from .switches import S as SW

BF16 = torch.bfloat16


def _fuse():
    """PICOTRON_FUSE=0 turns the epilogue fusions (RoPE in the q|k|v GEMM and the attention
    backward, SwiGLU in the gate|up / down GEMMs) off -- for A/B measurement only; both paths are
    HIP kernels with identical results."""
    return SW.fuse != 0


# ------------------------------------------------------------------------ gradient sinks
def _wgrad_target(p):
    """(buffer, epilogue) the wgrad GEMM of parameter p writes into."""
    mg = getattr(p, "main_grad", None)
    if mg is not None:   # DataParallelBucket's flat buffer: f32 (default) or bf16 (grad_type knob)
        return mg, (K.EPI_F32_ACC if mg.dtype == torch.float32 else K.EPI_BF16_ACC)
    if p.grad is None:
        p.grad = torch.empty_like(p)
        return p.grad, K.EPI_BF16
    return p.grad, K.EPI_BF16_ACC


def _grad_ready(p):
    """Tell the owner of p's gradient (DataParallelBucket) that this backward's grad is in place."""
    hook = getattr(p, "_pt_grad_ready", None)
    if hook is not None:
        hook(p)


# ------------------------------------------------------------------------ paired weight gradients
# The weight-gradient epilogues read-modify-write the gradient sink once per micro-batch: at
# SmolLM-1.7B 2.4 GB of bf16 .grad (DP = 1) or 4.8 GB of f32 main_grad (DataParallelBucket,
# data_parallel.py:122-144) read AND written 32 times per step.  Paired, micro-batch 2 i defers its
# weight gradients -- keeps their dY and X alive -- and micro-batch 2 i + 1 launches each as ONE GEMM
# over both micro-batches' tokens (K = 2 T, kernels.KPair: the A and B operands K-segmented), so the
# sinks are read-modify-written once per pair.  Same sums (the f32 accumulator covers both
# micro-batches before the one rounding into the sink: the same or closer to the fp32 sum).  The
# training loop drives it (train.train_step: `wgrad_pairing(phase)` around each backward at tp = 1;
# None = off, the reference's one-backward-at-a-time behaviour for any other caller).
class WgradPairing:
    phase = None   # None: launch now; 0: defer this backward's weight gradients; 1: pair them
    pending = {}   # parameter ids -> (dy2d, x2d, params) deferred by the previous micro-batch


def wgrad_pairing(phase):
    """Set the pairing phase of the next backward (train.train_step); returns the previous one."""
    old, WgradPairing.phase = WgradPairing.phase, phase
    return old


def flush_wgrad_pairs():
    """Launch (unpaired) every weight gradient a micro-batch deferred and no pair completed."""
    pend, WgradPairing.pending = WgradPairing.pending, {}
    ph, WgradPairing.phase = WgradPairing.phase, None
    try:
        for dy, x, params in pend.values():
            wgrad(dy, x, params)
    finally:
        WgradPairing.phase = ph


def pair_jobs(wjobs):
    """wjobs [(dy2d, x2d, params)] -> the jobs to launch in this backward: [] when it defers them
    (phase 0), each paired with the previous micro-batch's job of the same parameters (phase 1)."""
    ph = WgradPairing.phase
    if ph is None or not wjobs:
        return wjobs
    if ph == 0:
        for dy, x, params in wjobs:
            key = tuple(id(p) for p in params)
            if key in WgradPairing.pending:   # deferred twice without a pair: the older one now
                odx, ox, op = WgradPairing.pending.pop(key)
                wgrad(odx, ox, op)
            WgradPairing.pending[key] = (dy, x, params)
        return []
    out = []
    for dy, x, params in wjobs:
        prev = WgradPairing.pending.pop(tuple(id(p) for p in params), None)
        if prev is not None and (prev[0].shape != dy.shape or prev[1].shape != x.shape or
                                 prev[0].stride() != dy.stride() or prev[1].stride() != x.stride()):
            wgrad(*prev)            # not the same layout: the older one on its own first
            prev = None
        out.append((dy, x, params) if prev is None else (K.KPair(prev[0], dy), K.KPair(prev[1], x), params))
    return out


def wgrad(dy2d, x2d, params, notify=True):
    """dW_i = dY_i^T X for the column segments of dY; one launch when the sinks agree.  Parameters
    with requires_grad=False get no gradient (autograd leaves their .grad alone).  notify=False: a
    partial gradient (one token chunk of a chunked sequence-parallel layer, the sum is not complete
    yet): the owner is not told.  Under weight-gradient pairing (WgradPairing) the job may be
    deferred to, or paired with, the other micro-batch of its pair."""
    if WgradPairing.phase is not None:
        jobs = pair_jobs([(dy2d, x2d, params)])
        if not jobs:
            return
        (dy2d, x2d, params), = jobs
        ph = wgrad_pairing(None)   # settled: the per-parameter fallbacks launch it as it is
        try:
            return wgrad(dy2d, x2d, params, notify)
        finally:
            wgrad_pairing(ph)
    if not all(p.requires_grad for p in params):
        lo = 0
        for p in params:
            n = p.shape[0]
            if p.requires_grad:
                wgrad(dy2d[:, lo:lo + n], x2d, [p], notify)
            lo += n
        return
    targets = [_wgrad_target(p) for p in params]
    epis = {e for _, e in targets}
    if len(epis) == 1:
        K.linear_wgrad(dy2d, x2d, [t for t, _ in targets], epilogue=epis.pop())
    else:  # mixed sinks (one grad already allocated, another not): one launch per parameter
        lo = 0
        for (t, e), p in zip(targets, params):
            n = p.shape[0]
            K.linear_wgrad(dy2d[:, lo:lo + n], x2d, [t], epilogue=e)
            lo += n
    if notify:
        for p in params:
            _grad_ready(p)


def wgrad_group(jobs, notify=True):
    """Several wgrads [(dy2d, x2d, params), ...] in one grouped launch when every sink takes the
    same epilogue (else one wgrad() per job)."""
    if WgradPairing.phase is not None:
        jobs = pair_jobs(jobs)
        if not jobs:
            return
    ph = wgrad_pairing(None)   # the jobs are settled: the per-job fallbacks below launch them as they are
    try:
        _wgrad_group(jobs, notify)
    finally:
        wgrad_pairing(ph)


def _wgrad_group(jobs, notify):
    frozen = any(not p.requires_grad for _, _, params in jobs for p in params)
    targets = [] if frozen else [[_wgrad_target(p) for p in params] for _, _, params in jobs]
    epis = {e for tg in targets for _, e in tg}
    if frozen or len(epis) != 1:
        for dy2d, x2d, params in jobs:
            wgrad(dy2d, x2d, params, notify)
        return
    K.linear_wgrad_grouped([(dy2d, x2d, [t for t, _ in tg]) for (dy2d, x2d, _), tg in zip(jobs, targets)],
                           epilogue=epis.pop())
    if notify:
        for _, _, params in jobs:
            for p in params:
                _grad_ready(p)


def dgrad_with_wgrad(dy2d, weights, wjobs, gu=None, keep_parts=False, split_min=None, order=None, notify=True):
    """dX = dY . [W_0; ...] (with gu: the down_proj dX's SwiGLU backward, dg|du) AND the wgrads
    wjobs [(dy2d, x2d, params)] of the same layer in ONE launch (K.linear_dgrad_dual) when the
    shapes tile for it and every sink takes one epilogue; otherwise the separate launches.
    Returns dX / dg|du.  Under weight-gradient pairing a deferring micro-batch launches the dX alone
    (the split-K halves kept for the consumer as in the dual), the completing one the dual with the
    paired (K = 2 T) weight gradients."""
    if WgradPairing.phase is not None:
        wjobs = pair_jobs(wjobs)
        if not wjobs:
            if gu is not None:
                return K.linear_dgrad_swiglu(dy2d, weights[0], gu)
            return K.linear_dgrad(dy2d, weights, keep_parts=keep_parts, split_min=split_min)
    ph = wgrad_pairing(None)
    try:
        return _dgrad_with_wgrad(dy2d, weights, wjobs, gu, keep_parts, split_min, order, notify)
    finally:
        wgrad_pairing(ph)


def _dgrad_with_wgrad(dy2d, weights, wjobs, gu, keep_parts, split_min, order, notify):
    frozen = any(not p.requires_grad for _, _, params in wjobs for p in params)
    mns = [(dy.shape[1], x.shape[1]) for dy, x, _ in wjobs]
    dmn = (dy2d.shape[0], gu.shape[1] // 2 if gu is not None else weights[0].shape[1])
    if K.dual_enabled() and not frozen and K.dual_fits(dmn, mns):
        targets = [[_wgrad_target(p) for p in params] for _, _, params in wjobs]
        epis = {e for tg in targets for _, e in tg}
        if len(epis) == 1:
            epi = epis.pop()
            wk = [(dy, x, [t for t, _ in tg]) for (dy, x, _), tg in zip(wjobs, targets)]
            dx = K.linear_dgrad_dual(dy2d, weights, wk, epi, gu=gu, keep_parts=keep_parts, split_min=split_min,
                                     order=order)
            if dx is None:   # not tileable after all: the same sinks, separate launches
                dx = K.linear_dgrad_swiglu(dy2d, weights[0], gu) if gu is not None else K.linear_dgrad(dy2d, weights)
                K.linear_wgrad_grouped(wk, epilogue=epi)
        else:   # mixed sinks: one launch per parameter (the targets exist now)
            dx = K.linear_dgrad_swiglu(dy2d, weights[0], gu) if gu is not None else K.linear_dgrad(dy2d, weights)
            for (dy, x, params), tg in zip(wjobs, targets):
                lo = 0
                for p, (t, e) in zip(params, tg):
                    K.linear_wgrad(dy[:, lo:lo + p.shape[0]], x, [t], epilogue=e)
                    lo += p.shape[0]
        if notify:
            for _, _, params in wjobs:
                for p in params:
                    _grad_ready(p)
        return dx
    dx = K.linear_dgrad_swiglu(dy2d, weights[0], gu) if gu is not None else K.linear_dgrad(dy2d, weights)
    wgrad_group(wjobs, notify)
    return dx


# Deferred RMSNorm weight-gradient sums: inside an autograd backward, a norm whose gradient has
# no DataParallelBucket owner waiting on it leaves its per-block partial rows here, and one
# pt_rmsnorm_colsum_batch launch at the end of the backward (an engine final callback) sums them
# all into their sinks -- 2 L + 1 column-sum launches per micro-batch become one.  Norms whose
# weights' owner all-reduces during this backward (a _pt_grad_ready hook, and _pt_grad_sync() true:
# the last micro-batch of a step) keep the immediate sum, so their bucket's all-reduce overlaps the
# rest of the backward; under no_sync (the other grad_acc - 1 micro-batches) they defer too.  PICOTRON_NORM_DEFER=0 turns this off (A/B only).
_PENDING_DW = {}   # autograd graph task id -> [(partial, weight, stream)]


def _norm_defer_enabled():
    return SW.norm_defer != 0


def _norm_dw_sink(weight):
    """The weight gradient's sink as AccumulateGrad would treat it now: (buffer, epilogue)."""
    mg = getattr(weight, "main_grad", None)
    if mg is not None:
        return mg, (K.DW_ACC_F32 if mg.dtype == torch.float32 else K.DW_ACC_BF16)
    if weight.grad is None:
        weight.grad = torch.empty_like(weight)
        return weight.grad, 0
    return weight.grad, K.DW_ACC_BF16


def _sp_sum_partials(pending):
    """Sequence-parallel norms (entries with a tp group): each rank's column sums cover only its
    token rows, so their sum over the tp group is the weight gradient the reference computes on every
    rank.  Their partials are summed into one f32 [n, H] block per (width, stream, group), ONE
    all-reduce of it runs over the tp group, and each row re-enters the queue as a one-row partial
    (the sinks then see exactly the non-SP path's colsum).  Returns the rewritten entry list."""
    out, sp = [], {}
    for e in pending:
        if e[3] is None:
            out.append(e)
        else:
            part, weight, stream, tp = e
            sp.setdefault((part.shape[1], part.device, stream, id(tp.group)), []).append(e)
    for (cols, dev, stream, _), es in sp.items():
        with torch.cuda.stream(stream):
            tot = torch.zeros(len(es), cols, dtype=torch.float32, device=dev)
            for i in range(0, len(es), 32):
                K.rmsnorm_colsum_batch([(p, tot[j], K.DW_ACC_F32) for j, (p, _, _, _) in enumerate(es[i:i + 32], i)])
            es[0][3].all_reduce(tot)
            out += [(tot[j:j + 1], w, st, None, True) for j, (_, w, st, _) in enumerate(es)]
    return out


def _flush_norm_dw(task):
    """Sum every pending partial into its sink.  Sinks are resolved here, in backward order, so a
    .grad is only created (and stored into) once its sum is launched; a weight used by several
    norms of one backward gets a store and then accumulates, and jobs that share a sink go into
    separate, stream-ordered launches (generation g = the g-th job on that sink)."""
    groups, seen = {}, {}
    notify = []
    for part, weight, stream, *rest in _sp_sum_partials(_PENDING_DW.pop(task, [])):
        if rest and rest[-1] is True:   # a sequence-parallel norm's summed gradient: tell its owner
            notify.append(weight)
        buf, sink = _norm_dw_sink(weight)
        gen = seen.get(buf.data_ptr(), 0)
        seen[buf.data_ptr()] = gen + 1
        groups.setdefault((gen, part.shape[1], part.device, stream), []).append((part, buf, sink))
    for (_, _, _, stream), js in sorted(groups.items(), key=lambda kv: kv[0][0]):
        with torch.cuda.stream(stream):   # the stream the partials were produced on
            for i in range(0, len(js), 32):
                K.rmsnorm_colsum_batch(js[i:i + 32])
    for w in notify:
        _grad_ready(w)


def norm_bwd(dy2, z, weight, rstd, mode, dres=None, need_dw=True, sp=None):
    """RMSNorm backward with the weight gradient summed straight into p's sink (bf16 .grad store or
    accumulate -- autograd's AccumulateGrad -- or the f32 main_grad of DataParallelBucket).  A frozen
    weight (requires_grad=False) gets no gradient, as under autograd.  sp: the TPContext whose ranks
    hold the other token rows (sequence parallelism): the weight gradient is the sum over that group
    of this rank's column sums (_sp_sum_partials, at the end of the backward)."""
    if not (need_dw and weight.requires_grad):
        dx, _ = K.rmsnorm_bwd(dy2, z, weight, rstd, mode, dres=dres)
        return dx
    task = torch._C._current_graph_task_id()   # -1 outside an autograd backward
    if sp is not None and sp.world_size > 1:
        dx, partial = K.rmsnorm_bwd(dy2, z, weight, rstd, mode, dres=dres, defer_dw=True)
        entry = (partial, weight, torch.cuda.current_stream(z.device), sp)
        sync = getattr(weight, "_pt_grad_sync", None)
        waiting = getattr(weight, "_pt_grad_ready", None) is not None and (sync is None or sync())
        if task == -1 or waiting:
            # not inside an autograd backward, or an owner (a data-parallel wrapper) all-reduces this
            # backward and waits for it at its end: sum over tp and store now (one [1, H] all-reduce)
            for part, w, st, *_ in _sp_sum_partials([entry]):
                buf, sink = _norm_dw_sink(w)
                K.rmsnorm_colsum_batch([(part, buf, sink)])
                _grad_ready(w)
            return dx
        if task not in _PENDING_DW:
            _PENDING_DW[task] = []
            torch.autograd.Variable._execution_engine.queue_callback(lambda: _flush_norm_dw(task))
        _PENDING_DW[task].append(entry)
        return dx
    # an owner that all-reduces this backward (a data-parallel wrapper outside no_sync) is told at once
    sync = getattr(weight, "_pt_grad_sync", None)
    waiting = getattr(weight, "_pt_grad_ready", None) is not None and (sync is None or sync())
    if not waiting and z.is_cuda and task != -1 and _norm_defer_enabled():
        dx, partial = K.rmsnorm_bwd(dy2, z, weight, rstd, mode, dres=dres, defer_dw=True)
        if task not in _PENDING_DW:
            _PENDING_DW[task] = []
            torch.autograd.Variable._execution_engine.queue_callback(lambda: _flush_norm_dw(task))
        _PENDING_DW[task].append((partial, weight, torch.cuda.current_stream(z.device), None))
        return dx
    buf, sink = _norm_dw_sink(weight)
    dx, _ = K.rmsnorm_bwd(dy2, z, weight, rstd, mode, dres=dres, dw_out=buf, dw_sink=sink)
    _grad_ready(weight)
    return dx


# ------------------------------------------------------------------------ TP collectives
class TPContext:
    """The tp group as a layer sees it (process_group_manager.py:18,35-37 of the reference)."""

    def __init__(self, group=None, world_size=1, rank=0):
        self.group, self.world_size, self.rank = group, world_size, rank

    @staticmethod
    def current():
        from . import process_group_manager as pgm
        m = pgm.process_group_manager
        if m is None or m.tp_world_size == 1:
            return TPContext()
        return TPContext(m.tp_group, m.tp_world_size, m.tp_rank)

    def all_reduce(self, t, async_op=False):
        """Sum over the tp group (tp_communications.py:32,44).  Identity at tp=1."""
        if self.world_size == 1:
            return None
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=async_op)

    # ---- sequence parallelism (tensor_parallel/sequence_parallel.py): the residual stream between
    # the TP blocks is sharded by token rows over the tp group; the all-reduce of a row-parallel
    # output becomes a reduce-scatter onto the shards, a column-parallel input an all-gather of them
    def _nccl(self):
        return dist.get_backend(self.group) == "nccl"

    def all_gather_rows(self, t):
        """This rank's [n, ...] rows -> [world * n, ...] (rank i's rows at i * n)."""
        if self.world_size == 1:
            return t
        t = t.contiguous()
        out = torch.empty((self.world_size * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        self.all_gather_rows_into(out, t)
        return out

    def all_gather_rows_into(self, out, t, async_op=False):
        """t [n, ...] (this rank's rows) -> out [world * n, ...] (a contiguous buffer or row block of
        one; rank i's rows at i * n).  Returns the work handle (async_op, RCCL) or None (done)."""
        if self._nccl():
            return dist.all_gather_into_tensor(out, t.contiguous(), group=self.group, async_op=async_op)
        # gloo (CPU tests, one-GPU rehearsals): the list form, synchronous
        dist.all_gather(list(out.chunk(self.world_size)), t.contiguous(), group=self.group)
        return None

    def reduce_scatter_rows(self, t, async_op=False):
        """[world * n, ...] partial sums -> (this rank's [n, ...] rows of their sum, handle or None)."""
        if self.world_size == 1:
            return t, None
        n = t.shape[0] // self.world_size
        if self._nccl():
            out = torch.empty((n,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
            h = dist.reduce_scatter_tensor(out, t.contiguous(), op=dist.ReduceOp.SUM, group=self.group,
                                           async_op=async_op)
            return out, h
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)   # gloo: the sum, then my rows
        return t[self.rank * n:(self.rank + 1) * n], None

    def reduce_scatter_rows_into(self, out, t, async_op=False):
        """t [world * n, ...] partial sums -> out [n, ...] (a contiguous buffer or row block of one) =
        this rank's rows of their sum.  Returns the work handle (async_op, RCCL) or None (done)."""
        if self._nccl():
            return dist.reduce_scatter_tensor(out, t.contiguous(), op=dist.ReduceOp.SUM, group=self.group,
                                              async_op=async_op)
        n = out.shape[0]
        t = t.clone()
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)   # gloo: the sum, then my rows
        out.copy_(t[self.rank * n:(self.rank + 1) * n])
        return None

    # the chunked token-row layout (sequence parallelism with c chunks, tensor_parallel/
    # sequence_parallel.py): the flattened [T, ...] rows are c chunks of T / c rows (whole sequences);
    # rank r holds rows [r n, (r + 1) n) of every chunk (n = T / (c world)), chunk after chunk, so
    # chunk j's all-gather / reduce-scatter is one collective of its own that the layer issues as
    # soon as chunk j's producer is done and waits for only where chunk j's consumer starts
    def gather_chunk(self, full, shard, c, j, async_op=False):
        """Chunk j of the shard [T / world, ...] -> rows of chunk j of full [T, ...]; handle or None."""
        n = shard.shape[0] // c
        return self.all_gather_rows_into(full[j * n * self.world_size:(j + 1) * n * self.world_size],
                                         shard[j * n:(j + 1) * n], async_op=async_op)

    def scatter_chunk(self, shard, part, c, j, async_op=False):
        """Partial sums of chunk j's rows (part [T / c, ...]) -> chunk j's rows of the shard
        [T / world, ...] (their sum over the group); handle or None."""
        n = shard.shape[0] // c
        return self.reduce_scatter_rows_into(shard[j * n:(j + 1) * n], part, async_op=async_op)


def wait_all(handles):
    for h in handles:
        if h is not None:
            h.wait()


def _contig2d(x):
    x2 = x.reshape(-1, x.shape[-1])
    return x2 if x2.is_contiguous() else x2.contiguous()


# ------------------------------------------------------------------------ RMSNorm
class RMSNormFunction(torch.autograd.Function):
    """TritonRMSNorm (mode 0, model.py:51-65) / LlamaRMSNorm (mode 1, model.py:81-86)."""

    @staticmethod
    def forward(ctx, x, weight, eps, mode):
        x2 = _contig2d(x)
        y, rstd, _ = K.rmsnorm_fwd(x2, weight, eps, mode)
        ctx.save_for_backward(x2, weight, rstd)
        ctx.mode, ctx.shape = mode, x.shape
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, weight, rstd = ctx.saved_tensors
        dx = norm_bwd(_contig2d(dy), x2, weight, rstd, ctx.mode, need_dw=ctx.needs_input_grad[1])
        return dx.view(ctx.shape), None, None, None


class AddRMSNormFunction(torch.autograd.Function):
    """flash-attn layer_norm_fn(x, w, residual=r, prenorm=True, is_rms_norm=True) as reachable from
    TritonRMSNorm.forward (model.py:51-65): z = bf16(x + r); y = norm(z); returns (y, z)."""

    @staticmethod
    def forward(ctx, x, residual, weight, eps, mode):
        x2, r2 = _contig2d(x), _contig2d(residual)
        y, rstd, z = K.rmsnorm_fwd(x2, weight, eps, mode, residual=r2)
        ctx.save_for_backward(z, weight, rstd)
        ctx.mode, ctx.shape = mode, x.shape
        return y.view(x.shape), z.view(x.shape)

    @staticmethod
    def backward(ctx, dy, dz):
        z, weight, rstd = ctx.saved_tensors
        if dy is None:
            dy = torch.zeros(ctx.shape, dtype=z.dtype, device=z.device)
        dres = _contig2d(dz) if dz is not None else None
        dx = norm_bwd(_contig2d(dy), z, weight, rstd, ctx.mode, dres=dres, need_dw=ctx.needs_input_grad[2])
        dx = dx.view(ctx.shape)
        return dx, dx, None, None, None


# ------------------------------------------------------------------------ linear
class LinearFunction(torch.autograd.Function):
    """Y = X W^T (F.linear, no bias).  tp_reduce_fwd: sum Y over tp (RowParallelLinear's
    ReduceFromModelParallelRegion, tp_communications.py:44); tp_reduce_bwd: sum dX over tp
    (ColumnParallelLinear's CopyToModelParallelRegion, tp_communications.py:32), overlapped with the
    dW GEMM as LinearWithAsyncAllReduce does (tp_communications.py:83-101)."""

    @staticmethod
    def forward(ctx, x, weight, tp_reduce_fwd, tp_reduce_bwd):
        x2 = _contig2d(x)
        y = K.linear_fwd(x2, [weight])
        if tp_reduce_fwd:
            TPContext.current().all_reduce(y)
        ctx.save_for_backward(x2, weight)
        ctx.tp_reduce_bwd, ctx.xshape = tp_reduce_bwd, x.shape
        return y.view(*x.shape[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, weight = ctx.saved_tensors
        dy2 = _contig2d(dy)
        dx = handle = None
        if ctx.needs_input_grad[0]:
            dx = K.linear_dgrad(dy2, [weight])
            if ctx.tp_reduce_bwd:
                handle = TPContext.current().all_reduce(dx, async_op=True)
        if ctx.needs_input_grad[1]:
            wgrad(dy2, x2, [weight])
        if handle is not None:
            handle.wait()
        return (dx.view(ctx.xshape) if dx is not None else None), None, None, None


def linear(x, weight, tp_reduce_fwd=False, tp_reduce_bwd=False):
    return LinearFunction.apply(x, weight, tp_reduce_fwd, tp_reduce_bwd)


# ------------------------------------------------------------------------ lm_head + CE statistics
# The lm_head GEMM leaves, next to the logits, the CE forward's per-row (max, sum-exp) of the stored
# bf16 values for each 256- (128-) column output tile (csrc/gemm.hip EPI_CE_STATS).  They travel beside the logits, keyed by the
# logits' storage: F.cross_entropy on those logits (or a view of them, unmodified -- same version
# counter) combines V/256 pairs per row instead of streaming the [T, V] logits a second time; any
# other consumer sees ordinary logits.
_CE_STATS = {}


def _stash_ce_stats(y, stats):
    for key in [k for k, e in _CE_STATS.items() if e[0]() is None]:
        del _CE_STATS[key]
    _CE_STATS[y.data_ptr()] = (weakref.ref(y), y._version, y.numel(), stats)


def _take_ce_stats(lg):
    e = _CE_STATS.pop(lg.data_ptr(), None)
    if e is None:
        return None
    ref, version, numel, stats = e
    if ref() is None or lg._version != version or lg.numel() != numel or stats.shape[1] != lg.shape[0]:
        return None
    return stats


def ce_stats_enabled():
    return SW.ce_stats != 0


class LMHeadFunction(torch.autograd.Function):
    """final_proj(x) (model.py:270, no bias, tp 1) on the GEMM with the CE statistics epilogue; the
    backward is LinearFunction's."""

    @staticmethod
    def forward(ctx, x, weight, tp_reduce_bwd):
        x2 = _contig2d(x)
        y, stats = K.linear_ce_stats(x2, weight)
        _stash_ce_stats(y, stats)
        ctx.save_for_backward(x2, weight)
        ctx.xshape, ctx.tp_reduce_bwd = x.shape, tp_reduce_bwd
        return y.view(*x.shape[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, weight = ctx.saved_tensors
        dy2 = _contig2d(dy)
        dx = handle = None
        if ctx.needs_input_grad[0]:
            dx = K.linear_dgrad(dy2, [weight])
            if ctx.tp_reduce_bwd:   # a vocab shard (ColumnParallelLinear): sum dX over tp beside the dW GEMM
                handle = TPContext.current().all_reduce(dx, async_op=True)
        if ctx.needs_input_grad[1]:
            wgrad(dy2, x2, [weight])
        if handle is not None:
            handle.wait()
        return (dx.view(ctx.xshape) if dx is not None else None), None, None


def lm_head_linear(x, weight):
    """Y = x W^T for the lm_head: with the CE statistics when the shape tiles, else plain linear."""
    T = x.numel() // x.shape[-1]
    if (ce_stats_enabled() and x.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16
            and K.ce_stats_fusable(T, weight.shape[0]) and x.shape[-1] % 64 == 0):
        return LMHeadFunction.apply(x, weight, False)
    return linear(x, weight)


# ------------------------------------------------------------------------ vocab-parallel CE
# The reference's apply_tensor_parallel makes the lm_head ColumnParallelLinear(gather_output=True)
# (tensor_parallel.py:50): every rank all-gathers the [T, V] logits (tp_communications.py:51-72; at
# tp 8 and T 4096, 336 MiB into every rank per micro-batch) for F.cross_entropy (train.py:49).  Here
# that layer returns a stand-in of the gathered logits (same shape and dtype, no storage) carrying
# the vocab shards: F.cross_entropy on it -- or on its view(-1, V) / transpose(1, 2), the
# reference's two call sites -- reduces each shard to 16 bytes per row with the lm_head GEMM's
# statistics, all-gathers those, and differentiates the shard only (VocabParallelCEFunction); any
# other use gathers the logits exactly as the reference does, once, and runs on them.
def vp_ce_shape_ok(T, vocab_shard, K_in):
    return SW.vp_ce != 0 and K.ce_stats_fusable(T, vocab_shard) and K_in % 64 == 0


def lm_head_shard(x, weight):
    """The vocab shard's logits (ColumnParallelLinear's GEMM, dX summed over tp in its backward) and
    their per-tile CE statistics."""
    y = LMHeadFunction.apply(x, weight, True)
    return y, _take_ce_stats(_contig2d(y))


class _VPInfo:
    def __init__(self, shard, stats, vocab_lo, vocab, materialize):
        self.shard, self.stats, self.vocab_lo, self.vocab = shard, stats, vocab_lo, vocab
        self.materialize, self.full = materialize, None

    def gathered(self):
        if self.full is None:
            self.full = self.materialize()
        return self.full


def _standin(info, shape, path, requires_grad):
    """A data-less [shape] HipLogits (a 0-dim tensor expanded: no storage of that size) carrying the
    vocab shards `info` and the view path from the gathered logits.  It requires grad when the
    shard does (its own autograd history is a dummy: F.cross_entropy on it differentiates the shard
    through VocabParallelCEFunction, any other op through the gathered logits)."""
    ph = torch.empty((), dtype=info.shard.dtype, device=info.shard.device, requires_grad=requires_grad)
    out = ph.expand(*shape).as_subclass(HipLogits)
    out._pt_vp, out._pt_vp_path = info, path
    return out


def vp_logits(shard, stats, vocab_lo, vocab, materialize):
    """The stand-in for the gathered [..., vocab] logits of the vocab shard `shard` [..., Vs]
    (columns vocab_lo ..); `materialize()` gathers the real logits (GatherFromModelParallelRegion)."""
    return _standin(_VPInfo(shard, stats, vocab_lo, vocab, materialize), tuple(shard.shape[:-1]) + (vocab,), (),
                    shard.requires_grad)


def _vp_real(t):
    """A vocab-parallel stand-in (or a view of one) as the real gathered logits (same view)."""
    real = t._pt_vp.gathered()
    with torch._C.DisableTorchFunctionSubclass():
        for f, a, kw in t._pt_vp_path:
            real = f(real, *a, **kw)
    return real.as_subclass(HipLogits)


def _is_vp(t):
    return isinstance(t, HipLogits) and getattr(t, "_pt_vp", None) is not None


# metadata reads that are safe on the stand-in (no data)
_VP_META = frozenset([torch.Tensor.dim, torch.Tensor.size, torch.Tensor.numel, torch.Tensor.__len__])


class VocabParallelCEFunction(torch.autograd.Function):
    """F.cross_entropy(gathered logits, targets) from the vocab shards: per-row (max, sum-exp,
    target logit) of this rank's shard (pt_cross_entropy_vp_partial, from the lm_head GEMM's
    statistics), all-gathered over tp (16 B per row), combined in rank order
    (pt_cross_entropy_vp_combine) -- the same loss on every rank.  Backward: the shard's
    (exp(x - lse) - onehot) * scale, the columns of the gathered logits' gradient this rank's
    GatherFromModelParallelRegion backward (tp_communications.py:69-72) would keep."""

    @staticmethod
    def forward(ctx, shard, targets, stats, vocab_lo, vocab, ignore_index, reduction):
        lg = _contig2d(shard)
        tg = targets.reshape(-1)
        tp = TPContext.current()
        part = K.cross_entropy_vp_partial(lg, tg, stats, vocab_lo)
        parts = tp.all_gather_rows(part).view(tp.world_size, lg.shape[0], 4)
        odt = shard.dtype if shard.dtype in (torch.bfloat16, torch.float32) else torch.float32
        loss, inv_count, row_lse = K.cross_entropy_vp_combine(parts, tg, vocab, ignore_index, out_dtype=odt,
                                                              reduction=reduction)
        ctx.save_for_backward(lg, tg, row_lse, *([inv_count] if inv_count is not None else []))
        ctx.vocab_lo, ctx.ignore_index, ctx.shape, ctx.reduction = vocab_lo, ignore_index, shard.shape, reduction
        return loss if loss.dtype == shard.dtype else loss.to(shard.dtype)

    @staticmethod
    def backward(ctx, g):
        lg, tg, row_lse, *inv = ctx.saved_tensors
        if ctx.reduction == "none":
            scale = g.float().reshape(-1).contiguous()
        elif ctx.reduction == "sum":
            scale = g.float().reshape(1)
        else:
            scale = g.float().reshape(1) * inv[0]
        dl = K.cross_entropy_grad_lse_shard(lg, tg, row_lse, scale, ctx.vocab_lo, ctx.ignore_index)
        return dl.view(ctx.shape), None, None, None, None, None, None


_ROW_VIEWS = (torch.Tensor.view, torch.Tensor.reshape, torch.Tensor.flatten)


def _vp_path_form(path, ndim):
    """Which of the reference's two cross-entropy call forms the view path from the gathered
    [..., V] logits (ndim dims) is, so that the shard rows meet their targets in order: 'rows' --
    only view / reshape / flatten (on the contiguous gathered logits they never reorder rows:
    train.py:49's view(-1, V)) -- or 'bvs' -- exactly one transpose(1, 2) / permute(0, 2, 1) of a 3-D
    [B, S, V] (pipeline_parallel.py:103,153); None for any other path (rows possibly reordered: the
    caller gathers the logits and runs on them, as the reference does).  contiguous() reorders
    nothing and is skipped."""
    ops = [(f, a, kw) for f, a, kw in path if f is not torch.Tensor.contiguous]
    if all(f in _ROW_VIEWS for f, _, _ in ops):
        return "rows"
    if len(ops) != 1 or ndim != 3:
        return None
    f, a, kw = ops[0]
    dims = tuple(a) + tuple(kw.values())
    if len(dims) == 1 and isinstance(dims[0], (tuple, list)):
        dims = tuple(dims[0])
    dims = tuple(int(x) % 3 for x in dims)
    if f is torch.Tensor.transpose and sorted(dims) == [1, 2]:
        return "bvs"
    if f is torch.Tensor.permute and dims == (0, 2, 1):
        return "bvs"
    return None


def _vp_cross_entropy(input, target, reduction, ignore_index):
    """cross_entropy on a stand-in in one of the reference's two forms -- [N, V] rows (train.py:49)
    or [B, V, S] = transpose(1, 2) of [B, S, V] (pipeline_parallel.py:103,153) -- else None."""
    info = input._pt_vp
    shard, V = info.shard, info.vocab
    lead = tuple(shard.shape[:-1])
    rows = shard.numel() // shard.shape[-1]
    target = _plain(target)
    form = _vp_path_form(input._pt_vp_path, shard.dim())
    if form == "rows" and input.dim() == 2 and tuple(input.shape) == (rows, V) and target.dim() == 1 and \
            target.numel() == rows:
        out_shape = (rows,)
    elif form == "bvs" and input.dim() == 3 and len(lead) == 2 and tuple(input.shape) == (lead[0], V, lead[1]) and \
            tuple(target.shape) == lead:
        out_shape = lead
    else:
        return None
    out = VocabParallelCEFunction.apply(shard, target.reshape(-1), info.stats, info.vocab_lo, V, ignore_index,
                                        reduction)
    return out.view(out_shape) if reduction == "none" else out


# ------------------------------------------------------------------------ attention block
def ring_enabled():
    """model.py:148: the CONTEXT_PARALLEL switch set by apply_context_parallel."""
    return os.getenv("CONTEXT_PARALLEL", "0") == "1"


class AttnShape:
    """Views of the fused [T, q | k | v] projection as token-major [B, S, heads, d] tensors."""

    def __init__(self, B, S, nh, nkv, d, zz=False):
        self.B, self.S, self.nh, self.nkv, self.d = B, S, nh, nkv, d
        self.T = B * S
        self.wq, self.wkv = nh * d, nkv * d
        self.zz = zz    # the tokens are a zig-zag CP shard (context_parallel.apply_context_parallel)

    def q(self, t):
        return t[:, :self.wq].view(self.B, self.S, self.nh, self.d)

    def k(self, t):
        return t[:, self.wq:self.wq + self.wkv].view(self.B, self.S, self.nkv, self.d)

    def v(self, t):
        return t[:, self.wq + self.wkv:].view(self.B, self.S, self.nkv, self.d)


# head dims the attention kernels do not take (64 / 128; e.g. 60 = SmolLM-360M with 16 heads, as
# create_config.py's own example builds it): every head zero-padded to the next kernel width, each
# rotary half separately -- [x1 | 0 | x2 | 0] -- so that RoPE's (d, d + d/2) pairs stay pairs and the
# padded columns add nothing to q . k or to o (the scale stays 1/sqrt(d) of the real d).
ATTN_HEAD_DIMS = (64, 128)


def _head_pad_dim(d):
    return next((w for w in ATTN_HEAD_DIMS if d <= w), None)


def _pad_heads(t2d, heads, d, dp):
    """[T, heads * d] -> [T, heads, dp]: each head's halves at 0 and dp / 2, zeros between."""
    T, h, hp = t2d.shape[0], d // 2, dp // 2
    x = t2d.reshape(T, heads, d)
    out = torch.zeros(T, heads, dp, dtype=t2d.dtype, device=t2d.device)
    out[..., :h] = x[..., :h]
    out[..., hp:hp + h] = x[..., h:]
    return out


def _unpad_heads(tp, d):
    """Inverse of _pad_heads: [T, heads, dp] -> [T, heads * d] (contiguous)."""
    T, heads, dp = tp.shape
    h, hp = d // 2, dp // 2
    return torch.cat([tp[..., :h], tp[..., hp:hp + h]], dim=-1).reshape(T, heads * d)


def _pad_rope_table(t, d, dp):
    return _pad_heads(t, 1, d, dp).view(t.shape[0], dp)


def _attention_core_fwd_padded(qkv, sh, cos, sin, scale):
    d, dp = sh.d, _head_pad_dim(sh.d)
    heads = sh.nh + 2 * sh.nkv
    x = _pad_heads(qkv, heads, d, dp).view(sh.T, heads * dp)
    K.rope_(x, sh.nh + sh.nkv, dp, _pad_rope_table(cos, d, dp), _pad_rope_table(sin, d, dp), sh.S)
    # the rotated q|k back into qkv (in place, as the kernel-width path leaves them for the backward)
    qkv[:, :sh.wq + sh.wkv].copy_(_unpad_heads(x.view(sh.T, heads, dp)[:, :sh.nh + sh.nkv], d))
    shp = AttnShape(sh.B, sh.S, sh.nh, sh.nkv, dp)
    o, lse = K.attn_fwd(shp.q(x), shp.k(x), shp.v(x), scale, True)
    return _unpad_heads(o.view(sh.T, sh.nh, dp), d).view(sh.B, sh.S, sh.nh, d), lse


def _attention_core_bwd_padded(do, qkv, o, lse, sh, cos, sin, scale):
    d, dp = sh.d, _head_pad_dim(sh.d)
    heads = sh.nh + 2 * sh.nkv
    x = _pad_heads(qkv, heads, d, dp).view(sh.T, heads * dp)   # q|k already rotated (the forward)
    shp = AttnShape(sh.B, sh.S, sh.nh, sh.nkv, dp)
    dop = _pad_heads(do.reshape(sh.T, sh.wq), sh.nh, d, dp).view(sh.B, sh.S, sh.nh, dp)
    op = _pad_heads(o.reshape(sh.T, sh.wq), sh.nh, d, dp).view(sh.B, sh.S, sh.nh, dp)
    dxp = torch.empty_like(x)
    K.attn_bwd(dop, shp.q(x), shp.k(x), shp.v(x), op, lse, scale, True, dq=shp.q(dxp), dk=shp.k(dxp), dv=shp.v(dxp))
    K.rope_(dxp, sh.nh + sh.nkv, dp, _pad_rope_table(cos, d, dp), _pad_rope_table(sin, d, dp), sh.S, inverse=True)
    return _unpad_heads(dxp.view(sh.T, heads, dp), d)


def _req_head_dim(d, roped):
    if _head_pad_dim(d) is None or d % 2 or roped:
        raise RuntimeError(f"attention: head_dim {d} -- the kernels take 64 / 128 and pad even dims below 128")


def attention_core_fwd(qkv, sh, cos, sin, scale, roped=False):
    """RoPE on q|k in place (model.py:136-137; skipped when the projection epilogue already
    rotated them: roped), then causal flash attention (model.py:154) or the ring
    (model.py:148-151).  Returns (o [B,S,nh,d] bf16, lse f32 [B,nh,S])."""
    if sh.d not in ATTN_HEAD_DIMS and not ring_enabled():
        _req_head_dim(sh.d, roped)
        return _attention_core_fwd_padded(qkv, sh, cos, sin, scale)
    if not roped:
        K.rope_(qkv, sh.nh + sh.nkv, sh.d, cos, sin, sh.S)
    if ring_enabled():
        from .context_parallel.context_parallel import ring_attention_tokens
        return ring_attention_tokens(qkv, sh, scale, True, resident=sh.zz)
    return K.attn_fwd(sh.q(qkv), sh.k(qkv), sh.v(qkv), scale, True)


def attention_core_bwd(do, qkv, o, lse, sh, cos, sin, scale):
    """dq|dk|dv written into one [T, q|k|v] buffer, then the inverse rotation of dq|dk."""
    if sh.d not in ATTN_HEAD_DIMS and not ring_enabled():
        return _attention_core_bwd_padded(do, qkv, o, lse, sh, cos, sin, scale)
    dqkv = torch.empty_like(qkv)
    if ring_enabled():
        from .context_parallel.context_parallel import ring_attention_tokens_bwd
        ring_attention_tokens_bwd(do, qkv, o, lse, sh, scale, True, dqkv, resident=sh.zz)
        K.rope_(dqkv, sh.nh + sh.nkv, sh.d, cos, sin, sh.S, inverse=True)
    elif _fuse():  # the RoPE backward is fused into the dq / dk stores
        K.attn_bwd(do, sh.q(qkv), sh.k(qkv), sh.v(qkv), o, lse, scale, True,
                   dq=sh.q(dqkv), dk=sh.k(dqkv), dv=sh.v(dqkv), rope=(cos, sin))
    else:
        K.attn_bwd(do, sh.q(qkv), sh.k(qkv), sh.v(qkv), o, lse, scale, True,
                   dq=sh.q(dqkv), dk=sh.k(dqkv), dv=sh.v(dqkv))
        K.rope_(dqkv, sh.nh + sh.nkv, sh.d, cos, sin, sh.S, inverse=True)
    return dqkv


def attn_block_fwd(h2, wq, wk, wv, wo, cos, sin, sh, tp, reduce=True):
    """h2 [T,H] -> (a [T,H], saved).  Row-parallel out_proj: a = sum over tp of o W_o^T (reduce=False:
    this rank's partial, for the sequence-parallel reduce-scatter)."""
    scale = 1.0 / math.sqrt(sh.d)
    if _fuse() and K.rope_fusable(h2.shape[0], sh.d, sh.S, (wq.shape[0], wk.shape[0], wv.shape[0])):   # RoPE of q|k in the projection's epilogue
        qkv = K.linear_fwd_rope(h2, [wq, wk, wv], cos, sin, sh.S, sh.nh + sh.nkv, sh.d)
        o, lse = attention_core_fwd(qkv, sh, cos, sin, scale, roped=True)
    else:
        qkv = K.linear_fwd(h2, [wq, wk, wv])
        o, lse = attention_core_fwd(qkv, sh, cos, sin, scale)
    a = K.linear_fwd(o.view(sh.T, sh.wq), [wo])
    if reduce:
        tp.all_reduce(a)
    return a, (qkv, o, lse)


def _dual_qkv_enabled():
    return SW.dual_qkv != 0


def attn_block_bwd(da, h2, saved, wq, wk, wv, wo, cos, sin, sh, tp, need_dx=True, keep_parts=False, sp=False,
                   rs_out=None, notify=True):
    """keep_parts: the q|k|v dX may come back as K.SplitKParts (two f32 K halves) for a following
    rmsnorm backward to sum.  sp: the column-parallel dX is reduce-scattered onto this rank's token
    rows (sequence parallelism) instead of all-reduced.  rs_out: one token chunk of the chunked
    sequence-parallel layer -- the dX reduce-scatter writes rs_out and is NOT waited for: its handle
    is returned (the next chunk's work runs under it); notify=False: this chunk's weight gradients
    are partial sums (wgrad)."""
    qkv, o, lse = saved
    scale = 1.0 / math.sqrt(sh.d)
    do2 = K.linear_dgrad(da, [wo])
    dqkv = attention_core_bwd(do2.view(sh.B, sh.S, sh.nh, sh.d), qkv, o, lse, sh, cos, sin, scale)
    if need_dx and tp.world_size == 1 and _dual_qkv_enabled():
        # tp = 1 (no all-reduce to overlap): the q|k|v dX as two split-K halves (128 + 128 tiles of
        # 256x256, summed by the input norm's backward -- or by the sum pass without keep_parts) in
        # ONE launch with the q|k|v and o_proj dW (192 + 64 tiles): 512 tiles = 2 whole rounds of the
        # 256 CUs instead of a 128-tile dX launch and a 256-tile dW launch
        return dgrad_with_wgrad(dqkv, [wq, wk, wv], [(dqkv, h2, [wq, wk, wv]), (da, o.view(sh.T, sh.wq), [wo])],
                                keep_parts=keep_parts, split_min=1024)
    dh = handle = None
    if need_dx:
        dh = K.linear_dgrad(dqkv, [wq, wk, wv])
        if rs_out is not None:
            handle = tp.reduce_scatter_rows_into(rs_out, dh, async_op=True)
        elif sp:
            dh, handle = tp.reduce_scatter_rows(dh, async_op=True)
        else:
            handle = tp.all_reduce(dh, async_op=True)
    # dW of q|k|v and of o_proj in one launch: 192 + 64 tiles of 256x256 at SmolLM-1.7B dims,
    # where either alone leaves CUs idle (o_proj's wgrad was deferred from above; its inputs
    # da and o stay alive until here anyway)
    wgrad_group([(dqkv, h2, [wq, wk, wv]), (da, o.view(sh.T, sh.wq), [wo])], notify)
    if rs_out is not None:
        return handle
    if handle is not None:
        handle.wait()
    return dh


class AttentionFunction(torch.autograd.Function):
    """Attention.forward (model.py:122-162) as one node: fused q|k|v GEMM, in-place RoPE, flash
    attention, out_proj, with the Column/Row TP reductions."""

    @staticmethod
    def forward(ctx, x, wq, wk, wv, wo, cos, sin, nh, nkv, d):
        B, S, _ = x.shape
        sh = AttnShape(B, S, nh, nkv, d)
        h2 = _contig2d(x)
        a, saved = attn_block_fwd(h2, wq, wk, wv, wo, cos, sin, sh, TPContext.current())
        ctx.save_for_backward(h2, *saved, wq, wk, wv, wo, cos, sin)
        ctx.sh = sh
        return a.view(B, S, -1)

    @staticmethod
    def backward(ctx, da):
        h2, qkv, o, lse, wq, wk, wv, wo, cos, sin = ctx.saved_tensors
        sh = ctx.sh
        dh = attn_block_bwd(_contig2d(da), h2, (qkv, o, lse), wq, wk, wv, wo, cos, sin, sh, TPContext.current(),
                            need_dx=ctx.needs_input_grad[0])
        return (dh.view(sh.B, sh.S, -1) if dh is not None else None,) + (None,) * 9


# ------------------------------------------------------------------------ MLP block
def mlp_block_fwd(h2, wg, wu, wd, tp, residual=None, reduce=True):
    """h2 [T,H] -> down(silu(gate) * up) (+ residual, entering the tp sum once, from tp rank 0;
    reduce=False: this rank's partial, no residual, for the sequence-parallel reduce-scatter)."""
    I = wg.shape[0]
    if _fuse() and K.swiglu_fuse_pays(h2.shape[0], I, H=h2.shape[1]):   # SwiGLU in the gate|up GEMM's epilogue
        gu, hh = K.linear_swiglu_fwd(h2, wg, wu)
    else:
        gu = K.linear_fwd(h2, [wg, wu])
        hh = K.swiglu_fwd(gu[:, :I], gu[:, I:])
    res = residual if (residual is not None and tp.rank == 0) else None
    m = K.linear_fwd(hh, [wd], residual=res)
    if reduce:
        tp.all_reduce(m)
    return m, (gu, hh)


def _dual_gu_enabled():
    return SW.dual_gu != 0


# the gate|up dX + dW dual launch's XCD order: 1 = every XCD its dW tiles first (+0.3 % on the step
# over the staggered order the other dual launches keep; profiles/r04/ab_gu_order, five rounds)
GU_DUAL_ORDER = 1


def mlp_block_bwd(dm, h2, saved, wg, wu, wd, tp, need_dx=True, keep_parts=False, sp=False, rs_out=None,
                  notify=True):
    """keep_parts: the gate|up dX may come back as K.SplitKParts (its split-K halves unsummed) for a
    following rmsnorm backward to sum.  sp: the column-parallel dX is reduce-scattered onto this
    rank's token rows instead of all-reduced.  rs_out / notify: one token chunk of the chunked
    sequence-parallel layer (attn_block_bwd): returns the reduce-scatter's handle, not waited for."""
    gu, hh = saved
    I = wg.shape[0]
    if _fuse() and K.swiglu_fuse_pays(dm.shape[0], I, backward=True, H=dm.shape[1]):   # SwiGLU bwd in the down dX epilogue
        # ... in one launch with the down_proj dW: the epilogue's HBM-bound g|u / dg|du tail
        # overlaps the dW's MFMA work (K.linear_dgrad_dual)
        dgu = dgrad_with_wgrad(dm, [wd], [(dm, hh, [wd])], gu=gu, notify=notify)
    else:
        dhh = K.linear_dgrad(dm, [wd])
        dgu = torch.empty_like(gu)
        K.swiglu_bwd(dhh, gu[:, :I], gu[:, I:], dg=dgu[:, :I], du=dgu[:, I:])
        wgrad(dm, hh, [wd], notify)
    dh = handle = None
    split = SW.gu_splitk != 0
    if need_dx and tp.world_size == 1 and _dual_gu_enabled() and \
            (not split or K._splitk_halves(dgu.shape[0], h2.shape[1], dgu.shape[1]) is not None):
        # the gate|up dX and dW (512 tiles) in one dual launch (no TP all-reduce to overlap at
        # tp = 1): the dX as two split-K f32 halves (256 tiles: 3 whole rounds of the 256 CUs), or
        # (gu_splitk = 0) unsplit -- 128 tiles twice as long as a dW tile, beside which the other
        # CUs run four dW tiles each, and a bf16 dX for the norm backward to read.  XCD order 1
        # (every XCD its dW tiles first, GU_DUAL_ORDER): +0.3 % on the step over the staggered order
        # the down_proj dual keeps (profiles/r04/ab_gu_order, five interleaved rounds)
        return dgrad_with_wgrad(dgu, [wg, wu], [(dgu, h2, [wg, wu])], keep_parts=keep_parts,
                                split_min=None if split else 1 << 30, order=GU_DUAL_ORDER)
    if need_dx:
        dh = K.linear_dgrad(dgu, [wg, wu])
        if rs_out is not None:
            handle = tp.reduce_scatter_rows_into(rs_out, dh, async_op=True)
        elif sp:
            dh, handle = tp.reduce_scatter_rows(dh, async_op=True)
        else:
            handle = tp.all_reduce(dh, async_op=True)
    wgrad(dgu, h2, [wg, wu], notify)
    if rs_out is not None:
        return handle
    if handle is not None:
        handle.wait()
    return dh


class MLPFunction(torch.autograd.Function):
    """MLP.forward (model.py:184-186): gate|up in one GEMM, SwiGLU, down_proj."""

    @staticmethod
    def forward(ctx, x, wg, wu, wd):
        h2 = _contig2d(x)
        m, saved = mlp_block_fwd(h2, wg, wu, wd, TPContext.current())
        ctx.save_for_backward(h2, *saved, wg, wu, wd)
        ctx.shape = x.shape
        return m.view(*x.shape[:-1], -1)

    @staticmethod
    def backward(ctx, dm):
        h2, gu, hh, wg, wu, wd = ctx.saved_tensors
        dh = mlp_block_bwd(_contig2d(dm), h2, (gu, hh), wg, wu, wd, TPContext.current(),
                           need_dx=ctx.needs_input_grad[0])
        return (dh.view(ctx.shape) if dh is not None else None), None, None, None


# ------------------------------------------------------------------------ decoder layer
class DecoderLayerFunction(torch.autograd.Function):
    """DecoderLayer.forward (model.py:204-209) as one autograd node:

        h1 = norm1(x);  a = Attn(h1);  z = x + a  (fused into norm2);  h2 = norm2(z)
        out = z + MLP(h2)                  (residual fused into the down_proj epilogue)

    Backward runs the same kernels in reverse; the residual gradients are fused into the norm
    backward kernels (dres) and the TP dX all-reduces overlap the dW GEMMs.  zz: x is a zig-zag CP
    shard (cos / sin its positions' tables): the ring runs on it with no re-lay."""

    @staticmethod
    def forward(ctx, x, w1, w2, wq, wk, wv, wo, wg, wu, wd, cos, sin, eps, mode, nh, nkv, d, zz=False, sp=0):
        if sp:   # sp = the chunk count of the sequence-parallel layout (0: the replicated stream)
            return DecoderLayerFunction._forward_sp(ctx, x, w1, w2, wq, wk, wv, wo, wg, wu, wd, cos, sin, eps, mode,
                                                    nh, nkv, d, int(sp))
        ctx.sp = False
        B, S, H = x.shape
        sh = AttnShape(B, S, nh, nkv, d, zz)
        tp = TPContext.current()
        x2 = _contig2d(x)
        h1, rstd1, _ = K.rmsnorm_fwd(x2, w1, eps, mode)
        a, asaved = attn_block_fwd(h1, wq, wk, wv, wo, cos, sin, sh, tp)
        h2, rstd2, z = K.rmsnorm_fwd(a, w2, eps, mode, residual=x2)
        out, msaved = mlp_block_fwd(h2, wg, wu, wd, tp, residual=z)
        ctx.save_for_backward(x2, h1, rstd1, *asaved, z, h2, rstd2, *msaved,
                              w1, w2, wq, wk, wv, wo, wg, wu, wd, cos, sin)
        ctx.sh, ctx.mode = sh, mode
        return out.view(B, S, H)

    @staticmethod
    def _forward_sp(ctx, x, w1, w2, wq, wk, wv, wo, wg, wu, wd, cos, sin, eps, mode, nh, nkv, d, c):
        """Sequence-parallel TP layer (tensor_parallel/sequence_parallel.py): x is this rank's shard
        of the residual stream in the chunked token-row layout (TPContext.gather_chunk: c chunks of
        B / c whole sequences; rank r holds rows [r n, (r + 1) n) of each), viewed [B, S/tp, H].  The
        norms and residual adds run on the shard; the column-parallel inputs are all-gathered (the
        reference's replicated norm output), the row-parallel outputs reduce-scattered onto the shards
        (the reference's all-reduce, keeping this rank's rows):

            h1 = AG(norm1(x));  a = RS(attn(h1));  z = x + a (fused into norm2);  h2 = AG(norm2(z))
            out = z + RS(mlp(h2))

        chunk by chunk: every chunk's all-gather is issued at once (RCCL runs them in order on its
        stream), chunk j's block waits only for chunk j's rows, and its reduce-scatter is issued as
        soon as its GEMM is done -- so chunk j + 1's all-gather runs under chunk j's GEMMs and
        attention, chunk j's reduce-scatter under chunk j + 1's (tp_communications.py:35-49 moves the
        same bytes with nothing beside them).  The same values as the reference's layer
        (model.py:204-209), row by row; per rank the norms / adds touch T/tp rows instead of T."""
        tp = TPContext.current()
        B, Sl, H = x.shape
        W = tp.world_size
        S = Sl * W
        Tc = B // c * S                                # gathered rows per chunk
        sh = AttnShape(B // c, S, nh, nkv, d)
        x2 = _contig2d(x)
        h1r, rstd1, _ = K.rmsnorm_fwd(x2, w1, eps, mode)
        h1 = torch.empty(B * S, H, dtype=x2.dtype, device=x2.device)
        ag = [tp.gather_chunk(h1, h1r, c, j, async_op=True) for j in range(c)]
        ar = torch.empty_like(x2)
        asaved, rs = [], []
        for j in range(c):
            wait_all(ag[j:j + 1])
            a, sv = attn_block_fwd(h1[j * Tc:(j + 1) * Tc], wq, wk, wv, wo, cos, sin, sh, tp, reduce=False)
            asaved += list(sv)
            rs.append(tp.scatter_chunk(ar, a, c, j, async_op=True))
        wait_all(rs)
        h2r, rstd2, z = K.rmsnorm_fwd(ar, w2, eps, mode, residual=x2)
        h2 = torch.empty_like(h1)
        ag = [tp.gather_chunk(h2, h2r, c, j, async_op=True) for j in range(c)]
        mr = torch.empty_like(x2)
        msaved, rs = [], []
        for j in range(c):
            wait_all(ag[j:j + 1])
            m, sv = mlp_block_fwd(h2[j * Tc:(j + 1) * Tc], wg, wu, wd, tp, reduce=False)
            msaved += list(sv)
            rs.append(tp.scatter_chunk(mr, m, c, j, async_op=True))
        wait_all(rs)
        out = K.residual_add(z, mr)
        ctx.save_for_backward(x2, h1, rstd1, z, h2, rstd2, w1, w2, wq, wk, wv, wo, wg, wu, wd, cos, sin,
                              *asaved, *msaved)
        ctx.sh, ctx.mode, ctx.sp, ctx.c = sh, mode, True, c
        return out.view(B, Sl, H)

    @staticmethod
    def _backward_sp(ctx, dout):
        x2, h1, rstd1, z, h2, rstd2, w1, w2, wq, wk, wv, wo, wg, wu, wd, cos, sin, *rest = ctx.saved_tensors
        sh, mode, c = ctx.sh, ctx.mode, ctx.c
        asaved, msaved = rest[:3 * c], rest[3 * c:]
        tp = TPContext.current()
        Tc = sh.T
        dout2 = _contig2d(dout)                       # [T/tp, H]: the residual's gradient rows
        # the row-parallel down_proj sees every row: chunk j's rows gathered while chunk j - 1's MLP
        # backward runs; chunk j's dX reduce-scatter runs under chunk j + 1's
        dm = torch.empty_like(h2)
        ag = [tp.gather_chunk(dm, dout2, c, j, async_op=True) for j in range(c)]
        dh2 = torch.empty_like(dout2)
        rs = []
        for j in range(c):
            wait_all(ag[j:j + 1])
            rows = slice(j * Tc, (j + 1) * Tc)
            n = dout2.shape[0] // c
            rs.append(mlp_block_bwd(dm[rows], h2[rows], msaved[2 * j:2 * j + 2], wg, wu, wd, tp,
                                    rs_out=dh2[j * n:(j + 1) * n], notify=j == c - 1))
        wait_all(rs)
        dz = norm_bwd(dh2, z, w2, rstd2, mode, dres=dout2, sp=tp)
        da = torch.empty_like(h1)
        ag = [tp.gather_chunk(da, dz, c, j, async_op=True) for j in range(c)]
        dh1 = torch.empty_like(dout2)
        rs = []
        for j in range(c):
            wait_all(ag[j:j + 1])
            rows = slice(j * Tc, (j + 1) * Tc)
            n = dout2.shape[0] // c
            rs.append(attn_block_bwd(da[rows], h1[rows], asaved[3 * j:3 * j + 3], wq, wk, wv, wo, cos, sin, sh, tp,
                                     rs_out=dh1[j * n:(j + 1) * n], notify=j == c - 1))
        wait_all(rs)
        dx = norm_bwd(dh1, x2, w1, rstd1, mode, dres=dz, sp=tp)
        return (dx.view(dout.shape),) + (None,) * 18

    @staticmethod
    def backward(ctx, dout):
        if ctx.sp:
            return DecoderLayerFunction._backward_sp(ctx, dout)
        (x2, h1, rstd1, qkv, o, lse, z, h2, rstd2, gu, hh,
         w1, w2, wq, wk, wv, wo, wg, wu, wd, cos, sin) = ctx.saved_tensors
        sh, mode = ctx.sh, ctx.mode
        tp = TPContext.current()
        dout2 = _contig2d(dout)
        # the gate|up dX's split-K halves go straight into the norm backward (summed there)
        dh2 = mlp_block_bwd(dout2, h2, (gu, hh), wg, wu, wd, tp, keep_parts=K.norm_splitk_enabled())
        dz = norm_bwd(dh2, z, w2, rstd2, mode, dres=dout2)
        dh1 = attn_block_bwd(dz, h1, (qkv, o, lse), wq, wk, wv, wo, cos, sin, sh, tp, keep_parts=K.norm_splitk_enabled())
        dx = norm_bwd(dh1, x2, w1, rstd1, mode, dres=dz)   # (norm_bwd skips dW of frozen weights)
        return (dx.view(sh.B, sh.S, -1),) + (None,) * 18


# ------------------------------------------------------------------------ cross entropy
class EmbeddingFunction(torch.autograd.Function):
    """F.embedding (model.py:224-225) / VocabParallelEmbedding's masked lookup
    (tensor_parallel.py:246-270) with the backward written straight into the table's gradient sink:
    only the rows the micro-batch touches are read / written (csrc/embedding.hip)."""

    @staticmethod
    def forward(ctx, ids, weight, vocab_lo, vocab_hi, padding_idx):
        ctx.save_for_backward(ids)
        ctx.weight, ctx.lo, ctx.hi, ctx.pad = weight, vocab_lo, vocab_hi, padding_idx
        return K.embedding_fwd(ids, weight, vocab_lo, vocab_hi)

    @staticmethod
    def backward(ctx, dy):
        (ids,) = ctx.saved_tensors
        weight = ctx.weight
        if not weight.requires_grad:
            return None, None, None, None, None
        mg = getattr(weight, "main_grad", None)
        if mg is not None:
            buf, sink = mg, (K.DW_ACC_F32 if mg.dtype == torch.float32 else K.DW_ACC_BF16)
        else:
            if weight.grad is None:   # untouched rows of a fresh gradient are zero, as autograd's
                weight.grad = torch.zeros_like(weight)
            buf, sink = weight.grad, K.DW_ACC_BF16
        K.embedding_bwd(ids, _contig2d(dy), buf, sink, ctx.lo, ctx.hi, ctx.pad)
        _grad_ready(weight)
        return None, None, None, None, None


def embedding(ids, weight, vocab_lo=0, vocab_hi=None, padding_idx=None):
    hi = vocab_lo + weight.shape[0] if vocab_hi is None else vocab_hi
    return EmbeddingFunction.apply(ids, weight, vocab_lo, hi, padding_idx)


class CrossEntropyFunction(torch.autograd.Function):
    """F.cross_entropy(logits [N, V], targets [N]) as called at train.py:49 (reduction='mean'; 'sum'
    and 'none' for other consumers of the logits).  Forward streams the logits once for the per-row
    loss and LSE (saved, 16 KiB at 4096 rows) -- or takes both from the lm_head GEMM's statistics;
    backward writes (exp(x - lse) - onehot) * scale elementwise in one more read + write, with the
    scale (the incoming gradient, the reference's `/ grad_acc_steps`, times 1 / #valid for 'mean';
    per row for 'none') taken from device memory -- no host synchronisation."""

    @staticmethod
    def forward(ctx, logits, targets, ignore_index, reduction):
        lg = _contig2d(logits)
        tg = targets.reshape(-1)
        stats = _take_ce_stats(lg)   # the lm_head GEMM's statistics of exactly these logits, if any
        V = lg.shape[1]
        if V % 8:
            # the CE kernels stream 16-byte row chunks: a vocabulary off the 8-column grid (50257,
            # 32001) is padded with -inf columns -- exp(-inf - max) = 0 adds nothing to any row's sum;
            # their gradient columns are sliced off in the backward
            lgp = torch.full((lg.shape[0], (V + 7) // 8 * 8), float("-inf"), dtype=lg.dtype, device=lg.device)
            lgp[:, :V] = lg
            lg, stats = lgp, None
        ctx.vocab = V
        odt = logits.dtype if logits.dtype in (torch.bfloat16, torch.float32) else torch.float32
        if stats is not None:
            loss, inv_count, row_lse = K.cross_entropy_loss_lse_stats(lg, tg, stats, ignore_index, out_dtype=odt,
                                                                      reduction=reduction)
        else:
            loss, inv_count, row_lse = K.cross_entropy_loss_lse(lg, tg, ignore_index, out_dtype=odt,
                                                                reduction=reduction)
        ctx.save_for_backward(lg, tg, row_lse, *([inv_count] if inv_count is not None else []))
        ctx.ignore_index, ctx.shape, ctx.reduction = ignore_index, logits.shape, reduction
        return loss if loss.dtype == logits.dtype else loss.to(logits.dtype)

    @staticmethod
    def backward(ctx, g):
        lg, tg, row_lse, *inv = ctx.saved_tensors
        if ctx.reduction == "none":
            scale = g.float().reshape(-1).contiguous()
        elif ctx.reduction == "sum":
            scale = g.float().reshape(1)
        else:
            scale = g.float().reshape(1) * inv[0]
        dl = K.cross_entropy_grad_lse(lg, tg, row_lse, scale, ctx.ignore_index)
        if dl.shape[1] != ctx.vocab:
            dl = dl[:, :ctx.vocab]
        return dl.reshape(ctx.shape), None, None, None


def _plain(t):
    if isinstance(t, HipLogits) and getattr(t, "_pt_vp", None) is not None:
        t = _vp_real(t)   # a vocab-parallel stand-in has no data of its own: the gathered logits
    return t.as_subclass(torch.Tensor) if isinstance(t, (HipLogits, HipHidden)) else t


class HipLogits(torch.Tensor):
    """The lm_head output (model.py:270): an ordinary tensor -- same storage, same autograd history
    (Tensor.as_subclass) -- whose F.cross_entropy runs the fused HIP cross-entropy.  So the
    reference's unchanged callers, `F.cross_entropy(outputs.view(-1, V), targets)` (train.py:49) and
    `F.cross_entropy(output.transpose(1, 2), target)` (pipeline_parallel.py:103,153), reach
    csrc/cross_entropy.hip without an edit.  View-like methods keep the type (the callers reshape
    first); every other op returns plain tensors."""

    _KEEP = frozenset([torch.Tensor.view, torch.Tensor.reshape, torch.Tensor.transpose, torch.Tensor.permute,
                       torch.Tensor.flatten, torch.Tensor.contiguous])

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if func is torch.nn.functional.cross_entropy:
            return _dispatch_cross_entropy(*args, **kwargs)
        if func is torch.Tensor.contiguous and args and _is_vp(args[0]):
            # the stand-in stays one: recorded on its path (replayed on a gather, if ever), nothing
            # allocated -- a real contiguous() of the expanded stand-in would write a [T, V] buffer
            t = args[0]
            return _standin(t._pt_vp, tuple(t.shape), t._pt_vp_path + ((func, tuple(args[1:]), dict(kwargs)),),
                            t.requires_grad)
        if args and _is_vp(args[0]) and (func in cls._KEEP or func in _VP_META or
                                         getattr(func, "__name__", "") == "__get__"):
            # a view of the vocab-parallel stand-in stays one (its path replayed on a gather, if ever);
            # shape / dtype / device reads need no data
            out = super().__torch_function__(func, types, args, kwargs)
            if func in cls._KEEP and isinstance(out, HipLogits):
                out._pt_vp = args[0]._pt_vp
                out._pt_vp_path = args[0]._pt_vp_path + ((func, tuple(args[1:]), dict(kwargs)),)
            return out
        if any(_is_vp(a) for a in args) or any(_is_vp(v) for v in kwargs.values()):
            args = tuple(_vp_real(a) if _is_vp(a) else a for a in args)
            kwargs = {k: (_vp_real(v) if _is_vp(v) else v) for k, v in kwargs.items()}
            return HipLogits.__torch_function__(func, types, args, kwargs)
        if func in cls._KEEP:
            return super().__torch_function__(func, types, args, kwargs)
        with torch._C.DisableTorchFunctionSubclass():
            return func(*args, **kwargs)


class HipHidden(torch.Tensor):
    """The final norm's output (model.py:269 `self.final_norm(x)`): an ordinary tensor whose
    F.linear -- the call torch's nn.Linear.forward makes -- runs the HIP lm_head GEMM (with the CE
    statistics epilogue) and returns HipLogits.  This keeps the lm_head and the cross-entropy on the
    HIP path under callers that hold a plain nn.Linear final_proj: the one checkpoint.py:89-90
    installs, called directly by PipelineParallel.forward (pipeline_parallel.py:62-63), whose
    output then meets F.cross_entropy at pipeline_parallel.py:103,153.  Every other op returns
    plain tensors."""

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if func is torch.nn.functional.linear:
            return _dispatch_linear(*args, **kwargs)
        with torch._C.DisableTorchFunctionSubclass():
            return func(*args, **kwargs)


def _dispatch_linear(input, weight, bias=None):
    x, weight = _plain(input), _plain(weight)
    y = lm_head_linear(x, weight) if bias is None else linear(x, weight) + bias
    return as_logits(y)


def as_hidden(t):
    """Tag the final norm's output so an nn.Linear lm_head on it takes the HIP GEMM."""
    return t.as_subclass(HipHidden)


def _dispatch_cross_entropy(input, target, weight=None, size_average=None, ignore_index=-100, reduce=None,
                            reduction="mean", label_smoothing=0.0):
    if weight is not None or size_average is not None or reduce is not None or label_smoothing != 0.0 or \
            reduction not in ("mean", "sum", "none"):
        # not on picotron's path (train.py:49 / pipeline_parallel.py:103,153 call the plain form): class
        # weights, label smoothing and the legacy reduction flags are torch's own op on the same tensors
        if _is_vp(input):
            input = _vp_real(input)
        return torch.nn.functional.cross_entropy(_plain(input), _plain(target), weight=weight,
                                                 size_average=size_average, ignore_index=ignore_index,
                                                 reduce=reduce, reduction=reduction,
                                                 label_smoothing=label_smoothing)
    if _is_vp(input):   # the TP lm_head's stand-in (vp_logits)
        out = _vp_cross_entropy(input, target, reduction, ignore_index)
        if out is not None:
            return out
    return cross_entropy(_plain(input), _plain(target), reduction=reduction, ignore_index=ignore_index)


def as_logits(t):
    """Tag an lm_head output so F.cross_entropy on it (or on its views) takes the HIP kernel.
    (Tensor.as_subclass is not dispatched to __torch_function__: a HipLogits -- a vocab-parallel
    stand-in among them -- is returned as it is.)"""
    return t if isinstance(t, HipLogits) else t.as_subclass(HipLogits)


def cross_entropy(input, target, reduction="mean", ignore_index=-100):
    """Drop-in for F.cross_entropy(input, target, reduction=..., ignore_index=...) at the reference's
    two call sites (reduction='mean'):
      * train.py:49                     input [N, V], target [N];
      * pipeline_parallel.py:103,153    input = output.transpose(1, 2), i.e. [B, V, S] with the class
        dim 1 (a view of the [B, S, V] stage output), target [B, S].
    The [B, V, S] form is read as the [B*S, V] rows it views (no copy when the underlying [B, S, V]
    is contiguous); the gradient flows back through the same views.  reduction 'sum' and 'none'
    (per-row losses shaped like target, 0 at ignored rows) follow torch."""
    if reduction not in ("mean", "sum", "none"):
        raise ValueError(f"cross_entropy: reduction must be 'mean', 'sum' or 'none', got {reduction!r}")
    if _is_vp(input):   # the TP lm_head's stand-in: on the vocab shards, else on the gathered logits
        out = _vp_cross_entropy(input, target, reduction, ignore_index)
        if out is not None:
            return out
        input = _vp_real(input)
    input, target = _plain(input), _plain(target)
    if input.dim() == 3:
        B, V, S = input.shape
        if tuple(target.shape) != (B, S):
            raise ValueError(f"cross_entropy: input [B, V, S] = {tuple(input.shape)} needs target [B, S], got "
                             f"{tuple(target.shape)}")
        rows = input.transpose(1, 2).reshape(B * S, V)
        out = CrossEntropyFunction.apply(rows, target.reshape(-1), ignore_index, reduction)
        return out.view(B, S) if reduction == "none" else out
    if input.dim() != 2 or target.dim() != 1 or target.shape[0] != input.shape[0]:
        raise ValueError(f"cross_entropy: expected input [N, V] and target [N] (or [B, V, S] / [B, S]), got "
                         f"{tuple(input.shape)} / {tuple(target.shape)}")
    return CrossEntropyFunction.apply(input, target, ignore_index, reduction)
