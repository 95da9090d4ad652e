"""Tensor-level wrappers over the C ABI: validation, output allocation (by torch's caching
allocator -- kernels never allocate) and launch on torch's current stream.

Every function here runs the gfx950 kernels and nothing else; there is no CPU or eager
fallback.  Shapes/dtypes/strides are validated in Python before the call, as the reference
validates with asserts (e.g. picotron/model.py:95-96, tensor_parallel.py:81,151,226).
"""
import ctypes
import math

import sys

import torch

from . import _C
from .switches import S as SW

BF16 = torch.bfloat16


def _ptr(t):
    return None if t is None else t.data_ptr()


def _req(cond, msg):
    if not cond:
        raise ValueError(msg)


def _bf16_rowmajor(t, name):
    if isinstance(t, KPair):
        _bf16_rowmajor(t.a, name)
        _bf16_rowmajor(t.b, name)
        return
    _req(t.dtype == BF16, f"{name}: expected bfloat16, got {t.dtype}")
    _req(t.is_cuda, f"{name}: expected a device tensor")
    _req(t.dim() == 2 and t.stride(1) == 1, f"{name}: expected a 2-D row-major view")


# --------------------------------------------------------------------------------- RMSNorm
MODE_TRITON = 0   # flash-attn layer_norm_fn(is_rms_norm=True): bf16(x * rstd * w)
MODE_LLAMA = 1    # LlamaRMSNorm: w * bf16(x * rstd)


def rmsnorm_fwd(x, weight, eps, mode=MODE_TRITON, residual=None):
    """x [rows, cols] bf16 contiguous.  Returns (y, rstd, z) where z = bf16(x + residual) (or None)."""
    _bf16_rowmajor(x, "x")
    x = x.contiguous()
    rows, cols = x.shape
    lib = _C.lib()
    y = torch.empty_like(x)
    rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
    z = None
    if residual is not None:
        residual = residual.contiguous()
        _req(residual.shape == x.shape and residual.dtype == BF16, "residual shape/dtype")
        z = torch.empty_like(x)
    rc = lib.pt_rmsnorm_fwd(_ptr(x), _ptr(residual), _ptr(weight), _ptr(y), _ptr(z), _ptr(rstd), rows, cols,
                            float(eps), int(mode), _C.stream_ptr(x.device))
    _C.check(rc, "pt_rmsnorm_fwd")
    return y, rstd, z


DW_ACC_BF16, DW_ACC_F32 = 4, 8   # pt_rmsnorm_bwd dweight sinks (include/picotron_hip.h)


class SplitKParts:
    """A split-K dX GEMM's result before its sum pass: two f32 K halves [rows, cols] whose
    bf16(p0 + p1) is the dX (linear_dgrad_dual(keep_parts=True)).  rmsnorm_bwd takes it as its dy
    and sums in the norm kernel; anything else calls .sum() for the bf16 tensor."""

    def __init__(self, p0, p1):
        self.p0, self.p1 = p0, p1
        self.shape, self.device = p0.shape, p0.device

    def sum(self):
        out = torch.empty(self.shape, dtype=BF16, device=self.device)
        rc = _C.lib().pt_gemm_splitk_sum(_ptr(self.p0), _ptr(self.p1), None, _ptr(out), out.numel(),
                                         _C.stream_ptr(self.device))
        _C.check(rc, "pt_gemm_splitk_sum")
        return out


class KPair:
    """Two [T, n] row blocks a, b of one layout standing for their concatenation [2 T, n] along the
    token (K) dimension of a weight gradient: two micro-batches' dY (or X).  The wgrad launches take
    it as a K-segmented operand (pt_gemm_problem.A2 / b_seg_dim 1): dW = dY_a^T X_a + dY_b^T X_b in
    one K = 2 T GEMM (functional.pair_jobs).  Column slices stay pairs."""

    def __init__(self, a, b):
        _req(a.shape == b.shape and a.stride() == b.stride() and a.dtype == b.dtype and a.device == b.device,
             "KPair: two row blocks of one shape and layout")
        self.a, self.b = a, b
        self.shape = (2 * a.shape[0], a.shape[1])
        self.dtype, self.device = a.dtype, a.device

    def stride(self, i=None):
        return self.a.stride() if i is None else self.a.stride(i)

    def __getitem__(self, idx):
        return KPair(self.a[idx], self.b[idx])


def rmsnorm_bwd(dy, z, weight, rstd, mode=MODE_TRITON, dres=None, dw_out=None, dw_sink=0, defer_dw=False):
    """Returns (dx, dweight).  dres (same shape as dy) is added into dx when given.
    dw_out/dw_sink: write the weight gradient into an existing buffer -- 0 store (bf16),
    DW_ACC_BF16 accumulate into a bf16 .grad, DW_ACC_F32 accumulate into an f32 main_grad.
    defer_dw: no column sum; returns (dx, partial) -- the f32 per-block partial rows, to be summed
    into the sink later by rmsnorm_colsum_batch.  dy may be a SplitKParts (summed in the kernel)."""
    split = isinstance(dy, SplitKParts)
    if not split:
        dy = dy.contiguous()
    rows, cols = z.shape
    lib = _C.lib()
    nparts = lib.pt_rmsnorm_bwd_partials(rows, cols)
    _C.check(0 if nparts > 0 else nparts, "pt_rmsnorm_bwd_partials")
    partial = torch.empty(nparts, cols, dtype=torch.float32, device=z.device)
    dx = torch.empty_like(z)
    if defer_dw:
        dw_out, dw_sink = None, 0
    elif dw_out is None:
        dw_out, dw_sink = torch.empty(cols, dtype=BF16, device=z.device), 0
    if dw_out is not None:
        _req(dw_out.is_contiguous() and dw_out.numel() == cols, "dweight buffer must be contiguous [cols]")
        _req(dw_out.dtype == (torch.float32 if dw_sink == DW_ACC_F32 else BF16), "dweight buffer dtype")
    if dres is not None:
        dres = dres.contiguous()
    if split:
        _req(dy.p0.is_contiguous() and dy.p1.is_contiguous() and tuple(dy.shape) == (rows, cols), "split dy parts")
        rc = lib.pt_rmsnorm_bwd_splitk(_ptr(dy.p0), _ptr(dy.p1), _ptr(z), _ptr(weight), _ptr(rstd), _ptr(dres), _ptr(dx),
                                       _ptr(dw_out), _ptr(partial), rows, cols, int(mode) | int(dw_sink),
                                       _C.stream_ptr(z.device))
        _C.check(rc, "pt_rmsnorm_bwd_splitk")
    else:
        rc = lib.pt_rmsnorm_bwd(_ptr(dy), _ptr(z), _ptr(weight), _ptr(rstd), _ptr(dres), _ptr(dx), _ptr(dw_out),
                                _ptr(partial), rows, cols, int(mode) | int(dw_sink), _C.stream_ptr(z.device))
        _C.check(rc, "pt_rmsnorm_bwd")
    return dx, (partial if defer_dw else dw_out)


def rmsnorm_colsum_batch(jobs):
    """jobs: [(partial [nparts, cols] f32, dw_out, dw_sink)], all of one width, <= 32: the deferred
    weight-gradient sums of rmsnorm_bwd(defer_dw=True), one launch."""
    _req(0 < len(jobs) <= 32, "rmsnorm_colsum_batch: 1..32 jobs")
    cols = jobs[0][0].shape[1]
    for part, out, sink in jobs:
        _req(part.dtype == torch.float32 and part.is_contiguous() and part.shape[1] == cols, "partials [n, cols] f32")
        _req(out.is_contiguous() and out.numel() == cols, "dweight buffer must be contiguous [cols]")
        _req(out.dtype == (torch.float32 if sink == DW_ACC_F32 else BF16), "dweight buffer dtype")
    rc = _C.lib().pt_rmsnorm_colsum_batch(_C.ptrarr([_ptr(p) for p, _, _ in jobs]),
                                          _C.i32arr([p.shape[0] for p, _, _ in jobs]),
                                          _C.ptrarr([_ptr(o) for _, o, _ in jobs]),
                                          _C.i32arr([s for _, _, s in jobs]), len(jobs), cols,
                                          _C.stream_ptr(jobs[0][0].device))
    _C.check(rc, "pt_rmsnorm_colsum_batch")


# ------------------------------------------------------------------------------- embedding
def embedding_fwd(ids, weight, vocab_lo=0, vocab_hi=None):
    """out[t] = weight[ids[t] - vocab_lo] (zero rows for ids outside [vocab_lo, vocab_hi))."""
    _req(weight.dtype == BF16 and weight.stride(1) == 1, "embedding table: bf16 rows")
    vocab_hi = vocab_lo + weight.shape[0] if vocab_hi is None else vocab_hi
    flat = ids.reshape(-1).contiguous().to(torch.int64)
    H = weight.shape[1]
    out = torch.empty(flat.numel(), H, dtype=BF16, device=weight.device)
    rc = _C.lib().pt_embedding_fwd(_ptr(flat), flat.numel(), _ptr(weight), weight.stride(0), int(vocab_lo),
                                   int(vocab_hi), _ptr(out), out.stride(0), H, _C.stream_ptr(weight.device))
    _C.check(rc, "pt_embedding_fwd")
    return out.view(*ids.shape, H)


def embedding_bwd(ids, dy2d, dweight, sink, vocab_lo=0, vocab_hi=None, padding_idx=None):
    """Sum the dY rows of every id into dweight (sink: 0 / DW_ACC_BF16 / DW_ACC_F32); ids outside
    [vocab_lo, vocab_hi) and padding_idx contribute nothing (F.embedding's backward)."""
    _bf16_rowmajor(dy2d, "dy")
    flat = ids.reshape(-1).to(torch.int64).contiguous()
    vocab_hi = vocab_lo + dweight.shape[0] if vocab_hi is None else vocab_hi
    T = flat.numel()
    sorted_ids = torch.empty(T, dtype=torch.int64, device=flat.device)
    perm = torch.empty(T, dtype=torch.int64, device=flat.device)
    rc = _C.lib().pt_embedding_sort(_ptr(flat), T, int(vocab_lo), int(vocab_hi), int(padding_idx is not None),
                                    int(padding_idx if padding_idx is not None else 0), _ptr(sorted_ids), _ptr(perm),
                                    _C.stream_ptr(flat.device))
    if rc == -3:   # more tokens than the one-workgroup sort holds: torch's (stable) device sort
        skip = (flat < vocab_lo) | (flat >= vocab_hi)
        if padding_idx is not None:
            skip = skip | (flat == padding_idx)
        sorted_ids, perm = torch.sort(torch.where(skip, torch.full_like(flat, -1), flat), stable=True)
    else:
        _C.check(rc, "pt_embedding_sort")
    rc = _C.lib().pt_embedding_bwd(_ptr(sorted_ids), _ptr(perm), flat.numel(), _ptr(dy2d), dy2d.stride(0),
                                   int(vocab_lo), _ptr(dweight), dweight.stride(0), dy2d.shape[1], int(sink),
                                   _C.stream_ptr(dy2d.device))
    _C.check(rc, "pt_embedding_bwd")


# ----------------------------------------------------------------------------------- AdamW
def adamw_step(p, grad, exp_avg, exp_avg_sq, decay, w1, beta2, c2, bc2_sqrt, eps, step_size):
    """One fused AdamW update of tensor p in place (csrc/adamw.hip; torch foreach semantics)."""
    for t, nm in ((grad, "grad"), (exp_avg, "exp_avg"), (exp_avg_sq, "exp_avg_sq")):
        _req(t.dtype == p.dtype and t.numel() == p.numel() and t.device == p.device, f"adamw: {nm} must match param")
        _req(t.is_contiguous() or t.stride() == p.stride(), f"adamw: {nm} layout must match param")
    _req(p.is_contiguous(), "adamw: param must be contiguous")
    _req(grad.is_contiguous() and exp_avg.is_contiguous() and exp_avg_sq.is_contiguous(), "adamw: dense tensors")
    if p.dtype == BF16:
        dt = 0
    elif p.dtype == torch.float32:
        dt = 1
    else:
        raise _C.HipKernelError(f"adamw: unsupported dtype {p.dtype}")
    rc = _C.lib().pt_adamw_step(_ptr(p), _ptr(grad), _ptr(exp_avg), _ptr(exp_avg_sq), p.numel(), dt, float(decay),
                                float(w1), float(beta2), float(c2), float(bc2_sqrt), float(eps), float(step_size),
                                _C.stream_ptr(p.device))
    _C.check(rc, "pt_adamw_step")


_ADAM_DESC = {}


def adamw_step_multi(items, decay, w1, beta2, c2, bc2_sqrt, eps, step_size):
    """One launch of the fused AdamW update over a list of bf16 (param, grad, exp_avg, exp_avg_sq)
    tuples (pt_adamw_step_multi).  The device descriptor table is cached per pointer set (the
    tensors of a model stay put across steps; a re-allocated gradient makes a new table).  A new
    table is staged in pinned host memory and copied on the current stream without a host sync
    (the caching host allocator keeps the staging buffer alive until that copy has run)."""
    for p, g, m, v in items:
        for t in (p, g, m, v):
            _req(t.dtype == BF16 and t.is_contiguous() and t.numel() == p.numel() and t.data_ptr() % 16 == 0,
                 "adamw multi: contiguous, 16-byte aligned bf16 tensors of one length per parameter")
    key = tuple((p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel()) for p, g, m, v in items)
    ent = _ADAM_DESC.get(key)
    if ent is None:
        dev = items[0][0].device
        chunks = [0]
        for k in key:
            chunks.append(chunks[-1] + (k[4] + 7) // 8)
        desc_h = torch.tensor([list(k) for k in key], dtype=torch.int64).pin_memory()
        chunk_h = torch.tensor(chunks, dtype=torch.int64).pin_memory()
        ent = (desc_h.to(dev, non_blocking=True), chunk_h.to(dev, non_blocking=True), chunks[-1])
        if len(_ADAM_DESC) > 64:
            _ADAM_DESC.clear()
        _ADAM_DESC[key] = ent
    desc, chunk_t, total = ent
    rc = _C.lib().pt_adamw_step_multi(_ptr(desc), _ptr(chunk_t), len(items), int(total), float(decay), float(w1),
                                      float(beta2), float(c2), float(bc2_sqrt), float(eps), float(step_size),
                                      _C.stream_ptr(items[0][0].device))
    _C.check(rc, "pt_adamw_step_multi")


# ------------------------------------------------------------------------------------ RoPE
def rope_(x2d, nheads, head_dim, cos, sin, seq_len, inverse=False):
    """In-place rotate the first `nheads` heads of every row of x2d ([rows, row_stride] view)."""
    _req(x2d.dtype == BF16 and x2d.stride(-1) == 1, "rope: bf16 row-major view expected")
    _req(cos.dtype == BF16 and sin.dtype == BF16 and cos.stride(-1) == 1, "rope: bf16 cos/sin tables")
    _req(cos.shape[0] >= seq_len, "rope: table shorter than the sequence")
    rows = x2d.shape[0]
    rc = _C.lib().pt_rope(_ptr(x2d), rows, x2d.stride(0), nheads, head_dim, _ptr(cos), _ptr(sin), seq_len,
                          cos.stride(0), 1 if inverse else 0, _C.stream_ptr(x2d.device))
    _C.check(rc, "pt_rope")
    return x2d


# ---------------------------------------------------------------------------------- SwiGLU
def swiglu_fwd(g, u, out=None):
    rows, cols = g.shape
    h = out if out is not None else torch.empty(rows, cols, dtype=BF16, device=g.device)
    rc = _C.lib().pt_swiglu_fwd(_ptr(g), g.stride(0), _ptr(u), u.stride(0), _ptr(h), h.stride(0), rows, cols,
                                _C.stream_ptr(g.device))
    _C.check(rc, "pt_swiglu_fwd")
    return h


def swiglu_bwd(dh, g, u, dg=None, du=None):
    rows, cols = g.shape
    dh = dh if dh.stride(-1) == 1 else dh.contiguous()
    dg = dg if dg is not None else torch.empty(rows, cols, dtype=BF16, device=g.device)
    du = du if du is not None else torch.empty(rows, cols, dtype=BF16, device=g.device)
    rc = _C.lib().pt_swiglu_bwd(_ptr(dh), dh.stride(0), _ptr(g), g.stride(0), _ptr(u), u.stride(0), _ptr(dg),
                                dg.stride(0), _ptr(du), du.stride(0), rows, cols, _C.stream_ptr(g.device))
    _C.check(rc, "pt_swiglu_bwd")
    return dg, du


def residual_add(x, r):
    """bf16(x + r) of two contiguous bf16 tensors of one shape (model.py:208's residual add)."""
    _req(x.dtype == BF16 and r.dtype == BF16 and x.shape == r.shape and x.is_contiguous() and r.is_contiguous(),
         "residual_add: contiguous bf16 tensors of one shape")
    out = torch.empty_like(x)
    rc = _C.lib().pt_residual_add(_ptr(x), _ptr(r), _ptr(out), x.numel(), _C.stream_ptr(x.device))
    _C.check(rc, "pt_residual_add")
    return out


# ---------------------------------------------------------------------------- device status
STATUS_BAD_TARGET = 1   # PT_STATUS_BAD_TARGET (include/picotron_hip.h)
_STATUS = {}


def _dev_index(device):
    device = torch.device(device) if device is not None else torch.device("cuda")
    return device.index if device.index is not None else torch.cuda.current_device()


def status_word(device):
    """The per-device int32 status word data-validating kernels OR their error bits into."""
    _status_poll(device)   # an error an earlier launch posted raises before the next launch
    w = _STATUS.get(_dev_index(device))
    if w is None:
        w = torch.zeros(1, dtype=torch.int32, device=torch.device("cuda", _dev_index(device)))
        _STATUS[_dev_index(device)] = w
    return w


_STATUS_HOST = {}   # device index -> pinned int32 mirror of the status word (async D2H copies)


def _status_posted(device):
    """After a validating launch: copy the status word into its pinned host mirror on the same
    stream, without a host sync.  The next validating call reads the mirror (see _status_poll), so a
    bad target raises one call later even on the drop-in path, whose train.py never calls
    check_device_status -- as torch's own asynchronous device-side assert surfaces at a later op."""
    i = _dev_index(device)
    h = _STATUS_HOST.get(i)
    if h is None:
        h = _STATUS_HOST[i] = torch.zeros(1, dtype=torch.int32).pin_memory()
    h.copy_(status_word(device), non_blocking=True)


def _status_poll(device):
    """Raise if a copy that has already landed in the pinned mirror carries an error bit."""
    h = _STATUS_HOST.get(_dev_index(device))
    if h is not None and int(h[0]):
        check_device_status(device)


def device_status(device=None, reset=True):
    """Read (a host synchronisation) and optionally clear the status word of `device`."""
    w = _STATUS.get(_dev_index(device))
    if w is None:
        return 0
    v = int(w.item())
    if reset and v:
        w.zero_()
        h = _STATUS_HOST.get(_dev_index(device))
        if h is not None:
            h.zero_()   # every copy into it was enqueued before the item() sync above
    return v


def check_device_status(device=None):
    """Raise what torch's device-side asserts would have: called where the host synchronises anyway
    (train.train_step after the step's loss read) or by anyone after a suspicious NaN."""
    v = device_status(device)
    if v & STATUS_BAD_TARGET:
        raise _C.HipKernelError("cross_entropy: a target index is outside [0, vocab) and is not ignore_index "
                                "(torch: 'Assertion `t >= 0 && t < n_classes` failed'); its row loss and "
                                "gradient were set to NaN")
    if v:
        raise _C.HipKernelError(f"device status word {v:#x}")


# ---------------------------------------------------------------------------- cross entropy
def cross_entropy_fwd_bwd(logits, targets, scale=1.0, ignore_index=-100, inplace=True):
    """logits [rows, V] bf16, targets [rows] int64.  Returns (loss (f32 scalar tensor, mean over
    valid rows, *not* multiplied by scale), dlogits (aliases logits when inplace), inv_count)."""
    _bf16_rowmajor(logits, "logits")
    targets = targets.contiguous().to(torch.int64)
    rows, vocab = logits.shape
    valid = (targets != ignore_index)
    inv_count = (1.0 / valid.sum().clamp_min(1).to(torch.float32)).reshape(1)
    row_loss = torch.empty(rows, dtype=torch.float32, device=logits.device)
    dlogits = logits if inplace else torch.empty_like(logits)
    rc = _C.lib().pt_cross_entropy_fwd_bwd(_ptr(logits), logits.stride(0), _ptr(targets), _ptr(dlogits),
                                           dlogits.stride(0), _ptr(row_loss), rows, vocab, float(scale),
                                           _ptr(inv_count), int(ignore_index), _ptr(status_word(logits.device)), _C.stream_ptr(logits.device))
    _C.check(rc, "pt_cross_entropy_fwd_bwd")
    _status_posted(logits.device)
    loss = row_loss.sum() * inv_count[0]
    return loss, dlogits, inv_count


def cross_entropy_loss(logits, targets, ignore_index=-100):
    """Forward only: (mean loss f32 scalar tensor, inv_count [1] f32) -- one read of the logits."""
    _bf16_rowmajor(logits, "logits")
    rows, vocab = logits.shape
    _req(targets.dtype == torch.int64 and targets.numel() == rows, "targets: int64 [rows]")
    targets = targets.contiguous()
    inv_count = (1.0 / (targets != ignore_index).sum().clamp_min(1).to(torch.float32)).reshape(1)
    row_loss = torch.empty(rows, dtype=torch.float32, device=logits.device)
    rc = _C.lib().pt_cross_entropy_fwd_bwd(_ptr(logits), logits.stride(0), _ptr(targets), None, 0, _ptr(row_loss),
                                           rows, vocab, 1.0, None, int(ignore_index), _ptr(status_word(logits.device)), _C.stream_ptr(logits.device))
    _C.check(rc, "pt_cross_entropy_fwd_bwd(loss)")
    _status_posted(logits.device)
    return row_loss.sum() * inv_count[0], inv_count


def _ce_mean(row_loss, targets, ignore_index, out_dtype, reduce_sum=False):
    """(mean loss over the valid rows in out_dtype, inv_count [1] f32) in one launch
    (reduce_sum: the sum of the row losses, inv_count 1)."""
    rows = row_loss.numel()
    _req(out_dtype in (BF16, torch.float32), "cross_entropy: loss dtype bf16 / f32")
    inv_count = torch.empty(1, dtype=torch.float32, device=row_loss.device)
    loss = torch.empty((), dtype=out_dtype, device=row_loss.device)
    rc = _C.lib().pt_cross_entropy_mean(_ptr(row_loss), _ptr(targets), rows, int(ignore_index), None, _ptr(inv_count),
                                        _ptr(loss), int(out_dtype == BF16), int(bool(reduce_sum)),
                                        _C.stream_ptr(row_loss.device))
    _C.check(rc, "pt_cross_entropy_mean")
    return loss, inv_count


def _ce_reduce(row_loss, targets, ignore_index, out_dtype, reduction):
    """F.cross_entropy's reduction of the per-row losses (ignored rows hold 0): 'mean' / 'sum' in one
    launch -> (loss scalar, inv_count [1]); 'none' -> (row losses in out_dtype, None)."""
    if reduction == "none":
        return (row_loss if out_dtype == torch.float32 else row_loss.to(out_dtype)), None
    _req(reduction in ("mean", "sum"), f"cross_entropy: reduction {reduction!r}")
    return _ce_mean(row_loss, targets, ignore_index, out_dtype, reduce_sum=reduction == "sum")


def cross_entropy_loss_lse(logits, targets, ignore_index=-100, out_dtype=torch.float32, reduction="mean"):
    """Forward of the autograd pair: (mean loss f32 scalar tensor, inv_count [1] f32, row_lse [rows]
    f32) from one streaming read of the logits (online max / sum-exp)."""
    _bf16_rowmajor(logits, "logits")
    rows, vocab = logits.shape
    _req(targets.dtype == torch.int64 and targets.numel() == rows, "targets: int64 [rows]")
    targets = targets.contiguous()
    row_loss = torch.empty(rows, dtype=torch.float32, device=logits.device)
    row_lse = torch.empty(rows, dtype=torch.float32, device=logits.device)
    rc = _C.lib().pt_cross_entropy_fwd_lse(_ptr(logits), logits.stride(0), _ptr(targets), _ptr(row_loss),
                                           _ptr(row_lse), rows, vocab, int(ignore_index), _ptr(status_word(logits.device)), _C.stream_ptr(logits.device))
    _C.check(rc, "pt_cross_entropy_fwd_lse")
    _status_posted(logits.device)
    # no clamp: every target ignored gives 0 * inf = nan, as F.cross_entropy's mean does (grads 0)
    loss, inv_count = _ce_reduce(row_loss, targets, ignore_index, out_dtype, reduction)
    return loss, inv_count, row_lse


def cross_entropy_grad_lse(logits, targets, row_lse, scale_dev, ignore_index=-100):
    """dlogits = (exp(x - row_lse) - onehot) * scale_dev[0] (one f32 device scalar) or
    * scale_dev[row] (f32 [rows]: reduction='none'): elementwise, no row reduction."""
    _bf16_rowmajor(logits, "logits")
    rows, vocab = logits.shape
    targets = targets.contiguous()
    _req(scale_dev.dtype == torch.float32 and scale_dev.numel() in (1, rows), "scale: f32 device scalar or [rows]")
    _req(row_lse.dtype == torch.float32 and row_lse.is_contiguous() and row_lse.numel() == rows, "row_lse: f32 [rows]")
    scale_dev = scale_dev.contiguous()
    dl = torch.empty(rows, vocab, dtype=BF16, device=logits.device)
    rc = _C.lib().pt_cross_entropy_bwd_lse(_ptr(logits), logits.stride(0), _ptr(targets), _ptr(row_lse), _ptr(dl),
                                           dl.stride(0), rows, vocab, _ptr(scale_dev), int(scale_dev.numel() != 1),
                                           int(ignore_index), _C.stream_ptr(logits.device))
    _C.check(rc, "pt_cross_entropy_bwd_lse")
    return dl


def cross_entropy_grad(logits, targets, scale_dev, ignore_index=-100):
    """dlogits = (softmax - onehot) * scale_dev[0] (a device scalar, e.g. grad_output / #valid)."""
    _bf16_rowmajor(logits, "logits")
    rows, vocab = logits.shape
    targets = targets.contiguous()
    _req(scale_dev.dtype == torch.float32 and scale_dev.numel() == 1, "scale: f32 device scalar")
    scale_dev = scale_dev.contiguous()
    dl = torch.empty(rows, vocab, dtype=BF16, device=logits.device)
    row_loss = torch.empty(rows, dtype=torch.float32, device=logits.device)
    rc = _C.lib().pt_cross_entropy_fwd_bwd(_ptr(logits), logits.stride(0), _ptr(targets), _ptr(dl), dl.stride(0),
                                           _ptr(row_loss), rows, vocab, 1.0, _ptr(scale_dev), int(ignore_index),
                                           _ptr(status_word(logits.device)), _C.stream_ptr(logits.device))
    _C.check(rc, "pt_cross_entropy_fwd_bwd(grad)")
    _status_posted(logits.device)
    return dl


# ------------------------------------------------------------------------------------ GEMM
EPI_BF16, EPI_BF16_ACC, EPI_F32, EPI_F32_ACC, EPI_BF16_RES = 0, 1, 2, 3, 4


class GemmProbe:
    """Live timing of every GEMM launch (bench.py's roofline): a pair of HIP events recorded on
    the launch stream around each pt_gemm call, plus its algorithmic FLOPs (2*M*N*K)."""

    def __init__(self, only=None):
        self.records = []
        self.only = only   # a launch label: time only launches of that kind (bench.py's timed steps)

    def __enter__(self):
        global _PROBE
        _PROBE = self
        return self

    def __exit__(self, *exc):
        global _PROBE
        _PROBE = None

    def summary(self):
        torch.cuda.synchronize()
        ms = [r[0].elapsed_time(r[1]) for r in self.records]
        flops = [r[2] for r in self.records]
        byts = [r[3] for r in self.records]
        n = len(ms)
        return {"launches": n, "total_ms": sum(ms), "total_flop": sum(flops),
                "avg_ms": sum(ms) / max(n, 1), "avg_flop": sum(flops) / max(n, 1),
                "avg_alg_bytes": sum(byts) / max(n, 1)}

    def label_stats(self, label):
        """Launches of one label: {launches, total_ms, avg_ms, avg_flop, avg_alg_bytes}."""
        torch.cuda.synchronize()
        rs = [r for r in self.records if r[4] == label]
        n = max(len(rs), 1)
        ms = [r[0].elapsed_time(r[1]) for r in rs]
        return {"launches": len(rs), "total_ms": sum(ms), "avg_ms": sum(ms) / n,
                "avg_flop": sum(r[2] for r in rs) / n, "avg_alg_bytes": sum(r[3] for r in rs) / n}

    def by_label(self):
        """{label: (launches, total ms, TF/s)} -- which GEMM shapes / launch kinds take the time."""
        torch.cuda.synchronize()
        out = {}
        for r in self.records:
            n, t, f = out.get(r[4], (0, 0.0, 0.0))
            out[r[4]] = (n + 1, t + r[0].elapsed_time(r[1]), f + r[2])
        return {k: (n, round(t, 4), round(f / (t * 1e-3) / 1e12, 1)) for k, (n, t, f) in
                sorted(out.items(), key=lambda kv: -kv[1][1])}


def _alg_bytes(M, N, K, epilogue):
    """Algorithmic HBM bytes of one GEMM launch: A and B read once, C written once (read too when
    accumulating / adding a residual; f32 for the main_grad epilogues; the SwiGLU epilogues move
    two [M, N] bf16 tensors more)."""
    elem = 4 if epilogue in (EPI_F32, EPI_F32_ACC) else 2
    c = M * N * elem * (2 if epilogue in (EPI_BF16_ACC, EPI_F32_ACC, EPI_BF16_RES) else 1)
    if epilogue == 5:      # gate|up: reads x, Wg, Wu; writes g|u and h
        c = M * N * 2 + M * (N // 2) * 2
    elif epilogue == 6:    # down dX: reads g|u, writes dg|du
        c = 4 * M * N * 2
    return 2 * (M * K + N * K) + c


_PROBE = None


def _probe_for(label):
    """The active GemmProbe if it times launches of this label, else None."""
    p = _PROBE
    return p if p is not None and (p.only is None or p.only == label) else None


def _gemm(A, lda, a_kcontig, Bs, ldbs, b_bounds, b_kcontig, b_seg_dim, Cs, ldcs, c_bounds, M, N, K, epilogue,
          tile=-1, residual=None, ldr=0):
    lib = _C.lib()
    nb, nc = len(Bs), len(Cs)
    label = f"gemm {M}x{N}x{K} e{epilogue} t{tile}"
    probe = _probe_for(label)
    if probe is not None:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    rc = lib.pt_gemm(_ptr(A), lda, int(a_kcontig), _C.ptrarr([_ptr(b) for b in Bs]), _C.i64arr(ldbs),
                     _C.i64arr(b_bounds), nb, int(b_kcontig), int(b_seg_dim), _C.ptrarr([_ptr(c) for c in Cs]),
                     _C.i64arr(ldcs), _C.i64arr(c_bounds), nc, M, N, K, int(epilogue), _ptr(residual), int(ldr),
                     int(tile), _C.stream_ptr(A.device))
    _C.check(rc, f"pt_gemm(M={M}, N={N}, K={K}, a_k={a_kcontig}, b_k={b_kcontig}, epi={epilogue})")
    if probe is not None:
        ev1.record()
        probe.records.append((ev0, ev1, 2.0 * M * N * K, _alg_bytes(M, N, K, epilogue), label))


def _bounds(sizes):
    out = [0]
    for s in sizes:
        out.append(out[-1] + int(s))
    return out


# ------------------------------------------------------------------ shapes off the 64-element grid
# Every GEMM tile is a multiple of 64 in M, N and K (the smallest tile is 64x64, the K-tile 64), so a
# projection whose T, width or K is not (Llama-2-7B at tp 8: a vocab shard of 4000, an intermediate
# shard of 1376; an odd token count) runs on zero-padded copies: the padding adds zero products
# (the real outputs are the unpadded kernel's, bit for bit, K-order unchanged) and is sliced off.  The
# layer shapes of picotron's configs tile and never take this path.
GRID = 64


def _up(n):
    return -(-int(n) // GRID) * GRID


def _on_grid(*dims):
    return all(int(d) % GRID == 0 for d in dims)


def _pad2(t, rows, cols):
    """A zero-padded contiguous [rows, cols] copy of a 2-D tensor (or the tensor when it fits)."""
    if tuple(t.shape) == (rows, cols) and t.is_contiguous():
        return t
    out = torch.zeros(rows, cols, dtype=t.dtype, device=t.device)
    out[:t.shape[0], :t.shape[1]] = t
    return out


def _pad_cols_segments(t, rows, ns):
    """[r, sum ns] with column segments of widths ns -> [rows, sum _up(n)], each segment at its
    padded offset (the segments of a stacked q|k|v or gate|up output)."""
    out = torch.zeros(rows, sum(_up(n) for n in ns), dtype=t.dtype, device=t.device)
    src = dst = 0
    for n in ns:
        out[:t.shape[0], dst:dst + n] = t[:, src:src + n]
        src, dst = src + n, dst + _up(n)
    return out


def _unpad_cols_segments(tp, rows, ns):
    """Inverse of _pad_cols_segments: the real columns of every segment, [rows, sum ns] (a copy)."""
    if len(ns) == 1:
        return tp[:rows, :ns[0]]
    parts, off = [], 0
    for n in ns:
        parts.append(tp[:rows, off:off + n])
        off += _up(n)
    return torch.cat(parts, dim=1)


def _linear_fwd_padded(x2d, weights, out, residual):
    T, K = x2d.shape
    ns = [w.shape[0] for w in weights]
    Tp, Kp = _up(T), _up(K)
    rp = None if residual is None else _pad_cols_segments(residual, Tp, ns)
    yp = linear_fwd(_pad2(x2d, Tp, Kp), [_pad2(w, _up(n), Kp) for w, n in zip(weights, ns)], residual=rp)
    y = _unpad_cols_segments(yp, T, ns)
    if out is None:
        return y.contiguous()
    out.copy_(y)
    return out


def _linear_dgrad_padded(dy2d, weights, out, accumulate):
    T = dy2d.shape[0]
    Kin = weights[0].shape[1]
    ns = [w.shape[0] for w in weights]
    Tp, Kp = _up(T), _up(Kin)
    dxp = linear_dgrad(_pad_cols_segments(dy2d, Tp, ns), [_pad2(w, _up(n), Kp) for w, n in zip(weights, ns)])
    dx = dxp[:T, :Kin]
    if out is None:
        return dx.contiguous()
    if accumulate:   # EPI_BF16_ACC's bf16(old + bf16(new)): dx is already the bf16 product
        out.copy_(out + dx)
    else:
        out.copy_(dx)
    return out


def _linear_wgrad_padded(dy2d, x2d, outs, epilogue):
    """dW_i into the sinks outs with the epilogue's semantics: EPI_BF16 store, EPI_BF16_ACC
    bf16(old + bf16(new)), EPI_F32 store / EPI_F32_ACC old + new in f32 (the f32 product, unrounded)."""
    T = dy2d.shape[0]
    Kin = x2d.shape[1]
    ns = [o.shape[0] for o in outs]
    Tp, Kp = _up(T), _up(Kin)
    f32 = epilogue in (EPI_F32, EPI_F32_ACC)
    tmp = [torch.empty(_up(n), Kp, dtype=torch.float32 if f32 else BF16, device=dy2d.device) for n in ns]
    linear_wgrad(_pad_cols_segments(dy2d, Tp, ns), _pad2(x2d, Tp, Kp), tmp, EPI_F32 if f32 else EPI_BF16)
    for o, t, n in zip(outs, tmp, ns):
        if epilogue in (EPI_BF16_ACC, EPI_F32_ACC):
            o.copy_(o + t[:n, :Kin])
        else:
            o.copy_(t[:n, :Kin])
    return outs


def _problem(A, lda, Bs, ldbs, b_bounds, b_seg_dim, Cs, ldcs, c_bounds, M, N, K):
    pr = _C.GemmProblem()
    pr.A, pr.lda = _ptr(A), int(lda)
    for i, (b, ld) in enumerate(zip(Bs, ldbs)):
        pr.B[i], pr.ldb[i] = _ptr(b), int(ld)
    for i, v in enumerate(b_bounds):
        pr.b_bounds[i] = int(v)
    pr.nb, pr.b_seg_dim = len(Bs), int(b_seg_dim)
    for i, (c, ld) in enumerate(zip(Cs, ldcs)):
        pr.C[i], pr.ldc[i] = _ptr(c), int(ld)
    for i, v in enumerate(c_bounds):
        pr.c_bounds[i] = int(v)
    pr.nc = len(Cs)
    pr.M, pr.N, pr.K = int(M), int(N), int(K)
    return pr


def _ksplit_enabled():
    return SW.ksplit != 0


def wgrad_ksplit(mnks, extra_tiles=0):
    """K-slices for a group of wgrad problems [(M, N, K)] (K = the token count) that leaves CUs idle:
    the TP-shard weight gradients (TP = 8 at SmolLM-1.7B: q|k|v dW 24 + o_proj dW 8 tiles of 256x256,
    down_proj dW 32, gate|up dW 64, on 256 CUs) run as ksplit slices of K / ksplit -- the largest
    power of two keeping every slice >= 512 deep and the launch within one round of the 256 CUs
    (2 ... 16) -- into f32 partials that pt_gemm_splitk_reduce sums into the sink.  1 = unsplit:
    shapes that already fill half the CUs, or do not tile by 256.  extra_tiles: tiles of other
    problems sharing the launch (a dual launch's dX), counted in the round."""
    if not _ksplit_enabled() or any(m % 256 or n % 256 for m, n, _ in mnks):
        return 1
    tiles = sum((m // 256) * (n // 256) for m, n, _ in mnks)
    if tiles >= 128:
        return 1
    s = 1
    while s < 16 and tiles * s * 2 + extra_tiles <= 256 and \
            all(k % (s * 2 * 64) == 0 and k // (s * 2) >= 512 for _, _, k in mnks):
        s *= 2
    return s


def swiglu_dx_ksplit(T, I, H):
    """K-slices for the down_proj dX with the SwiGLU backward (dual launch beside the down_proj dW)
    when its 256x256 tiles fill under half the CUs -- the TP shards (TP = 8 at SmolLM-1.7B: 64
    tiles with K 2048, the launch's critical path beside 128 dW slices of K 1024): the largest power
    of two keeping the dX slices within half a round and >= 512 deep, the SwiGLU backward then in
    the reduce pass (pt_gemm_splitk_reduce mode 6).  1 = unsplit (the fused epilogue)."""
    if not _ksplit_enabled() or not SW.swiglu_splitk or T % 256 or I % 256:
        return 1
    tiles = (T // 256) * (I // 256)
    s = 1
    while s < 8 and tiles * s * 2 <= 128 and H % (s * 2 * 64) == 0 and H // (s * 2) >= 512:
        s *= 2
    return s


def hq_form(mnks, extra_tiles=0):
    """K-slices (1 or 2) for a group of few-tile problems [(M, N, K)] on the 128x128 k-substep tile
    (15), or 0 when it does not apply.  It applies where the phased 256x256 tiles leave most of the 256
    CUs idle -- fewer than 96 of them over the group: the TP shards (TP = 8 at SmolLM-1.7B: the q|k|v
    forward 48 tiles, the o_proj dX 16, the q|k|v + o_proj dW 32, gate|up dW 64) -- and every problem
    tiles by 128.  A 128x128 tile puts four times the workgroups on the CUs at the same K, so most
    of these fill the chip without K-slices; 2 slices where the 128x128 tiles still fill at most half
    a round and K >= 4096 (the q|k|v + o_proj and down_proj dW: 128 tiles).  Measured per launch
    (tools/tp_gemm_ab.py, profiles/r05/tp_gemm_ab_r05c.log), against the 256x256 K-slice forms:
    q|k|v forward 22.1 vs 34.4 us, o_proj dX 20.7 vs 25.8, q|k|v + o dW 34.4 vs 42.6, gate|up dW
    40.6 vs 49.9, down_proj dW 31.6 vs 38.6."""
    if not _ksplit_enabled() or any(m % 128 or n % 128 for m, n, _ in mnks):
        return 0
    t12 = sum((m // 256) * (n // 256) if m % 256 == 0 and n % 256 == 0 else (m * n) // 65536 for m, n, _ in mnks)
    if t12 >= 96 or any(m < 2048 and k < 2048 for m, _, k in mnks):
        return 0
    t15 = sum((m // 128) * (n // 128) for m, n, _ in mnks) + extra_tiles
    if t15 * 2 <= 256 and all(k >= 4096 and k % 256 == 0 for _, _, k in mnks):
        return 2
    return 1


def _gemm_ksplit(A, lda, a_kcontig, Bs, ldbs, b_bounds, b_kcontig, b_seg_dim, out, M, N, K, s, tile, epilogue,
                 residual=None, ldr=0):
    """C = A . B as s K-slices into f32 partials (one grouped launch of `tile`), then the reduce
    pass through `epilogue` (EPI_BF16 / EPI_BF16_ACC / EPI_BF16_RES) into out [M, N]."""
    dev = A.device
    ws = torch.empty(s * M * N, dtype=torch.float32, device=dev)
    probs = (_C.GemmProblem * 1)()
    pr = _problem(A, lda, Bs, ldbs, b_bounds, b_seg_dim, [ws], [N], [0, M], M, N, K)
    pr.ksplit, pr.kpart_stride = s, M * N
    probs[0] = pr
    label = f"gemm {M}x{N}x{K} ks{s}"
    probe = _probe_for(label)
    if probe is not None:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
    _ksplit_launch(probs, 1, a_kcontig, b_kcontig, tile, [_sink([out], [0, M], epilogue, residual, ldr)], dev)
    if probe is not None:
        ev1.record()
        probe.records.append((ev0, ev1, 2.0 * M * N * K, _alg_bytes(M, N, K, epilogue), label))
    return out


def _reduce_sink_ok(out, residual=None):
    """pt_gemm_splitk_reduce writes 16-B (f32) / 8-B (bf16) row chunks and reads the residual the same
    way: a sink (or residual) it cannot address so -- a misaligned view -- keeps the unsplit GEMM,
    decided before anything is launched (the reduce pass would refuse it after the partial GEMM)."""
    for t in (out,) if residual is None else (out, residual):
        if t.stride(1) != 1 or t.stride(0) % 4 or t.data_ptr() % (16 if t.dtype == torch.float32 else 8):
            return False
    return True


def _sink(outs, bounds, mode, residual=None, ldr=0):
    """(outs, row bounds, epilogue, residual, ldr) of a split-K problem's real sink."""
    return outs, bounds, mode, residual, ldr


def _ksplit_launch(probs, n, a_kcontig, b_kcontig, tile, sinks, dev):
    """The split-K problems (f32 partials, one grouped launch), then one reduce pass per problem into
    its sink through the GEMM's own epilogue (pt_gemm_splitk_reduce: the partials summed in slice
    order over the whole chip).  (Finishing a tile inside the launch -- its last-arriving slice
    summing the partials, tools/diag/ksplit_fused.patch -- measured 12-20 % slower at TP = 8: one
    workgroup per tile then does the whole reduction after the other slices have left the CUs.)"""
    stream = _C.stream_ptr(dev)
    rc = _C.lib().pt_gemm_grouped(probs, n, int(a_kcontig), int(b_kcontig), EPI_F32, int(tile), stream)
    _C.check(rc, f"pt_gemm_grouped({n} problems, split-K {probs[0].ksplit})")
    for j in range(n):
        pr = probs[j]
        outs, bounds, mode, residual, ldr = sinks[j]
        rc = _C.lib().pt_gemm_splitk_reduce(ctypes.c_void_p(pr.C[0]), pr.ksplit, pr.kpart_stride, pr.M, pr.N,
                                            _C.ptrarr([_ptr(o) for o in outs]), _C.i64arr([o.stride(0) for o in outs]),
                                            _C.i64arr(bounds), len(outs), int(mode), _ptr(residual), int(ldr), stream)
        _C.check(rc, "pt_gemm_splitk_reduce")


def _wgrad_ksplit_run(jobs, epilogue, s, tile=-1):
    """The wgrad jobs [(dy2d, x2d, outs)] as s-way split-K problems of ONE grouped launch (f32
    partials in one workspace; tile -1: the auto pick), then one reduce pass per job into its outs
    through `epilogue`."""
    dev = jobs[0][0].device
    sizes = [dy.shape[1] * x.shape[1] for dy, x, _ in jobs]
    ws = torch.empty(s * sum(sizes), dtype=torch.float32, device=dev)
    probs = (_C.GemmProblem * len(jobs))()
    flops = nbytes = 0.0
    base = 0
    views = []
    for j, (dy2d, x2d, outs) in enumerate(jobs):
        T, N = dy2d.shape
        Kin = x2d.shape[1]
        part = ws[base:base + s * N * Kin]
        views.append(part)
        pr = _problem(dy2d, dy2d.stride(0), [x2d], [x2d.stride(0)], [0, Kin], 0, [part], [Kin], [0, N], N, Kin, T)
        pr.ksplit, pr.kpart_stride = s, N * Kin
        probs[j] = pr
        base += s * N * Kin
        flops += 2.0 * N * Kin * T
        nbytes += _alg_bytes(N, Kin, T, epilogue)
    probe = _probe_for("_wgrad_ksplit_run")
    if probe is not None:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
    sinks = [_sink(outs, _bounds([o.shape[0] for o in outs]), epilogue) for _, _, outs in jobs]
    _ksplit_launch(probs, len(jobs), 0, 0, tile, sinks, dev)
    if probe is not None:
        ev1.record()
        probe.records.append((ev0, ev1, flops, nbytes, "_wgrad_ksplit_run"))


def _wgrad_problem(dy2d, x2d, outs):
    """The GemmProblem of dW = dY^T X into outs (row segments of dW): dY and X plain [T, n] or KPair
    (two micro-batches: A K-segmented at T through A2, B through two K-segments)."""
    Nw, Kin = dy2d.shape[1], x2d.shape[1]
    ns = [o.shape[0] for o in outs]
    _req(sum(ns) == Nw and x2d.shape[0] == dy2d.shape[0], "wgrad: output rows must cover dY's width")
    Cs, ldcs, cb = outs, [o.stride(0) for o in outs], _bounds(ns)
    if isinstance(dy2d, KPair):
        _req(isinstance(x2d, KPair), "wgrad: dY and X paired together")
        t = dy2d.a.shape[0]
        pr = _problem(dy2d.a, dy2d.stride(0), [x2d.a, x2d.b], [x2d.stride(0)] * 2, [0, t, 2 * t], 1, Cs, ldcs, cb,
                      Nw, Kin, 2 * t)
        pr.A2, pr.a_k2 = _ptr(dy2d.b), t
        return pr
    return _problem(dy2d, dy2d.stride(0), [x2d], [x2d.stride(0)], [0, Kin], 0, Cs, ldcs, cb, Nw, Kin, dy2d.shape[0])


def _is_paired(jobs):
    return any(isinstance(dy, KPair) for dy, _, _ in jobs)


_ACC_OF = {EPI_BF16: EPI_BF16_ACC, EPI_BF16_ACC: EPI_BF16_ACC, EPI_F32: EPI_F32_ACC, EPI_F32_ACC: EPI_F32_ACC}


def _wgrad_unpaired(jobs, epilogue):
    """Paired wgrad jobs as two launches each: the first micro-batch's half through `epilogue`, the
    second's accumulating onto it."""
    for dy, x, outs in jobs:
        if isinstance(dy, KPair):
            linear_wgrad_grouped([(dy.a, x.a, outs)], epilogue)
            linear_wgrad_grouped([(dy.b, x.b, outs)], _ACC_OF[epilogue])
        else:
            linear_wgrad_grouped([(dy, x, outs)], epilogue)


def linear_wgrad_grouped(jobs, epilogue=EPI_BF16, tile=-1):
    """Several wgrad GEMMs (dW_i = dY_i^T X for each job (dy2d, x2d, outs)) in ONE launch
    (pt_gemm_grouped): e.g. dW of q|k|v (192 tiles) + dW of o_proj (64 tiles) fill 256 CUs.  A group
    that would leave most CUs idle (TP shards) runs split-K (wgrad_ksplit)."""
    if not all(_on_grid(dy.shape[0], x.shape[1], *[o.shape[0] for o in outs]) for dy, x, outs in jobs):
        # a job off the 64-grid: every job on its own (linear_wgrad pads; a pair as its two halves)
        if _is_paired(jobs):
            _wgrad_unpaired(jobs, epilogue)
        else:
            for dy, x, outs in jobs:
                linear_wgrad(dy, x, outs, epilogue)
        return
    paired = _is_paired(jobs)
    if paired:
        tile = 12   # the K-segmented A: the 256x256 8-phase kernel only
    if tile < 0 and epilogue in (EPI_BF16, EPI_BF16_ACC, EPI_F32_ACC):
        mnks = [(dy.shape[1], x.shape[1], dy.shape[0]) for dy, x, _ in jobs]
        hq = hq_form(mnks) if all(o.shape[0] % 128 == 0 for _, _, outs in jobs for o in outs) else 0
        sinks_ok = all(_reduce_sink_ok(o) for _, _, outs in jobs for o in outs)
        if hq == 2 and sinks_ok:
            return _wgrad_ksplit_run(jobs, epilogue, 2, tile=15)
        if hq == 1:
            tile = 15
        else:
            s = wgrad_ksplit(mnks)
            if s > 1 and sinks_ok:
                return _wgrad_ksplit_run(jobs, epilogue, s)
    probs = (_C.GemmProblem * len(jobs))()
    flops = nbytes = 0.0
    for j, (dy2d, x2d, outs) in enumerate(jobs):
        _bf16_rowmajor(dy2d, "dy")
        _bf16_rowmajor(x2d, "x")
        T, N = dy2d.shape
        Kin = x2d.shape[1]
        probs[j] = _wgrad_problem(dy2d, x2d, outs)
        flops += 2.0 * N * Kin * T
        nbytes += _alg_bytes(N, Kin, T, epilogue)
    probe = _probe_for("linear_wgrad_grouped")
    if probe is not None:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
    rc = _C.lib().pt_gemm_grouped(probs, len(jobs), 0, 0, int(epilogue), int(tile), _C.stream_ptr(jobs[0][0].device))
    if rc == -3 and paired:   # a shape the 256x256 tile does not cover: each micro-batch's half on its own
        _wgrad_unpaired(jobs, epilogue)
        rc = 0
    _C.check(rc, f"pt_gemm_grouped({len(jobs)} problems, epi={epilogue})")
    if probe is not None:
        ev1.record()
        probe.records.append((ev0, ev1, flops, nbytes, "linear_wgrad_grouped"))


def linear_fwd(x2d, weights, out=None, tile=-1, residual=None):
    """Y = x . [W_0; W_1; ...]^T  -> [T, sum N_i] (one launch; F.linear of model.py:124-126,186).
    residual [T, N]: Y = residual + x W^T (the residual add of model.py:208 in the epilogue)."""
    _bf16_rowmajor(x2d, "x")
    T, K = x2d.shape
    for w in weights:
        _req(w.dtype == BF16 and w.is_contiguous() and w.shape[1] == K, "weight must be contiguous [N, K] bf16")
    ns = [w.shape[0] for w in weights]
    N = sum(ns)
    if not _on_grid(T, K, *ns):
        if residual is not None:
            _req(tuple(residual.shape) == (T, N), "residual shape")
        return _linear_fwd_padded(x2d, weights, out, residual)
    y = out if out is not None else torch.empty(T, N, dtype=BF16, device=x2d.device)
    _req(y.stride(1) == 1 and y.shape == (T, N), "out shape")
    epi, ldr = EPI_BF16, 0
    if residual is not None:
        _bf16_rowmajor(residual, "residual")
        _req(tuple(residual.shape) == (T, N), "residual shape")
        epi, ldr = EPI_BF16_RES, residual.stride(0)
    if out is None and tile < 0 and _splitk_enabled() and len(weights) <= 4 and \
            (residual is None or residual.is_contiguous()):
        h = _splitk_halves(T, N, K)
        if h is not None:
            return _linear_fwd_splitk(x2d, weights, h, y, residual)
    hq = hq_form([(T, N, K)]) if tile < 0 and all(n % 128 == 0 for n in ns) else 0
    if hq == 1:
        tile = 15
    elif hq == 2 and _reduce_sink_ok(y, residual):
        return _gemm_ksplit(x2d, x2d.stride(0), 1, weights, [K] * len(weights), _bounds(ns), 1, 0, y, T, N, K, 2, 15,
                            epi, residual=residual, ldr=ldr)
    _gemm(x2d, x2d.stride(0), 1, weights, [K] * len(weights), _bounds(ns), 1, 0, [y], [y.stride(0)], [0, T],
          T, N, K, epi, tile, residual=residual, ldr=ldr)
    return y


EPI_SWIGLU_FWD, EPI_SWIGLU_BWD = 5, 6


def rope_fusable(T, head_dim, seq_len, widths=()):
    """The RoPE-fused q|k|v projection tiles head_dim 64 (the wave tile width) with T % 256, and the
    phased kernels need every q / k / v segment boundary on a 128-column tile edge (e.g. TP shards
    of 2 q heads + 1 kv head of 64 do not tile: the separate RoPE kernel runs instead)."""
    return head_dim == 64 and T % 256 == 0 and T % seq_len == 0 and all(w % 128 == 0 for w in widths)


# fewer 256x256 tiles than this: q|k|v + RoPE as a plain GEMM + rope kernel (PICOTRON_ROPE_FUSE_MIN_TILES)


def linear_fwd_rope(x2d, weights, cos, sin, seq_len, rot_heads, head_dim):
    """Y = x . [W_0; ...]^T with the first rot_heads heads of every row rotated by RoPE in the GEMM
    epilogue (model.py:124-126 + 136-137: the q|k|v projection, then apply_rotary_emb on q and k)."""
    _bf16_rowmajor(x2d, "x")
    T, K = x2d.shape
    for w in weights:
        _req(w.dtype == BF16 and w.is_contiguous() and w.shape[1] == K, "weight must be contiguous [N, K] bf16")
    _req(cos.dtype == BF16 and sin.dtype == BF16 and cos.stride(-1) == 1 and sin.stride(0) == cos.stride(0),
         "rope tables: bf16 [S, d]")
    _req(cos.shape[0] >= seq_len and rope_fusable(T, head_dim, seq_len), "linear_fwd_rope: shape")
    ns = [w.shape[0] for w in weights]
    N = sum(ns)
    if (T // 256) * (N // 256) < SW.rope_fuse_min_tiles:
        # a TP shard's q|k|v (TP = 8: N 768, 48 tiles of 256x256 on 256 CUs): the phased kernels
        # the RoPE epilogue needs would leave most CUs idle; the plain GEMM picks a smaller tile and
        # csrc/rope.hip rotates q|k after it (bit-identical to the fused epilogue)
        y = linear_fwd(x2d, weights)
        return rope_(y, rot_heads, head_dim, cos, sin, seq_len)
    y = torch.empty(T, N, dtype=BF16, device=x2d.device)
    probe = _probe_for("linear_fwd_rope")
    if probe is not None:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
    rc = _C.lib().pt_gemm_rope(_ptr(x2d), x2d.stride(0), _C.ptrarr([_ptr(w) for w in weights]), _C.i64arr([K] * len(weights)),
                               _C.i64arr(_bounds(ns)), len(weights), _ptr(y), y.stride(0), T, N, K, _ptr(cos), _ptr(sin),
                               cos.stride(0), seq_len, rot_heads * head_dim, head_dim, -1, _C.stream_ptr(x2d.device))
    _C.check(rc, "pt_gemm_rope")
    if probe is not None:
        ev1.record()
        probe.records.append((ev0, ev1, 2.0 * T * N * K, _alg_bytes(T, N, K, EPI_BF16), "linear_fwd_rope"))
    return y


EPI_CE_STATS = 8


def ce_stats_block(T, V):
    """Column tile of the lm_head GEMM's CE statistics: 256 (8-phase 256x256 kernel) when V divides,
    else 128 (4-phase 256x128); None when the shape does not tile (T % 256)."""
    if T % 256:
        return None
    return 256 if V % 256 == 0 else (128 if V % 128 == 0 else None)


def ce_stats_fusable(T, V):
    return ce_stats_block(T, V) is not None


def linear_ce_stats(x2d, weight):
    """lm_head (model.py:270) with the CE forward's statistics in the GEMM epilogue: returns (logits
    [T, V] bf16, stats [V / block, T, 2] f32 = per column tile and row (max, sum exp(x - max)) of
    the stored bf16 logits)."""
    _bf16_rowmajor(x2d, "x")
    T, K = x2d.shape
    V = weight.shape[0]
    _req(weight.dtype == BF16 and weight.is_contiguous() and weight.shape[1] == K, "weight must be contiguous [V, K] bf16")
    block = ce_stats_block(T, V)
    _req(block is not None and K % 64 == 0, "linear_ce_stats: T % 256, V % 128, K % 64")
    y = torch.empty(T, V, dtype=BF16, device=x2d.device)
    stats = torch.empty(V // block, T, 2, dtype=torch.float32, device=x2d.device)
    probe = _probe_for("linear_ce_stats")
    if probe is not None:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
    rc = _C.lib().pt_gemm_ce_stats(_ptr(x2d), x2d.stride(0), _ptr(weight), K, _ptr(y), y.stride(0), _ptr(stats),
                                   block, T, V, K, _C.stream_ptr(x2d.device))
    _C.check(rc, "pt_gemm_ce_stats")
    if probe is not None:
        ev1.record()
        probe.records.append((ev0, ev1, 2.0 * T * V * K, _alg_bytes(T, V, K, EPI_BF16), "linear_ce_stats"))
    return y, stats


def cross_entropy_loss_lse_stats(logits, targets, stats, ignore_index=-100, out_dtype=torch.float32,
                                 reduction="mean"):
    """cross_entropy_loss_lse from the lm_head GEMM's statistics (linear_ce_stats): same outputs,
    the logits are not streamed again (only x[row, target] is read)."""
    _bf16_rowmajor(logits, "logits")
    rows, vocab = logits.shape
    _req(targets.dtype == torch.int64 and targets.numel() == rows, "targets: int64 [rows]")
    _req(stats.dtype == torch.float32 and stats.is_contiguous() and stats.dim() == 3 and stats.shape[1:] == (rows, 2)
         and vocab % stats.shape[0] == 0, "stats: f32 [nblk, rows, 2]")
    targets = targets.contiguous()
    row_loss = torch.empty(rows, dtype=torch.float32, device=logits.device)
    row_lse = torch.empty(rows, dtype=torch.float32, device=logits.device)
    rc = _C.lib().pt_cross_entropy_fwd_stats(_ptr(logits), logits.stride(0), _ptr(targets), _ptr(stats),
                                             stats.shape[0], _ptr(row_loss), _ptr(row_lse), rows, vocab,
                                             int(ignore_index), _ptr(status_word(logits.device)),
                                             _C.stream_ptr(logits.device))
    _C.check(rc, "pt_cross_entropy_fwd_stats")
    _status_posted(logits.device)
    loss, inv_count = _ce_reduce(row_loss, targets, ignore_index, out_dtype, reduction)
    return loss, inv_count, row_lse


def cross_entropy_vp_partial(logits_shard, targets, stats, vocab_lo):
    """One tp rank's share of the vocab-parallel CE: per row float4 (max, sum exp(x - max), x[target]
    or 0, 1 or 0: the target in this shard) of the shard logits [rows, Vs] (columns vocab_lo ..), from
    the lm_head GEMM's statistics (linear_ce_stats) -- the logits are read at x[target] only."""
    _bf16_rowmajor(logits_shard, "logits")
    rows, vs = logits_shard.shape
    _req(targets.dtype == torch.int64 and targets.numel() == rows, "targets: int64 [rows]")
    _req(stats.dtype == torch.float32 and stats.is_contiguous() and stats.dim() == 3 and stats.shape[1:] == (rows, 2)
         and vs % stats.shape[0] == 0, "stats: f32 [nblk, rows, 2]")
    targets = targets.contiguous()
    part = torch.empty(rows, 4, dtype=torch.float32, device=logits_shard.device)
    rc = _C.lib().pt_cross_entropy_vp_partial(_ptr(logits_shard), logits_shard.stride(0), _ptr(targets), _ptr(stats),
                                              stats.shape[0], _ptr(part), rows, vs, int(vocab_lo),
                                              _C.stream_ptr(logits_shard.device))
    _C.check(rc, "pt_cross_entropy_vp_partial")
    return part


def cross_entropy_vp_combine(parts, targets, vocab, ignore_index=-100, out_dtype=torch.float32, reduction="mean"):
    """Every tp rank's partials [tp, rows, 4] (rank order) -> (loss, inv_count, row_lse) as
    cross_entropy_loss_lse_stats returns them for the whole [rows, vocab] logits."""
    _req(parts.dtype == torch.float32 and parts.is_contiguous() and parts.dim() == 3 and parts.shape[2] == 4,
         "parts: f32 [tp, rows, 4]")
    tp, rows = parts.shape[0], parts.shape[1]
    _req(targets.dtype == torch.int64 and targets.numel() == rows, "targets: int64 [rows]")
    targets = targets.contiguous()
    row_loss = torch.empty(rows, dtype=torch.float32, device=parts.device)
    row_lse = torch.empty(rows, dtype=torch.float32, device=parts.device)
    rc = _C.lib().pt_cross_entropy_vp_combine(_ptr(parts), tp, _ptr(targets), _ptr(row_loss), _ptr(row_lse), rows,
                                              int(vocab), int(ignore_index), _ptr(status_word(parts.device)),
                                              _C.stream_ptr(parts.device))
    _C.check(rc, "pt_cross_entropy_vp_combine")
    _status_posted(parts.device)
    loss, inv_count = _ce_reduce(row_loss, targets, ignore_index, out_dtype, reduction)
    return loss, inv_count, row_lse


def cross_entropy_grad_lse_shard(logits_shard, targets, row_lse, scale_dev, vocab_lo, ignore_index=-100):
    """cross_entropy_grad_lse on a vocab shard (columns vocab_lo ..): the one-hot only where the
    target falls in the shard; row_lse is the whole vocabulary's."""
    _bf16_rowmajor(logits_shard, "logits")
    rows, vs = logits_shard.shape
    targets = targets.contiguous()
    _req(scale_dev.dtype == torch.float32 and scale_dev.numel() in (1, rows), "scale: f32 device scalar or [rows]")
    _req(row_lse.dtype == torch.float32 and row_lse.is_contiguous() and row_lse.numel() == rows, "row_lse: f32 [rows]")
    scale_dev = scale_dev.contiguous()
    dl = torch.empty(rows, vs, dtype=BF16, device=logits_shard.device)
    rc = _C.lib().pt_cross_entropy_bwd_lse_shard(_ptr(logits_shard), logits_shard.stride(0), _ptr(targets),
                                                 _ptr(row_lse), _ptr(dl), dl.stride(0), rows, vs, int(vocab_lo),
                                                 _ptr(scale_dev), int(scale_dev.numel() != 1), int(ignore_index),
                                                 _C.stream_ptr(logits_shard.device))
    _C.check(rc, "pt_cross_entropy_bwd_lse_shard")
    return dl


def swiglu_fusable(T, I, backward=False, H=None):
    """Shapes the SwiGLU-fused projections tile (8-phase kernel: T % 256, I % 128 (fwd) / 256 (bwd),
    and the hidden size H -- the GEMM's K -- on the 64 K-tile grid)."""
    return T % 256 == 0 and I % (256 if backward else 128) == 0 and (H is None or H % GRID == 0)


# fewer 256-row x (128 fwd / 256 bwd)-column tiles than this: the SwiGLU runs as its own kernel
# beside a plain GEMM (whose auto tile fills the CUs) -- a TP shard's I (TP = 8: 1024; 128 tiles
# on 256 CUs); bit-identical either way.  The backward keeps its fused dual launch at every width
# (TP = 8 proxy: 8.95 vs 9.08 ms per micro-batch split).  PICOTRON_SWIGLU_FUSE_MIN_TILES / _BWD_MIN_TILES.


def swiglu_fuse_pays(T, I, backward=False, H=None):
    """swiglu_fusable and enough tiles that the fused (8-phase 256x256) launch fills the CUs."""
    tiles = (T // 256) * (I // (256 if backward else 128))
    return swiglu_fusable(T, I, backward, H) and \
        tiles >= (SW.swiglu_bwd_min_tiles if backward else SW.swiglu_fuse_min_tiles)


def linear_swiglu_fwd(x2d, wg, wu):
    """gate|up projection with SwiGLU in the GEMM epilogue (model.py:186): returns (gu [T, 2I] =
    [x Wg^T | x Wu^T], h = bf16(bf16(silu(g)) * u) [T, I]) in one launch."""
    _bf16_rowmajor(x2d, "x")
    T, K = x2d.shape
    I = wg.shape[0]
    for w in (wg, wu):
        _req(w.dtype == BF16 and w.is_contiguous() and tuple(w.shape) == (I, K), "gate/up weights [I, K] bf16")
    _req(swiglu_fusable(T, I, H=x2d.shape[1]), "linear_swiglu_fwd: T % 256, I % 128 and H % 64 required")
    gu = torch.empty(T, 2 * I, dtype=BF16, device=x2d.device)
    h = torch.empty(T, I, dtype=BF16, device=x2d.device)
    _gemm(x2d, x2d.stride(0), 1, [wg, wu], [K, K], [0, I, 2 * I], 1, 0, [h, gu], [I, 2 * I], [0, T], T, 2 * I, K,
          EPI_SWIGLU_FWD)
    return gu, h


def linear_dgrad_swiglu(dy2d, wd, gu):
    """dh = dY W_down (model.py:186 backward) with the SwiGLU backward in the epilogue: returns
    dgu = [dg | du] [T, 2I] (dh is never materialised)."""
    _bf16_rowmajor(dy2d, "dy")
    _bf16_rowmajor(gu, "gu")
    T, H = dy2d.shape
    I = wd.shape[1]
    _req(wd.dtype == BF16 and wd.is_contiguous() and wd.shape[0] == H, "down weight [H, I] bf16")
    _req(tuple(gu.shape) == (T, 2 * I), "gu must be [T, 2I]")
    _req(swiglu_fusable(T, I, backward=True, H=dy2d.shape[1]), "linear_dgrad_swiglu: T % 256, I % 256 and H % 64 required")
    dgu = torch.empty(T, 2 * I, dtype=BF16, device=dy2d.device)
    _gemm(dy2d, dy2d.stride(0), 1, [wd], [I], [0, I], 0, 0, [dgu], [dgu.stride(0)], [0, T], T, I, H, EPI_SWIGLU_BWD,
          residual=gu, ldr=gu.stride(0))
    return dgu


def _splitk_enabled():
    return SW.splitk2 != 0


def _splitk_min():
    return SW.splitk2_min


def _splitk_halves(M, N, K, min_half=None):
    """K of each half when C [M, N] = A [M, K] . B pays to split in two K halves (None if not): one
    round of 256x256 tiles for both halves together and at least PICOTRON_SPLITK2_MIN (8192) of K per
    half -- where the 256x256 8-phase rate (~17 % above the 256x128 one at long K) pays for the f32
    partials and the sum pass.  min_half overrides that floor (a caller whose halves share a launch
    with other work and whose consumer sums them)."""
    if M % 256 or N % 256 or 2 * (M // 256) * (N // 256) > 256 or K % 128:
        return None
    h = K // 2
    return h if h >= (_splitk_min() if min_half is None else min_half) else None


def _segments(sizes, lo, hi):
    """(index, offset inside it, length) of the pieces of the concatenation of `sizes` in [lo, hi)"""
    out, base = [], 0
    for i, n in enumerate(sizes):
        a, b = max(lo, base), min(hi, base + n)
        if a < b:
            out.append((i, a - base, b - a))
        base += n
    return out


def _splitk_run(probs, b_kcontig, parts, residual, out, flops, nbytes, device):
    probe = _probe_for("_splitk_run")
    if probe is not None:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
    stream = _C.stream_ptr(device)
    rc = _C.lib().pt_gemm_grouped(probs, 2, 1, b_kcontig, EPI_F32, 12, stream)
    _C.check(rc, "pt_gemm_grouped(split-K)")
    rc = _C.lib().pt_gemm_splitk_sum(_ptr(parts[0]), _ptr(parts[1]), _ptr(residual), _ptr(out), out.numel(), stream)
    _C.check(rc, "pt_gemm_splitk_sum")
    if probe is not None:
        ev1.record()
        probe.records.append((ev0, ev1, flops, nbytes, "_splitk_run"))
    return out


def _linear_dgrad_splitk(dy2d, weights, h, dx, keep_parts=False):
    """dX = bf16(dY[:, :h] . W[:h] + dY[:, h:] . W[h:]) with W = [W_0; W_1; ...] (the halves may cut
    through a weight): two f32 problems on 256x256 tiles in one grouped launch, then the sum pass
    (keep_parts: no sum pass, the SplitKParts for a consumer that sums them)."""
    T, N = dy2d.shape
    Kin = weights[0].shape[1]
    ns = [w.shape[0] for w in weights]
    parts = [torch.empty(T, Kin, dtype=torch.float32, device=dy2d.device) for _ in range(2)]
    probs = (_C.GemmProblem * 2)()
    for i, (lo, hi) in enumerate(((0, h), (h, N))):
        segs = _segments(ns, lo, hi)
        bs = [weights[j][a:a + n] for j, a, n in segs]
        probs[i] = _problem(dy2d[:, lo:], dy2d.stride(0), bs, [Kin] * len(bs), _bounds([n for _, _, n in segs]), 1,
                            [parts[i]], [Kin], [0, T], T, Kin, hi - lo)
    if keep_parts:
        rc = _C.lib().pt_gemm_grouped(probs, 2, 1, 0, EPI_F32, 12, _C.stream_ptr(dy2d.device))
        _C.check(rc, "pt_gemm_grouped(split-K halves)")
        return SplitKParts(parts[0], parts[1])
    return _splitk_run(probs, 0, parts, None, dx, 2.0 * T * Kin * N, _alg_bytes(T, Kin, N, EPI_BF16), dy2d.device)


def _linear_fwd_splitk(x2d, weights, h, y, residual):
    """Y = bf16(x[:, :h] . W[:, :h]^T + x[:, h:] . W[:, h:]^T) (+ residual as EPI_BF16_RES): two f32
    problems on 256x256 tiles in one grouped launch, then the sum pass (which adds the residual)."""
    T, K = x2d.shape
    ns = [w.shape[0] for w in weights]
    N = sum(ns)
    parts = [torch.empty(T, N, dtype=torch.float32, device=x2d.device) for _ in range(2)]
    probs = (_C.GemmProblem * 2)()
    for i, (lo, hi) in enumerate(((0, h), (h, K))):
        probs[i] = _problem(x2d[:, lo:], x2d.stride(0), [w[:, lo:] for w in weights], [K] * len(weights), _bounds(ns),
                            0, [parts[i]], [N], [0, T], T, N, hi - lo)
    return _splitk_run(probs, 1, parts, residual, y, 2.0 * T * N * K, _alg_bytes(T, N, K, EPI_BF16), x2d.device)


def linear_dgrad(dy2d, weights, out=None, accumulate=False, tile=-1, keep_parts=False, split_min=None):
    """dX = dY . [W_0; W_1; ...]  where dY = [dY_0 | dY_1 | ...] is [T, sum N_i].  split_min / keep_parts
    as linear_dgrad_dual's (the dX of a dual launch whose weight gradients were deferred)."""
    _bf16_rowmajor(dy2d, "dy")
    T, N = dy2d.shape
    Kin = weights[0].shape[1]
    ns = [w.shape[0] for w in weights]
    _req(sum(ns) == N, "dgrad: dY width must equal the stacked weight rows")
    if not _on_grid(T, Kin, *ns):
        return _linear_dgrad_padded(dy2d, weights, out, accumulate)
    if out is None and not accumulate and tile < 0 and _splitk_enabled() and len(weights) <= 3:
        h = _splitk_halves(T, Kin, N, split_min)
        if h is not None and all(w.dtype == BF16 and w.is_contiguous() for w in weights) and \
                all(n % 64 == 0 for n in ns):
            return _linear_dgrad_splitk(dy2d, weights, h, torch.empty(T, Kin, dtype=BF16, device=dy2d.device),
                                        keep_parts=keep_parts)
    dx = out if out is not None else torch.empty(T, Kin, dtype=BF16, device=dy2d.device)
    hq = hq_form([(T, Kin, N)]) if tile < 0 and all(n % 64 == 0 for n in ns) else 0
    if hq == 1:
        tile = 15
    elif hq == 2 and _reduce_sink_ok(dx):
        return _gemm_ksplit(dy2d, dy2d.stride(0), 1, weights, [Kin] * len(weights), _bounds(ns), 0, 1, dx, T, Kin,
                            N, 2, 15, EPI_BF16_ACC if accumulate else EPI_BF16)
    _gemm(dy2d, dy2d.stride(0), 1, weights, [Kin] * len(weights), _bounds(ns), 0, 1, [dx], [dx.stride(0)],
          [0, T], T, Kin, N, EPI_BF16_ACC if accumulate else EPI_BF16, tile)
    return dx


def dual_enabled():
    """PICOTRON_DUAL=0 launches a layer's dX and dW GEMMs separately (A/B measurement only)."""
    return SW.dual != 0


# the dual launch's XCD order unless a caller picks one: 0 = dX tiles first in every XCD, 1 = dW
# first, 2 = staggered -- even XCDs dX first, odd XCDs dW first, so half the chip is in the dX tiles'
# HBM-bound SwiGLU-backward tail at a time (+0.8 % on the step over 0 / 1, profiles/r03/dual_order_ab.txt)
DUAL_ORDER = 2


def dual_fits(dgrad_mn, wgrad_mns):
    """Whether pt_gemm_dual tiles these problems: every [M, N] by 256 x 256 and each group's tile
    count a multiple of 8 (equal shares per XCD)."""
    def ok(mns):
        return all(m % 256 == 0 and n % 256 == 0 for m, n in mns) and sum(m * n for m, n in mns) // 65536 % 8 == 0
    return ok([dgrad_mn]) and ok(wgrad_mns)


def norm_splitk_enabled():
    """The post-attention norm backward takes the gate|up dX's split-K halves directly
    (PICOTRON_NORM_SPLITK=0: the sum pass + the plain norm backward, A/B only)."""
    return SW.norm_splitk != 0


def linear_dgrad_dual(dy2d, weights, wjobs, wepilogue, gu=None, order=None, keep_parts=False, split_min=None):
    """dX = dY . [W_0; ...] (or, with gu, the SwiGLU backward dg|du of the down_proj dX:
    linear_dgrad_swiglu) AND the wgrads wjobs [(dy2d, x2d, outs)] (linear_wgrad, epilogue
    wepilogue) in ONE launch (pt_gemm_dual).  Returns dX / dg|du, or None (nothing launched) when
    the problems do not tile for it -- the caller then launches them separately."""
    _bf16_rowmajor(dy2d, "dy")
    T, N = dy2d.shape
    dxs = 1   # K-slices of a few-tile SwiGLU dX (finished by the reduce pass's SwiGLU backward)
    if gu is not None:
        wd = weights[0]
        I = wd.shape[1]
        _bf16_rowmajor(gu, "gu")
        _req(len(weights) == 1 and wd.is_contiguous() and wd.shape[0] == N and tuple(gu.shape) == (T, 2 * I),
             "dual: down weight [H, I], gu [T, 2I]")
        dx = torch.empty(T, 2 * I, dtype=BF16, device=dy2d.device)
        dxs = swiglu_dx_ksplit(T, I, N)
        if dxs > 1:   # TP shard widths: dh as K-slices into f32 partials beside the dW slices
            dxpart = torch.empty(dxs * T * I, dtype=torch.float32, device=dy2d.device)
            p0 = _problem(dy2d, dy2d.stride(0), [wd], [I], [0, I], 0, [dxpart], [I], [0, T], T, I, N)
            p0.ksplit, p0.kpart_stride = dxs, T * I
            e0 = EPI_F32
        else:
            p0 = _problem(dy2d, dy2d.stride(0), [wd], [I], [0, I], 0, [dx], [dx.stride(0)], [0, T], T, I, N)
            p0.residual, p0.ldr = _ptr(gu), gu.stride(0)
            e0 = EPI_SWIGLU_BWD
        flops, nbytes = 2.0 * T * I * N, _alg_bytes(T, I, N, EPI_SWIGLU_BWD)
    else:
        Kin = weights[0].shape[1]
        ns = [w.shape[0] for w in weights]
        _req(sum(ns) == N, "dgrad: dY width must equal the stacked weight rows")
        dx = torch.empty(T, Kin, dtype=BF16, device=dy2d.device)
        p0 = _problem(dy2d, dy2d.stride(0), weights, [Kin] * len(weights), _bounds(ns), 1, [dx], [dx.stride(0)],
                      [0, T], T, Kin, N)
        e0, flops, nbytes = EPI_BF16, 2.0 * T * Kin * N, _alg_bytes(T, Kin, N, EPI_BF16)
        h = _splitk_halves(T, Kin, N, split_min) if _splitk_enabled() else None
        if h is not None and all(w.dtype == BF16 and w.is_contiguous() for w in weights) and \
                all(n % 64 == 0 for n in ns):
            # the dX as two f32 K halves (split-K, finished by the sum pass after the launch)
            parts = [torch.empty(T, Kin, dtype=torch.float32, device=dy2d.device) for _ in range(2)]
            p0s = (_C.GemmProblem * 2)()
            for i, (lo, hi) in enumerate(((0, h), (h, N))):
                segs = _segments(ns, lo, hi)
                bs = [weights[j][a:a + n] for j, a, n in segs]
                p0s[i] = _problem(dy2d[:, lo:], dy2d.stride(0), bs, [Kin] * len(bs), _bounds([n for _, _, n in segs]),
                                  1, [parts[i]], [Kin], [0, T], T, Kin, hi - lo)
            e0 = EPI_F32
    if e0 != EPI_F32 or dxs > 1:
        p0s = (_C.GemmProblem * 1)(p0)
    # the probe's label of this launch kind (bench.py's roofline picks the dominant kernel by label)
    label = f"dual dX {T}x{p0s[0].N if e0 != EPI_F32 or dxs > 1 else dx.shape[1]}x{N} e{e0} + dW " + \
        ",".join(f"{dy.shape[1]}x{x.shape[1]}x{dy.shape[0]}" for dy, x, _ in wjobs) + f" e{wepilogue}"
    p1s = (_C.GemmProblem * len(wjobs))()
    # the TP shards' few-tile dW as split-K slices beside the dX tiles (f32 partials, reduced below)
    dx_tiles = sum(p.M // 256 * (p.N // 256) * max(1, p.ksplit) for p in p0s)
    ws = wgrad_ksplit([(dy.shape[1], x.shape[1], dy.shape[0]) for dy, x, _ in wjobs], extra_tiles=dx_tiles) \
        if wepilogue in (EPI_BF16, EPI_BF16_ACC, EPI_F32_ACC) and not _is_paired(wjobs) else 1
    # the reduce pass writes 16-B (f32) / 8-B (bf16) row chunks: a sink it cannot address that way (a
    # misaligned .grad / main_grad view) keeps the unsplit dW, decided before anything is launched
    if ws > 1 and not all(_reduce_sink_ok(o) for _, _, outs in wjobs for o in outs):
        ws = 1
    wparts = []
    for j, (wdy, x2d, outs) in enumerate(wjobs):
        _bf16_rowmajor(wdy, "dy")
        _bf16_rowmajor(x2d, "x")
        Tw, Nw = wdy.shape
        Kin = x2d.shape[1]
        ns = [o.shape[0] for o in outs]
        _req(sum(ns) == Nw and x2d.shape[0] == Tw, "wgrad: output rows must cover dY's width")
        if isinstance(wdy, KPair):   # two micro-batches' weight gradient, K = 2 T (the 8-phase tile: A2)
            p1s[j] = _wgrad_problem(wdy, x2d, outs)
        elif ws > 1:
            part = torch.empty(ws * Nw * Kin, dtype=torch.float32, device=dy2d.device)
            wparts.append(part)
            p1s[j] = _problem(wdy, wdy.stride(0), [x2d], [x2d.stride(0)], [0, Kin], 0, [part], [Kin], [0, Nw], Nw,
                              Kin, Tw)
            p1s[j].ksplit, p1s[j].kpart_stride = ws, Nw * Kin
        else:
            p1s[j] = _problem(wdy, wdy.stride(0), [x2d], [x2d.stride(0)], [0, Kin], 0, outs,
                              [o.stride(0) for o in outs], _bounds(ns), Nw, Kin, Tw)
        flops += 2.0 * Nw * Kin * Tw
        nbytes += _alg_bytes(Nw, Kin, Tw, wepilogue)
    probe = _probe_for(label)
    if probe is not None:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
    if order is None:
        order = DUAL_ORDER
        # unsplit dX tiles longer (in K) than the dW tiles: dX first on every XCD, the dW tiles
        # chaining on the other CUs around them (a dW-first XCD would start its dX tiles last)
        if e0 == EPI_BF16 and wjobs and N > max(dy.shape[0] for dy, _, _ in wjobs):
            order = 0
    rc = _C.lib().pt_gemm_dual(p0s, len(p0s), 1, 0, e0, p1s, len(wjobs), 0, 0, EPI_F32 if ws > 1 else int(wepilogue),
                               int(order), _C.stream_ptr(dy2d.device))
    if rc == -3:   # PT_EUNSUPPORTED: outside the dual tiling (e.g. C segments not on 256 rows)
        return None
    _C.check(rc, f"pt_gemm_dual(dX epi {e0}, {len(wjobs)} wgrads epi {wepilogue}, split {ws})")
    for (wdy, x2d, outs), part in zip(wjobs, wparts):
        Nw, Kin = wdy.shape[1], x2d.shape[1]
        ns = [o.shape[0] for o in outs]
        rc = _C.lib().pt_gemm_splitk_reduce(_ptr(part), ws, Nw * Kin, Nw, Kin, _C.ptrarr([_ptr(o) for o in outs]),
                                            _C.i64arr([o.stride(0) for o in outs]), _C.i64arr(_bounds(ns)), len(outs),
                                            int(wepilogue), None, 0, _C.stream_ptr(dy2d.device))
        _C.check(rc, "pt_gemm_splitk_reduce")
    if dxs > 1:   # dg|du = the SwiGLU backward of the summed dh slices
        rc = _C.lib().pt_gemm_splitk_reduce(_ptr(dxpart), dxs, T * I, T, I, _C.ptrarr([_ptr(dx)]),
                                            _C.i64arr([dx.stride(0)]), _C.i64arr([0, T]), 1, EPI_SWIGLU_BWD,
                                            _ptr(gu), gu.stride(0), _C.stream_ptr(dy2d.device))
        _C.check(rc, "pt_gemm_splitk_reduce(SwiGLU backward)")
    elif e0 == EPI_F32:
        if keep_parts:   # the consumer (rmsnorm_bwd) sums the halves
            dx = SplitKParts(parts[0], parts[1])
        else:
            rc = _C.lib().pt_gemm_splitk_sum(_ptr(parts[0]), _ptr(parts[1]), None, _ptr(dx), dx.numel(),
                                             _C.stream_ptr(dy2d.device))
            _C.check(rc, "pt_gemm_splitk_sum")
    if probe is not None:
        ev1.record()
        probe.records.append((ev0, ev1, flops, nbytes, label))
    return dx


def linear_wgrad(dy2d, x2d, outs, epilogue=EPI_BF16, tile=-1):
    """dW_i = dY_i^T . X for the column segments dY_i of dY (widths = outs[i].shape[0]); one launch.
    dY / X may be KPair (two micro-batches in one K = 2 T launch)."""
    if isinstance(dy2d, KPair):
        linear_wgrad_grouped([(dy2d, x2d, outs)], epilogue)
        return outs
    _bf16_rowmajor(dy2d, "dy")
    _bf16_rowmajor(x2d, "x")
    T, N = dy2d.shape
    Kin = x2d.shape[1]
    ns = [o.shape[0] for o in outs]
    _req(sum(ns) == N, "wgrad: output rows must cover dY's width")
    if not _on_grid(T, Kin, *ns):
        return _linear_wgrad_padded(dy2d, x2d, outs, epilogue)
    if tile < 0 and epilogue in (EPI_BF16, EPI_BF16_ACC, EPI_F32_ACC):
        hq = hq_form([(N, Kin, T)]) if all(n % 128 == 0 for n in ns) else 0
        sinks_ok = all(_reduce_sink_ok(o) for o in outs)
        if hq == 2 and sinks_ok:
            _wgrad_ksplit_run([(dy2d, x2d, outs)], epilogue, 2, tile=15)
            return outs
        if hq == 1:
            tile = 15
        elif wgrad_ksplit([(N, Kin, T)]) > 1 and sinks_ok:
            _wgrad_ksplit_run([(dy2d, x2d, outs)], epilogue, wgrad_ksplit([(N, Kin, T)]))
            return outs
    _gemm(dy2d, dy2d.stride(0), 0, [x2d], [x2d.stride(0)], [0, Kin], 0, 0, outs, [o.stride(0) for o in outs],
          _bounds(ns), N, Kin, T, epilogue, tile)
    return outs


# ------------------------------------------------------------------------------- LSE merge
def lse_merge(out, block_out, lse, block_lse):
    """(out_new f32, lse_new) = update_out_and_lse's non-first step (context_parallel.py:157-187) over
    contiguous out / block_out [..., D] and lse / block_lse [...] (lse in bf16 or f32)."""
    _req(out.dtype == torch.float32 and out.is_cuda, "lse_merge: out must be an f32 device tensor")
    _req(block_out.shape == out.shape and block_out.dtype in (BF16, torch.float32), "lse_merge: block_out")
    _req(lse.dtype == block_lse.dtype and lse.dtype in (BF16, torch.float32), "lse_merge: lse dtypes")
    D = out.shape[-1]
    rows = out.numel() // D
    _req(lse.numel() == rows and block_lse.numel() == rows, "lse_merge: one lse per output row")
    out, block_out, lse, block_lse = (t.contiguous() for t in (out, block_out, lse, block_lse))
    out_new = torch.empty_like(out)
    lse_new = torch.empty_like(lse)
    rc = _C.lib().pt_lse_merge(_ptr(out), _ptr(block_out), 0 if block_out.dtype == BF16 else 1, _ptr(lse),
                               _ptr(block_lse), 0 if lse.dtype == BF16 else 1, _ptr(out_new), _ptr(lse_new), rows, D,
                               _C.stream_ptr(out.device))
    _C.check(rc, "pt_lse_merge")
    return out_new, lse_new


# ------------------------------------------------------------------------------- attention
def _str3(t):
    _req(t.dim() == 4 and t.stride(3) == 1, "attention tensors are [B, S, H, D] views with d contiguous")
    return _C.i64arr([t.stride(0), t.stride(1), t.stride(2)])


def _lse_ld(t, B, H, Sq, name="lse"):
    """Row stride of an f32 [B, H, Sq] LSE / delta tensor: dense, or the Sq-column slice of a longer
    [B, H, S] one (the zig-zag ring's half blocks); the kernels index (b, h) rows lse_ld apart."""
    _req(t.dtype == torch.float32 and tuple(t.shape) == (B, H, Sq) and t.stride(2) == 1
         and t.stride(1) >= Sq and (B == 1 or t.stride(0) == H * t.stride(1)) and (H == 1 or t.stride(1) > 0),
         f"{name} must be f32 [B, H, Sq] with unit column stride and (b, h) rows evenly spaced")
    return t.stride(1) if H > 1 else (t.stride(0) if B > 1 else Sq)


# causal attention over a sequence length off the kernels' 128-row query blocks (attention.hip
# check_common: Sq % 128): q / k / v zero-padded to the next multiple.  Causality keeps the padded
# keys out of every real query's softmax, and the padded queries' rows are sliced off (forward) or
# carry dO = 0 and LSE = +inf, so P = 0 and they add nothing to dK / dV (backward): the real rows'
# results are the kernels' own on the real data.
ATTN_Q_BLOCK = 128


def _attn_padded_len(S):
    return -(-int(S) // ATTN_Q_BLOCK) * ATTN_Q_BLOCK


def _pad_seq(t, Sp, fill=0.0):
    """[B, S, ...] -> a contiguous [B, Sp, ...] copy whose rows past S are `fill`."""
    out = torch.full((t.shape[0], Sp) + tuple(t.shape[2:]), fill, dtype=t.dtype, device=t.device)
    out[:, :t.shape[1]] = t
    return out


def _attn_off_block(causal, Sq, Sk, lse, B, H):
    return causal and Sq == Sk and Sq % ATTN_Q_BLOCK != 0 and (lse is None or _lse_ld(lse, B, H, Sq) == Sq)


def attn_fwd(q, k, v, scale, causal, out=None, lse=None, merge=False):
    """q [B,Sq,H,D], k/v [B,Sk,Hkv,D] (token-major views).  Returns (out, lse[B,H,Sq] f32).
    merge=True: `out` is an f32 accumulator and `lse` the running LSE; this block is merged in.
    lse may be the Sq-column slice of a longer [B, H, S] LSE (rows evenly spaced)."""
    B, Sq, H, D = q.shape
    Sk, HKV = k.shape[1], k.shape[2]
    if not merge and _attn_off_block(causal, Sq, Sk, lse, B, H):
        Sp = _attn_padded_len(Sq)
        op, lp = attn_fwd(_pad_seq(q, Sp), _pad_seq(k, Sp), _pad_seq(v, Sp), scale, True)
        if out is None:
            out = op[:, :Sq].contiguous()
        else:
            out.copy_(op[:, :Sq])
        if lse is None:
            lse = lp[:, :, :Sq].contiguous()
        else:
            lse.copy_(lp[:, :, :Sq])
        return out, lse
    if out is None:
        out = torch.empty(B, Sq, H, D, dtype=BF16, device=q.device)
    if lse is None:
        lse = torch.empty(B, H, Sq, dtype=torch.float32, device=q.device)
    ld = _lse_ld(lse, B, H, Sq)
    ws = _attn_split_ws(B, H, HKV, Sq, Sk, D, causal, 0, q.device) if (not merge and ld == Sq) else None
    if ws is not None:   # few heads (a TP shard): split work items + merge (pt_attn_split_plan)
        rc = _C.lib().pt_attn_fwd_split(_ptr(q), _str3(q), _ptr(k), _str3(k), _ptr(v), _str3(v), _ptr(out),
                                        _str3(out), _ptr(lse), B, H, HKV, Sq, Sk, D, float(scale), int(bool(causal)),
                                        _ptr(ws), ws.numel(), _C.stream_ptr(q.device))
        _C.check(rc, "pt_attn_fwd_split")
        return out, lse
    rc = _C.lib().pt_attn_fwd(_ptr(q), _str3(q), _ptr(k), _str3(k), _ptr(v), _str3(v), _ptr(out), _str3(out),
                              _ptr(lse), B, H, HKV, Sq, Sk, D, float(scale), int(bool(causal)), int(bool(merge)),
                              ld, _C.stream_ptr(q.device))
    _C.check(rc, "pt_attn_fwd")
    return out, lse


def _attn_split_ws(B, H, HKV, Sq, Sk, D, causal, backward, device):
    """The workspace (uint8) of the few-head split forms when they apply to this shape, else None."""
    nb = ctypes.c_int64(0)
    rc = _C.lib().pt_attn_split_plan(B, H, HKV, Sq, Sk, D, int(bool(causal)), int(backward), ctypes.byref(nb))
    _C.check(min(rc, 0), "pt_attn_split_plan")
    return torch.empty(nb.value, dtype=torch.uint8, device=device) if rc == 1 else None


def attn_delta(dout, out, delta=None):
    """delta[b, h, q] = sum_d dO * O  (f32 [B, H, Sq]) for the backward (FA2 'D'); into `delta` (a
    dense or row-strided [B, H, Sq] f32 tensor) when given."""
    B, Sq, H, D = out.shape
    if delta is None:
        delta = torch.empty(B, H, Sq, dtype=torch.float32, device=out.device)
    ld = _lse_ld(delta, B, H, Sq, "delta")
    rc = _C.lib().pt_attn_bwd_delta(_ptr(dout), _str3(dout), _ptr(out), _str3(out), _ptr(delta), B, H, Sq, D, ld,
                                    _C.stream_ptr(out.device))
    _C.check(rc, "pt_attn_bwd_delta")
    return delta


def attn_bwd_part(dout, q, k, v, lse, delta, scale, causal, dq=None, dk=None, dv=None, grad_f32=True):
    """Only dQ (dk = dv = None) or only dK / dV (dq = None) of one attention block, accumulated into the
    given f32 (grad_f32) or stored into bf16 tensors (pt_attn_bwd_part); lse / delta: the queries'
    rows (f32 [B, H, Sq], any row stride shared by both)."""
    B, Sq, H, D = q.shape
    Sk, HKV = k.shape[1], k.shape[2]
    parts = (1 if dq is not None else 0) | (2 if dk is not None else 0)
    _req(parts in (1, 2) and (dk is None) == (dv is None), "attn_bwd_part: dq alone, or dk and dv")
    ld = _lse_ld(lse, B, H, Sq)
    _req(_lse_ld(delta, B, H, Sq, "delta") == ld, "attn_bwd_part: delta and lse rows must share a stride")
    z = _C.i64arr([0, 0, 0])
    rc = _C.lib().pt_attn_bwd_part(_ptr(q), _str3(q), _ptr(k), _str3(k), _ptr(v), _str3(v), _ptr(dout), _str3(dout),
                                   _ptr(lse), _ptr(delta), _ptr(dq), _str3(dq) if dq is not None else z, _ptr(dk),
                                   _str3(dk) if dk is not None else z, _ptr(dv), _str3(dv) if dv is not None else z,
                                   B, H, HKV, Sq, Sk, D, float(scale), int(bool(causal)), int(bool(grad_f32)), ld,
                                   parts, _C.stream_ptr(q.device))
    _C.check(rc, "pt_attn_bwd_part")


def attn_bwd(dout, q, k, v, out, lse, scale, causal, dq=None, dk=None, dv=None, grad_f32=False, delta=None,
             rope=None):
    """rope = (cos, sin) [S, d] bf16 tables: dq / dk are stored rotated back by -theta (the RoPE
    backward fused into the attention backward; positions = sequence index)."""
    B, Sq, H, D = q.shape
    Sk, HKV = k.shape[1], k.shape[2]
    if not grad_f32 and _attn_off_block(causal, Sq, Sk, lse, B, H) and \
            (delta is None or _lse_ld(delta, B, H, Sq, "delta") == Sq):
        Sp = _attn_padded_len(Sq)
        lsep = torch.full((B, H, Sp), float("inf"), dtype=torch.float32, device=q.device)
        lsep[:, :, :Sq] = lse
        dlp = None
        if delta is not None:
            dlp = torch.zeros(B, H, Sp, dtype=torch.float32, device=q.device)
            dlp[:, :, :Sq] = delta
        rp = None
        if rope is not None:   # tables long enough for the padded rows (their values are never used)
            rp = tuple(t if t.shape[0] >= Sp else _pad_seq(t.unsqueeze(0), Sp)[0] for t in rope)
        dqp, dkp, dvp, dlt = attn_bwd(_pad_seq(dout, Sp), _pad_seq(q, Sp), _pad_seq(k, Sp), _pad_seq(v, Sp),
                                      _pad_seq(out, Sp), lsep, scale, True, delta=dlp, rope=rp)
        res = []
        for given, got in ((dq, dqp), (dk, dkp), (dv, dvp)):
            if given is None:
                res.append(got[:, :Sq].contiguous())
            else:
                given.copy_(got[:, :Sq])
                res.append(given)
        return res[0], res[1], res[2], dlt[:, :, :Sq]
    lib = _C.lib()
    fuse_delta = delta is None and not grad_f32 and out.dtype == BF16 and SW.fuse_delta != 0
    if delta is None and not fuse_delta:
        ld0 = _lse_ld(lse, B, H, Sq)
        delta = attn_delta(dout, out, torch.empty(B, H, ld0, dtype=torch.float32, device=q.device)[:, :, :Sq]
                           if ld0 != Sq else None)
    if delta is not None:
        _req(_lse_ld(delta, B, H, Sq, "delta") == _lse_ld(lse, B, H, Sq), "attn_bwd: delta and lse rows must share a stride")
    gdt = torch.float32 if grad_f32 else BF16
    if dq is None:
        dq = (torch.zeros if grad_f32 else torch.empty)(B, Sq, H, D, dtype=gdt, device=q.device)
    if dk is None:
        dk = (torch.zeros if grad_f32 else torch.empty)(B, Sk, HKV, D, dtype=gdt, device=q.device)
    if dv is None:
        dv = (torch.zeros if grad_f32 else torch.empty)(B, Sk, HKV, D, dtype=gdt, device=q.device)
    rc_cos = rc_sin = None
    rstride = 0
    if rope is not None:
        rc_cos, rc_sin = rope
        _req(rc_cos.dtype == BF16 and rc_sin.dtype == BF16 and rc_cos.stride(-1) == 1 and rc_cos.shape[0] >= Sq,
             "attn_bwd rope tables: bf16 [S, d]")
        _req(rc_sin.stride(0) == rc_cos.stride(0), "attn_bwd rope tables share a stride")
        rstride = rc_cos.stride(0)
    ld = _lse_ld(lse, B, H, Sq)
    if fuse_delta:   # D = rowsum(dO * O) inside the dQ kernel (no separate pass)
        _req(out.shape == q.shape, "attn_bwd: out must be [B, Sq, H, D]")
        _req(ld == Sq, "attn_bwd: the fused-delta form takes a dense lse")
        delta = torch.empty(B, H, Sq, dtype=torch.float32, device=q.device)
        ws = _attn_split_ws(B, H, HKV, Sq, Sk, D, causal, 1, q.device)
        if ws is not None:   # few heads (a TP shard): split work items + reduce passes
            rc = lib.pt_attn_bwd_split(_ptr(q), _str3(q), _ptr(k), _str3(k), _ptr(v), _str3(v), _ptr(out), _str3(out),
                                       _ptr(dout), _str3(dout), _ptr(lse), _ptr(delta), _ptr(dq), _str3(dq), _ptr(dk),
                                       _str3(dk), _ptr(dv), _str3(dv), B, H, HKV, Sq, Sk, D, float(scale),
                                       int(bool(causal)), _ptr(rc_cos), _ptr(rc_sin), rstride, _ptr(ws), ws.numel(),
                                       _C.stream_ptr(q.device))
            _C.check(rc, "pt_attn_bwd_split")
            return dq, dk, dv, delta
        rc = lib.pt_attn_bwd_fused_delta(_ptr(q), _str3(q), _ptr(k), _str3(k), _ptr(v), _str3(v), _ptr(out), _str3(out),
                                         _ptr(dout), _str3(dout), _ptr(lse), _ptr(delta), _ptr(dq), _str3(dq), _ptr(dk),
                                         _str3(dk), _ptr(dv), _str3(dv), B, H, HKV, Sq, Sk, D, float(scale),
                                         int(bool(causal)), _ptr(rc_cos), _ptr(rc_sin), rstride, ld,
                                         _C.stream_ptr(q.device))
        _C.check(rc, "pt_attn_bwd_fused_delta")
        return dq, dk, dv, delta
    rc = lib.pt_attn_bwd(_ptr(q), _str3(q), _ptr(k), _str3(k), _ptr(v), _str3(v), _ptr(dout), _str3(dout),
                         _ptr(lse), _ptr(delta), _ptr(dq), _str3(dq), _ptr(dk), _str3(dk), _ptr(dv), _str3(dv),
                         B, H, HKV, Sq, Sk, D, float(scale), int(bool(causal)), int(bool(grad_f32)),
                         _ptr(rc_cos), _ptr(rc_sin), rstride, ld, _C.stream_ptr(q.device))
    _C.check(rc, "pt_attn_bwd")
    return dq, dk, dv, delta
