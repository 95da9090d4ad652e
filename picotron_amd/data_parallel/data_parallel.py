"""Data parallelism: naive per-parameter and bucketed gradient all-reduce over cp_dp_group.

Mirrors picotron/data_parallel/data_parallel.py (okoge-kaz/picotron @ 2025-03-02):
DataParallelNaive (:10-60) and DataParallelBucket (:62-170) with the same interface
(`require_backward_grad_sync`, `no_sync()`, `reset()`, `backward(...)` for the PP engine,
`bucket_manager`), fp32 `main_grad` accumulation and the post-backward callback that waits for the
buckets and sets `p.grad = main_grad.to(p.dtype)` (:153-165).

Two gradient paths feed the buckets:
  * parameters whose gradient comes from autograd (the embedding) use the reference's hook on the
    gradient accumulator (:93-144): main_grad += grad; grad = None;
  * parameters consumed by the fused kernels (every projection and norm weight) have their
    gradient written into main_grad by the kernel epilogue itself; the kernels then call
    `param._pt_grad_ready`, which does the reference hook's remaining work (queue the
    post-backward callback, mark the parameter ready); `param._pt_grad_sync()` tells them whether
    this backward all-reduces at all (outside `no_sync`), so the norm weights' column sums can be
    batched at the end of the micro-batches that do not.
"""
import contextlib

import torch
import torch.distributed as dist
from torch import nn
from torch.autograd import Variable

from .. import process_group_manager as pgm
from .bucket import BucketManager


def _cp_averaged(module):
    """The wrapper averages gradients over cp_dp_group, cp ranks included: the residual stream of a
    context-parallel model may then stay in the zig-zag layout (context_parallel.enable_zigzag_residual)."""
    if pgm.current().cp_world_size > 1:
        from ..context_parallel.context_parallel import enable_zigzag_residual
        enable_zigzag_residual(module)


class DataParallelNaive(nn.Module):
    """data_parallel.py:10-60: all-reduce (mean over cp_dp_group) every parameter's gradient once it
    is final for the backward.  Two triggers, as in DataParallelBucket: autograd's post-accumulate
    hook for gradients autograd accumulates, and `param._pt_grad_ready` for the weights whose
    gradient a fused kernel wrote itself (those never reach an AccumulateGrad node).
    (The reference's hook receives the parameter and all-reduces the parameter tensor, not its
    .grad -- a no-op on replicated weights; this averages the gradient, the documented intent.)"""

    def __init__(self, module):
        super().__init__()
        self.module = module
        self.require_backward_grad_sync = True
        _cp_averaged(module)
        for p in self.module.parameters():
            if p.requires_grad:
                p.register_post_accumulate_grad_hook(self._allreduce_grads)
                p._pt_grad_ready = self._allreduce_grads
                p._pt_grad_sync = self._sync_wanted

    def forward(self, *inputs, **kwargs):
        return self.module(*inputs, **kwargs)

    def _sync_wanted(self):
        """Whether this backward all-reduces (the fused kernels then report each gradient at once)."""
        return self.require_backward_grad_sync

    def _allreduce_grads(self, param):
        if self.require_backward_grad_sync and param.grad is not None:
            m = pgm.current()
            dist.all_reduce(param.grad, op=dist.ReduceOp.SUM, group=m.cp_dp_group)
            param.grad /= m.cp_dp_world_size

    @contextlib.contextmanager
    def no_sync(self):
        self.require_backward_grad_sync = False
        yield
        self.require_backward_grad_sync = True


class DataParallelBucket(nn.Module):
    def __init__(self, module, bucket_cap_mb=25, grad_type=torch.float32):
        super().__init__()
        self.module = module
        self.require_backward_grad_sync = True
        grad_size = 2 if grad_type == torch.bfloat16 else 4
        bucket_size = bucket_cap_mb * 1024 * 1024 // grad_size
        self.bucket_manager = BucketManager(module.parameters(), pgm.current().cp_dp_group, bucket_size, grad_type)
        self.register_backward_hook()
        _cp_averaged(module)
        self._post_backward_callback_set = False

    def forward(self, *inputs, **kwargs):
        return self.module(*inputs, **kwargs)

    def backward(self, input_tensor, output_tensor, output_tensor_grad):
        return self.module.backward(input_tensor, output_tensor, output_tensor_grad)

    def register_backward_hook(self):
        self.grad_accs = []
        for param in self.module.parameters():
            if param.requires_grad:
                param_tmp = param.expand_as(param)
                grad_acc_fn = param_tmp.grad_fn.next_functions[0][0]
                grad_acc_fn.register_hook(self._make_param_hook(param))
                self.grad_accs.append(grad_acc_fn)
                param._pt_grad_ready = self._fused_grad_ready
                param._pt_grad_sync = self._sync_wanted

    def _ready(self, param):
        if self.require_backward_grad_sync:
            if not self._post_backward_callback_set:
                Variable._execution_engine.queue_callback(self._post_backward)
                self._post_backward_callback_set = True
            self.bucket_manager.mark_param_as_ready(param)

    def _make_param_hook(self, param):
        def param_hook(*unused):
            # A fused kernel returns no gradient for its weights (it has written main_grad
            # itself and called _fused_grad_ready); the accumulator node still runs, with grad None.
            if param.requires_grad and param.grad is not None:
                param.main_grad.add_(param.grad.data)
                param.grad = None
                self._ready(param)
        return param_hook

    def _fused_grad_ready(self, param):
        self._ready(param)

    def _sync_wanted(self):
        return self.require_backward_grad_sync

    @contextlib.contextmanager
    def no_sync(self):
        self.require_backward_grad_sync = False
        yield
        self.require_backward_grad_sync = True

    def _post_backward(self):
        self.bucket_manager.wait()
        self._post_backward_callback_set = False
        for p in self.module.parameters():
            if p.requires_grad:
                p.grad = p.main_grad.to(p.dtype)

    def reset(self):
        self.bucket_manager.reset()
