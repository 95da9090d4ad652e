"""Megatron f/g conjugate collectives over the tp group (RCCL on MI355X).

Mirrors picotron/tensor_parallel/tp_communications.py (okoge-kaz/picotron @ 2025-03-02):
CopyToModelParallelRegion (:19-33), ReduceFromModelParallelRegion (:35-49),
GatherFromModelParallelRegion (:51-72), LinearWithAsyncAllReduce (:74-101),
linear_with_all_reduce / linear_with_async_all_reduce (:103-109).  The GEMMs inside the linear
helpers are the gfx950 MFMA kernel (functional.LinearFunction), which always overlaps the dX
all-reduce with the dW GEMM (the async variant's schedule) -- so both helpers share it.
"""
import torch
import torch.distributed as dist

from .. import functional as FN
from .. import process_group_manager as pgm


def split_tensor_along_last_dim(tensor, num_partitions):
    last_dim = tensor.dim() - 1
    assert tensor.size()[last_dim] % num_partitions == 0, f"{tensor.size()[last_dim]} is not divisible by {num_partitions}"
    return torch.split(tensor, tensor.size()[last_dim] // num_partitions, dim=last_dim)


class CopyToModelParallelRegion(torch.autograd.Function):
    """f: identity forward, all-reduce backward."""

    @staticmethod
    def forward(ctx, x):
        return x

    @staticmethod
    def backward(ctx, grad_output):
        m = pgm.current()
        if m.tp_world_size == 1:
            return grad_output
        dist.all_reduce(grad_output, op=dist.ReduceOp.SUM, group=m.tp_group)
        return grad_output


class ReduceFromModelParallelRegion(torch.autograd.Function):
    """g: all-reduce forward, identity backward."""

    @staticmethod
    def forward(ctx, x):
        m = pgm.current()
        if m.tp_world_size == 1:
            return x
        dist.all_reduce(x, op=dist.ReduceOp.SUM, group=m.tp_group)
        return x

    @staticmethod
    def backward(ctx, grad_output):
        return grad_output


class GatherFromModelParallelRegion(torch.autograd.Function):
    """All-gather along the last dim forward, split backward."""

    @staticmethod
    def forward(ctx, x):
        m = pgm.current()
        if m.tp_world_size == 1:
            return x
        x = x.contiguous()
        tensor_list = [torch.empty_like(x) for _ in range(m.tp_world_size)]
        tensor_list[m.tp_rank] = x
        dist.all_gather(tensor_list, x, group=m.tp_group)
        return torch.cat(tensor_list, dim=x.dim() - 1).contiguous()

    @staticmethod
    def backward(ctx, grad_output):
        m = pgm.current()
        if m.tp_world_size == 1:
            return grad_output
        return split_tensor_along_last_dim(grad_output, m.tp_world_size)[m.tp_rank].contiguous()


def linear_with_all_reduce(x, weight, bias):
    out = FN.linear(x, weight, tp_reduce_bwd=True)
    return out if bias is None else out + bias


class LinearWithAsyncAllReduce:
    """tp_communications.py:74-101: dX all-reduce launched before, and overlapped with, dW.
    That is FN.LinearFunction's backward schedule, so `apply` builds the same graph node."""

    @staticmethod
    def apply(input_, weight, bias):
        return linear_with_all_reduce(input_, weight, bias)


def linear_with_async_all_reduce(x, weight, bias):
    return LinearWithAsyncAllReduce.apply(x, weight, bias)
