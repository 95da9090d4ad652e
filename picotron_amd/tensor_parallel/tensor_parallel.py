"""Megatron 1-D tensor parallelism: Column / Row parallel linears and the vocab-parallel embedding.

Mirrors picotron/tensor_parallel/tensor_parallel.py (okoge-kaz/picotron @ 2025-03-02):
apply_tensor_parallel (:9-52), ColumnParallelLinear (:54-123), RowParallelLinear (:125-189),
VocabParallelEmbedding (:191-270) -- same constructors, shard shapes ([out/tp, in] and
[out, in/tp]), master-weight initialisation and split, forward semantics.  The GEMMs are the gfx950
MFMA kernel; the collectives are RCCL over xGMI.  Inside a fused DecoderLayer the shards are read
directly by functional.DecoderLayerFunction, which sums the q/k/v (and gate/up) dX inside the GEMM
and all-reduces once per block instead of once per linear (exact by linearity).
"""
import math
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import functional as FN
from .. import process_group_manager as pgm
from .sequence_parallel import enable_sequence_parallel
from .tp_communications import (GatherFromModelParallelRegion, ReduceFromModelParallelRegion,
                                linear_with_all_reduce, linear_with_async_all_reduce)


def apply_tensor_parallel(model):
    def _replace_module(_module, _linear_proj_name, _style, args={}):
        assert _style in ["column", "row", "vocab"]
        linear_layer = getattr(_module, _linear_proj_name)
        if _style == "column":
            new = ColumnParallelLinear(in_features=linear_layer.in_features, out_features=linear_layer.out_features,
                                       bias=linear_layer.bias is not None, gather_output=args.get("gather_output", False))
        elif _style == "row":
            new = RowParallelLinear(in_features=linear_layer.in_features, out_features=linear_layer.out_features,
                                    bias=linear_layer.bias is not None)
        else:
            new = VocabParallelEmbedding(num_embeddings=linear_layer.num_embeddings,
                                         embedding_dim=linear_layer.embedding_dim)
        if getattr(linear_layer, "_pt_lm_head", False):   # keep F.cross_entropy on the HIP kernel
            new._pt_lm_head = True
        setattr(_module, _linear_proj_name, new)

    mapping = [
        ("attention", "q_proj", "column"),
        ("attention", "k_proj", "column"),
        ("attention", "v_proj", "column"),
        ("attention", "out_proj", "row"),
        ("mlp", "up_proj", "column"),
        ("mlp", "gate_proj", "column"),
        ("mlp", "down_proj", "row"),
    ]
    for layer in model.decoder_layers:
        for module_name, linear_proj_name, style in mapping:
            _replace_module(getattr(layer, module_name), linear_proj_name, style)
    _replace_module(model, "embedding", "vocab")
    _replace_module(model, "final_proj", "column", args={"gather_output": True})
    # MI355X-first addition: the residual stream sharded by token rows between the TP blocks
    # (sequence_parallel.py: same values, the norms / adds on T / tp rows per rank)
    enable_sequence_parallel(model)
    return model


class ColumnParallelLinear(torch.nn.Module):
    """Y_i = X W_i^T (+ b_i); W_i = rows [tp_rank * out/tp, (tp_rank+1) * out/tp) of the master W."""

    def __init__(self, in_features: int, out_features: int, bias: bool = False, gather_output: bool = False,
                 async_all_reduce: bool = False) -> None:
        super().__init__()
        m = pgm.current()
        self.tp_world_size, self.tp_rank = m.tp_world_size, m.tp_rank
        self.in_features, self.out_features = in_features, out_features
        assert out_features % self.tp_world_size == 0, "Hidden dimension must be divisible by the tensor parallel world size"
        self.output_size_per_partition = out_features // self.tp_world_size
        self.gather_output = gather_output
        self.async_all_reduce = async_all_reduce
        self.weight = nn.Parameter(torch.empty(self.output_size_per_partition, self.in_features))
        if bias:
            self.bias = nn.Parameter(torch.zeros(self.output_size_per_partition))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        master_weight = torch.empty(self.out_features, self.in_features, dtype=self.weight.dtype,
                                    device=self.weight.device, requires_grad=False)
        bound = math.sqrt(1 / master_weight.size(1))
        torch.nn.init.uniform_(master_weight, -bound, bound)
        weight_list = torch.split(master_weight, self.output_size_per_partition, dim=0)
        self.weight.data = weight_list[self.tp_rank].contiguous()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = FN._plain(x)
        if (self.gather_output and getattr(self, "_pt_lm_head", False) and self.tp_world_size > 1
                and self.bias is None and x.dtype == torch.bfloat16 and self.weight.dtype == torch.bfloat16
                and FN.vp_ce_shape_ok(x.numel() // x.shape[-1], self.output_size_per_partition, x.shape[-1])):
            # the lm_head: F.cross_entropy on the vocab shards, the logits gathered only if something
            # else reads them (functional.vp_logits)
            y, stats = FN.lm_head_shard(x, self.weight)
            if stats is not None:
                return FN.vp_logits(y, stats, self.tp_rank * self.output_size_per_partition, self.out_features,
                                    lambda: GatherFromModelParallelRegion.apply(y))
            return FN.as_logits(GatherFromModelParallelRegion.apply(y))
        if self.async_all_reduce:
            output = linear_with_async_all_reduce(x, self.weight, self.bias)
        else:
            output = linear_with_all_reduce(x, self.weight, self.bias)
        if self.gather_output:
            output = GatherFromModelParallelRegion.apply(output)
        return FN.as_logits(output) if getattr(self, "_pt_lm_head", False) else output


class RowParallelLinear(nn.Module):
    """Y = sum_i X_i W_i^T + b; X_i = the tp_rank-th column block of the (already split) input."""

    def __init__(self, in_features: int, out_features: int, bias: bool):
        super().__init__()
        m = pgm.current()
        self.tp_world_size, self.tp_rank = m.tp_world_size, m.tp_rank
        self.in_features, self.out_features = in_features, out_features
        assert in_features % self.tp_world_size == 0, "Hidden dimension must be divisible by the tensor parallel world size"
        self.input_size_per_partition = in_features // self.tp_world_size
        self.weight = nn.Parameter(torch.empty(self.out_features, self.input_size_per_partition))
        if bias:
            self.bias = nn.Parameter(torch.zeros(self.out_features))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        master_weight = torch.empty(self.out_features, self.in_features, dtype=self.weight.dtype,
                                    device=self.weight.device, requires_grad=False)
        bound = math.sqrt(1 / master_weight.size(1))
        torch.nn.init.uniform_(master_weight, -bound, bound)
        weight_list = torch.split(master_weight, self.input_size_per_partition, dim=1)
        self.weight.data = weight_list[self.tp_rank].contiguous()

    def forward(self, x):
        output = FN.linear(x, self.weight, tp_reduce_fwd=True)
        return output if self.bias is None else output + self.bias


class VocabParallelEmbedding(nn.Module):
    """tensor_parallel.py:191-270: masked lookup into this rank's vocab slice + all-reduce."""

    def __init__(self, num_embeddings: int, embedding_dim: int, padding_idx: Optional[int] = None,
                 max_norm: Optional[float] = None, norm_type: float = 2.0, scale_grad_by_freq: bool = False,
                 sparse: bool = False):
        super().__init__()
        m = pgm.current()
        self.tp_world_size, self.tp_rank = m.tp_world_size, m.tp_rank
        self.num_embeddings, self.embedding_dim = num_embeddings, embedding_dim
        self.padding_idx, self.max_norm, self.norm_type = padding_idx, max_norm, norm_type
        self.scale_grad_by_freq, self.sparse = scale_grad_by_freq, sparse
        self.vocab_start_index, self.vocab_end_index = self._vocab_range_from_global_vocab_size(
            self.num_embeddings, self.tp_rank, self.tp_world_size)
        self.num_embeddings_per_partition = self.vocab_end_index - self.vocab_start_index
        self.weight = nn.Parameter(torch.empty(self.num_embeddings_per_partition, self.embedding_dim))
        self.reset_parameters()

    def _vocab_range_from_global_vocab_size(self, global_vocab_size: int, rank: int, world_size: int):
        assert global_vocab_size % world_size == 0, f"{global_vocab_size} is not divisible by {world_size}"
        per = global_vocab_size // world_size
        return rank * per, rank * per + per

    def reset_parameters(self):
        master_weight = torch.empty(self.num_embeddings, self.embedding_dim, dtype=self.weight.dtype,
                                    device=self.weight.device, requires_grad=False)
        torch.nn.init.normal_(master_weight, mean=0.0, std=1.0)
        weight_list = torch.split(master_weight, self.num_embeddings_per_partition, dim=0)
        self.weight.data = weight_list[self.tp_rank].contiguous()

    def forward(self, x):
        if self.max_norm is not None or self.scale_grad_by_freq or self.sparse:
            raise NotImplementedError("VocabParallelEmbedding: max_norm / scale_grad_by_freq / sparse are not used "
                                      "by picotron")
        # the masked lookup (ids outside this rank's slice -> zero rows, no gradient) in one kernel
        output_parallel = FN.embedding(x, self.weight, self.vocab_start_index, self.vocab_end_index,
                                       self.padding_idx)
        state = getattr(self, "_pt_sp_state", None)
        if state is not None:   # sequence parallelism: reduce-scatter the partial lookups into the shards
            from .sequence_parallel import enter
            return enter(state, output_parallel, partial=True)
        return ReduceFromModelParallelRegion.apply(output_parallel)
