"""Sequence parallelism for the TP group: the residual stream sharded by token rows between blocks.

The reference keeps every TP rank's residual stream whole: the RMSNorms, the residual adds and the
row-parallel all-reduces (tp_communications.py:35-49, ReduceFromModelParallelRegion) all work on the
full [B*S, H] activation on every rank (model.py:204-209 after tensor_parallel.py:9-52).  Here, with
tp > 1, each rank holds only its T / tp token rows between the TP blocks (Megatron-style sequence
parallelism): a row-parallel output is reduce-scattered onto the shards instead of all-reduced (the
same sum, each rank keeping its rows), a column-parallel input is all-gathered from the shards
(the same replicated tensor the reference feeds it), and the norms / residual adds touch T / tp rows
per rank.  The values every rank's GEMMs see are the reference's; the communication volume is the
all-reduce's (an all-reduce IS a reduce-scatter + all-gather); only the norm weights' gradients
change hands (summed over the tp group, functional._sp_sum_partials).

Entry / exit as the zig-zag CP residual (context_parallel.enable_zigzag_residual): a forward hook on
the embedding keeps this rank's rows of its (all-reduced, replicated) output, a pre-hook on the final
norm all-gathers them back, so Llama.forward and the logits are unchanged.  Shard = token rows
[r T/tp, (r + 1) T/tp) of the flattened batch, viewed [B, S/tp, H] (a reshape of those rows, not a
slice of every sequence).  A batch whose S does not divide by tp runs unsharded (the entry hook
decides per forward; the layers and the exit follow it).

Enabled by apply_tensor_parallel at tp > 1 when neither context nor pipeline parallelism is on (their
own layouts / stage shapes are not sharded this way) -- switch `tp_sp` (PICOTRON_TP_SP=0: the
reference's replicated stream, A/B only).
"""
import torch

from .. import functional as FN
from .. import process_group_manager as pgm
from ..switches import S as SW

_STATE = {"local_len": 0}   # this forward's shard length (S / tp), 0 = unsharded


def local_len():
    return _STATE["local_len"]


def sp_supported():
    m = pgm.current()
    return m.tp_world_size > 1 and m.cp_world_size == 1 and m.pp_world_size == 1 and SW.tp_sp != 0


class ScatterToSequenceRegion(torch.autograd.Function):
    """[B, S, H] replicated -> this rank's [B, S/tp, H] token rows; backward: the all-gather of the
    shards' gradients (every rank's upstream -- the vocab-parallel embedding -- needs all rows)."""

    @staticmethod
    def forward(ctx, x):
        tp = FN.TPContext.current()
        B, S, H = x.shape
        n = B * S // tp.world_size
        ctx.shape = x.shape
        return x.reshape(B * S, H)[tp.rank * n:(tp.rank + 1) * n].clone().view(B, S // tp.world_size, H)

    @staticmethod
    def backward(ctx, g):
        tp = FN.TPContext.current()
        B, S, H = ctx.shape
        return tp.all_gather_rows(g.reshape(-1, H)).view(B, S, H)


class GatherFromSequenceRegion(torch.autograd.Function):
    """[B, S/tp, H] shards -> [B, S, H] on every rank; backward: this rank's rows of the (replicated)
    gradient -- the final norm and the lm_head's input gradient are the same on every tp rank."""

    @staticmethod
    def forward(ctx, x):
        tp = FN.TPContext.current()
        B, Sl, H = x.shape
        ctx.n = B * Sl
        return tp.all_gather_rows(x.reshape(-1, H)).view(B, Sl * tp.world_size, H)

    @staticmethod
    def backward(ctx, g):
        tp = FN.TPContext.current()
        B, S, H = g.shape
        n = ctx.n
        return g.reshape(B * S, H)[tp.rank * n:(tp.rank + 1) * n].contiguous().view(B, S // tp.world_size, H)


def _entry_hook(module, inputs, output):
    tp = FN.TPContext.current().world_size
    if output.dim() == 3 and output.shape[1] % tp == 0:
        _STATE["local_len"] = output.shape[1] // tp
        return ScatterToSequenceRegion.apply(FN._plain(output))
    _STATE["local_len"] = 0
    return output


def _exit_hook(module, args):
    x = args[0]
    if x.dim() == 3 and _STATE["local_len"] and x.shape[1] == _STATE["local_len"]:
        _STATE["local_len"] = 0
        return (GatherFromSequenceRegion.apply(FN._plain(x)),) + tuple(args[1:])
    return None


def enable_sequence_parallel(model):
    """Shard `model`'s residual stream over the tp group between its TP blocks (see the module
    docstring).  Returns True when enabled."""
    if not sp_supported() or getattr(model, "_pt_sequence_parallel", False):
        return getattr(model, "_pt_sequence_parallel", False)
    from ..model import DecoderLayer
    for name, mod in model.named_modules():
        leaf = name.rsplit(".", 1)[-1]
        if isinstance(mod, DecoderLayer):
            mod.tp_sequence_parallel = True
        elif leaf == "embedding" and not isinstance(mod, torch.nn.Identity):
            mod.register_forward_hook(_entry_hook)
        elif leaf == "final_norm" and not isinstance(mod, torch.nn.Identity):
            mod.register_forward_pre_hook(_exit_hook)
    model._pt_sequence_parallel = True
    return True
