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

Layout (functional.TPContext.gather_chunk): the flattened [B*S, H] rows are c chunks of B / c whole
sequences, and rank r holds rows [r n, (r + 1) n) of every chunk (n = B S / (c tp)), chunk after
chunk, viewed [B, S/tp, H].  Each chunk's collective is its own, so a layer overlaps chunk j + 1's
all-gather with chunk j's GEMMs and chunk j's reduce-scatter with chunk j + 1's
(functional.DecoderLayerFunction._forward_sp).  c = `layout_chunks`: by default as many chunks (up
to 8) as keep >= 8192 token rows each -- the shard GEMMs at fewer rows cost more than the hidden
collectives save -- so one chunk at mbs 4 or 8 x seq 1024 (rank r then holds rows
[r T/tp, (r+1) T/tp)), two at mbs 16, four at mbs 32; the `tp_sp_chunks` switch forces a count.

Entry / exit, as the zig-zag CP residual (context_parallel.enable_zigzag_residual): the vocab-parallel
embedding's masked lookup is reduce-scattered straight into the shards (the reference all-reduces it,
tensor_parallel.py:270: half the bytes, the same sum); a pre-hook on the final norm all-gathers the
shards back, so Llama.forward and the logits are unchanged.  A batch whose S does not divide by tp runs
unsharded (the entry decides per forward; the layers and the exit follow it).  The decision lives in
one SPState per model (reset by a pre-hook at every model forward), not in module globals.

Enabled by apply_tensor_parallel at tp > 1 when neither context nor pipeline parallelism is on (their
own layouts / stage shapes are not sharded this way) -- switch `tp_sp` (PICOTRON_TP_SP=0: the
reference's replicated stream, A/B only).
"""
import torch

from .. import functional as FN
from .. import process_group_manager as pgm
from ..switches import S as SW


class SPState:
    """One model's sequence-parallel decision for the current forward: the shard length S / tp
    (0 = unsharded) and the layout's chunk count."""

    def __init__(self):
        self.local_len, self.chunks = 0, 1

    def reset(self):
        self.local_len, self.chunks = 0, 1


def sp_supported():
    m = pgm.current()
    return m.tp_world_size > 1 and m.cp_world_size == 1 and m.pp_world_size == 1 and SW.tp_sp != 0


# auto chunking keeps every chunk at least this many token rows: the TP-shard GEMMs lose too much
# below it.  TP = 8 SmolLM-1.7B proxy, replayed ms per micro-batch (profiles/r06/notes_r06.md):
# mbs 8 (8192 rows) 10.2 in one chunk, 15.6 in two; mbs 16: 19.3 / 20.8; mbs 32: 35.7 / 39.0 / 40.5
# in 1 / 2 / 4 chunks -- a chunk of 4096 rows costs half again, one of >= 8192 rows 8-14 %, against the
# (c - 1) / c of the exposed collectives (~5.4 ms per 4096 tokens at 250 GB/s) it takes off the path
CHUNK_MIN_ROWS = 8192
CHUNK_MAX = 8


def layout_chunks(B, S, tp):
    """Chunks of the token-row layout for a [B, S] batch over tp ranks: 0 = not shardable (S % tp),
    else the largest power of two c <= the tp_sp_chunks switch (0 = auto: <= CHUNK_MAX, and each
    chunk >= CHUNK_MIN_ROWS rows) dividing B with (B / c) S % tp == 0."""
    if S % tp:
        return 0
    auto = SW.tp_sp_chunks <= 0
    c = CHUNK_MAX if auto else SW.tp_sp_chunks
    while c > 1 and (B % c or (B // c * S) % tp or (auto and B // c * S < CHUNK_MIN_ROWS)):
        c //= 2
    return c


def shard_rows(t2d, tp, c):
    """This rank's rows of a replicated [T, ...] tensor in the c-chunk layout."""
    T = t2d.shape[0]
    n = T // (c * tp.world_size)
    return torch.cat([t2d[j * T // c + tp.rank * n: j * T // c + (tp.rank + 1) * n] for j in range(c)])


def gather_rows(xr, tp, c):
    """The shards [T/tp, ...] (c-chunk layout) -> the replicated [T, ...] on every rank."""
    out = torch.empty((xr.shape[0] * tp.world_size,) + tuple(xr.shape[1:]), dtype=xr.dtype, device=xr.device)
    FN.wait_all([tp.gather_chunk(out, xr, c, j, async_op=True) for j in range(c)])
    return out


class ScatterToSequenceRegion(torch.autograd.Function):
    """[B, S, H] replicated -> this rank's [B, S/tp, H] token rows (c-chunk layout); backward: the
    all-gather of the shards' gradients (every rank's upstream needs all rows)."""

    @staticmethod
    def forward(ctx, x, c=1):
        tp = FN.TPContext.current()
        B, S, H = x.shape
        ctx.shape, ctx.c = x.shape, c
        return shard_rows(x.reshape(B * S, H), tp, c).view(B, S // tp.world_size, H)

    @staticmethod
    def backward(ctx, g):
        tp = FN.TPContext.current()
        B, S, H = ctx.shape
        return gather_rows(g.reshape(-1, H).contiguous(), tp, ctx.c).view(B, S, H), None


class ReduceScatterToSequenceRegion(torch.autograd.Function):
    """The vocab-parallel embedding's entry into the sharded stream: [B, S, H] partial sums (this
    rank's masked lookup) -> this rank's [B, S/tp, H] rows of their sum over tp (the reference's
    all-reduce, tensor_parallel.py:270, keeping only these rows: half its bytes); backward: the
    all-gather of the shards' gradients (the masked lookup's backward needs every row)."""

    @staticmethod
    def forward(ctx, x, c=1):
        tp = FN.TPContext.current()
        B, S, H = x.shape
        ctx.shape, ctx.c = x.shape, c
        x2 = x.reshape(B * S, H)
        Tc = B * S // c
        out = torch.empty(B * S // tp.world_size, H, dtype=x.dtype, device=x.device)
        FN.wait_all([tp.scatter_chunk(out, x2[j * Tc:(j + 1) * Tc], c, j, async_op=True) for j in range(c)])
        return out.view(B, S // tp.world_size, H)

    @staticmethod
    def backward(ctx, g):
        tp = FN.TPContext.current()
        B, S, H = ctx.shape
        return gather_rows(g.reshape(-1, H).contiguous(), tp, ctx.c).view(B, S, H), None


class GatherFromSequenceRegion(torch.autograd.Function):
    """[B, S/tp, H] shards -> [B, S, H] on every rank; backward: this rank's rows of the (replicated)
    gradient -- the final norm and the lm_head's input gradient are the same on every tp rank."""

    @staticmethod
    def forward(ctx, x, c=1):
        tp = FN.TPContext.current()
        B, Sl, H = x.shape
        ctx.c = c
        return gather_rows(x.reshape(-1, H).contiguous(), tp, c).view(B, Sl * tp.world_size, H)

    @staticmethod
    def backward(ctx, g):
        tp = FN.TPContext.current()
        B, S, H = g.shape
        return shard_rows(g.reshape(B * S, H), tp, ctx.c).view(B, S // tp.world_size, H), None


def enter(state, output, partial=False):
    """The entry of a forward: the embedding's [B, S, H] output (partial=True: this rank's masked
    lookup, not yet summed over tp) -> this rank's shard, or -- S not divisible by tp -- the
    replicated stream (summed here when partial)."""
    tp = FN.TPContext.current()
    c = layout_chunks(output.shape[0], output.shape[1], tp.world_size) if output.dim() == 3 else 0
    if not c:
        state.reset()
        if partial:
            from .tp_communications import ReduceFromModelParallelRegion
            return ReduceFromModelParallelRegion.apply(output)
        return output
    state.local_len, state.chunks = output.shape[1] // tp.world_size, c
    if partial:
        return ReduceScatterToSequenceRegion.apply(FN._plain(output), c)
    return ScatterToSequenceRegion.apply(FN._plain(output), c)


def enable_sequence_parallel(model):
    """Shard `model`'s residual stream over the tp group between its TP blocks (see the module
    docstring).  Returns True when enabled."""
    if not sp_supported() or getattr(model, "_pt_sequence_parallel", False):
        return getattr(model, "_pt_sequence_parallel", False)
    from ..model import DecoderLayer
    from .tensor_parallel import VocabParallelEmbedding
    state = SPState()

    def entry_hook(module, inputs, output):
        return enter(state, output)

    def exit_hook(module, args):
        x = args[0]
        if x.dim() == 3 and state.local_len and x.shape[1] == state.local_len:
            c = state.chunks
            state.reset()
            return (GatherFromSequenceRegion.apply(FN._plain(x), c),) + tuple(args[1:])
        return None

    for name, mod in model.named_modules():
        leaf = name.rsplit(".", 1)[-1]
        if isinstance(mod, DecoderLayer):
            mod.tp_sequence_parallel = True
            mod._pt_sp_state = state
        elif isinstance(mod, VocabParallelEmbedding):
            mod._pt_sp_state = state          # its forward reduce-scatters into the shards
        elif leaf == "embedding" and not isinstance(mod, torch.nn.Identity):
            mod.register_forward_hook(entry_hook)
        elif leaf == "final_norm" and not isinstance(mod, torch.nn.Identity):
            mod.register_forward_pre_hook(exit_hook)
    # a forward that raised between the entry and the exit leaves no stale shard length behind
    model.register_forward_pre_hook(lambda module, args: state.reset())
    model._pt_sequence_parallel = True
    model._pt_sp_state = state
    return True
