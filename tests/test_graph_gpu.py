"""The HIP-graph launch mode of the tensor-parallel path (train.GraphedTrainStep, bench.py --graph):
a replayed micro-batch must compute exactly what the eager one does.

Both run on a one-rank RCCL group (the one-GPU box), so the collectives inside the captured graph
are real RCCL launches on RCCL's stream with the async fork / join edges the layers issue:
  * the whole training step of a small Llama (train_step vs GraphedTrainStep, AdamW between
    steps, fresh zero_grad(set_to_none=True) each step): losses and weights bit-identical;
  * one micro-batch of TP = 2 shard layers (bench.OneRankTP: every all-gather / reduce-scatter /
    all-reduce an RCCL launch on the one-rank group; the chunked sequence-parallel layout; the
    vocab-parallel cross-entropy): loss and every gradient bit-identical, eager vs replay."""
import math
import os
import types

import pytest
import torch

from tests import _dist

pytestmark = pytest.mark.gpu
CFG = dict(hidden_size=256, intermediate_size=512, num_attention_heads=4, num_key_value_heads=2, vocab_size=512,
           rms_norm_eps=1e-5, rope_theta=10000.0, num_hidden_layers=2, max_position_embeddings=256)


def _step_graph_vs_eager(rank, world):
    os.environ["FLASH_ATTEN"] = "1"
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.model import Llama
    from picotron_amd.optim import AdamW
    from picotron_amd.train import GraphedTrainStep, SyntheticMicroBatchDataLoader, train_step
    pgm.setup_process_group_manager(1, 1, 1, 1)
    cfg = types.SimpleNamespace(**CFG)
    dev = torch.device("cuda", 0)
    runs = {}
    for mode in ("eager", "graph"):
        torch.manual_seed(0)
        with torch.device(dev):
            model = Llama(cfg)
        model.to(torch.bfloat16)
        opt = AdamW(model.parameters(), lr=1e-3)
        loader = SyntheticMicroBatchDataLoader(2, 256, 4, CFG["vocab_size"], dev, seed=7, fresh=True)
        step = GraphedTrainStep(model, loader, dev) if mode == "graph" else None
        losses = []
        from picotron_amd import switches
        # one weight-gradient launch per micro-batch on both sides: a replay repeats one captured
        # micro-batch, so train_step's pairing (tp = 1 only) does not apply to the graphed step
        with switches.override(wgrad_pair=0):
            for _ in range(3):
                opt.zero_grad()
                losses.append(step() if step is not None else train_step(model, loader, dev))
                opt.step()
        torch.cuda.synchronize()
        runs[mode] = (losses, [p.detach().clone() for p in model.parameters()])
        if step is not None:
            assert step.graph is not None
    (le, pe), (lg, pg) = runs["eager"], runs["graph"]
    assert le == lg, (le, lg)
    for a, b in zip(pe, pg):
        assert torch.equal(a, b)


def test_graphed_train_step_equals_eager():
    _dist.run(_step_graph_vs_eager, 1, device="cuda", backend="nccl")


def _tp_graph_vs_eager(rank, world, chunks):
    import bench
    from picotron_amd import functional as FN
    from picotron_amd import process_group_manager as pgm
    from picotron_amd import switches
    from picotron_amd.tensor_parallel import sequence_parallel as SPM
    pgm.setup_process_group_manager(1, 1, 1, 1)
    tp, B, S, H, I, V, L, d = 2, 4, 256, 256, 512, 1024, 2, 64
    nh = nkv = 4 // tp
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)

    def u(o, i):
        return torch.nn.Parameter(((torch.rand(o, i, device=dev, generator=g) * 2 - 1) / math.sqrt(i)).to(torch.bfloat16))
    stack = [[torch.nn.Parameter(torch.ones(H, device=dev, dtype=torch.bfloat16)) for _ in range(2)] +
             [u(nh * d, H), u(nkv * d, H), u(nkv * d, H), u(H, nh * d), u(I // tp, H), u(I // tp, H), u(H, I // tp)]
             for _ in range(L)]
    emb = torch.nn.Parameter(torch.randn(V // tp, H, device=dev, generator=g).to(torch.bfloat16))
    head = u(V // tp, H)
    params = [p for w in stack for p in w] + [emb, head]
    from picotron_amd.model import get_cos_sin
    os.environ["DEVICE"] = "cuda"
    cos, sin = get_cos_sin(S, d, base=10000.0)
    ids = torch.randint(0, V // tp, (B, S), device=dev, generator=g)
    tgt = torch.randint(0, V, (B * S,), device=dev, generator=g)
    loss_buf = torch.zeros((), dtype=torch.float32, device=dev)
    with switches.override(tp_sp_chunks=chunks):
        c = SPM.layout_chunks(B, S, tp)
    assert c == chunks

    def micro_batch():
        x = SPM.ReduceScatterToSequenceRegion.apply(FN.embedding(ids, emb), c)
        for w in stack:
            x = FN.DecoderLayerFunction.apply(x, *w, cos, sin, 1e-5, 0, nh, nkv, d, False, c)
        x = SPM.GatherFromSequenceRegion.apply(x, c)
        lg, stats = FN.lm_head_shard(x.reshape(B * S, H), head)
        assert stats is not None
        full = FN.vp_logits(lg, stats, 0, V, lambda: None)
        loss = FN.cross_entropy(full, tgt)
        loss.backward()
        loss_buf.copy_(loss.detach().float())

    current = FN.TPContext.current
    FN.TPContext.current = staticmethod(lambda: bench.OneRankTP(torch.distributed.group.WORLD, tp))
    try:
        micro_batch()                                   # eager (allocates every .grad)
        torch.cuda.synchronize()
        eager = [loss_buf.clone()] + [p.grad.clone() for p in params]
        assert all(torch.isfinite(t).all() for t in eager)
        for p in params:
            p.grad.zero_()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            micro_batch()                               # warm-up on a side stream, as the capture wants
        torch.cuda.current_stream().wait_stream(side)
        from picotron_amd.train import quiesce_collectives
        quiesce_collectives(dev)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            micro_batch()
        for p in params:
            p.grad.zero_()
        graph.replay()
        torch.cuda.synchronize()
        replay = [loss_buf.clone()] + [p.grad.clone() for p in params]
    finally:
        FN.TPContext.current = current
    for i, (a, b) in enumerate(zip(eager, replay)):
        assert torch.equal(a, b), i


@pytest.mark.parametrize("chunks", [4, 2, 1])   # 4: the layout of bench.py's TP default (mbs 32)
def test_graphed_tp_layers_equal_eager(chunks):
    _dist.run(_tp_graph_vs_eager, 1, chunks, device="cuda", backend="nccl")
