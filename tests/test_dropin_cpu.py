"""The drop-in boundary on the host (CPU): the `picotron` overlay (dropin/picotron) that lets the
reference's unchanged train.py import the hot path, the HipLogits dispatch of F.cross_entropy, and
the process grid's group families."""
import os
import subprocess
import sys

import pytest
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REFERENCE = os.environ.get("PICOTRON_REFERENCE", "/root/reference")


def _run(code, with_reference):
    path = [os.path.join(ROOT, "dropin")] + ([REFERENCE] if with_reference else [])
    env = dict(os.environ, PYTHONPATH=os.pathsep.join(path), DEVICE="cpu", LOCAL_RANK="0")
    env.pop("PICOTRON_REFERENCE", None)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd="/tmp", env=env, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_overlay_aliases_the_hot_path_modules():
    """`import picotron.X` yields picotron_amd's module OBJECT for every replaced module, so module
    globals (process_group_manager) are shared with whoever imports the reference's names."""
    out = _run("""
import importlib, picotron
names = ["process_group_manager", "model", "tensor_parallel.tensor_parallel", "tensor_parallel.tp_communications",
         "context_parallel.context_parallel", "context_parallel.cp_communications",
         "data_parallel.data_parallel", "data_parallel.bucket", "pipeline_parallel.pp_communications"]
for n in names:
    assert importlib.import_module("picotron." + n) is importlib.import_module("picotron_amd." + n), n
import picotron.process_group_manager as pgm
m = pgm.setup_process_group_manager(1, 1, 1, 1)
import picotron_amd.process_group_manager as apgm
assert apgm.process_group_manager is m
from picotron.tensor_parallel.tensor_parallel import apply_tensor_parallel, ColumnParallelLinear, RowParallelLinear
from picotron.context_parallel.context_parallel import (apply_context_parallel, ring_attention, update_out_and_lse,
    ring_attention_forward, ring_attention_backward, update_rope_for_context_parallel)
from picotron.model import (Llama, DecoderLayer, Attention, MLP, TritonRMSNorm, LlamaRMSNorm, Embedding,
    get_cos_sin, apply_rotary_pos_emb, flash_attention)
from picotron.data_parallel.data_parallel import DataParallelBucket, DataParallelNaive
print("ok")
""", with_reference=False)
    assert out.strip().endswith("ok")


@pytest.mark.skipif(not os.path.isdir(os.path.join(REFERENCE, "picotron")), reason="no reference checkout here")
def test_overlay_serves_the_reference_callers():
    """With the checkout on the path, the modules the overlay does not replace (pipeline engine,
    checkpoint init, utils) come from the checkout and see the build's process-group global; the
    reference's PipelineParallel wraps the build's Llama (train.py:174-186 order) on a 1-rank grid."""
    out = _run("""
import types, torch, torch.distributed as dist
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % __import__("random").randint(20000, 40000),
                        rank=0, world_size=1)
import picotron, picotron.process_group_manager as pgm
from picotron.pipeline_parallel.pipeline_parallel import PipelineParallel
import picotron.utils as U
import picotron.checkpoint as ck
assert PipelineParallel.__module__ == "picotron.pipeline_parallel.pipeline_parallel"
import picotron.pipeline_parallel.pipeline_parallel as PPm
import picotron_amd.pipeline_parallel.pp_communications as PC
assert PPm.pipeline_communicate is PC.pipeline_communicate
assert PPm.bidirectional_pipeline_communicate is PC.bidirectional_pipeline_communicate
assert U.pgm is pgm and ck.pgm is pgm
pgm.setup_process_group_manager(tp_size=1, cp_size=1, pp_size=1, dp_size=1)
from picotron.model import Llama
from picotron.tensor_parallel.tensor_parallel import apply_tensor_parallel
cfg = types.SimpleNamespace(hidden_size=128, intermediate_size=256, num_attention_heads=2, num_key_value_heads=2,
    vocab_size=256, rms_norm_eps=1e-5, rope_theta=10000.0, num_hidden_layers=2, max_position_embeddings=64)
m = Llama(cfg)
m = apply_tensor_parallel(m)
pp = PipelineParallel(m, cfg)
assert list(pp.decoder_layers.keys()) == ["0", "1"] and pp.final_proj is m.final_proj
print("ok")
""", with_reference=True)
    assert out.strip().endswith("ok")


def test_hip_logits_route_f_cross_entropy(monkeypatch):
    """F.cross_entropy on the lm_head output (or its view / [B, V, S] transpose) calls
    functional.cross_entropy; other ops return plain tensors."""
    from picotron_amd import functional as FN
    seen = []

    def fake(input, target, reduction="mean", ignore_index=-100):
        seen.append((type(input), tuple(input.shape), tuple(target.shape)))
        return F.cross_entropy(input, target, reduction=reduction, ignore_index=ignore_index)
    monkeypatch.setattr(FN, "cross_entropy", fake)
    x = torch.randn(2, 3, 5, requires_grad=True)
    lg = FN.as_logits(x * 2)
    t = torch.randint(0, 5, (2, 3))
    l1 = F.cross_entropy(lg.view(-1, 5), t.reshape(-1))
    l2 = F.cross_entropy(lg.transpose(1, 2), t)
    assert [s[0] for s in seen] == [torch.Tensor, torch.Tensor]          # plain tensors reach the kernel path
    assert seen[0][1:] == ((6, 5), (6,)) and seen[1][1:] == ((2, 5, 3), (2, 3))
    assert torch.allclose(l1, l2)
    assert type(lg * 1) is torch.Tensor and type(lg.view(6, 5)) is FN.HipLogits
    l1.backward()
    assert x.grad is not None and x.grad.shape == x.shape
    # not on picotron's path: torch's own op on the plain tensors
    ls = F.cross_entropy(lg.view(-1, 5), t.reshape(-1), label_smoothing=0.1)
    assert type(ls) is torch.Tensor
    assert torch.allclose(ls, F.cross_entropy((x * 2).detach().view(-1, 5), t.reshape(-1), label_smoothing=0.1))
    assert len(seen) == 2


def test_hip_hidden_routes_f_linear(monkeypatch):
    """The final norm's output (HipHidden): torch's nn.Linear on it -- the lm_head checkpoint.py:89-90
    installs, which PipelineParallel.forward calls directly (pipeline_parallel.py:63) -- goes to
    functional.lm_head_linear and returns HipLogits; every other op returns plain tensors."""
    from picotron_amd import functional as FN
    seen = []

    def fake(x, w):
        seen.append((type(x), tuple(x.shape), tuple(w.shape)))
        return x @ w.t()
    monkeypatch.setattr(FN, "lm_head_linear", fake)
    h = FN.as_hidden(torch.randn(2, 3, 8, requires_grad=True))
    lin = torch.nn.Linear(8, 5, bias=False)
    y = lin(h)
    assert isinstance(y, FN.HipLogits) and seen == [(torch.Tensor, (2, 3, 8), (5, 8))]
    assert torch.allclose(y.as_subclass(torch.Tensor), h.as_subclass(torch.Tensor) @ lin.weight.t())
    assert type(h * 2) is torch.Tensor and type(h.view(6, 8)) is torch.Tensor
    y.sum().backward()
    assert lin.weight.grad is not None


def test_cross_entropy_argument_forms():
    from picotron_amd import functional as FN
    with pytest.raises(ValueError):
        FN.cross_entropy(torch.zeros(2, 5, 3), torch.zeros(3, 2, dtype=torch.long))
    with pytest.raises(ValueError):
        FN.cross_entropy(torch.zeros(4, 5), torch.zeros(4, 2, dtype=torch.long))
    with pytest.raises(ValueError):
        FN.cross_entropy(torch.zeros(4, 5), torch.zeros(4, dtype=torch.long), reduction="average")


@pytest.mark.parametrize("dims", [(2, 1, 2, 2), (1, 2, 2, 2), (2, 2, 1, 2), (1, 1, 4, 2)])
def test_axis_groups_match_the_reference_enumeration(dims):
    """process_group_manager.py:18-23's comprehensions, restated, against the permute/reshape form."""
    from picotron_amd.process_group_manager import CP, DP, PP, TP, _axis_groups
    dp, pp, cp, tp = dims
    g = torch.arange(dp * pp * cp * tp).view(dp, pp, cp, tp)
    want = {
        "tp": [g[d, p, c, :].tolist() for d in range(dp) for p in range(pp) for c in range(cp)],
        "cp": [g[d, p, :, t].tolist() for d in range(dp) for p in range(pp) for t in range(tp)],
        "pp": [g[d, :, c, t].tolist() for d in range(dp) for c in range(cp) for t in range(tp)],
        "dp": [g[:, p, c, t].tolist() for p in range(pp) for c in range(cp) for t in range(tp)],
        "cp_dp": [g[:, p, :, t].flatten().tolist() for p in range(pp) for t in range(tp)],
        "pp_dp": [g[:, :, c, t].flatten().tolist() for c in range(cp) for t in range(tp)],
    }
    axes = {"tp": (TP,), "cp": (CP,), "pp": (PP,), "dp": (DP,), "cp_dp": (DP, CP), "pp_dp": (DP, PP)}
    for name, ax in axes.items():
        assert _axis_groups(g, ax) == want[name], name


def test_plan_buckets_rule():
    from picotron_amd.data_parallel.bucket import plan_buckets
    places, totals = plan_buckets([3, 4, 10, 2, 2, 1, 0, 9], 8)
    assert places == [(0, 3, 0), (3, 7, 0), (0, 10, 1), (0, 2, 2), (2, 4, 2), (4, 5, 2), (5, 5, 2), (0, 9, 3)]
    assert totals == [7, 10, 5, 9]
