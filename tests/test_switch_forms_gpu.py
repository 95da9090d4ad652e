"""Every measurement switch's non-default form (picotron_amd/switches.py) through the whole GPU path,
against the CPU oracle: a 2-layer Llama (T = 2 x 1024 tokens, H 1024, I 4096 or 2048, d 64, GQA 16 / 8
heads) at shapes where the switched launches are taken -- the fused RoPE / SwiGLU epilogues and the
split-K halves forced on by their thresholds (tools/switch_kernels.py traces, per case, the launches
that differ: profiles/r05/switch_kernels_r05k.txt) -- with loss, logits and every parameter gradient within north_star's bf16
tolerance (norm-relative 2e-2), as test_model_gpu.test_llama_loss_and_grads_match_oracle.  The
oracle (oracle/picotron_oracle.py) runs once for all cases on the same bf16 weights and tokens."""
import types

import pytest
import torch
import torch.nn.functional as F

from oracle import picotron_oracle as O

pytestmark = pytest.mark.gpu
BF = torch.bfloat16
TOL = 2e-2
# two shapes: "a" (I 4096: the split-K halves, the few-tile forms at M = 2048) and "b" (I 2048: the
# SwiGLU-backward dX in K-slices needs (T / 256) (I / 256) <= 64)
CONFIGS = {"a": dict(S=1024, H=1024, I=4096, nh=16, nkv=8, V=2048), "b": dict(S=1024, H=1024, I=2048, nh=16, nkv=8, V=2048)}
# the switch forms the default path does not take (switches.DEFAULTS holds the defaults), each as the
# overrides on top of FORCE; the order is that of tools/switch_kernels.py, which traces what each changes
CASES = [("a", {})] + [("a", {k: v}) for k, v in (
    ("fuse", 0), ("norm_defer", 0), ("ce_stats", 0), ("dual_qkv", 0), ("dual_gu", 0), ("gu_splitk", 0), ("ksplit", 0),
    ("splitk2", 0), ("dual", 0), ("norm_splitk", 0), ("fuse_delta", 0), ("attn_pair", 0), ("gemm_mix", 0))] + [
    ("b", {}), ("b", dict(swiglu_splitk=0)),
]
# (gemm_kh, the K-halves tile 14 for 256x128 launches at K >= 4096, is not reached at shapes this
# small: test_kernels_gpu.py covers gemm_kh = 0 on the launch directly)
# thresholds lowered so that these shapes take the fused / split launches the switches choose between
FORCE = dict(rope_fuse_min_tiles=0, swiglu_fuse_min_tiles=0, splitk2_min=2048)


def case_id(case):
    cfg, kw = case
    return cfg + ("-" + "-".join(f"{k}{v}" for k, v in kw.items()) if kw else "-default")


def rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def build(name):
    """The 2-layer Llama of shape `name` on cuda:0 (bf16, seeded) and its tokens."""
    import os
    os.environ.update(DEVICE="cuda", LOCAL_RANK="0", CONTEXT_PARALLEL="0", FLASH_ATTEN="1")
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.model import Llama
    pgm.setup_process_group_manager(1, 1, 1, 1)
    torch.manual_seed(0)
    c = CONFIGS[name]
    cfg = types.SimpleNamespace(hidden_size=c["H"], intermediate_size=c["I"], num_attention_heads=c["nh"],
                                num_key_value_heads=c["nkv"], vocab_size=c["V"], rms_norm_eps=1e-5, rope_theta=10000.0,
                                num_hidden_layers=2, max_position_embeddings=c["S"])
    with torch.device("cuda"):
        model = Llama(cfg)
    model.to(BF)
    ids = torch.randint(0, c["V"], (2, c["S"] + 1), generator=torch.Generator().manual_seed(3))
    return model, cfg, ids


@pytest.fixture(scope="module")
def models():
    import os
    old = {k: os.environ.get(k) for k in ("DEVICE", "LOCAL_RANK", "CONTEXT_PARALLEL", "FLASH_ATTEN")}
    cache = {}

    def get(name):
        if name not in cache:
            model, cfg, ids = build(name)
            p = {k: v.detach().float().cpu().requires_grad_(True) for k, v in model.named_parameters()}
            cos, sin = O.get_cos_sin(ids.shape[1] - 1, cfg.hidden_size // cfg.num_attention_heads, base=10000.0)
            lr = O.llama_forward(ids[:, :-1], p, dict(vars(cfg)), cos.float(), sin.float(),
                                 norm=O.rmsnorm_flash_semantics)
            loss_r = F.cross_entropy(lr.reshape(-1, cfg.vocab_size), ids[:, 1:].reshape(-1))
            loss_r.backward()
            cache[name] = (model, cfg, ids, dict(loss=loss_r.item(), logits=lr.detach(),
                                                 grads={k: v.grad for k, v in p.items()}))
        return cache[name]
    yield get
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def run(model, cfg, ids):
    from picotron_amd import functional as FN
    model.zero_grad(set_to_none=True)
    logits = model(ids[:, :-1].cuda())
    loss = FN.cross_entropy(logits.view(-1, cfg.vocab_size), ids[:, 1:].reshape(-1).cuda())
    loss.backward()
    torch.cuda.synchronize()
    return loss.float().item(), logits.detach().float().cpu(), {n: q.grad.float().cpu() for n, q in model.named_parameters()}


@pytest.mark.parametrize("case", CASES, ids=[case_id(c) for c in CASES])
def test_switch_form_matches_oracle(models, case):
    from picotron_amd import switches
    name, over = case
    model, cfg, ids, ref = models(name)
    assert all(k in switches.DEFAULTS for k in over)
    with switches.override(**FORCE, **over):
        loss, logits, grads = run(model, cfg, ids)
    assert abs(loss - ref["loss"]) < TOL * abs(ref["loss"]), (over, loss, ref["loss"])
    assert rel(logits, ref["logits"]) < TOL, over
    for n, g in grads.items():
        assert rel(g, ref["grads"][n]) < TOL, (over, n)
