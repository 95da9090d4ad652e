"""Pin the CPU oracle against golden vectors generated from the reference itself
(tests/golden/make_golden.py).  CPU only."""
import math
import os

import pytest
import torch

from oracle import picotron_oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    return torch.load(os.path.join(GOLD, f"{name}.pt"), weights_only=True)


def close(a, b, rtol=1e-5, atol=1e-6):
    torch.testing.assert_close(a.float(), b.float(), rtol=rtol, atol=atol)


@pytest.mark.parametrize("tag", ["f32", "bf16"])
def test_rmsnorm_llama_golden(tag):
    g = load(f"G1_{tag}")
    x = g["x"].clone().requires_grad_(True)
    w = g["w"].clone().requires_grad_(True)
    y = O.rmsnorm_llama(x, w, float(g["eps"]))
    y.backward(g["dy"])
    tol = dict(rtol=0, atol=0) if tag == "f32" else dict(rtol=1e-2, atol=1e-2)
    close(y, g["y"], **({"rtol": 1e-6, "atol": 1e-6} if tag == "f32" else tol))
    close(x.grad, g["dx"], rtol=1e-5 if tag == "f32" else 2e-2, atol=1e-5 if tag == "f32" else 2e-2)
    close(w.grad, g["dw"], rtol=1e-5 if tag == "f32" else 2e-2, atol=1e-5 if tag == "f32" else 5e-2)


def test_cos_sin_tables_golden():
    g = load("G2_tables")
    c, s = O.get_cos_sin(16, 32, base=10000.0)
    assert torch.equal(c, g["cos_16_32"]) and torch.equal(s, g["sin_16_32"])
    c, s = O.get_cos_sin(64, 128)
    assert torch.equal(c, g["cos_64_128_default"]) and torch.equal(s, g["sin_64_128_default"])


def test_rope_golden():
    g = load("G2")
    x = g["x"].clone().requires_grad_(True)
    y = O.apply_rotary_pos_emb(x, g["cos"].float(), g["sin"].float())
    y.backward(g["dy"])
    close(y, g["y"])
    close(x.grad, g["dx"])


def test_attention_golden():
    g = load("G3")
    p = {k: g[k].clone().requires_grad_(True) for k in ["q_proj.weight", "k_proj.weight", "v_proj.weight",
                                                       "out_proj.weight"]}
    x = g["x"].clone().requires_grad_(True)
    y = O.attention(x, p["q_proj.weight"], p["k_proj.weight"], p["v_proj.weight"], p["out_proj.weight"],
                    g["cos"].float(), g["sin"].float(), 4, 2)
    y.backward(g["dy"])
    close(y, g["y"], rtol=1e-4, atol=1e-5)
    close(x.grad, g["dx"], rtol=1e-4, atol=1e-5)
    for k, v in p.items():
        close(v.grad, g[f"grad.{k}"], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("tag", ["f32", "bf16"])
def test_ring_pieces_golden(tag):
    g = load(f"G4_{tag}")
    sc = 1 / math.sqrt(16)
    tol = dict(rtol=1e-5, atol=1e-6) if tag == "f32" else dict(rtol=0, atol=0)
    o_c, l_c = O.ring_attention_forward(g["q"], g["k"], g["v"], sc, True)
    o_f, l_f = O.ring_attention_forward(g["q"], g["k"], g["v"], sc, False)
    close(o_c, g["o_causal"], **tol); close(l_c, g["lse_causal"], **tol)
    close(o_f, g["o_full"], **tol); close(l_f, g["lse_full"], **tol)
    out, lse = O.update_out_and_lse(None, None, o_c, l_c)
    out, lse = O.update_out_and_lse(out, lse, o_f, l_f)
    close(out, g["merged_out"], **tol); close(lse, g["merged_lse"], **tol)
    dq, dk, dv = O.ring_attention_backward(g["dO"], g["q"], g["k"], g["v"], out.to(g["q"].dtype),
                                           lse.squeeze(-1), sc, True)
    close(dq, g["dq"], **tol); close(dk, g["dk"], **tol); close(dv, g["dv"], **tol)


def test_mlp_golden():
    g = load("G5")
    p = {k: g[k].clone().requires_grad_(True) for k in ["up_proj.weight", "gate_proj.weight", "down_proj.weight"]}
    x = g["x"].clone().requires_grad_(True)
    y = O.mlp(x, p["gate_proj.weight"], p["up_proj.weight"], p["down_proj.weight"])
    y.backward(g["dy"])
    close(y, g["y"], rtol=1e-5, atol=1e-6)
    close(x.grad, g["dx"], rtol=1e-5, atol=1e-6)
    for k, v in p.items():
        close(v.grad, g[f"grad.{k}"], rtol=1e-5, atol=1e-6)


def test_decoder_layer_golden():
    g = load("G6")
    names = [k for k in g if not k.startswith("grad.") and k not in ("x", "y", "dy", "dx", "cos", "sin")]
    p = {k: g[k].clone().requires_grad_(True) for k in names}
    x = g["x"].clone().requires_grad_(True)
    y = O.decoder_layer(x, p, g["cos"].float(), g["sin"].float(), 4, 2, 1e-5)
    y.backward(g["dy"])
    close(y, g["y"], rtol=1e-4, atol=1e-5)
    close(x.grad, g["dx"], rtol=1e-4, atol=1e-5)
    for k, v in p.items():
        close(v.grad, g[f"grad.{k}"], rtol=1e-4, atol=1e-4)


def test_cross_entropy_golden():
    g = load("G9")
    logits = g["logits"].clone().requires_grad_(True)
    loss = torch.nn.functional.cross_entropy(logits.view(16, -1), g["targets"].reshape(-1)) / int(g["grad_acc"])
    loss.backward()
    close(loss, g["loss"], rtol=0, atol=0)
    close(logits.grad, g["dlogits"], rtol=0, atol=0)
    # the oracle's fp32 statement agrees with the reference's bf16 result to bf16 precision
    lo = O.cross_entropy(g["logits"], g["targets"], int(g["grad_acc"]))
    close(lo, g["loss"], rtol=1e-2, atol=1e-2)


def test_llama_forward_golden():
    g = load("G10")
    cfg = dict(hidden_size=64, intermediate_size=128, num_attention_heads=4, num_key_value_heads=2,
               rms_norm_eps=1e-5, vocab_size=96, num_hidden_layers=2)
    params = {k[len("param."):]: v for k, v in g.items() if k.startswith("param.")}
    cos, sin = O.get_cos_sin(16, 16, base=10000.0)
    logits = O.llama_forward(g["ids"][:, :-1], params, cfg, cos.float(), sin.float())
    close(logits, g["logits"], rtol=1e-4, atol=1e-4)
    loss = torch.nn.functional.cross_entropy(logits.reshape(-1, 96), g["ids"][:, 1:].reshape(-1))
    close(loss, g["loss"], rtol=1e-5, atol=1e-5)


def test_tensor_parallel_golden():
    """G7 (the reference's tests/test_tensor_parallel.py pin, tp=2 on gloo): the oracle's dense
    linear reproduces the dense layer, and the Column / Row shards are the dense result's slices and
    partial sums -- the semantics the GPU test checks the HIP Column/Row modules against."""
    g = load("G7")
    for t in ("", "async."):
        x, w, b = g[f"rank0.{t}x"], g[f"rank0.{t}dense_w"], g[f"rank0.{t}dense_b"]
        close(O.linear(x, w) + b, g[f"rank0.{t}y_dense"], rtol=1e-5, atol=1e-5)
        for r in (0, 1):
            assert torch.equal(g[f"rank{r}.{t}y_col"], g[f"rank{r}.{t}y_dense"])        # test_tensor_parallel.py:54
            close(g[f"rank{r}.{t}y_row"], g[f"rank{r}.{t}y_dense"], rtol=1e-5, atol=1e-5)
            close(g[f"rank{r}.{t}dw_col"], g[f"rank{r}.{t}dw_dense"].chunk(2, 0)[r])
            close(g[f"rank{r}.{t}dw_row"], g[f"rank{r}.{t}dw_dense"].chunk(2, 1)[r])
            close(g[f"rank{r}.{t}dx_col"], g[f"rank{r}.{t}dx_dense"])
            close(g[f"rank{r}.{t}dx_row"], g[f"rank{r}.{t}dx_dense"].chunk(2, -1)[r])
            close(g[f"rank{r}.{t}db_row"], g[f"rank{r}.{t}db_dense"])
    # VocabParallelEmbedding: the two ranks' vocab slices sum to the dense lookup
    w_full = torch.cat([g["rank0.emb_w"], g["rank1.emb_w"]], 0)
    close(g["rank0.emb_y"], torch.nn.functional.embedding(g["rank0.emb_ids"], w_full), rtol=0, atol=0)


def test_data_parallel_bucket_golden():
    """G8 (DataParallelBucket at dp=2, grad_acc 2): every rank's averaged grad equals the oracle's
    gradient of the mean loss over both ranks' micro-batches."""
    g = load("G8")
    cfg = dict(hidden_size=128, intermediate_size=256, num_attention_heads=2, num_key_value_heads=2,
               rms_norm_eps=1e-5, vocab_size=256, num_hidden_layers=2)
    params = {k[len("rank0.param."):]: v.clone().requires_grad_(True) for k, v in g.items()
              if k.startswith("rank0.param.")}
    cos, sin = O.get_cos_sin(128, 64, base=10000.0)
    ids = g["rank0.ids"]
    dp, ga = ids.shape[0], ids.shape[1]
    for r in range(dp):
        for i in range(ga):
            t = ids[r, i]
            lo = O.llama_forward(t[:, :-1], params, cfg, cos.float(), sin.float())
            (torch.nn.functional.cross_entropy(lo.reshape(-1, 256), t[:, 1:].reshape(-1)) / (ga * dp)).backward()
    for r in range(dp):
        for n, p in params.items():
            close(g[f"rank{r}.grad.{n}"], p.grad, rtol=1e-4, atol=1e-5)


def test_ring_step_golden_g4b():
    """G4b: rank 1's ring step (causal diagonal + full off-diagonal block, update_out_and_lse) as
    the reference computes it, in f32 and bf16 -- the oracle's pieces reproduce both."""
    for tag in ("f32", "bf16"):
        g = load(f"G4b_{tag}")
        sc = 1 / math.sqrt(64)
        o_c, l_c = O.ring_attention_forward(g["q1"], g["k1"], g["v1"], sc, True)
        o_f, l_f = O.ring_attention_forward(g["q1"], g["k0"], g["v0"], sc, False)
        out, lse = O.update_out_and_lse(None, None, o_c, l_c)
        out, lse = O.update_out_and_lse(out, lse, o_f, l_f)
        # bitwise in this container; another host's CPU GEMM can differ by an f32 ulp in an element
        tol = dict(rtol=1e-5, atol=1e-6) if tag == "f32" else dict(rtol=4e-6, atol=1e-7)
        close(out, g["out"], **tol)
        close(lse, g["lse"], **tol)


def test_g10m_fixtures_are_reference_loss_curves():
    """G10m_{tp2,cp2,dp2}: 4 finite, falling losses, identical on both ranks (the logged, cp_dp-
    averaged value), and the same initial weights in every topology."""
    import torch
    base = None
    for tag in ("tp2", "cp2", "dp2"):
        g = load(f"G10m_{tag}")
        l0, l1 = g["rank0.losses"], g["rank1.losses"]
        assert torch.equal(l0, l1) and l0.numel() == 4 and torch.isfinite(l0).all()
        assert (l0[1:] < l0[:-1]).all()
        w = {k: v for k, v in g.items() if k.startswith("rank0.param.")}
        if base is None:
            base = w
        assert w.keys() == base.keys() and all(torch.equal(w[k], base[k]) for k in w)


@pytest.mark.parametrize("prec", ["G11", "G11f32"])
def test_g11_fixtures_are_reference_50_step_curves(prec):
    """G11_* (bf16: the reference's GPU training precision) and G11f32_*: the reference's own 50-step
    loss curves on a fresh bigram batch per step (make_golden.g11_curve): finite, falling from ln 256
    towards the data's entropy, identical on both ranks, the single-rank and tp2 curves close (fp32:
    equal to reduction-order precision), and the bf16 run within 5 % of the fp32 one."""
    curves = {}
    for tag in ("1", "tp2", "cp2", "dp2"):
        g = load(f"{prec}_{tag}")
        l0 = g["rank0.losses"]
        assert l0.numel() == 50 and torch.isfinite(l0).all()
        assert abs(l0[0].item() - math.log(256)) < 0.3 and l0[-1].item() < 0.45 * l0[0].item()
        if tag != "1":
            assert torch.equal(l0, g["rank1.losses"])
        if prec == "G11":
            f32 = load(f"G11f32_{tag}")["rank0.losses"]
            assert ((l0 - f32).abs() / f32).max().item() < 0.05
        curves[tag] = l0
    assert (curves["tp2"] - curves["1"]).abs().max().item() < (1e-3 if prec == "G11f32" else 0.05)


@pytest.mark.parametrize("name", ["G11_cp2s512", "G11_cp2s512avg"])
def test_g11_cp2_seq512_fixture_is_a_reference_curve(name):
    """G11_cp2s512(avg) (make_golden.g11_curve at seq 512, cp2, bf16; avg: the cp ranks' gradients
    averaged by the reference's DataParallelBucket): the reference's ring over 256-token shards -- 50
    finite losses, the logged value identical on both ranks, falling like G11_cp2."""
    g = load(name)
    l0 = g["rank0.losses"]
    assert l0.numel() == 50 and torch.isfinite(l0).all() and torch.equal(l0, g["rank1.losses"])
    assert abs(l0[0].item() - math.log(256)) < 0.3 and l0[-1].item() < 0.45 * l0[0].item()
    assert tuple(g["rank0.ids"].shape) == (50, 2, 2, 2, 513)


def test_oracle_reproduces_g11_first_steps():
    """G11f32_1: the oracle's fp32 train step (llama_forward + CE / grad_acc + torch AdamW lr 1e-3) on G11_1's
    token stream from G10m's initial weights reproduces the reference's first 3 logged losses."""
    g = load("G11f32_1")
    w = load("G10m_tp2")
    cfg = dict(hidden_size=128, intermediate_size=256, num_attention_heads=2, num_key_value_heads=2,
               rms_norm_eps=1e-5, vocab_size=256, num_hidden_layers=2)
    params = {k[len("rank0.param."):]: v.clone().requires_grad_(True) for k, v in w.items()
              if k.startswith("rank0.param.")}
    opt = torch.optim.AdamW(list(params.values()), lr=1e-3)
    cos, sin = O.get_cos_sin(256, 64, base=10000.0)
    ids = g["rank0.ids"].long()
    for step in range(3):
        opt.zero_grad()
        acc = 0.0
        for i in range(2):
            t = ids[step, 0, i]
            lo = O.llama_forward(t[:, :-1], params, cfg, cos.float(), sin.float())
            loss = torch.nn.functional.cross_entropy(lo.reshape(-1, 256), t[:, 1:].reshape(-1)) / 2
            loss.backward()
            acc += loss.item()
        opt.step()
        assert abs(acc - g["rank0.losses"][step].item()) < 1e-4 * abs(acc), (step, acc)


@pytest.mark.parametrize("name", ["G12_tiny", "G12_smollm", "G12f32_smollm"])
def test_g12_fixtures_are_reference_grid_curves(name):
    """G12_* / G12f32_smollm: the reference's dp2 tp2 pp2 1F1B run (8 gloo processes,
    make_golden.g12_grid): every rank sits at its own (dp, pp, cp, tp) grid point
    (process_group_manager.py:13: view(dp, pp, cp, tp), tp fastest), the last-stage ranks log the same
    falling curve, the first stage logs 0."""
    g = load(name)
    seen = set()
    for r in range(8):
        d, p, c, t = g[f"rank{r}.grid"].tolist()
        assert r == ((d * 2 + p) * 1 + c) * 2 + t
        seen.add((d, p, t))
        lo = g[f"rank{r}.losses"]
        if p == 0:
            assert not lo.any()
        else:
            assert torch.equal(lo, g["rank2.losses"]) and (lo[1:] < lo[:-1]).all()
    assert len(seen) == 8


def test_g12_smollm_precision_gap_is_pinned():
    """G12f32_smollm (config 1's literal fp32, the README's --use_cpu precision) against G12_smollm
    (the same run in the reference's bf16 GPU training precision): the same first loss, and the bf16
    curve below the fp32 one by a gap that grows with the steps -- 0.9 / 2.2 / 3.6 % at steps 1-3 --
    set by bf16 AdamW updates of about one ulp at lr 1e-4, not by any implementation.  The HIP path's
    bf16 curve sits within 1 % of G12_smollm and within this gap of G12f32_smollm
    (tests/test_golden_gpu.py::test_dp2_tp2_pp2_1f1b_loss_curve_matches_reference_g12)."""
    f32, bf = load("G12f32_smollm")["rank2.losses"], load("G12_smollm")["rank2.losses"]
    gap = ((f32 - bf) / f32).tolist()
    assert abs(gap[0]) < 1e-4
    assert all(0.005 < g < 0.05 for g in gap[1:]) and gap[1] < gap[2] < gap[3], gap


def test_oracle_reproduces_g12_tiny_grid_curve():
    """G12_tiny (the reference's dp2 tp2 pp2 1F1B, 5 layers, mbs 4 seq 128 ga 2, lr 1e-2): the oracle
    restating what the grid computes -- each dp replica's gradient is the SUM over its micro-batches
    of the mean CE (pipeline_parallel.py:103,153, not / grad_acc), DataParallelBucket averages the two
    replicas (bucket.py all-reduce / cp_dp size), TP / PP change no arithmetic -- from the same
    deterministic full weights reproduces all 6 logged losses (mean over dp of the stage's loss)."""
    from tests import _g12
    g = load("G12_tiny")
    c = _g12.CFGS["tiny"]
    params = {k: v.clone().requires_grad_(True) for k, v in _g12.full_params("tiny").items()}
    opt = torch.optim.AdamW(list(params.values()), lr=_g12.RUN["tiny"]["lr"])
    S, V = c["max_position_embeddings"], c["vocab_size"]
    cos, sin = O.get_cos_sin(S, c["hidden_size"] // c["num_attention_heads"], base=c["rope_theta"])
    ids = _g12.tokens(V, S)
    for step in range(_g12.RUN["tiny"]["steps"]):
        opt.zero_grad()
        acc = 0.0
        for d in range(2):
            for i in range(_g12.GA):
                t = ids[d, i]
                lo = O.llama_forward(t[:, :-1], params, c, cos.float(), sin.float())
                loss = torch.nn.functional.cross_entropy(lo.transpose(1, 2), t[:, 1:])
                (loss / 2).backward()
                acc += loss.item() / _g12.GA / 2
        opt.step()
        ref = g["rank2.losses"][step].item()
        assert abs(acc - ref) < 1e-4 * abs(ref), (step, acc, ref)


def test_oracle_reproduces_g10m_pp2_pipeline_curve():
    """G10m_pp2 / G10m_pp2afab: the reference's PipelineParallel at pp 2 (1F1B and AFAB: the same
    curve, 5.71 -> 3.04) from G10m's initial weights.  The oracle restating the engine's loss -- each
    micro-batch's mean CE, NOT divided by grad_acc (pipeline_parallel.py:103,153), gradients summed
    over the micro-batches, torch AdamW lr 1e-2 -- reproduces all 4 logged losses."""
    a, b = load("G10m_pp2"), load("G10m_pp2afab")
    assert torch.equal(a["rank1.losses"], b["rank1.losses"]) and not a["rank0.losses"].any()
    w = load("G10m_tp2")
    assert all(torch.equal(a[k], w[k]) for k in a if k.startswith("rank0.param."))
    cfg = dict(hidden_size=128, intermediate_size=256, num_attention_heads=2, num_key_value_heads=2,
               rms_norm_eps=1e-5, vocab_size=256, num_hidden_layers=2)
    params = {k[len("rank0.param."):]: v.clone().requires_grad_(True) for k, v in a.items()
              if k.startswith("rank0.param.")}
    opt = torch.optim.AdamW(list(params.values()), lr=1e-2)
    cos, sin = O.get_cos_sin(256, 64, base=10000.0)
    gen = torch.Generator().manual_seed(1234)      # make_golden._g10m_data: one batch, every step
    ids = torch.randint(0, 256, (1, 2, 2, 2, 257), generator=gen)[0, 0]
    for step in range(4):
        opt.zero_grad()
        acc = 0.0
        for i in range(2):
            lo = O.llama_forward(ids[i][:, :-1], params, cfg, cos.float(), sin.float())
            loss = torch.nn.functional.cross_entropy(lo.transpose(1, 2), ids[i][:, 1:])
            loss.backward()
            acc += loss.item() / 2
        opt.step()
        ref = a["rank1.losses"][step].item()
        assert abs(acc - ref) < 1e-4 * abs(ref), (step, acc, ref)
