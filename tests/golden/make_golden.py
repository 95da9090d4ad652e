"""Generate the golden vectors that pin the CPU oracle (oracle/picotron_oracle.py).

Run IN THE BUILD CONTAINER ONLY (the reference checkout is not on the GPU box):
    python tests/golden/make_golden.py  [--ref /root/reference]

It imports the reference's own modules from the read-only checkout and evaluates them on tiny
seeded inputs (CPU, FLASH_ATTEN=0, the reference's eager path).  flash_attn (requirements.txt:6)
is not installed, so its three import names are satisfied by empty placeholder modules -- only
FLASH_ATTEN=0 code runs.  Outputs are plain tensor dicts saved with torch.save and read back with
torch.load(weights_only=True).  No reference source is copied; only inputs/outputs are stored.
"""
import argparse
import math
import os
import sys
import types

import torch

OUT = os.path.dirname(os.path.abspath(__file__))


def _install_stubs():
    for name in ["flash_attn", "flash_attn.flash_attn_interface", "flash_attn.layers", "flash_attn.layers.rotary",
                 "flash_attn.ops", "flash_attn.ops.triton", "flash_attn.ops.triton.layer_norm"]:
        m = types.ModuleType(name)
        m.flash_attn_func = m.apply_rotary_emb = m.layer_norm_fn = None
        sys.modules[name] = m


def _fake_pgm(pgm_mod):
    pgm_mod.process_group_manager = types.SimpleNamespace(
        tp_world_size=1, tp_rank=0, cp_world_size=1, cp_rank=0, pp_world_size=1, pp_rank=0,
        dp_world_size=1, cp_dp_world_size=1, pp_is_first_stage=True, pp_is_last_stage=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    os.environ.update(DEVICE="cpu", LOCAL_RANK="0", FLASH_ATTEN="0")
    sys.path.insert(0, args.ref)
    _install_stubs()
    import picotron.process_group_manager as pgm
    _fake_pgm(pgm)
    from picotron import model as M
    from picotron.context_parallel import context_parallel as CP

    g = torch.Generator().manual_seed(1234)
    gold = {}

    # G1: LlamaRMSNorm fwd/bwd (fp32 and bf16)
    for dt in (torch.float32, torch.bfloat16):
        tag = "f32" if dt == torch.float32 else "bf16"
        x = torch.randn(6, 64, generator=g).to(dt).requires_grad_(True)
        norm = M.LlamaRMSNorm(64, eps=1e-5)
        with torch.no_grad():
            norm.weight.copy_(1 + 0.1 * torch.randn(64, generator=g))
        norm = norm.to(dt)
        y = norm(x)
        dy = torch.randn(y.shape, generator=g).to(dt)
        y.backward(dy)
        gold[f"G1_{tag}"] = dict(x=x.detach(), w=norm.weight.detach(), eps=torch.tensor(1e-5), y=y.detach(), dy=dy,
                                 dx=x.grad.detach(), dw=norm.weight.grad.detach())

    # G2: get_cos_sin + apply_rotary_pos_emb fwd/bwd, [B, H, S, D]
    cos, sin = M.get_cos_sin(16, 32, base=10000.0)
    x = torch.randn(2, 3, 16, 32, generator=g, requires_grad=True)
    y = M.apply_rotary_pos_emb(x, cos.float(), sin.float())
    dy = torch.randn(y.shape, generator=g)
    y.backward(dy)
    gold["G2"] = dict(cos=cos, sin=sin, x=x.detach(), y=y.detach(), dy=dy, dx=x.grad.detach(), base=torch.tensor(1e4))
    cos5, sin5 = M.get_cos_sin(64, 128, base=500000.0)
    gold["G2_tables"] = dict(cos_16_32=cos, sin_16_32=sin, cos_64_128_default=cos5, sin_64_128_default=sin5)

    # tiny config shared by G3/G5/G6
    cfg = types.SimpleNamespace(hidden_size=64, intermediate_size=128, num_attention_heads=4, num_key_value_heads=2,
                                rms_norm_eps=1e-5, max_position_embeddings=16, rope_theta=10000.0, vocab_size=96,
                                num_hidden_layers=2)
    torch.manual_seed(42)

    # G3: Attention fwd/bwd (SDPA path, GQA 4/2)
    att = M.Attention(cfg, layer_idx=0)
    cos, sin = M.get_cos_sin(16, 16, base=10000.0)
    x = torch.randn(2, 16, 64, generator=g, requires_grad=True)
    y = att(x, cos.float(), sin.float())
    dy = torch.randn(y.shape, generator=g)
    y.backward(dy)
    gold["G3"] = dict(x=x.detach(), y=y.detach(), dy=dy, dx=x.grad.detach(), cos=cos, sin=sin,
                      **{f"{n}": p.detach() for n, p in att.named_parameters()},
                      **{f"grad.{n}": p.grad.detach() for n, p in att.named_parameters()})

    # G4: ring pure functions (fp32 and bf16 -- bf16 keeps the reference's bf16 LSE)
    for dt in (torch.float32, torch.bfloat16):
        tag = "f32" if dt == torch.float32 else "bf16"
        q, k, v = (torch.randn(1, 2, 8, 16, generator=g).to(dt) for _ in range(3))
        sc = 1 / math.sqrt(16)
        o_c, l_c = CP.ring_attention_forward(q, k, v, sc, True)
        o_f, l_f = CP.ring_attention_forward(q, k, v, sc, False)
        out, lse = CP.update_out_and_lse(None, None, o_c, l_c)
        out, lse = CP.update_out_and_lse(out, lse, o_f, l_f)
        dO = torch.randn(q.shape, generator=g).to(dt)
        dq, dk, dv = CP.ring_attention_backward(dO, q, k, v, out.to(dt), lse.squeeze(-1), sc, True)
        gold[f"G4_{tag}"] = dict(q=q, k=k, v=v, o_causal=o_c, lse_causal=l_c, o_full=o_f, lse_full=l_f,
                                 merged_out=out, merged_lse=lse, dO=dO, dq=dq, dk=dk, dv=dv)

    # G5: MLP fwd/bwd
    mlp = M.MLP(cfg)
    x = torch.randn(2, 5, 64, generator=g, requires_grad=True)
    y = mlp(x)
    dy = torch.randn(y.shape, generator=g)
    y.backward(dy)
    gold["G5"] = dict(x=x.detach(), y=y.detach(), dy=dy, dx=x.grad.detach(),
                      **{n: p.detach() for n, p in mlp.named_parameters()},
                      **{f"grad.{n}": p.grad.detach() for n, p in mlp.named_parameters()})

    # G6: DecoderLayer fwd/bwd
    layer = M.DecoderLayer(cfg, layer_idx=0)
    x = torch.randn(2, 16, 64, generator=g, requires_grad=True)
    layer.cos, layer.sin = layer.cos.float(), layer.sin.float()
    y = layer(x)
    dy = torch.randn(y.shape, generator=g)
    y.backward(dy)
    gold["G6"] = dict(x=x.detach(), y=y.detach(), dy=dy, dx=x.grad.detach(), cos=layer.cos, sin=layer.sin,
                      **{n: p.detach() for n, p in layer.named_parameters()},
                      **{f"grad.{n}": p.grad.detach() for n, p in layer.named_parameters()})

    # G9: cross entropy on bf16 logits / grad_acc (train.py:46-49)
    logits = torch.randn(2, 8, 96, generator=g).to(torch.bfloat16).requires_grad_(True)
    tgt = torch.randint(0, 96, (2, 8), generator=g)
    loss = torch.nn.functional.cross_entropy(logits.view(16, -1), tgt.reshape(-1), reduction="mean") / 4
    loss.backward()
    gold["G9"] = dict(logits=logits.detach(), targets=tgt, loss=loss.detach(), dlogits=logits.grad.detach(),
                      grad_acc=torch.tensor(4))

    # G10: tiny Llama forward + CE loss (single rank), weights from the reference's own init
    torch.manual_seed(7)
    llama = M.Llama(cfg)
    for layer in llama.decoder_layers:
        layer.cos, layer.sin = layer.cos.float(), layer.sin.float()
    ids = torch.randint(0, 96, (2, 17), generator=g)
    logits = llama(ids[:, :-1])
    loss = torch.nn.functional.cross_entropy(logits.reshape(-1, 96), ids[:, 1:].reshape(-1))
    loss.backward()
    gold["G10"] = dict(ids=ids, logits=logits.detach(), loss=loss.detach(),
                       **{f"param.{n}": p.detach() for n, p in llama.named_parameters()},
                       **{f"grad.{n}": p.grad.detach() for n, p in llama.named_parameters()})

    for name, d in gold.items():
        torch.save({k: (v.contiguous() if torch.is_tensor(v) else v) for k, v in d.items()},
                   os.path.join(OUT, f"{name}.pt"))
    print("wrote", sorted(gold))


if __name__ == "__main__":
    main()
