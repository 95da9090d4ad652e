"""Fused AdamW (csrc/adamw.hip) against torch.optim.AdamW -- the reference's optimizer
(train.py:209) -- on the same bf16 / f32 tensors over several steps, through the C ABI."""
import pytest
import torch

DEV = "cuda"
pytestmark = pytest.mark.gpu


def _run(opt_cls, shapes, dtype, steps, seed=0, **kw):
    g = torch.Generator().manual_seed(seed)
    params = [torch.nn.Parameter(torch.randn(s, generator=g).to(dtype).to(DEV)) for s in shapes]
    grads = [[(torch.randn(s, generator=g) * 0.1).to(dtype).to(DEV) for s in shapes] for _ in range(steps)]
    opt = opt_cls(params, **kw)
    for k in range(steps):
        for p, gr in zip(params, grads[k]):
            p.grad = gr.clone()
        opt.step()
    torch.cuda.synchronize()
    return params, opt


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_adamw_matches_torch_foreach(dtype):
    from picotron_amd.optim import AdamW
    shapes = [(2048,), (1000,), (512, 2048), (37,), (3, 5, 7)]
    kw = dict(lr=3e-4, weight_decay=0.01)
    ref, ropt = _run(lambda ps, **k: torch.optim.AdamW(ps, foreach=True, **k), shapes, dtype, 4, **kw)
    out, oopt = _run(AdamW, shapes, dtype, 4, **kw)
    for pr, po in zip(ref, out):
        sr, so = ropt.state[pr], oopt.state[po]
        assert float(sr["step"]) == float(so["step"]) == 4.0
        for a, b in ((pr, po), (sr["exp_avg"], so["exp_avg"]), (sr["exp_avg_sq"], so["exp_avg_sq"])):
            a, b = a.detach().float().cpu(), b.detach().float().cpu()
            diff = (a != b)
            if dtype == torch.bfloat16:
                # op-for-op the same roundings to bf16: identical but where an f32 contraction
                # difference crosses a rounding boundary
                assert diff.float().mean().item() < 1e-3, diff.float().mean().item()
                assert ((a - b).abs() <= 1e-2 * a.abs().clamp_min(1e-3)).all()
            else:  # f32 storage: contraction differences stay at the f32 ulp level
                assert torch.allclose(a, b, rtol=1e-5, atol=1e-7), (a - b).abs().max().item()


def test_adamw_state_dict_roundtrip():
    """Same state layout as torch.optim.AdamW: a torch optimizer's state_dict loads into ours."""
    from picotron_amd.optim import AdamW
    shapes = [(256,), (64, 32)]
    ref, ropt = _run(lambda ps, **k: torch.optim.AdamW(ps, foreach=True, **k), shapes, torch.bfloat16, 2, lr=1e-3)
    ours = AdamW([torch.nn.Parameter(p.detach().clone()) for p in ref], lr=1e-3)
    ours.load_state_dict(ropt.state_dict())
    g = [torch.randn_like(p) for p in ref]
    for p, q, gg in zip(ref, ours.param_groups[0]["params"], g):
        p.grad, q.grad = gg.clone(), gg.clone()
    ropt.step()
    ours.step()
    torch.cuda.synchronize()
    for p, q in zip(ref, ours.param_groups[0]["params"]):
        assert (p.float() - q.float()).abs().max().item() <= 1e-2 * p.float().abs().max().item()


def test_multi_tensor_launch_equals_per_tensor():
    """pt_adamw_step_multi (one launch over the list, ragged tails included) == pt_adamw_step per
    tensor, bit for bit; a re-made gradient (new pointer) gets a new descriptor table."""
    from picotron_amd import kernels as K
    g = torch.Generator().manual_seed(3)
    shapes = [(2048,), (1001,), (512, 2048), (37,), (3, 5, 7), (8,)]

    def mk():
        return [torch.randn(s, generator=g).to(torch.bfloat16).to(DEV) for s in shapes]
    P, G, M, V = mk(), mk(), [t.abs() * 0.01 for t in mk()], [t.abs() * 1e-4 for t in mk()]
    sc = dict(decay=1 - 3e-4 * 0.01, w1=0.1, beta2=0.999, c2=0.001, bc2_sqrt=(1 - 0.999 ** 3) ** 0.5, eps=1e-8,
              step_size=-3e-4 / (1 - 0.9 ** 3))
    a = [[t.clone() for t in L] for L in (P, G, M, V)]
    b = [[t.clone() for t in L] for L in (P, G, M, V)]
    for i in range(len(shapes)):
        K.adamw_step(a[0][i], a[1][i], a[2][i], a[3][i], **sc)
    K.adamw_step_multi(list(zip(*b)), **sc)
    torch.cuda.synchronize()
    for la, lb in zip(a, b):
        for x, y in zip(la, lb):
            assert torch.equal(x, y)
    b[1] = [t.clone() for t in G]   # new gradient tensors: new pointers
    K.adamw_step_multi(list(zip(*b)), **sc)
    for i in range(len(shapes)):
        K.adamw_step(a[0][i], G[i].clone(), a[2][i], a[3][i], **sc)
    torch.cuda.synchronize()
    for la, lb in zip((a[0], a[2], a[3]), (b[0], b[2], b[3])):
        for x, y in zip(la, lb):
            assert torch.equal(x, y)
