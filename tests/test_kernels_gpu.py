"""Kernel parity on the GPU: each gfx950 kernel (through the C ABI) against the CPU oracle /
torch fp32 on the same seeded inputs.  Tolerances: bf16 outputs within rel 2e-2 of the fp32
reference (north_star), stated per test."""
import math

import pytest
import torch

from oracle import picotron_oracle as O
from picotron_amd import switches

pytestmark = pytest.mark.gpu

DEV = "cuda"
BF = torch.bfloat16


def rel_err(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def maxabs(a, b):
    return (a.float().cpu() - b.float().cpu()).abs().max().item()


@pytest.fixture(autouse=True)
def _seed():
    torch.manual_seed(0)


# --------------------------------------------------------------------------- RMSNorm
@pytest.mark.parametrize("rows,cols", [(64, 64), (300, 2048), (128, 4096), (8, 512), (64, 5120), (300, 8192),
                                       (16, 16384), (1000, 4104)])
@pytest.mark.parametrize("mode", [0, 1])
def test_rmsnorm_fwd_bwd(rows, cols, mode):
    """(the rows wider than 4096: rmsnorm.hip's wide-row kernels -- Llama-2-13B 5120, 70B 8192)"""
    from picotron_amd import kernels as K
    x = torch.randn(rows, cols).to(BF)
    w = (1 + 0.1 * torch.randn(cols)).to(BF)
    dy = torch.randn(rows, cols).to(BF)
    # reference in fp32 on the same bf16 inputs
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    ref = O.rmsnorm_flash_semantics(xr, wr, 1e-5) if mode == 0 else O.rmsnorm_llama(xr, wr, 1e-5)
    ref.backward(dy.float())
    y, rstd, _ = K.rmsnorm_fwd(x.to(DEV), w.to(DEV), 1e-5, mode)
    dx, dw = K.rmsnorm_bwd(dy.to(DEV), x.to(DEV), w.to(DEV), rstd, mode)
    torch.cuda.synchronize()
    assert rel_err(y, ref) < 5e-3
    assert rel_err(dx, xr.grad) < 1e-2
    assert rel_err(dw, wr.grad) < 1e-2


@pytest.mark.parametrize("rows,cols,mode", [(4096, 2048, 0), (300, 2048, 1), (256, 512, 0), (64, 4096, 0),
                                            (300, 5120, 0), (64, 8192, 1)])
def test_rmsnorm_bwd_from_splitk_parts(rows, cols, mode):
    """dy given as two f32 split-K halves (pt_rmsnorm_bwd_splitk) == their bf16 sum pass followed
    by the plain backward, bit for bit (dx with the residual gradient, dweight)."""
    from picotron_amd import kernels as K
    z = torch.randn(rows, cols).to(BF).to(DEV)
    w = (1 + 0.1 * torch.randn(cols)).to(BF).to(DEV)
    dres = torch.randn(rows, cols).to(BF).to(DEV)
    parts = K.SplitKParts(torch.randn(rows, cols, device=DEV), torch.randn(rows, cols, device=DEV))
    _, rstd, _ = K.rmsnorm_fwd(z, w, 1e-5, mode)
    dx1, dw1 = K.rmsnorm_bwd(parts, z, w, rstd, mode, dres=dres)
    dx2, dw2 = K.rmsnorm_bwd(parts.sum(), z, w, rstd, mode, dres=dres)
    torch.cuda.synchronize()
    assert torch.equal(dx1, dx2) and torch.equal(dw1, dw2)


@pytest.mark.parametrize("cols", [2048, 8192])
def test_rmsnorm_fused_residual(cols):
    from picotron_amd import kernels as K
    rows = 256
    x, r = torch.randn(rows, cols).to(BF), torch.randn(rows, cols).to(BF)
    w = torch.ones(cols).to(BF)
    y, rstd, z = K.rmsnorm_fwd(x.to(DEV), w.to(DEV), 1e-5, 0, residual=r.to(DEV))
    zr = (x + r)  # bf16 add, as the reference's residual (model.py:207-208)
    assert torch.equal(z.cpu(), zr)
    assert rel_err(y, O.rmsnorm_flash_semantics(zr, w, 1e-5)) < 5e-3
    dy, dres = torch.randn(rows, cols).to(BF), torch.randn(rows, cols).to(BF)
    dx, _ = K.rmsnorm_bwd(dy.to(DEV), z, w.to(DEV), rstd, 0, dres=dres.to(DEV))
    zf = zr.float().requires_grad_(True)
    O.rmsnorm_flash_semantics(zf, w.float(), 1e-5).backward(dy.float())
    assert rel_err(dx, zf.grad + dres.float()) < 1e-2


@pytest.mark.parametrize("rows", [4096, 1000, 5000])
def test_rmsnorm_dweight_sinks(rows):
    """dweight written into an existing sink: bf16 store, bf16 accumulate (= autograd's grad +
    bf16(new)), f32 accumulate (main_grad); the partial-row sum is deterministic (bitwise repeat)."""
    from picotron_amd import kernels as K
    cols = 2048
    x, dy = torch.randn(rows, cols).to(BF).to(DEV), torch.randn(rows, cols).to(BF).to(DEV)
    w = (1 + 0.1 * torch.randn(cols)).to(BF).to(DEV)
    _, rstd, _ = K.rmsnorm_fwd(x, w, 1e-5, 0)
    _, dw = K.rmsnorm_bwd(dy, x, w, rstd, 0)
    _, dw2 = K.rmsnorm_bwd(dy, x, w, rstd, 0)
    assert torch.equal(dw, dw2)
    xr = x.float().cpu().requires_grad_(True)
    wr = w.float().cpu().requires_grad_(True)
    O.rmsnorm_flash_semantics(xr, wr, 1e-5).backward(dy.float().cpu())
    assert rel_err(dw, wr.grad) < 1e-2
    old = torch.randn(cols).to(BF).to(DEV)
    acc = old.clone()
    K.rmsnorm_bwd(dy, x, w, rstd, 0, dw_out=acc, dw_sink=K.DW_ACC_BF16)
    assert torch.equal(acc, old + dw)
    oldf = torch.randn(cols, device=DEV)
    accf = oldf.clone()
    _, _ = K.rmsnorm_bwd(dy, x, w, rstd, 0, dw_out=accf, dw_sink=K.DW_ACC_F32)
    assert rel_err(accf - oldf, dw.float()) < 1e-2


def test_rmsnorm_colsum_batch_equals_per_norm():
    """deferred weight-gradient sums (partials kept, one batched launch) == the per-norm sums, bit for
    bit, for every sink; dx unchanged"""
    from picotron_amd import kernels as K
    rows, cols = 4096, 2048
    sinks = [0, K.DW_ACC_BF16, K.DW_ACC_F32, K.DW_ACC_BF16]
    jobs, want = [], []
    for i, sink in enumerate(sinks):
        x, dy = torch.randn(rows, cols).to(BF).to(DEV), torch.randn(rows, cols).to(BF).to(DEV)
        w = (1 + 0.1 * torch.randn(cols)).to(BF).to(DEV)
        _, rstd, _ = K.rmsnorm_fwd(x, w, 1e-5, i % 2)
        init = torch.randn(cols, device=DEV).to(torch.float32 if sink == K.DW_ACC_F32 else BF)
        ref = init.clone()
        dx_ref, _ = K.rmsnorm_bwd(dy, x, w, rstd, i % 2, dw_out=ref, dw_sink=sink)
        dx, partial = K.rmsnorm_bwd(dy, x, w, rstd, i % 2, defer_dw=True)
        assert torch.equal(dx, dx_ref)
        out = init.clone()
        jobs.append((partial, out, sink))
        want.append(ref)
    K.rmsnorm_colsum_batch(jobs)
    torch.cuda.synchronize()
    for (_, out, _), ref in zip(jobs, want):
        assert torch.equal(out, ref)


def test_rmsnorm_deferred_dw_through_autograd(monkeypatch):
    """a stack of norms under autograd: with the deferral (one batched column sum at the end of the
    backward) the weight grads are bit-identical to the immediate per-norm sums"""
    from picotron_amd import functional as FN
    rows, cols, n = 1024, 2048, 5
    x0 = torch.randn(rows, cols).to(BF).to(DEV)
    ws = [torch.nn.Parameter((1 + 0.1 * torch.randn(cols)).to(BF).to(DEV)) for _ in range(n)]
    dy = torch.randn(rows, cols).to(BF).to(DEV)
    grads = {}
    for defer in ("1", "0"):
        monkeypatch.setattr(switches.S, "norm_defer", int(defer))
        for w in ws:
            w.grad = None
        x = x0.clone().requires_grad_(True)
        h = x
        for w in ws:
            h = FN.RMSNormFunction.apply(h, w, 1e-5, 0)
        h.backward(dy)
        assert not FN._PENDING_DW
        grads[defer] = [w.grad.clone() for w in ws] + [x.grad.clone()]
    for a, b in zip(grads["1"], grads["0"]):
        assert torch.equal(a, b)


# ------------------------------------------------------------------------------ RoPE
@pytest.mark.parametrize("d", [64, 128])
def test_rope_fused_qk_rows(d):
    from picotron_amd import kernels as K
    B, S, nh, nkv = 2, 64, 4, 2
    cos, sin = O.get_cos_sin(S, d, base=10000.0)
    qkv = torch.randn(B * S, (nh + 2 * nkv) * d).to(BF)
    ref = qkv.clone()
    # reference: rotate q and k heads ([B, H, S, D] layout), flash semantics (one rounding)
    for lo, n in ((0, nh), (nh * d, nkv)):
        t = ref[:, lo:lo + n * d].view(B, S, n, d).transpose(1, 2)
        t2 = O.rotary_flash_semantics(t, cos, sin)
        ref[:, lo:lo + n * d] = t2.transpose(1, 2).reshape(B * S, n * d)
    dq = qkv.to(DEV)
    K.rope_(dq, nh + nkv, d, cos.to(DEV), sin.to(DEV), S)
    torch.cuda.synchronize()
    assert maxabs(dq, ref) <= 2 * 2 ** -7 * ref.abs().max().item()
    assert torch.equal(dq[:, (nh + nkv) * d:].cpu(), qkv[:, (nh + nkv) * d:])  # v untouched
    # inverse restores the input to bf16 rounding
    K.rope_(dq, nh + nkv, d, cos.to(DEV), sin.to(DEV), S, inverse=True)
    assert rel_err(dq, qkv) < 1e-2


# ---------------------------------------------------------------------------- SwiGLU
def test_swiglu_fwd_bwd_strided():
    from picotron_amd import kernels as K
    T, I = 512, 1024
    gu = torch.randn(T, 2 * I).to(BF)
    g, u = gu[:, :I], gu[:, I:]
    dh = torch.randn(T, I).to(BF)
    gr, ur = g.clone().requires_grad_(True), u.clone().requires_grad_(True)
    h_ref = torch.nn.functional.silu(gr) * ur   # bf16 eager, as model.py:186
    h_ref.backward(dh)
    d = gu.to(DEV)
    h = K.swiglu_fwd(d[:, :I], d[:, I:])
    dg, du = K.swiglu_bwd(dh.to(DEV), d[:, :I], d[:, I:])
    torch.cuda.synchronize()
    assert maxabs(h, h_ref) <= 1e-2 * h_ref.abs().max().item()
    assert rel_err(dg, gr.grad) < 1e-2 and rel_err(du, ur.grad) < 1e-2


# ---------------------------------------------------------------------- cross entropy
@pytest.mark.parametrize("V", [96, 49152, 32000, 80000])
def test_cross_entropy_fused(V):
    from picotron_amd import kernels as K
    T, ga = 64, 4
    logits = (3 * torch.randn(T, V)).to(BF)
    tgt = torch.randint(0, V, (T,))
    tgt[5] = -100
    lr = logits.float().requires_grad_(True)
    loss_ref = torch.nn.functional.cross_entropy(lr, tgt) / ga
    loss_ref.backward()
    dl = logits.to(DEV)
    loss, grad, _ = K.cross_entropy_fwd_bwd(dl, tgt.to(DEV), scale=1.0 / ga, inplace=True)
    torch.cuda.synchronize()
    assert abs(loss.item() / ga - loss_ref.item()) < 1e-3 * max(1, abs(loss_ref.item()))
    assert grad.data_ptr() == dl.data_ptr()
    assert rel_err(grad, lr.grad) < 1e-2
    assert grad[5].float().abs().max().item() == 0.0


def test_cross_entropy_golden_vector():
    """against the reference's own bf16 F.cross_entropy / grad_acc (tests/golden/G9)."""
    import os
    from picotron_amd import kernels as K
    g = torch.load(os.path.join(os.path.dirname(__file__), "golden", "G9.pt"), weights_only=True)
    lg = g["logits"].view(16, -1).to(DEV).clone()
    loss, grad, _ = K.cross_entropy_fwd_bwd(lg, g["targets"].reshape(-1).to(DEV), scale=1.0 / int(g["grad_acc"]))
    assert abs(loss.item() / int(g["grad_acc"]) - g["loss"].float().item()) < 2e-2 * abs(g["loss"].float().item())
    assert rel_err(grad, g["dlogits"].view(16, -1)) < 2e-2


# ------------------------------------------------------------------------------ GEMM
def _ref_mm(a, b):
    return a.float().cpu() @ b.float().cpu()


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 256), (4096, 2048, 2048), (128, 384, 128),
                                   (64, 64, 128)])
def test_gemm_fwd_nt(M, N, K):
    from picotron_amd import kernels as K_
    x = torch.randn(M, K).to(BF)
    w = (torch.randn(N, K) / math.sqrt(K)).to(BF)
    y = K_.linear_fwd(x.to(DEV), [w.to(DEV)])
    torch.cuda.synchronize()
    assert rel_err(y, _ref_mm(x, w.t())) < 1e-2


@pytest.mark.parametrize("tile", [2, 3, 12, 13, 14, 15])
def test_gemm_every_tile_every_layout(tile):
    from picotron_amd import kernels as K_
    M, N, K = 512, 512, 256
    a = torch.randn(M, K).to(BF)
    b = (torch.randn(N, K) / 16).to(BF)
    y = K_.linear_fwd(a.to(DEV), [b.to(DEV)], tile=tile)
    assert rel_err(y, _ref_mm(a, b.t())) < 1e-2
    # NN: dX = dY W   (dY [M, N], W [N, K])
    dy = torch.randn(M, N).to(BF)
    dx = K_.linear_dgrad(dy.to(DEV), [b.to(DEV)], tile=tile)
    assert rel_err(dx, _ref_mm(dy, b)) < 1e-2
    # TN: dW = dY^T X  (dY [M, N], X [M, K]) -> [N, K]
    dw = torch.empty(N, K, dtype=BF, device=DEV)
    K_.linear_wgrad(dy.to(DEV), a.to(DEV), [dw], tile=tile)
    torch.cuda.synchronize()
    assert rel_err(dw, _ref_mm(dy.t(), a)) < 1e-2


@pytest.mark.parametrize("T,K,ns", [(100, 72, [40, 24]), (4000 // 8, 1376 // 8, [4000 // 8]), (192, 1376, [96]),
                                    (256, 256, [200]), (512, 4096, [4000]), (512, 1376, [4096])])
def test_gemm_off_grid_shapes_run_padded(T, K, ns):
    """Projections whose T, K or output widths are not multiples of 64 (no GEMM tile covers them:
    Llama-2-7B at tp 8 has a vocab shard of 4000 and an intermediate shard of 1376) run on
    zero-padded copies (kernels._linear_*_padded): forward with stacked segments and the residual
    epilogue, dX plain and accumulated, dW stored / bf16-accumulated / f32-accumulated, and a
    micro-batch pair's dW (KPair) -- each against torch fp32 on the same bf16 inputs."""
    from picotron_amd import kernels as K_
    N = sum(ns)
    x = torch.randn(T, K).to(BF)
    ws = [(torch.randn(n, K) / math.sqrt(K)).to(BF) for n in ns]
    res = torch.randn(T, N).to(BF)
    dy = torch.randn(T, N).to(BF)
    W = torch.cat([w.float() for w in ws])
    y = K_.linear_fwd(x.to(DEV), [w.to(DEV) for w in ws])
    assert y.shape == (T, N) and rel_err(y, x.float() @ W.t()) < 1e-2
    yr = K_.linear_fwd(x.to(DEV), [w.to(DEV) for w in ws], residual=res.to(DEV))
    assert rel_err(yr, res.float() + x.float() @ W.t()) < 1e-2
    dx = K_.linear_dgrad(dy.to(DEV), [w.to(DEV) for w in ws])
    assert dx.shape == (T, K) and rel_err(dx, dy.float() @ W) < 1e-2
    acc = torch.randn(T, K).to(BF).to(DEV)
    want = acc.float().cpu() + dy.float() @ W
    K_.linear_dgrad(dy.to(DEV), [w.to(DEV) for w in ws], out=acc, accumulate=True)
    assert rel_err(acc, want) < 1e-2
    ref = dy.float().t() @ x.float()
    for epi, dt in ((K_.EPI_BF16, BF), (K_.EPI_BF16_ACC, BF), (K_.EPI_F32_ACC, torch.float32)):
        outs = [torch.randn(n, K).to(dt).to(DEV) for n in ns]
        base = torch.cat([o.float().cpu() for o in outs]) if epi != K_.EPI_BF16 else 0
        K_.linear_wgrad(dy.to(DEV), x.to(DEV), outs, epi)
        got = torch.cat([o.float().cpu() for o in outs])
        assert rel_err(got, base + ref) < 1e-2, epi
    # a micro-batch pair's weight gradient (train_step's pairing) off the grid: its two halves
    dy2, x2 = torch.randn(T, N).to(BF), torch.randn(T, K).to(BF)
    outs = [torch.zeros(n, K, dtype=BF, device=DEV) for n in ns]
    K_.linear_wgrad(K_.KPair(dy.to(DEV), dy2.to(DEV)), K_.KPair(x.to(DEV), x2.to(DEV)), outs, K_.EPI_BF16)
    assert rel_err(torch.cat([o.float().cpu() for o in outs]), ref + dy2.float().t() @ x2.float()) < 1e-2


def test_gemm_retired_tiles_are_refused():
    """Tile ids 4, 5, 8, 9 (the simple 256-row kernels, never auto-picked, spilling at 256x256) are
    not in the library: asking for one is PT_EUNSUPPORTED, not a silent other kernel."""
    from picotron_amd import kernels as K_
    from picotron_amd._C import HipKernelError
    a = torch.randn(512, 256).to(BF).to(DEV)
    b = torch.randn(512, 256).to(BF).to(DEV)
    for t in (4, 5, 8, 9):
        with pytest.raises(HipKernelError, match="UNSUPPORTED"):
            K_.linear_fwd(a, [b], tile=t)


@pytest.mark.parametrize("tile", [12, 13, 14, 15])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 192), (768, 512, 512), (256, 512, 2048),
                                   (512, 256, 320), (256, 256, 128)])
def test_gemm_8phase_shapes(M, N, K, tile):
    """the phased kernels (tile 12: 256x256, 13: 256x128, 14: 256x128 K-halves, 15: 128x128 K-halves,
    4-deep ring): 1-5 and 8 / 32 K-tiles (every remainder of the 2-, 3- and 4-buffer loops), every
    layout"""
    from picotron_amd import kernels as K_
    a = torch.randn(M, K).to(BF)
    b = (torch.randn(N, K) / 16).to(BF)
    bn = 256 if tile == 12 else 128
    y = K_.linear_fwd(a.to(DEV), [b.to(DEV)], tile=tile)
    assert rel_err(y, _ref_mm(a, b.t())) < 1e-2
    dy = torch.randn(M, N).to(BF)
    if K % bn == 0:
        dx = K_.linear_dgrad(dy.to(DEV), [b.to(DEV)], tile=tile)
        assert rel_err(dx, _ref_mm(dy, b)) < 1e-2
    dw = torch.empty(N, K, dtype=BF, device=DEV)
    if N % 256 == 0 and K % bn == 0:
        K_.linear_wgrad(dy.to(DEV), a.to(DEV), [dw], tile=tile)
        torch.cuda.synchronize()
        assert rel_err(dw, _ref_mm(dy.t(), a)) < 1e-2
    # exactness: A = I picks rows of B^T
    eye = torch.eye(M, K).to(BF)
    y = K_.linear_fwd(eye.to(DEV), [b.to(DEV)], tile=tile)
    torch.cuda.synchronize()
    assert torch.equal(y.cpu()[:min(M, K)], b.t()[:min(M, K)])


@pytest.mark.parametrize("T,N,K", [(4096, 2048, 2048), (4096, 2048, 8192), (1024, 384, 1024)])
def test_gemm_khalves_tile_at_layer_shapes(T, N, K):
    """Tile 14 (256x128, the K-tile's two k-substeps over two wave groups, partials summed through
    LDS) on the layer's 256x128 launches -- o_proj forward / dX (K 2048), down_proj forward with the
    residual (K 8192) -- against the fp32 reference and the 4-phase tile 13 (a different f32
    summation order: within bf16 rounding of it), and the auto pick under switch gemm_kh."""
    from picotron_amd import kernels as K_
    from picotron_amd import switches
    g = torch.Generator().manual_seed(T + N + K)
    x = torch.randn(T, K, generator=g).to(BF)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(BF)
    res = torch.randn(T, N, generator=g).to(BF)
    xd, wd, rd = x.to(DEV), w.to(DEV), res.to(DEV)
    ref = _ref_mm(x, w.t())
    y14 = K_.linear_fwd(xd, [wd], tile=14)
    y13 = K_.linear_fwd(xd, [wd], tile=13)
    assert rel_err(y14, ref) < 1e-2 and rel_err(y14, y13.float().cpu()) < 1e-2
    yr = K_.linear_fwd(xd, [wd], tile=14, residual=rd)
    assert rel_err(yr, (res.float() + y14.float().cpu()).to(BF).float()) < 1e-2
    dy = torch.randn(T, N, generator=g).to(BF)
    w2 = (torch.randn(N, K, generator=g) / N ** 0.5).to(BF)
    dx = K_.linear_dgrad(dy.to(DEV), [w2.to(DEV)], tile=14)
    assert rel_err(dx, _ref_mm(dy, w2)) < 1e-2
    ya = K_.linear_fwd(xd, [wd])      # the auto pick: tile 14 at K >= 4096 (variant gemm_kh)
    with switches.override(gemm_kh=0):
        yb = K_.linear_fwd(xd, [wd])
    torch.cuda.synchronize()
    assert rel_err(ya, ref) < 1e-2 and rel_err(yb, ref) < 1e-2


def test_swiglu_dx_ksplit_beside_dw_slices():
    """TP = 8 shard widths (I 1024): the down_proj dX with the SwiGLU backward runs as two K-slices
    beside the dW slices in the dual launch and the reduce pass applies the SwiGLU backward (mode 6).
    dg|du within bf16 rounding of the fused single-pass form and of the fp32 reference; the dW slices
    are the same launch either way (bit-identical)."""
    from picotron_amd import kernels as K_
    T, H, I = 4096, 2048, 1024
    assert K_.swiglu_dx_ksplit(T, I, H) == 2
    g = torch.Generator().manual_seed(5)
    dm = torch.randn(T, H, generator=g).to(BF).to(DEV)
    hh = torch.randn(T, I, generator=g).to(BF).to(DEV)
    wd = (torch.randn(H, I, generator=g) / I ** 0.5).to(BF).to(DEV)
    gu = torch.randn(T, 2 * I, generator=g).to(BF).to(DEV)
    outs = []
    for v in (0, 1):
        gw = torch.zeros(H, I, dtype=BF, device=DEV)
        with switches.override(swiglu_splitk=v):
            dgu = K_.linear_dgrad_dual(dm, [wd], [(dm, hh, [gw])], K_.EPI_BF16_ACC, gu=gu)
        torch.cuda.synchronize()
        outs.append((dgu.clone(), gw.clone()))
    assert rel_err(outs[1][0], outs[0][0]) < 1e-2
    assert torch.equal(outs[1][1], outs[0][1])
    dh = (dm.float() @ wd.float()).to(BF).float()
    gg, uu = gu[:, :I].float(), gu[:, I:].float()
    sg = torch.sigmoid(gg)
    du = dh * (gg * sg).to(BF).float()
    dg = (dh * uu).to(BF).float() * (sg * (1 + gg * (1 - sg)))
    assert rel_err(outs[1][0], torch.cat([dg, du], dim=1)) < 2e-2


@pytest.mark.parametrize("epi", [0, 1, 3])
def test_gemm_grouped_wgrad(epi):
    """dW of q|k|v (3 outputs) and dW of o_proj in one pt_gemm_grouped launch == separate GEMMs"""
    from picotron_amd import kernels as K_
    T, H, nkv = 512, 512, 256
    dqkv, h = torch.randn(T, H + 2 * nkv).to(BF).to(DEV), torch.randn(T, H).to(BF).to(DEV)
    da, o = torch.randn(T, H).to(BF).to(DEV), torch.randn(T, H).to(BF).to(DEV)
    dt = torch.float32 if epi == 3 else BF
    init = [torch.randn(n, H).to(dt).to(DEV) for n in (H, nkv, nkv, H)]
    outs = [t.clone() for t in init]
    K_.linear_wgrad_grouped([(dqkv, h, outs[:3]), (da, o, outs[3:])], epilogue=epi)
    refs = [t.clone() for t in init]
    K_.linear_wgrad(dqkv, h, refs[:3], epilogue=epi)
    K_.linear_wgrad(da, o, refs[3:], epilogue=epi)
    torch.cuda.synchronize()
    for a, b in zip(outs, refs):
        assert torch.equal(a, b)
    full = _ref_mm(dqkv.t().cpu(), h.cpu())
    base = init[0].float().cpu() if epi else 0
    assert rel_err(outs[0], full[:H] + base) < 1e-2


@pytest.mark.parametrize("epi", [0, 1, 3])
def test_wgrad_ksplit_tp8_shapes(epi, monkeypatch):
    """The TP = 8 shard weight gradients (SmolLM-1.7B: q|k|v dW [768, 2048] + o_proj dW [2048, 256]
    in one group, 32 tiles; down_proj dW [2048, 1024], 32 tiles) as split-K slices (f32 partials +
    pt_gemm_splitk_reduce into the bf16 store / bf16 accumulate / f32 accumulate sinks) against the
    unsplit launch (PICOTRON_KSPLIT=0) and an f32 reference: equal up to the f32 summation order."""
    from picotron_amd import kernels as K_
    T, H, q, o_in, I = 4096, 2048, 256, 256, 1024
    dqkv, h = torch.randn(T, 3 * q).to(BF).to(DEV), torch.randn(T, H).to(BF).to(DEV)
    da, o = torch.randn(T, H).to(BF).to(DEV), torch.randn(T, o_in).to(BF).to(DEV)
    dm, hh = torch.randn(T, H).to(BF).to(DEV), torch.randn(T, I).to(BF).to(DEV)
    assert K_.wgrad_ksplit([(3 * q, H, T), (H, o_in, T)]) == 8
    assert K_.wgrad_ksplit([(H, I, T)]) == 8 and K_.wgrad_ksplit([(2 * I, H, T)]) == 4
    dt = torch.float32 if epi == 3 else BF
    init = [torch.randn(n, k).to(dt).to(DEV) for n, k in ((q, H), (q, H), (q, H), (H, o_in), (H, I))]
    outs, refs = [t.clone() for t in init], [t.clone() for t in init]
    K_.linear_wgrad_grouped([(dqkv, h, outs[:3]), (da, o, outs[3:4])], epilogue=epi)
    K_.linear_wgrad(dm, hh, outs[4:], epilogue=epi)
    monkeypatch.setattr(switches.S, "ksplit", 0)
    K_.linear_wgrad_grouped([(dqkv, h, refs[:3]), (da, o, refs[3:4])], epilogue=epi)
    K_.linear_wgrad(dm, hh, refs[4:], epilogue=epi)
    torch.cuda.synchronize()
    full = [dqkv[:, :q].t().float() @ h.float(), dqkv[:, q:2 * q].t().float() @ h.float(),
            dqkv[:, 2 * q:].t().float() @ h.float(), da.t().float() @ o.float(), dm.t().float() @ hh.float()]
    for a, b, f, i0 in zip(outs, refs, full, init):
        want = f + (i0.float() if epi else 0)
        assert rel_err(a, want) < 4e-3 and rel_err(b, want) < 4e-3
        assert maxabs(a, b) <= 2 * b.float().abs().max().item() * (2 ** -8 if dt == BF else 2 ** -20)


@pytest.mark.parametrize("epi", [1, 3])
def test_gemm_dual_with_ksplit_wgrad(epi, monkeypatch):
    """TP = 8 down_proj backward: the SwiGLU-backward dX (64 tiles) beside the split-K down_proj dW
    (32 tiles x 4 slices: one round with the dX tiles; f32 partials + reduce) in one dual launch == the unsplit dual launch up to
    the dW's f32 summation order; the dX bit for bit (its own K-slicing, swiglu_splitk, is off here:
    test_swiglu_dx_ksplit_beside_dw_slices covers it)."""
    from picotron_amd import kernels as K_
    monkeypatch.setattr(switches.S, "swiglu_splitk", 0)
    T, H, I = 4096, 2048, 1024
    dm = torch.randn(T, H).to(BF).to(DEV)
    wd = (torch.randn(H, I) / math.sqrt(I)).to(BF).to(DEV)
    gu = torch.randn(T, 2 * I).to(BF).to(DEV)
    hh = torch.randn(T, I).to(BF).to(DEV)
    dt = torch.float32 if epi == 3 else BF
    init = torch.randn(H, I).to(dt).to(DEV)
    out_a, out_b = init.clone(), init.clone()
    dx_a = K_.linear_dgrad_dual(dm, [wd], [(dm, hh, [out_a])], epi, gu=gu)
    monkeypatch.setattr(switches.S, "ksplit", 0)
    dx_b = K_.linear_dgrad_dual(dm, [wd], [(dm, hh, [out_b])], epi, gu=gu)
    torch.cuda.synchronize()
    assert dx_a is not None and dx_b is not None and torch.equal(dx_a, dx_b)
    want = dm.t().float() @ hh.float() + init.float()
    assert rel_err(out_a, want) < 4e-3
    assert maxabs(out_a, out_b) <= 2 * out_b.float().abs().max().item() * (2 ** -8 if dt == BF else 2 ** -20)


@pytest.mark.parametrize("mode", [0, 1, 2, 3, 4])
def test_splitk_reduce_modes(mode):
    """pt_gemm_splitk_reduce: the sum of the partials in part order through each sink epilogue,
    into two row segments with their own leading dimensions."""
    from picotron_amd import _C, kernels as K_
    parts = torch.randn(3, 512, 256, device=DEV)
    total = parts[0] + parts[1] + parts[2]
    f32 = mode in (2, 3)
    dt = torch.float32 if f32 else BF
    seg = [torch.randn(384, 264, device=DEV).to(dt)[:, :256], torch.randn(128, 256, device=DEV).to(dt)]
    init = [t.clone() for t in seg]
    res = torch.randn(512, 256, device=DEV).to(BF)
    rc = _C.lib().pt_gemm_splitk_reduce(K_._ptr(parts), 3, 512 * 256, 512, 256, _C.ptrarr([K_._ptr(t) for t in seg]),
                                        _C.i64arr([t.stride(0) for t in seg]), _C.i64arr([0, 384, 512]), 2, mode,
                                        K_._ptr(res) if mode == 4 else None, 256, _C.stream_ptr(torch.device(DEV)))
    assert rc == 0
    torch.cuda.synchronize()
    got = torch.cat([seg[0], seg[1]]).float()
    old = torch.cat(init).float()
    if mode == 0:
        want = total.to(BF).float()
    elif mode == 1:
        want = (old + total.to(BF).float()).to(BF).float()
    elif mode == 2:
        want = total
    elif mode == 3:
        want = old + total
    else:
        want = (res.float() + total.to(BF).float()).to(BF).float()
    assert torch.equal(got, want)


@pytest.mark.parametrize("T,H,I", [(256, 256, 128), (512, 512, 1024), (1024, 256, 384)])
def test_gemm_swiglu_fused(T, H, I):
    """gate|up GEMM with SwiGLU in the epilogue == GEMM + swiglu kernel, bit for bit; and the down
    dX GEMM with the SwiGLU backward in the epilogue == dgrad GEMM + swiglu bwd kernel"""
    from picotron_amd import kernels as K_
    x = torch.randn(T, H).to(BF).to(DEV)
    wg, wu = [(torch.randn(I, H) / math.sqrt(H)).to(BF).to(DEV) for _ in range(2)]
    gu, h = K_.linear_swiglu_fwd(x, wg, wu)
    gu_ref = K_.linear_fwd(x, [wg, wu], tile=12 if I % 256 == 0 else 2)
    h_ref = K_.swiglu_fwd(gu_ref[:, :I], gu_ref[:, I:])
    torch.cuda.synchronize()
    assert torch.equal(gu, gu_ref)
    assert torch.equal(h, h_ref)
    if I % 256:
        return
    wd = (torch.randn(H, I) / math.sqrt(I)).to(BF).to(DEV)
    dm = torch.randn(T, H).to(BF).to(DEV)
    dgu = K_.linear_dgrad_swiglu(dm, wd, gu)
    dh = K_.linear_dgrad(dm, [wd], tile=12)
    dg, du = K_.swiglu_bwd(dh, gu[:, :I], gu[:, I:])
    torch.cuda.synchronize()
    assert torch.equal(dgu[:, :I], dg)
    assert torch.equal(dgu[:, I:], du)


def test_mlp_block_split_swiglu_equals_fused(monkeypatch):
    """Below the tile thresholds (a TP = 8 shard) the MLP runs its SwiGLU forward / backward as
    separate kernels beside plain GEMMs: output, dX and all three dW bit-identical to the fused
    epilogues."""
    from picotron_amd import functional as FN
    from picotron_amd import kernels as K_
    T, H, I = 1024, 256, 512
    x = torch.randn(T, H).to(BF).to(DEV)
    ws = [(torch.randn(o, i) / math.sqrt(i)).to(BF).to(DEV) for o, i in ((I, H), (I, H), (H, I))]
    dm = torch.randn(T, H).to(BF).to(DEV)
    outs = []
    for thr in (0, 1 << 30):
        monkeypatch.setattr(switches.S, "swiglu_fuse_min_tiles", thr)
        monkeypatch.setattr(switches.S, "swiglu_bwd_min_tiles", thr)
        wl = [w.clone().requires_grad_(True) for w in ws]
        tp = FN.TPContext()
        m, saved = FN.mlp_block_fwd(x, *wl, tp)
        dx = FN.mlp_block_bwd(dm, x, saved, *wl, tp)
        torch.cuda.synchronize()
        outs.append([m.clone(), dx.clone()] + [w.grad.clone() for w in wl])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("swiglu", [True, False])
@pytest.mark.parametrize("epi", [0, 1, 3])
@pytest.mark.parametrize("order", [0, 1, 2])
def test_gemm_dual_equals_separate(swiglu, epi, order, monkeypatch):
    """pt_gemm_dual (a dX group and a wgrad group in one launch, every dispatch order) == the two
    groups as separate 256x256 launches, bit for bit: the down_proj dX with the SwiGLU backward
    beside its dW, and a K-segmented q|k|v dX beside the q|k|v + o_proj dWs (unsplit dW: the split-K
    dW beside a dX is test_gemm_dual_with_ksplit_wgrad)"""
    from picotron_amd import kernels as K_
    monkeypatch.setattr(switches.S, "ksplit", 0)
    T, H = 1024, 512
    dt = torch.float32 if epi == 3 else BF
    if swiglu:
        I = 1024
        dm = torch.randn(T, H).to(BF).to(DEV)
        wd = (torch.randn(H, I) / math.sqrt(I)).to(BF).to(DEV)
        gu = torch.randn(T, 2 * I).to(BF).to(DEV)
        hh = torch.randn(T, I).to(BF).to(DEV)
        init = [torch.randn(H, I).to(dt).to(DEV)]
        wj = lambda outs: [(dm, hh, outs)]
        outs = [t.clone() for t in init]
        dx = K_.linear_dgrad_dual(dm, [wd], wj(outs), epi, gu=gu, order=order)
        ref_dx = K_.linear_dgrad_swiglu(dm, wd, gu)
    else:
        H, nkv = 1024, 512
        dqkv = torch.randn(T, H + 2 * nkv).to(BF).to(DEV)
        ws = [(torch.randn(n, H) / math.sqrt(H)).to(BF).to(DEV) for n in (H, nkv, nkv)]
        h, da, o = [torch.randn(T, H).to(BF).to(DEV) for _ in range(3)]
        init = [torch.randn(n, H).to(dt).to(DEV) for n in (H, nkv, nkv, H)]
        outs = [t.clone() for t in init]
        wj = lambda o_: [(dqkv, h, o_[:3]), (da, o, o_[3:])]
        dx = K_.linear_dgrad_dual(dqkv, ws, wj(outs), epi, order=order)
        ref_dx = K_.linear_dgrad(dqkv, ws, tile=12)
    assert dx is not None
    refs = [t.clone() for t in init]
    K_.linear_wgrad_grouped(wj(refs), epilogue=epi, tile=12)
    torch.cuda.synchronize()
    assert torch.equal(dx, ref_dx)
    for a, b in zip(outs, refs):
        assert torch.equal(a, b)


def test_gemm_dual_unsupported_returns_none():
    """a group whose tile count is not a multiple of 8 is refused before anything runs"""
    from picotron_amd import kernels as K_
    T, H = 256, 512   # dX: 1 x 2 tiles
    dy = torch.randn(T, H).to(BF).to(DEV)
    w = torch.randn(H, H).to(BF).to(DEV)
    out = torch.zeros(H, H, dtype=BF, device=DEV)
    assert not K_.dual_fits((T, H), [(H, H)])
    assert K_.linear_dgrad_dual(dy, [w], [(dy, dy, [out])], 0) is None
    torch.cuda.synchronize()
    assert not out.any()


@pytest.mark.parametrize("T,Kin,ns,kmin", [(1024, 2048, [8192, 8192], 8192), (512, 2048, [16384], 8192),
                                           (4096, 2048, [8192, 8192], 8192), (4096, 2048, [2048] * 3, 1024)])
def test_dgrad_splitk(T, Kin, ns, kmin, monkeypatch):
    """dgrad split in two K halves (f32 partials on 256x256 tiles + the sum pass; the last shape's
    halves cut through the middle weight, as q|k|v's) against the single pass (PICOTRON_SPLITK2=0)
    and an f32 reference: the same up to the f32 summation order (one bf16 rounding either way)"""
    from picotron_amd import kernels as K_
    monkeypatch.setattr(switches.S, "splitk2_min", kmin)
    dy = torch.randn(T, sum(ns)).to(BF).to(DEV)
    ws = [(torch.randn(n, Kin) / math.sqrt(sum(ns))).to(BF).to(DEV) for n in ns]
    assert K_._splitk_halves(T, Kin, sum(ns)) is not None
    dx = K_.linear_dgrad(dy, ws)
    monkeypatch.setattr(switches.S, "splitk2", 0)
    ref1 = K_.linear_dgrad(dy, ws)
    ref = (dy.float() @ torch.cat(ws).float())
    torch.cuda.synchronize()
    assert rel_err(dx, ref) < 4e-3
    assert maxabs(dx, ref1) <= 2 * ref1.float().abs().max().item() * 2 ** -8
    assert rel_err(dx, ref1) < 4e-3


@pytest.mark.parametrize("epi", [1, 3])
def test_gemm_dual_splitk_dgrad(epi):
    """the split-K gate|up dX (two f32 K halves) and the gate|up dW in one dual launch == the split-K
    dX and the wgrad launched separately, bit for bit"""
    from picotron_amd import kernels as K_
    T, H, I = 1024, 2048, 8192
    dgu = torch.randn(T, 2 * I).to(BF).to(DEV)
    h2 = torch.randn(T, H).to(BF).to(DEV)
    wg, wu = [(torch.randn(I, H) / math.sqrt(2 * I)).to(BF).to(DEV) for _ in range(2)]
    dt = torch.float32 if epi == 3 else BF
    init = [torch.randn(I, H).to(dt).to(DEV) for _ in range(2)]
    outs_a, outs_b = [t.clone() for t in init], [t.clone() for t in init]
    assert K_._splitk_halves(T, H, 2 * I) is not None
    dx = K_.linear_dgrad_dual(dgu, [wg, wu], [(dgu, h2, outs_a)], epi)
    assert dx is not None
    dx_ref = K_.linear_dgrad(dgu, [wg, wu])
    K_.linear_wgrad(dgu, h2, outs_b, epilogue=epi)
    torch.cuda.synchronize()
    assert torch.equal(dx, dx_ref)
    for a, b in zip(outs_a, outs_b):
        assert torch.equal(a, b)


@pytest.mark.parametrize("residual", [False, True])
def test_fwd_splitk(residual, monkeypatch):
    """forward GEMM split in two K halves, the residual add (EPI_BF16_RES: bf16(R + bf16(acc))) in
    the sum pass, against the single pass and an f32 reference (down_proj's shape: K 8192)"""
    from picotron_amd import kernels as K_
    monkeypatch.setattr(switches.S, "splitk2_min", 4096)
    T, K, N = 4096, 8192, 2048
    x = torch.randn(T, K).to(BF).to(DEV)
    w = (torch.randn(N, K) / math.sqrt(K)).to(BF).to(DEV)
    r = torch.randn(T, N).to(BF).to(DEV) if residual else None
    assert K_._splitk_halves(T, N, K) is not None
    y = K_.linear_fwd(x, [w], residual=r)
    monkeypatch.setattr(switches.S, "splitk2", 0)
    y1 = K_.linear_fwd(x, [w], residual=r)
    ref = x.float() @ w.float().t() + (r.float() if residual else 0)
    torch.cuda.synchronize()
    assert rel_err(y, ref) < 4e-3
    assert rel_err(y, y1) < 4e-3
    assert maxabs(y, y1) <= 2 * y1.float().abs().max().item() * 2 ** -8


@pytest.mark.parametrize("nh,nkv,S,fuse", [(4, 2, 256, True), (8, 8, 128, True), (16, 16, 512, True),
                                            (32, 32, 1024, True), (4, 4, 2048, False)])
def test_gemm_rope_fused(monkeypatch, nh, nkv, S, fuse):
    """q|k|v projection with RoPE in the epilogue == projection + rope kernel, bit for bit (the
    third and fourth shapes take the mixed 256x256 / 256x128 launch, the first two a single tile
    shape; fuse=False: a TP-shard width below the fusion threshold, plain GEMM + rope kernel)"""
    from picotron_amd import kernels as K_
    monkeypatch.setattr(switches.S, "rope_fuse_min_tiles", 0 if fuse else 96)
    d, B = 64, 2
    T, H = B * S, 256
    x = torch.randn(T, H).to(BF).to(DEV)
    ws = [(torch.randn(n * d, H) / math.sqrt(H)).to(BF).to(DEV) for n in (nh, nkv, nkv)]
    cos, sin = [t.to(DEV) for t in O.get_cos_sin(S, d, base=10000.0)]
    y = K_.linear_fwd_rope(x, ws, cos, sin, S, nh + nkv, d)
    ref = K_.linear_fwd(x, ws)
    K_.rope_(ref, nh + nkv, d, cos, sin, S)
    torch.cuda.synchronize()
    assert torch.equal(y, ref)


@pytest.mark.parametrize("D", [64, 128])
def test_attention_bwd_rope_fused(D):
    """attention backward with the RoPE backward fused into the dq / dk stores == attention
    backward + inverse rope kernel, bit for bit"""
    from picotron_amd import kernels as K_
    B, S, H, HKV = 2, 256, 4, 2
    T = B * S
    qkv = torch.randn(T, (H + 2 * HKV) * D).to(BF).to(DEV)
    sh = lambda t, lo, n: t.view(B, S, -1)[:, :, lo * D:(lo + n) * D].view(B, S, n, D)
    q, k, v = sh(qkv, 0, H), sh(qkv, H, HKV), sh(qkv, H + HKV, HKV)
    do = torch.randn(B, S, H, D).to(BF).to(DEV)
    cos, sin = [t.to(DEV) for t in O.get_cos_sin(S, D, base=10000.0)]
    scale = D ** -0.5
    o, lse = K_.attn_fwd(q, k, v, scale, True)
    d1 = torch.empty_like(qkv)
    K_.attn_bwd(do, q, k, v, o, lse, scale, True, dq=sh(d1, 0, H), dk=sh(d1, H, HKV), dv=sh(d1, H + HKV, HKV),
                rope=(cos, sin))
    d2 = torch.empty_like(qkv)
    K_.attn_bwd(do, q, k, v, o, lse, scale, True, dq=sh(d2, 0, H), dk=sh(d2, H, HKV), dv=sh(d2, H + HKV, HKV))
    K_.rope_(d2, H + HKV, D, cos, sin, S, inverse=True)
    torch.cuda.synchronize()
    assert torch.equal(d1, d2)


def test_gemm_segmented_qkv():
    """fused q|k|v forward, dX over stacked weights, dW into three outputs: one launch each."""
    from picotron_amd import kernels as K_
    T, H, nkv = 1024, 512, 256
    x = torch.randn(T, H).to(BF)
    ws = [(torch.randn(n, H) / math.sqrt(H)).to(BF) for n in (H, nkv, nkv)]
    wd = [w.to(DEV) for w in ws]
    y = K_.linear_fwd(x.to(DEV), wd)
    ref = _ref_mm(x, torch.cat(ws).t())
    assert rel_err(y, ref) < 1e-2
    dy = torch.randn(T, H + 2 * nkv).to(BF)
    dx = K_.linear_dgrad(dy.to(DEV), wd)
    assert rel_err(dx, _ref_mm(dy, torch.cat(ws))) < 1e-2
    outs = [torch.empty_like(w) for w in wd]
    K_.linear_wgrad(dy.to(DEV), x.to(DEV), outs)
    ref_w = _ref_mm(dy.t(), x)
    lo = 0
    for o, w in zip(outs, ws):
        assert rel_err(o, ref_w[lo:lo + w.shape[0]]) < 1e-2
        lo += w.shape[0]


def test_gemm_accumulate_epilogues():
    from picotron_amd import kernels as K_
    T, N, K = 512, 256, 256
    dy, x = torch.randn(T, N).to(BF), torch.randn(T, K).to(BF)
    base = torch.randn(N, K)
    # f32 accumulate (main_grad)
    acc = base.clone().to(DEV)
    K_.linear_wgrad(dy.to(DEV), x.to(DEV), [acc], epilogue=K_.EPI_F32_ACC)
    assert rel_err(acc, base + _ref_mm(dy.t(), x)) < 1e-3
    # bf16 accumulate (param.grad in bf16 across micro-batches)
    accb = base.to(BF).to(DEV)
    K_.linear_wgrad(dy.to(DEV), x.to(DEV), [accb], epilogue=K_.EPI_BF16_ACC)
    assert rel_err(accb, base.to(BF).float() + _ref_mm(dy.t(), x)) < 1e-2


def test_gemm_asymmetric_exact():
    """A = I with an asymmetric B catches a transposed C write (guide §3)."""
    from picotron_amd import kernels as K_
    n = 256
    eye = torch.eye(n).to(BF)
    b = torch.arange(n * n, dtype=torch.float32).reshape(n, n).remainder(251).to(BF)
    y = K_.linear_fwd(eye.to(DEV), [b.to(DEV)])   # y = I . b^T
    assert torch.equal(y.cpu(), b.t().contiguous())


# ------------------------------------------------------------------------- attention
def _qkv(B, S, H, HKV, D, fused=True):
    T = B * S
    buf = torch.randn(T, (H + 2 * HKV) * D).to(BF)
    d = buf.to(DEV)
    q = d[:, :H * D].view(B, S, H, D)
    k = d[:, H * D:(H + HKV) * D].view(B, S, HKV, D)
    v = d[:, (H + HKV) * D:].view(B, S, HKV, D)
    return q, k, v


def _ref_attn(q, k, v, causal, scale):
    # [B,S,H,D] -> [B,H,S,D], GQA by repeat_interleave (model.py:142-143)
    rep = q.shape[2] // k.shape[2]
    qq = q.float().cpu().transpose(1, 2)
    kk = k.float().cpu().transpose(1, 2).repeat_interleave(rep, 1)
    vv = v.float().cpu().transpose(1, 2).repeat_interleave(rep, 1)
    return qq, kk, vv


@pytest.mark.parametrize("B,S,H,HKV,D,causal", [(2, 128, 4, 4, 64, True), (1, 256, 4, 2, 64, True),
                                                 (2, 256, 2, 2, 128, True), (1, 128, 2, 1, 128, False),
                                                 (1, 512, 2, 2, 64, False), (2, 1024, 2, 2, 64, True)])
def test_attention_fwd_bwd(B, S, H, HKV, D, causal):
    from picotron_amd import kernels as K_
    q, k, v = _qkv(B, S, H, HKV, D)
    scale = 1 / math.sqrt(D)
    o, lse = K_.attn_fwd(q, k, v, scale, causal)
    qq, kk, vv = _ref_attn(q, k, v, causal, scale)
    qq.requires_grad_(True); kk.requires_grad_(True); vv.requires_grad_(True)
    o_ref, lse_ref = O.attention_lse(qq, kk, vv, scale, causal)
    assert rel_err(o, o_ref.transpose(1, 2)) < 1e-2
    assert maxabs(lse, lse_ref) < 1e-2
    do = torch.randn(o.shape).to(BF)
    (o_ref * do.float().transpose(1, 2)).sum().backward()
    dq, dk, dv, _ = K_.attn_bwd(do.to(DEV), q, k, v, o, lse, scale, causal)
    torch.cuda.synchronize()
    rep = H // HKV
    dk_ref = kk.grad.view(B, HKV, rep, S, D).sum(2).transpose(1, 2)
    dv_ref = vv.grad.view(B, HKV, rep, S, D).sum(2).transpose(1, 2)
    assert rel_err(dq, qq.grad.transpose(1, 2)) < 2e-2
    assert rel_err(dk, dk_ref) < 2e-2
    assert rel_err(dv, dv_ref) < 2e-2


@pytest.mark.parametrize("D,causal", [(60, True), (80, False), (96, True)])
def test_flash_attention_api_padded_head_dims(D, causal):
    """model.flash_attention (flash_attn_func's call form) at head dims the kernels do not take:
    zero-padded to 64 / 128 (scale of the real D), out and dq / dk / dv against the oracle."""
    from picotron_amd.model import flash_attention
    B, S, H = 2, 256, 4
    g = torch.Generator().manual_seed(3)
    q, k, v, do = (torch.randn(B, H, S, D, generator=g).to(BF) for _ in range(4))
    qd, kd, vd = (t.to(DEV).requires_grad_(True) for t in (q, k, v))
    out = flash_attention(qd, kd, vd, causal)                        # [B, S, H, D]
    out.backward(do.transpose(1, 2).to(DEV))
    qr, kr, vr = (t.float().requires_grad_(True) for t in (q, k, v))
    o_ref, _ = O.attention_lse(qr, kr, vr, 1 / math.sqrt(D), causal)
    o_ref.backward(do.float())
    assert out.shape == (B, S, H, D) and rel_err(out, o_ref.transpose(1, 2)) < 1e-2
    for got, ref in ((qd.grad, qr.grad), (kd.grad, kr.grad), (vd.grad, vr.grad)):
        assert rel_err(got, ref) < 2e-2


@pytest.mark.parametrize("B,S,H,HKV,D", [(2, 200, 4, 2, 64), (1, 1000, 4, 4, 128), (2, 72, 2, 1, 64)])
def test_attention_off_block_sequence_lengths(B, S, H, HKV, D):
    """Causal attention at sequence lengths off the kernels' 128-row query blocks (kernels.attn_fwd /
    attn_bwd zero-pad q / k / v; the padded keys are causally invisible, the padded queries carry
    dO = 0 and LSE = +inf): out, lse and dq / dk / dv against the oracle."""
    from picotron_amd import kernels as K_
    q, k, v = _qkv(B, S, H, HKV, D)
    scale = 1 / math.sqrt(D)
    o, lse = K_.attn_fwd(q, k, v, scale, True)
    assert o.shape == (B, S, H, D) and lse.shape == (B, H, S)
    qq, kk, vv = _ref_attn(q, k, v, True, scale)
    qq.requires_grad_(True); kk.requires_grad_(True); vv.requires_grad_(True)
    o_ref, lse_ref = O.attention_lse(qq, kk, vv, scale, True)
    assert rel_err(o, o_ref.transpose(1, 2)) < 1e-2
    assert maxabs(lse, lse_ref) < 1e-2
    do = torch.randn(o.shape).to(BF)
    (o_ref * do.float().transpose(1, 2)).sum().backward()
    dq, dk, dv, _ = K_.attn_bwd(do.to(DEV), q, k, v, o, lse, scale, True)
    torch.cuda.synchronize()
    rep = H // HKV
    assert rel_err(dq, qq.grad.transpose(1, 2)) < 2e-2
    assert rel_err(dk, kk.grad.view(B, HKV, rep, S, D).sum(2).transpose(1, 2)) < 2e-2
    assert rel_err(dv, vv.grad.view(B, HKV, rep, S, D).sum(2).transpose(1, 2)) < 2e-2


@pytest.mark.parametrize("B,S,H,HKV,D,causal,f32,rope", [
    (2, 1024, 4, 4, 64, True, False, True), (1, 512, 4, 2, 64, True, False, False),
    (1, 384, 2, 1, 64, True, False, False), (1, 512, 2, 2, 128, True, False, True),
    (1, 1024, 4, 2, 128, False, True, False), (2, 256, 2, 2, 64, False, True, False),
    (1, 2048, 2, 2, 128, True, False, False)])
def test_attention_dkdv_wave_pair_split_is_bit_identical(monkeypatch, B, S, H, HKV, D, causal, f32, rope):
    """The dK/dV kernel split over wave pairs (score wave -> P|dS hand-off -> accumulator wave) runs
    the same MFMA operands in the same order as the one-wave kernel: dq, dk, dv bit-identical
    (causal pairing on and off, GQA, d 64 / 128, f32 ring accumulators, fused RoPE backward)."""
    from picotron_amd import kernels as K_
    q, k, v = _qkv(B, S, H, HKV, D)
    scale = 1 / math.sqrt(D)
    o, lse = K_.attn_fwd(q, k, v, scale, causal)
    do = torch.randn(o.shape).to(BF).to(DEV)
    rp = None
    if rope:
        rp = tuple(t.to(DEV) for t in O.get_cos_sin(S, D, base=10000.0))
    outs = []
    for mask in (0, 3):
        with switches.override(attn_split=mask):
            if f32:
                g = [torch.full((B, S, n, D), 0.25, device=DEV) for n in (H, HKV, HKV)]
                K_.attn_bwd(do, q, k, v, o, lse, scale, causal, dq=g[0], dk=g[1], dv=g[2], grad_f32=True)
            else:
                g = K_.attn_bwd(do, q, k, v, o, lse, scale, causal, rope=rp)[:3]
            torch.cuda.synchronize()
        outs.append([t.clone() for t in g])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_attention_ring_merge_matches_full():
    """Two key blocks merged by the fused update_out_and_lse epilogue == attention over both
    (context_parallel.py:157-187), and the backward with the global LSE sums to the full grads."""
    from picotron_amd import kernels as K_
    B, S, H, D = 1, 256, 2, 64
    q, k, v = _qkv(B, 2 * S, H, H, D)
    scale = 1 / math.sqrt(D)
    q2 = q[:, S:]                       # queries of the second shard
    acc = torch.zeros(B, S, H, D, dtype=torch.float32, device=DEV)
    lse = torch.full((B, H, S), float("-inf"), device=DEV)
    K_.attn_fwd(q2, k[:, S:], v[:, S:], scale, True, out=acc, lse=lse, merge=True)   # diagonal block
    K_.attn_fwd(q2, k[:, :S], v[:, :S], scale, False, out=acc, lse=lse, merge=True)  # earlier block
    qq, kk, vv = _ref_attn(q, k, v, True, scale)
    o_ref, lse_ref = O.attention_lse(qq, kk, vv, scale, True)
    assert rel_err(acc, o_ref[:, :, S:].transpose(1, 2)) < 1e-2
    assert maxabs(lse, lse_ref[:, :, S:]) < 1e-2


# ------------------------------------------------------------------------------ embedding
@pytest.mark.parametrize("lo,hi,pad", [(0, 512, None), (128, 384, None), (0, 512, 7)])
def test_embedding_fwd_bwd_matches_torch(lo, hi, pad):
    """masked lookup + backward into the grad sink == F.embedding (+ VocabParallel masking) and
    autograd's dense backward / AccumulateGrad, over two micro-batches with repeated ids"""
    import torch.nn.functional as F
    from picotron_amd import functional as FN
    V, H, T = 512, 256, 1024
    g = torch.Generator().manual_seed(0)
    w0 = torch.randn(hi - lo, H, generator=g).to(BF).to(DEV)
    ids = [torch.randint(0, 64, (T,), generator=g).to(DEV), torch.randint(0, V, (T,), generator=g).to(DEV)]
    dys = [torch.randn(T, H, generator=g).to(BF).to(DEV) for _ in range(2)]
    w = torch.nn.Parameter(w0.clone())
    wr = torch.nn.Parameter(w0.clone())
    for t, dy in zip(ids, dys):
        y = FN.embedding(t, w, lo, hi, pad)
        mask = (t < lo) | (t >= hi)
        yr = F.embedding(torch.where(mask, torch.zeros_like(t), t - lo), wr,
                         None if pad is None else pad - lo).masked_fill(mask[:, None], 0.0)
        assert torch.equal(y, yr)
        y.backward(dy)
        yr.backward(dy)
    torch.cuda.synchronize()
    assert rel_err(w.grad, wr.grad.float().cpu()) < 1e-2
    a, b = w.grad.float(), wr.grad.float()
    # f32 sums in a different order, then three bf16 roundings on each side (sum of micro-batch 1,
    # sum of micro-batch 2, their sum): each error <= 2^-9 x the absolute mass of the dY rows summed
    # (cancellation can make the result itself tiny, so the bound is on the mass, not the result)
    mass = torch.zeros(hi - lo, H, device=DEV)
    for t, dy in zip(ids, dys):
        keep = (t >= lo) & (t < hi) & (t != (-1 if pad is None else pad))
        mass.index_add_(0, (t - lo)[keep], dy.float().abs()[keep])
    assert ((a - b).abs() <= 2.0 ** -6 * mass + 1e-6).all()
    # bit-exact against the kernel's documented order: f32 sum over the tokens of an id in ascending
    # position, rounded to bf16 once, added to the bf16 gradient with one more rounding
    gref = torch.zeros(hi - lo, H, dtype=BF)
    for t, dy in zip(ids, dys):
        acc = torch.zeros(hi - lo, H)
        tc, dc = t.cpu(), dy.float().cpu()
        for i in range(T):
            r = int(tc[i])
            if lo <= r < hi and r != pad:
                acc[r - lo] += dc[i]
        gref = (gref.float() + acc.to(BF).float()).to(BF)
    assert torch.equal(w.grad.cpu(), gref)


@pytest.mark.parametrize("V", [96, 49152, 32000, 80000, 8])
def test_cross_entropy_lse_pair(V):
    """The autograd pair (streaming forward saving the row LSE, elementwise backward) against
    torch fp32 F.cross_entropy / grad_acc, with an ignore_index row, and against the reference's
    own bf16 golden vector G9."""
    from picotron_amd import kernels as K
    T, ga = 64, 4
    logits = (3 * torch.randn(T, V)).to(BF)
    tgt = torch.randint(0, V, (T,))
    tgt[5] = -100
    lr = logits.float().requires_grad_(True)
    loss_ref = torch.nn.functional.cross_entropy(lr, tgt) / ga
    loss_ref.backward()
    lg, tg = logits.to(DEV), tgt.to(DEV)
    loss, inv_count, lse = K.cross_entropy_loss_lse(lg, tg)
    lse_ref = torch.logsumexp(logits.float(), dim=1)
    assert (lse.cpu() - lse_ref).abs().max().item() < 1e-4 * max(1.0, lse_ref.abs().max().item())
    grad = K.cross_entropy_grad_lse(lg, tg, lse, inv_count / ga)
    torch.cuda.synchronize()
    assert abs(loss.item() / ga - loss_ref.item()) < 1e-3 * max(1, abs(loss_ref.item()))
    assert rel_err(grad, lr.grad) < 1e-2
    assert grad[5].float().abs().max().item() == 0.0
    assert torch.equal(lg.cpu(), logits)                      # logits untouched (user-visible)


def test_cross_entropy_lse_pair_golden_vector():
    import os
    from picotron_amd import kernels as K
    g = torch.load(os.path.join(os.path.dirname(__file__), "golden", "G9.pt"), weights_only=True)
    lg = g["logits"].view(16, -1).to(DEV)
    tg = g["targets"].reshape(-1).to(DEV)
    ga = int(g["grad_acc"])
    loss, inv_count, lse = K.cross_entropy_loss_lse(lg, tg)
    grad = K.cross_entropy_grad_lse(lg, tg, lse, inv_count / ga)
    assert abs(loss.item() / ga - g["loss"].float().item()) < 2e-2 * abs(g["loss"].float().item())
    assert rel_err(grad, g["dlogits"].view(16, -1)) < 2e-2


@pytest.mark.parametrize("ns,T,Kin,acc", [([2048, 2048, 2048], 4096, 2048, False), ([8192, 8192], 4096, 2048, True),
                                           ([4096], 2048, 1024, False)])
def test_dgrad_k_segmented(ns, T, Kin, acc):
    """dX = dY . [W_0; ...] with K-segmented B (the q|k|v and gate|up dX at SmolLM dims) vs torch
    fp32, store and bf16-accumulate epilogues, auto tile vs the 256x128 kernel (tile 13)."""
    from picotron_amd import kernels as K
    N = sum(ns)
    dy = torch.randn(T, N, device=DEV).to(BF)
    ws = [(torch.randn(n, Kin, device=DEV) * 0.02).to(BF) for n in ns]
    ref = dy.float() @ torch.cat(ws, 0).float()
    base = torch.randn(T, Kin, device=DEV).to(BF) if acc else None
    dx = K.linear_dgrad(dy, ws, out=base.clone() if acc else None, accumulate=acc)
    want = ref + base.float() if acc else ref
    assert rel_err(dx, want) < 1e-2
    one = K.linear_dgrad(dy, ws, out=base.clone() if acc else None, accumulate=acc, tile=13)
    assert rel_err(dx, one.float()) < 5e-3


@pytest.mark.parametrize("T,lo,hi,pad", [(4096, 0, 49152, None), (1000, 100, 300, 150), (17, 0, 8, 3),
                                         (16384, 0, 49152, 7), (5000, 0, 70000, None), (20000, 0, 512, None)])
def test_embedding_sort_equals_torch_stable_sort(T, lo, hi, pad):
    """pt_embedding_sort (one-workgroup LSD radix sort of (key, position), 4 key bits per pass) ==
    torch.sort(stable) of the keyed ids, bit for bit -- at the most tokens it holds (16384) and with a
    key width that is not a multiple of 4 bits (hi 70000: 17 bits); T > 16384 takes torch's device
    sort (same result by construction)."""
    from picotron_amd import _C
    from picotron_amd import kernels as K
    g = torch.Generator().manual_seed(T)
    ids = torch.randint(0, max(hi + 50, 64), (T,), generator=g).to(DEV)
    skip = (ids < lo) | (ids >= hi)
    if pad is not None:
        skip = skip | (ids == pad)
    ref_ids, ref_perm = torch.sort(torch.where(skip, torch.full_like(ids, -1), ids), stable=True)
    s_ids = torch.empty(T, dtype=torch.int64, device=DEV)
    perm = torch.empty(T, dtype=torch.int64, device=DEV)
    rc = _C.lib().pt_embedding_sort(K._ptr(ids), T, lo, hi, int(pad is not None), pad or 0, K._ptr(s_ids),
                                    K._ptr(perm), _C.stream_ptr(ids.device))
    if T > 16384:
        assert rc == -3
        return
    assert rc == 0
    assert torch.equal(s_ids, ref_ids) and torch.equal(perm, ref_perm)


def test_cross_entropy_mean_kernel():
    """pt_cross_entropy_mean: mean over the valid rows (ignore_index excluded), 1/#valid, bf16 / f32
    output; all rows ignored -> NaN (torch's mean of an empty selection)."""
    from picotron_amd import kernels as K
    rows = 4096
    rl = torch.rand(rows, device=DEV) * 5
    tg = torch.randint(0, 100, (rows,), device=DEV)
    tg[::7] = -100
    rl[::7] = 0.0
    valid = (tg != -100).sum().item()
    for dt in (torch.float32, BF):
        loss, inv = K._ce_mean(rl, tg, -100, dt)
        assert loss.dtype == dt and abs(inv.item() - 1.0 / valid) < 1e-9
        ref = rl.double().sum().item() / valid
        assert abs(loss.float().item() - ref) <= (1e-6 if dt == torch.float32 else 2 ** -8) * ref
    loss, _ = K._ce_mean(torch.zeros_like(rl), torch.full_like(tg, -100), -100, torch.float32)  # rows all 0
    assert math.isnan(loss.item())


@pytest.mark.parametrize("M,N,K,kind,residual", [(4096, 768, 2048, "fwd", False), (4096, 256, 2048, "dgrad", False),
                                                 (4096, 512, 2048, "fwd", True), (2048, 384, 1024, "fwd", False)])
def test_fewtile_forms_match_single_pass(monkeypatch, M, N, K, kind, residual):
    """The TP-shard forward / dX GEMMs whose tiles leave most CUs idle (SmolLM-1.7B at TP = 8: the
    q|k|v forward 4096 x 768 x 2048, the o_proj dX 4096 x 256 x 2048) run on the 128x128 k-substep
    tile, as 2 K-slices + the reduce pass where its tiles still fill half a round (kernels.hq_form):
    against an f32 reference and the unsplit launch (PICOTRON_KSPLIT=0), equal up to the f32
    summation order (<= 2 bf16 ulps)."""
    from picotron_amd import kernels as K_
    assert K_.hq_form([(M, N, K) if kind == "fwd" else (M, N, K)]) >= 1, (M, N, K)
    if kind == "fwd":
        x = torch.randn(M, K).to(BF).to(DEV)
        ws = [(torch.randn(n, K) / math.sqrt(K)).to(BF).to(DEV) for n in (N // 2, N // 2)]
        r = torch.randn(M, N).to(BF).to(DEV) if residual else None
        run = lambda: K_.linear_fwd(x, ws, residual=r)  # noqa: E731
        ref = x.float() @ torch.cat(ws).float().t() + (r.float() if residual else 0)
    else:
        dy = torch.randn(M, K).to(BF).to(DEV)
        w = (torch.randn(K, N) / math.sqrt(K)).to(BF).to(DEV)
        run = lambda: K_.linear_dgrad(dy, [w])  # noqa: E731
        ref = dy.float() @ w.float()
    y = run()
    monkeypatch.setattr(switches.S, "ksplit", 0)
    y1 = run()
    torch.cuda.synchronize()
    assert rel_err(y, ref) < 4e-3
    assert maxabs(y, y1) <= 2 * y1.float().abs().max().item() * 2 ** -8


@pytest.mark.parametrize("B,S,H,HKV,causal,rope", [(4, 1024, 4, 4, True, True), (2, 1024, 4, 2, True, False),
                                                   (1, 512, 2, 2, False, False), (4, 1024, 4, 4, True, False)])
@pytest.mark.parametrize("chunk", [2, 4, 6])
def test_attention_few_head_split_forms(B, S, H, HKV, causal, rope, chunk):
    """The few-head split forms (pt_attn_split_plan: the regular launch would put < 128 workgroups on
    the 256 CUs -- a TP = 8 shard of SmolLM-1.7B is B 4 x 4 heads): forward work items of `chunk`
    K/V tiles + the LSE merge, backward dQ / dK|dV items + reduce passes (the RoPE backward in the
    reduce), against the regular kernels (attn_kv_chunk = 0) to f32-summation-order rounding and
    against the fp32 oracle at bf16 tolerance."""
    from picotron_amd import kernels as K_
    D = 64
    q, k, v = _qkv(B, S, H, HKV, D)
    scale = 1 / math.sqrt(D)
    do = torch.randn(B, S, H, D).to(BF).to(DEV)
    rp = tuple(t.to(DEV) for t in O.get_cos_sin(S, D, base=10000.0)) if rope else None
    res = {}
    for ck in (0, chunk):
        with switches.override(attn_kv_chunk=ck):
            assert (K_._attn_split_ws(B, H, HKV, S, S, D, causal, 0, DEV) is not None) == (ck > 0)
            o, lse = K_.attn_fwd(q, k, v, scale, causal)
            dq, dk, dv, delta = K_.attn_bwd(do, q, k, v, o, lse, scale, causal, rope=rp)
        torch.cuda.synchronize()
        res[ck] = [t.clone() for t in (o, lse, dq, dk, dv, delta)]
    for name, a, b in zip(("o", "lse", "dq", "dk", "dv", "delta"), res[chunk], res[0]):
        assert torch.isfinite(a.float()).all(), name
        assert rel_err(a, b.float().cpu()) < 4e-3, name      # f32 summation order, then bf16 rounding
    qq, kk, vv = _ref_attn(q, k, v, causal, scale)
    qq.requires_grad_(True); kk.requires_grad_(True); vv.requires_grad_(True)
    o_ref, lse_ref = O.attention_lse(qq, kk, vv, scale, causal)
    o, lse, dq, dk, dv, _ = res[chunk]
    assert rel_err(o, o_ref.transpose(1, 2)) < 1e-2 and maxabs(lse, lse_ref) < 1e-2
    if not rope:
        (o_ref * do.float().cpu().transpose(1, 2)).sum().backward()
        rep = H // HKV
        assert rel_err(dq, qq.grad.transpose(1, 2)) < 2e-2
        assert rel_err(dk, kk.grad.view(B, HKV, rep, S, D).sum(2).transpose(1, 2)) < 2e-2
        assert rel_err(dv, vv.grad.view(B, HKV, rep, S, D).sum(2).transpose(1, 2)) < 2e-2




@pytest.mark.parametrize("epi", ["bf16", "bf16_acc", "f32_acc"])
def test_paired_wgrad_k_segments(epi):
    """Weight-gradient pairing (functional.WgradPairing): dW = dY_a^T X_a + dY_b^T X_b of two
    micro-batches as ONE K = 2 T GEMM whose A (pt_gemm_problem.A2) and B (two K-segments) operands
    are the two micro-batches' row blocks (kernels.KPair) -- grouped (q|k|v + o_proj shapes, column
    slices of one dY buffer as the model passes them) and beside a dX group in the dual launch --
    against the fp32 sum and against the two separate launches (equal up to the f32 summation order:
    the pair rounds into the sink once)."""
    from picotron_amd import kernels as K_
    T, H = 1024, 512
    g = torch.Generator().manual_seed(3)

    def rnd(*s, sc=1.0):
        return (torch.randn(*s, generator=g) * sc).to(BF).to(DEV)
    dqkv = [rnd(T, 3 * H) for _ in range(2)]             # two micro-batches' dY [T, q|k|v]
    xs = [rnd(T, H) for _ in range(2)]
    da = [rnd(T, H) for _ in range(2)]
    os_ = [rnd(T, H) for _ in range(2)]
    f32 = epi == "f32_acc"
    dt = torch.float32 if f32 else BF
    e = {"bf16": K_.EPI_BF16, "bf16_acc": K_.EPI_BF16_ACC, "f32_acc": K_.EPI_F32_ACC}[epi]
    base = [(torch.randn(3 * H, H, generator=g) * 0.1).to(dt).to(DEV), (torch.randn(H, H, generator=g) * 0.1).to(dt).to(DEV)]
    init = [b.clone() if epi != "bf16" else torch.zeros_like(b) for b in base]
    ref = [init[0].float() + sum(dqkv[i].float().t() @ xs[i].float() for i in range(2)),
           init[1].float() + sum(da[i].float().t() @ os_[i].float() for i in range(2))]
    # grouped: q|k|v as three row segments of one output, o_proj beside it
    outs = [b.clone() for b in base]
    segs = [outs[0][:H], outs[0][H:2 * H], outs[0][2 * H:]]
    K_.linear_wgrad_grouped([(K_.KPair(dqkv[0], dqkv[1]), K_.KPair(xs[0], xs[1]), segs),
                             (K_.KPair(da[0], da[1]), K_.KPair(os_[0], os_[1]), [outs[1]])], epilogue=e)
    # the separate launches (the unpaired path: first half through e, second accumulating)
    sep = [b.clone() for b in base]
    acc = {K_.EPI_BF16: K_.EPI_BF16_ACC}.get(e, e)
    K_.linear_wgrad_grouped([(dqkv[0], xs[0], [sep[0]]), (da[0], os_[0], [sep[1]])], epilogue=e)
    K_.linear_wgrad_grouped([(dqkv[1], xs[1], [sep[0]]), (da[1], os_[1], [sep[1]])], epilogue=acc)
    # dual: a dX group (q|k|v dX: dY . W) beside the paired dW group
    w = rnd(3 * H, H, sc=0.05)
    dual = [b.clone() for b in base]
    dx = K_.linear_dgrad_dual(dqkv[1], [w], [(K_.KPair(dqkv[0], dqkv[1]), K_.KPair(xs[0], xs[1]), [dual[0]]),
                                             (K_.KPair(da[0], da[1]), K_.KPair(os_[0], os_[1]), [dual[1]])], e)
    torch.cuda.synchronize()
    assert dx is not None and rel_err(dx, dqkv[1].float() @ w.float()) < 4e-3
    tol = 2e-3 if f32 else 6e-3
    for got in (outs, dual):
        for o, r in zip(got, ref):
            assert rel_err(o, r) < tol, epi
    for o, s_, r in zip(outs, sep, ref):   # the pair is no further from the fp32 sum than two launches
        assert rel_err(o, r) <= rel_err(s_, r) * 1.05 + 1e-6
    for a, b in zip(outs, dual):
        assert torch.equal(a, b)               # the same tiles, the same K order


@pytest.mark.parametrize("ga", [4, 3])
def test_paired_wgrad_training_matches_unpaired_and_oracle(ga):
    """train_step with weight-gradient pairing (default) vs without (PICOTRON_WGRAD_PAIR=0) on a small
    Llama, ga micro-batches of one step (4: 2 pairs; 3: a pair and a last micro-batch launched on its
    own), bf16 .grad sinks and fp32 main_grad (a one-rank
    DataParallelBucket is not needed: the main_grad sink is exercised by test_golden_gpu's G8): the
    loss is identical and every gradient agrees to bf16 rounding; both agree with the fp32 oracle's
    accumulated gradients at north_star's tolerance."""
    import types
    import torch.nn.functional as F
    from picotron_amd import process_group_manager as pgm
    from picotron_amd.model import Llama
    from picotron_amd.train import SyntheticMicroBatchDataLoader, train_step
    pgm.setup_process_group_manager(1, 1, 1, 1)
    cfg = types.SimpleNamespace(hidden_size=256, intermediate_size=512, num_attention_heads=4, num_key_value_heads=2,
                                vocab_size=512, rms_norm_eps=1e-5, rope_theta=10000.0, num_hidden_layers=2,
                                max_position_embeddings=256)
    res = {}
    for pair in (1, 0):
        torch.manual_seed(0)
        with torch.device(DEV):
            model = Llama(cfg)
        model.to(BF)
        loader = SyntheticMicroBatchDataLoader(2, 256, ga, cfg.vocab_size, torch.device(DEV), seed=5)
        with switches.override(wgrad_pair=pair):
            loss = train_step(model, loader, DEV)
        torch.cuda.synchronize()
        res[pair] = (loss, {n: p.grad.float().cpu() for n, p in model.named_parameters()})
        if pair:
            params = {n: p.detach().float().cpu().requires_grad_(True) for n, p in model.named_parameters()}
            ids_all = [(loader._inputs[i].cpu(), loader._targets[i].cpu()) for i in range(ga)]
    assert abs(res[1][0] - res[0][0]) < 1e-6 * abs(res[0][0])
    for n in res[0][1]:
        assert rel_err(res[1][1][n], res[0][1][n]) < 1e-2, n
    c = dict(vars(cfg))
    cos, sin = O.get_cos_sin(256, 64, base=10000.0)
    for x, t in ids_all:
        lo = O.llama_forward(x, params, c, cos.float(), sin.float(), norm=O.rmsnorm_flash_semantics)
        (F.cross_entropy(lo.reshape(-1, cfg.vocab_size), t.reshape(-1)) / ga).backward()
    for n, p in params.items():
        assert rel_err(res[1][1][n], p.grad) < 2e-2, n
