"""Host-side launch-shape choices of picotron_amd.kernels (pure functions, no GPU): the K-slice
counts of the TP-shard GEMMs and of the SwiGLU-backward dX, and the split-K halves of the long-K
dX projections -- at the shapes the layer and the TP = 8 proxy launch."""
from picotron_amd import kernels as K
from picotron_amd import switches

T, H, I, V = 4096, 2048, 8192, 49152


def test_swiglu_dx_ksplit_only_at_tp_shard_widths():
    assert K.swiglu_dx_ksplit(T, I // 8, H) == 2          # TP = 8: 64 tiles -> 2 slices (128)
    assert K.swiglu_dx_ksplit(T, I, H) == 1               # TP = 1: 512 tiles, fused epilogue
    assert K.swiglu_dx_ksplit(T, I // 2, H) == 1          # TP = 2: 256 tiles
    assert K.swiglu_dx_ksplit(T, I // 4, H) == 1          # TP = 4: 128 tiles (already half a round)
    assert K.swiglu_dx_ksplit(T, 5504 // 8, 4096) == 1    # not on 256-column tiles
    with switches.override(swiglu_splitk=0):
        assert K.swiglu_dx_ksplit(T, I // 8, H) == 1


def test_wgrad_ksplit_fills_one_round():
    q, o = 3 * H // 8, H // 8
    assert K.wgrad_ksplit([(q, H, T), (H, o, T)]) == 8    # 24 + 8 tiles x 8 = 256
    assert K.wgrad_ksplit([(2 * I // 8, H, T)]) == 4      # gate|up dW: 64 tiles x 4
    assert K.wgrad_ksplit([(H, I // 8, T)], extra_tiles=128) == 4   # down dW: 32 tiles x 4 beside 128 dX slices
    assert K.wgrad_ksplit([(2 * I, H, T)]) == 1           # TP = 1: 512 tiles
    with switches.override(ksplit=0):
        assert K.wgrad_ksplit([(q, H, T), (H, o, T)]) == 1


def test_splitk_halves_for_long_k_dx():
    assert K._splitk_halves(T, H, 2 * I) == I              # gate|up dX: two K-8192 halves
    assert K._splitk_halves(T, H, V) == V // 2             # lm_head dX
    assert K._splitk_halves(T, H, H) is None               # o_proj dX: K 2048
    assert K._splitk_halves(T, H, 3 * H, min_half=1024) == 3 * H // 2   # q|k|v dX beside its dW


def test_reduce_sink_alignment_decided_before_launch():
    """A split-K sink the reduce pass cannot address in 8-B (bf16) / 16-B (f32) row chunks -- or a
    misaligned residual -- keeps the unsplit GEMM (decided before the partial GEMM)."""
    import torch
    buf = torch.empty(64 * 64 + 8, dtype=torch.bfloat16)
    ok = buf[:64 * 64].view(64, 64)
    assert K._reduce_sink_ok(ok)
    assert not K._reduce_sink_ok(buf[1:1 + 64 * 64].view(64, 64))            # 2-B offset
    assert K._reduce_sink_ok(ok, residual=ok)
    assert not K._reduce_sink_ok(ok, residual=buf[2:2 + 64 * 64].view(64, 64))   # 4-B offset residual
    f = torch.empty(64 * 64 + 4, dtype=torch.float32)
    assert not K._reduce_sink_ok(f[2:2 + 64 * 64].view(64, 64))              # 8-B offset f32
    assert not K._reduce_sink_ok(ok.t())                                     # column-major


def test_hq_form_for_tp_shards():
    """The 128x128 k-substep tile (15) for the few-tile TP-shard GEMMs, 2 K-slices where its tiles
    fill at most half a round at K >= 4096; not for the TP = 1 shapes or the shards that already tile."""
    assert K.hq_form([(T, 3 * H // 8, H)]) == 1                  # q|k|v forward: 192 tiles of 128x128
    assert K.hq_form([(T, H // 8, H)]) == 1                      # o_proj dX: 64 tiles
    assert K.hq_form([(3 * H // 8, H, T), (H, H // 8, T)]) == 2  # q|k|v + o_proj dW: 128 tiles x 2
    assert K.hq_form([(2 * I // 8, H, T)]) == 1                  # gate|up dW: 256 tiles
    assert K.hq_form([(T, H, H // 8)]) == 0                      # o_proj forward: 128 256x256 tiles
    assert K.hq_form([(T, 3 * H, H)]) == 0                       # TP = 1
    assert K.hq_form([(1024, 256, 1024)]) == 0                   # small shapes keep the old forms
    assert K.hq_form([(T, 192, H)]) == 0                         # not on 128-column tiles
    with switches.override(ksplit=0):
        assert K.hq_form([(T, 3 * H // 8, H)]) == 0
