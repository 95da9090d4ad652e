"""Host logic of the TP lm_head's vocab-parallel stand-in (functional.vp_logits): the [.., V] object
ColumnParallelLinear(gather_output=True) returns instead of gathered logits.  Metadata reads and the
reference's view forms keep it a stand-in without touching data; anything else gathers the logits
once (the materialize callback: GatherFromModelParallelRegion on the product path) and replays the
views on them.  The HIP cross-entropy on it is covered by tests/test_parallel_gpu.py."""
import torch

from picotron_amd import functional as FN


def _standin(calls):
    y = torch.randn(2, 3, 8, requires_grad=True)

    def gather():
        calls.append(1)
        return torch.cat([y, 2 * y], dim=-1)
    return y, FN.vp_logits(y, None, 0, 16, gather)


def test_metadata_and_views_do_not_gather():
    calls = []
    y, st = _standin(calls)
    assert FN._is_vp(st) and st.shape == (2, 3, 16) and st.dtype == y.dtype and st.dim() == 3
    assert st.size(-1) == 16 and st.numel() == 96
    v = st.view(-1, 16)
    t = st.transpose(1, 2)
    assert FN._is_vp(v) and FN._is_vp(t) and v.shape == (6, 16) and t.shape == (2, 16, 3)
    assert FN.as_logits(st) is st          # Tensor.as_subclass would drop the stand-in
    assert not calls


def test_other_ops_gather_once_and_replay_views():
    calls = []
    y, st = _standin(calls)
    full = torch.cat([y, 2 * y], dim=-1).detach()
    v = st.view(-1, 16)
    assert torch.equal(v[4].detach(), full.view(-1, 16)[4])
    assert torch.equal(st.transpose(1, 2).float().detach(), full.transpose(1, 2))
    p = FN._plain(v)
    assert type(p) is torch.Tensor and p.stride() == (16, 1) and torch.equal(p.detach(), full.view(-1, 16))
    assert len(calls) == 1                 # gathered once, cached on the stand-in
    st.float().sum().backward()            # the gathered logits keep the shard's autograd graph
    assert torch.allclose(y.grad, torch.full_like(y, 3.0))


def test_unsupported_cross_entropy_form_falls_back():
    calls = []
    y, st = _standin(calls)
    # [B, S, V] with class dim S is not one of the reference's two call forms: no vocab-parallel path
    assert FN._vp_cross_entropy(st, torch.zeros(2, 16, dtype=torch.long), "mean", -100) is None
    assert not calls


def test_reordering_views_are_not_served_by_the_shard_rows():
    """the shard path is taken only when the view path keeps the shard rows in order
    (view / reshape / flatten, or one transpose(1, 2) / permute(0, 2, 1) of [B, S, V]); a path that
    reorders rows -- e.g. sequence-major rows with matching targets -- falls back to the gathered
    logits (None here: the caller gathers)."""
    calls = []
    y, st = _standin(calls)
    tgt2 = torch.zeros(6, dtype=torch.long)
    assert FN._vp_path_form(st.view(-1, 16)._pt_vp_path, 3) == "rows"
    assert FN._vp_path_form(st.reshape(6, 16).contiguous()._pt_vp_path, 3) == "rows"
    assert FN._vp_path_form(st.transpose(1, 2)._pt_vp_path, 3) == "bvs"
    assert FN._vp_path_form(st.transpose(-1, -2)._pt_vp_path, 3) == "bvs"
    assert FN._vp_path_form(st.permute(0, 2, 1)._pt_vp_path, 3) == "bvs"
    assert FN._vp_path_form(st.permute((0, 2, 1))._pt_vp_path, 3) == "bvs"
    seq_major = st.transpose(0, 1).reshape(-1, 16)
    assert FN._is_vp(seq_major) and FN._vp_path_form(seq_major._pt_vp_path, 3) is None
    assert FN._vp_cross_entropy(seq_major, tgt2, "mean", -100) is None
    assert FN._vp_path_form(st.permute(1, 0, 2)._pt_vp_path, 3) is None
    assert FN._vp_path_form(st.transpose(1, 2).reshape(-1, 16)._pt_vp_path, 3) is None
    assert not calls


def test_contiguous_keeps_the_stand_in_without_storage():
    """contiguous() on the stand-in is recorded, not run (a real one would write a
    [T, V] buffer), and replayed if the logits are ever gathered; the stand-in requires grad as its
    shard does."""
    calls = []
    y, st = _standin(calls)
    c = st.contiguous()
    assert FN._is_vp(c) and c.shape == st.shape
    with torch._C.DisableTorchFunctionSubclass():   # (a storage read through the subclass would gather)
        assert c.untyped_storage().nbytes() <= 8
    assert c._pt_vp is st._pt_vp and c._pt_vp_path[-1][0] is torch.Tensor.contiguous
    assert st.requires_grad and c.requires_grad
    assert not calls
    full = torch.cat([y, 2 * y], dim=-1).detach()
    assert torch.equal(c.transpose(1, 2).contiguous().float().detach(), full.transpose(1, 2))
    assert len(calls) == 1
