"""Host logic of weight-gradient pairing (functional.WgradPairing / pair_jobs, train.train_step's
phases): which micro-batch defers its weight-gradient jobs, how the next one pairs them (kernels.KPair:
the two micro-batches' row blocks of one layout), and the phase sequence train_step drives.  The
K-segmented GEMM itself and the training numerics are GPU tests (test_kernels_gpu.py)."""
import torch

from picotron_amd import functional as FN
from picotron_amd import kernels as K


def _job(T, n, k, params):
    return (torch.randn(T, n), torch.randn(T, k), params)


def test_defer_then_pair():
    w1, w2 = torch.nn.Parameter(torch.zeros(4, 3)), torch.nn.Parameter(torch.zeros(6, 3))
    a, b = _job(8, 4, 3, [w1]), _job(8, 6, 3, [w2])
    old = FN.wgrad_pairing(0)
    try:
        assert FN.pair_jobs([a, b]) == [] and len(FN.WgradPairing.pending) == 2
        FN.wgrad_pairing(1)
        c, d = _job(8, 4, 3, [w1]), _job(8, 6, 3, [w2])
        out = FN.pair_jobs([c, d])
        assert not FN.WgradPairing.pending and len(out) == 2
        (dy, x, params), _ = out
        assert isinstance(dy, K.KPair) and dy.a is a[0] and dy.b is c[0] and x.a is a[1] and x.b is c[1]
        assert dy.shape == (16, 4) and params == [w1]
        sl = dy[:, 1:3]                                   # a column slice stays a pair
        assert isinstance(sl, K.KPair) and torch.equal(sl.a, a[0][:, 1:3]) and torch.equal(sl.b, c[0][:, 1:3])
        # a job of parameters nobody deferred passes through unpaired
        e = _job(8, 4, 3, [torch.nn.Parameter(torch.zeros(4, 3))])
        assert FN.pair_jobs([e]) == [e]
        FN.wgrad_pairing(None)
        assert FN.pair_jobs([e]) == [e]                   # phase None: as given
    finally:
        FN.wgrad_pairing(old)
        FN.WgradPairing.pending.clear()


def test_train_step_phase_sequence():
    """Micro-batches (0, 1), (2, 3), ... pair; an odd last micro-batch runs alone (phase None)."""
    from picotron_amd.train import pairing_phase

    def phases(ga):
        return [pairing_phase(i, ga) for i in range(ga)]
    assert phases(4) == [0, 1, 0, 1]
    assert phases(5) == [0, 1, 0, 1, None]
    assert phases(1) == [None]
    assert phases(32).count(1) == 16
