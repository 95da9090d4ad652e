"""Measurement switches of the HIP path, read ONCE from the environment when the package is imported.

Every switch selects between HIP kernels with the same results (fused vs separate epilogues,
split-K vs one pass, one launch vs two); the defaults are the production path, and nothing on the
hot path reads the environment again.  `PICOTRON_<NAME>` (upper case) sets a switch for a whole
process (an A/B run); tests and tools change one for a block with `override(name=value)`.
Every non-default form runs through the whole GPU path against the oracle in
tests/test_switch_forms_gpu.py (ring_zigzag / tp_sp_chunks in test_parallel_gpu.py, gemm_kh and
wgrad_pair in test_kernels_gpu.py);
tools/switch_kernels.py traces which launches each changes (profiles/r05/switch_kernels_r05k.txt).

The native switches (attention causal pairing, dK/dV kernel form, few-head split chunk; GEMM
tile-row grouping, mixed-tile q|k|v launch, K-halves tile) live in the library; `apply_native`
pushes them through `pt_set_variant` when the library is loaded, and `override` pushes a changed one at once.
"""
import contextlib
import os
import sys

DEFAULTS = {
    # functional.py: the fused epilogues (RoPE in the q|k|v GEMM and attention backward, SwiGLU in the
    # gate|up / down GEMMs), deferred norm-weight column sums, lm_head CE statistics, the q|k|v and
    # gate|up dX + dW dual launches (the latter's dX as split-K halves or unsplit)
    "fuse": 1, "norm_defer": 1, "ce_stats": 1, "dual_qkv": 1, "dual_gu": 1, "gu_splitk": 1,
    # kernels.py: weight-gradient / few-tile forward and dX K-slices (the SwiGLU-backward dX's too), split-K dgrad halves (and their minimum K), dX + dW dual
    # launches and their XCD order, the norm backward fed by split-K halves, the attention
    # backward's fused delta, and the tile-count thresholds below which the RoPE / SwiGLU epilogues
    # run as separate kernels (TP shard widths)
    "ksplit": 1, "swiglu_splitk": 1, "splitk2": 1, "splitk2_min": 8192, "dual": 1, "norm_splitk": 1,
    "fuse_delta": 1, "rope_fuse_min_tiles": 96, "swiglu_fuse_min_tiles": 192, "swiglu_bwd_min_tiles": 0,
    # context_parallel.py: the zig-zag (load-balanced) ring where it tiles, the residual stream kept
    # in that layout across the decoder stack, the full-mesh K|V / dK|dV exchange instead of the ring
    "ring_zigzag": 1, "zigzag_residual": 1, "ring_mesh": 1,
    # tensor_parallel/sequence_parallel.py: the residual stream sharded by token rows over the tp group,
    # in a layout of (up to) this many chunks, whose collectives overlap the other chunks' GEMMs
    # (0 = auto: chunks of >= 8192 token rows, at most 8)
    "tp_sp": 1, "tp_sp_chunks": 0,
    # functional.py: the TP lm_head's F.cross_entropy on the vocab shards (no logits all-gather)
    "vp_ce": 1,
    # functional.py / train.py: the weight gradients of micro-batch pairs as one K = 2 T launch each
    # (train_step at tp = pp = 1; 0 = one launch per micro-batch, the reference's order)
    "wgrad_pair": 1,
    # native (libpicotron_hip.so, pt_set_variant)
    "attn_pair": 1, "attn_split": 2, "gemm_mix": 1, "gemm_kh": 2, "attn_kv_chunk": 4,
}
NATIVE = ("attn_pair", "attn_split", "gemm_mix", "gemm_kh", "attn_kv_chunk")


class _Switches:
    def __init__(self):
        for k, d in DEFAULTS.items():
            v = os.environ.get("PICOTRON_" + k.upper())
            setattr(self, k, int(v) if v not in (None, "") else d)

    def __repr__(self):
        return "Switches(" + ", ".join(f"{k}={getattr(self, k)}" for k in DEFAULTS) + ")"


S = _Switches()


def apply_native(lib):
    """Push the native switches into a freshly loaded library (called by _C.load_library)."""
    for k in NATIVE:
        rc = lib.pt_set_variant(k.encode(), int(getattr(S, k)))
        if rc != 0:
            # an older build (whole-step A/B of library builds) without this variant runs the form
            # its default names; any other value is an error
            if lib.pt_get_variant(k.encode()) < 0 and getattr(S, k) == DEFAULTS[k]:
                print(f"[picotron_amd] library has no variant {k!r}; its default ({DEFAULTS[k]}) form assumed",
                      file=sys.stderr)
                continue
            raise RuntimeError(f"pt_set_variant({k!r}, {getattr(S, k)}) failed: {rc}")


@contextlib.contextmanager
def override(**kw):
    """Set switches for the duration of a block (tests / A/B tools), native ones included."""
    unknown = set(kw) - set(DEFAULTS)
    if unknown:
        raise KeyError(f"unknown switches {sorted(unknown)}")
    old = {k: getattr(S, k) for k in kw}
    try:
        for k, v in kw.items():
            setattr(S, k, int(v))
        _push([k for k in kw if k in NATIVE])
        yield S
    finally:
        for k, v in old.items():
            setattr(S, k, v)
        _push([k for k in kw if k in NATIVE])


def _push(names):
    if not names:
        return
    from . import _C
    lib = _C.load_library()
    for k in names:
        lib.pt_set_variant(k.encode(), int(getattr(S, k)))
