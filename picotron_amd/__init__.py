"""picotron_amd -- picotron's Llama decoder-layer hot path, native to MI355X (gfx950 / CDNA4).

The package keeps the module interfaces of the reference (okoge-kaz/picotron): model.py,
tensor_parallel/, context_parallel/, data_parallel/ and process_group_manager.py, so a picotron
training loop can import them in place of the reference's.  Underneath, every dense contraction,
norm, rotary, activation, attention and loss op is a hand-written HIP kernel for gfx950
(csrc/*.hip, built into lib/libpicotron_hip.so and bound by ctypes through the C ABI declared in
include/picotron_hip.h), and the collectives are torch.distributed's "nccl" backend, i.e. RCCL.

Nothing here falls back to eager/CPU compute: without the HIP library or a visible device, the ops
raise.
"""
__all__ = ["model", "functional", "kernels", "tensor_parallel", "context_parallel", "data_parallel",
           "process_group_manager", "train"]
