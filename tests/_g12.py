"""G12 helpers shared by the CPU oracle test and the GPU grid test: the fixture generator's
deterministic full weights and token batch (tests/golden/make_golden.py, loaded by path -- it imports
nothing from the reference at module level)."""
import importlib.util
import os

_spec = importlib.util.spec_from_file_location(
    "_make_golden", os.path.join(os.path.dirname(__file__), "golden", "make_golden.py"))
MG = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(MG)

CFGS, RUN, GA, MBS = MG.G12_CFGS, MG.G12_RUN, MG.G12_GA, MG.G12_MBS
full_param, tokens, full_shape = MG.g12_full_param, MG.g12_tokens, MG._g12_full_shape


def full_params(size):
    """Every full (unsharded) parameter of G12's `size` model, in the reference's state_dict naming."""
    c = CFGS[size]
    names = ["embedding.weight", "final_norm.weight", "final_proj.weight"]
    for i in range(c["num_hidden_layers"]):
        names += [f"decoder_layers.{i}.{s}.weight" for s in (
            "input_layernorm", "post_attention_layernorm", "attention.q_proj", "attention.k_proj", "attention.v_proj",
            "attention.out_proj", "mlp.up_proj", "mlp.gate_proj", "mlp.down_proj")]
    return {n: full_param(n, full_shape(n, _Shape(c["hidden_size"]), c)) for n in names}


class _Shape:
    """Stands in for a parameter whose shape full_shape() needs only for the norms (H)."""
    def __init__(self, h):
        self.shape = (h,)
