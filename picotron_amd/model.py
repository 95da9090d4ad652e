"""Llama modules with the reference's model.py API, running on the gfx950 kernels.

Mirrors picotron/model.py of okoge-kaz/picotron @ 2025-03-02: the same class names, constructor
and forward signatures, attribute names (q_proj ... down_proj, input_layernorm,
post_attention_layernorm, attention, mlp, decoder_layers, embedding, final_norm, final_proj, cos,
sin), parameter registration order, state_dict keys, initialisation (model.py:110-120,173-182,
221-222) and env switches (FLASH_ATTEN picks the RMSNorm flavour, model.py:192,248;
CONTEXT_PARALLEL picks ring attention, model.py:148).  So apply_tensor_parallel,
apply_context_parallel, DataParallelBucket and the checkpoint name maps operate on it unchanged.

The compute is different: DecoderLayer.forward is ONE autograd node (functional.DecoderLayerFunction)
built from hand-written HIP kernels -- fused q|k|v and gate|up GEMMs, in-place RoPE on the
projection output, flash attention on strided views (no repeat_interleave, no transposes), the
residual adds fused into the RMSNorm and down_proj kernels.  Attention / MLP / the norms can still
be called on their own (each is its own Function).  The token embedding is csrc/embedding.hip
(masked lookup; sorted-segment backward).
"""
import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import functional as FN
from . import kernels as K
from . import process_group_manager as pgm
from .context_parallel import context_parallel


def _flash():
    return os.getenv("FLASH_ATTEN", "1") == "1"


# ---------------------------------------------------------------------------- rotary
class _RotaryBHSD(torch.autograd.Function):
    """apply_rotary_pos_emb on a [B, H, S, D] tensor (model.py:12-19) through the rope kernel."""

    @staticmethod
    def forward(ctx, x, cos, sin):
        B, H, S, D = x.shape
        xt = x.transpose(1, 2).contiguous()          # token-major copy; the kernel rotates in place
        K.rope_(xt.view(B * S, H * D), H, D, cos, sin, S)
        ctx.save_for_backward(cos, sin)
        return xt.transpose(1, 2)

    @staticmethod
    def backward(ctx, g):
        cos, sin = ctx.saved_tensors
        B, H, S, D = g.shape
        gt = g.transpose(1, 2).contiguous()
        K.rope_(gt.view(B * S, H * D), H, D, cos, sin, S, inverse=True)
        return gt.transpose(1, 2), None, None


def apply_rotary_pos_emb(x, cos, sin):
    """model.py:12-19: x [B, H, S, D]; cos/sin [S, D] bf16 tables from get_cos_sin."""
    return _RotaryBHSD.apply(x, cos.to(torch.bfloat16).contiguous(), sin.to(torch.bfloat16).contiguous())


def get_cos_sin(seq_length, head_dim, base=500000.0):
    """model.py:21-31: inverse frequencies on the CPU in fp32, pos*theta on the device, tables in
    DTYPE (bf16 unless DTYPE says otherwise), each half repeated -> [seq_length, head_dim]."""
    assert head_dim % 2 == 0
    theta = 1.0 / (base ** (torch.arange(0, head_dim, 2, dtype=torch.int64).float().to("cpu") / head_dim))
    dtype = torch.bfloat16 if os.getenv("DTYPE", "bfloat16") == "bfloat16" else torch.float32
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    device = torch.device("cuda", local_rank) if os.getenv("DEVICE", "cuda") == "cuda" else torch.device("cpu")
    position = torch.arange(seq_length).to(device).unsqueeze(1).float()
    theta = theta.to(device)
    ang = position.float() * theta.float()
    return torch.cos(ang).to(dtype).repeat(1, 2), torch.sin(ang).to(dtype).repeat(1, 2)


def _pad_d(t, dp):
    """[..., D] -> [..., dp] zero-padded (a head dim the kernels do not take: no RoPE pairing here)."""
    return t if t.shape[-1] == dp else torch.nn.functional.pad(t, (0, dp - t.shape[-1]))


class _FlashAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal):
        # q/k/v: [B, S, H, D] views (d contiguous); a D other than 64 / 128 runs zero-padded (the
        # padded columns add nothing to q . k and are sliced off o; the scale is the real D's)
        D = q.shape[-1]
        scale = 1.0 / math.sqrt(D)
        dp = FN._head_pad_dim(D) if D not in FN.ATTN_HEAD_DIMS else D
        if dp is None:
            raise RuntimeError(f"flash_attention: head_dim {D} -- the kernels take 64 / 128 and pad dims below 128")
        qp, kp, vp = (_pad_d(t, dp) for t in (q, k, v))
        o, lse = K.attn_fwd(qp, kp, vp, scale, causal)
        ctx.save_for_backward(qp, kp, vp, o, lse)
        ctx.scale, ctx.causal, ctx.D = scale, causal, D
        return o[..., :D] if dp != D else o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        D = ctx.D
        do = _pad_d(do, o.shape[-1])
        if do.stride(-1) != 1:
            do = do.contiguous()
        dq, dk, dv, _ = K.attn_bwd(do, q, k, v, o, lse, ctx.scale, ctx.causal)
        if o.shape[-1] != D:
            dq, dk, dv = dq[..., :D], dk[..., :D], dv[..., :D]
        return dq, dk, dv, None


def flash_attention(q, k, v, causal=True):
    """model.py:33-37: q/k/v [B, H, S, D] -> out [B, S, H, D] (flash_attn_func semantics)."""
    return _FlashAttention.apply(q.permute(0, 2, 1, 3), k.permute(0, 2, 1, 3), v.permute(0, 2, 1, 3), causal)


# ---------------------------------------------------------------------------- norms / linear
class TritonRMSNorm(nn.Module):
    """model.py:39-65 (flash-attn layer_norm_fn, is_rms_norm=True): y = bf16(x * rstd * w)."""

    def __init__(self, hidden_size, eps=1e-5, device=None, dtype=None):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.empty(hidden_size, device=device, dtype=dtype))
        self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        nn.init.ones_(self.weight)

    def forward(self, hidden_states, residual=None, dropout_p=0.0, prenorm=False, residual_in_fp32=False,
                return_dropout_mask=False):
        if dropout_p != 0.0 or residual_in_fp32 or return_dropout_mask:
            raise NotImplementedError("TritonRMSNorm: dropout / fp32 residual are not on the picotron path")
        if residual is None:
            y = _tag_final(self, FN.RMSNormFunction.apply(FN._plain(hidden_states), self.weight, self.eps, 0))
            return (y, hidden_states) if prenorm else y
        y, z = FN.AddRMSNormFunction.apply(hidden_states, residual, self.weight, self.eps, 0)
        return (y, z) if prenorm else y


class LlamaRMSNorm(nn.Module):
    """model.py:67-86: w * bf16(x_fp32 * rsqrt(mean(x^2) + eps))."""

    def __init__(self, hidden_size, eps=1e-5):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(hidden_size))
        self.variance_epsilon = eps
        self.reset_parameters()

    def reset_parameters(self):
        nn.init.ones_(self.weight)

    def forward(self, hidden_states):
        return _tag_final(self, FN.RMSNormFunction.apply(FN._plain(hidden_states), self.weight,
                                                         self.variance_epsilon, 1))


def _tag_final(norm, y):
    """Llama's final_norm hands its output on as functional.HipHidden, so whatever module holds the
    lm_head -- also a torch nn.Linear called directly (PipelineParallel.forward,
    pipeline_parallel.py:62-63, after checkpoint.py:89-90) -- runs the HIP lm_head GEMM."""
    return FN.as_hidden(y) if getattr(norm, "_pt_final_norm", False) else y


def _norm_mode(norm):
    return 0 if isinstance(norm, TritonRMSNorm) else 1


def _norm_eps(norm):
    return norm.eps if isinstance(norm, TritonRMSNorm) else norm.variance_epsilon


class Linear(nn.Module):
    """nn.Linear(in, out, bias) as used by model.py:100-103,167-169,247; forward on the MFMA GEMM.
    Same attributes (in_features, out_features, weight, bias) so apply_tensor_parallel
    (tensor_parallel.py:11-33) can read and replace it."""

    def __init__(self, in_features, out_features, bias=False, device=None, dtype=None):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = nn.Parameter(torch.empty(out_features, in_features, device=device, dtype=dtype))
        if bias:
            self.bias = nn.Parameter(torch.empty(out_features, device=device, dtype=dtype))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        # nn.Linear's default: kaiming_uniform(a=sqrt(5)) == U(-1/sqrt(in), 1/sqrt(in))
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            bound = 1 / math.sqrt(self.in_features) if self.in_features > 0 else 0
            nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, x):
        x = FN._plain(x)
        if getattr(self, "_pt_lm_head", False) and self.bias is None:
            return FN.as_logits(FN.lm_head_linear(x, self.weight))
        y = FN.linear(x, self.weight)
        y = y if self.bias is None else y + self.bias
        # the lm_head (Llama tags its final_proj): keep F.cross_entropy on the HIP kernel also when
        # a caller other than Llama.forward runs it (PipelineParallel.forward, model.py:63)
        return FN.as_logits(y) if getattr(self, "_pt_lm_head", False) else y


def _init_uniform_fan_in(tensor):
    """model.py:112-115 / 175-178: U(-sqrt(1/size(1)), sqrt(1/size(1)))."""
    bound = math.sqrt(1 / tensor.size(1))
    torch.nn.init.uniform_(tensor, -bound, bound)


# ---------------------------------------------------------------------------- blocks
class Attention(nn.Module):
    """model.py:88-162."""

    def __init__(self, config, layer_idx):
        super().__init__()
        m = pgm.current()
        self.hidden_size = config.hidden_size
        self.num_heads = config.num_attention_heads
        self.num_key_values = config.num_key_value_heads
        self.head_dim = self.hidden_size // self.num_heads
        assert config.num_attention_heads % m.tp_world_size == 0, "num_attention_heads should be divisible by tp world size"
        assert config.num_key_value_heads % m.tp_world_size == 0, "num_key_value_heads should be divisible by  tp world size"
        self.num_local_heads = config.num_attention_heads // m.tp_world_size
        self.num_local_kv_heads = config.num_key_value_heads // m.tp_world_size
        self.q_proj = Linear(config.hidden_size, self.num_heads * self.head_dim, bias=False)
        self.k_proj = Linear(config.hidden_size, self.num_key_values * self.head_dim, bias=False)
        self.v_proj = Linear(config.hidden_size, self.num_key_values * self.head_dim, bias=False)
        self.out_proj = Linear(config.hidden_size, config.hidden_size, bias=False)
        self.layer_idx = layer_idx
        self.reset_parameters()

    def reset_parameters(self):
        for t in (self.q_proj.weight, self.k_proj.weight, self.v_proj.weight, self.out_proj.weight):
            _init_uniform_fan_in(t)

    def weights(self):
        return self.q_proj.weight, self.k_proj.weight, self.v_proj.weight, self.out_proj.weight

    def forward(self, x, cos, sin, attention_mask=None, position_ids=None):
        return FN.AttentionFunction.apply(x, *self.weights(), cos, sin, self.num_local_heads,
                                          self.num_local_kv_heads, self.head_dim)


class MLP(nn.Module):
    """model.py:164-186 (parameter order up, gate, down as in the reference)."""

    def __init__(self, config) -> None:
        super().__init__()
        self.up_proj = Linear(config.hidden_size, config.intermediate_size, bias=False)
        self.gate_proj = Linear(config.hidden_size, config.intermediate_size, bias=False)
        self.down_proj = Linear(config.intermediate_size, config.hidden_size, bias=False)
        self.reset_parameters()

    def reset_parameters(self):
        for t in (self.up_proj.weight, self.gate_proj.weight, self.down_proj.weight):
            _init_uniform_fan_in(t)

    def forward(self, x):
        return FN.MLPFunction.apply(x, self.gate_proj.weight, self.up_proj.weight, self.down_proj.weight)


class DecoderLayer(nn.Module):
    """model.py:188-209: RMSNorm -> Attention -> residual -> RMSNorm -> MLP -> residual."""

    def __init__(self, config, layer_idx):
        super().__init__()
        RMSNorm = TritonRMSNorm if _flash() else LlamaRMSNorm
        self.input_layernorm = RMSNorm(config.hidden_size, eps=config.rms_norm_eps)
        self.post_attention_layernorm = RMSNorm(config.hidden_size, eps=config.rms_norm_eps)
        self.attention = Attention(config, layer_idx=layer_idx)
        self.mlp = MLP(config)
        self.layer_idx = layer_idx
        head_dim = config.hidden_size // config.num_attention_heads
        self._rope_args = (config.max_position_embeddings, head_dim, config.rope_theta)
        self.cos, self.sin = get_cos_sin(config.max_position_embeddings, head_dim=head_dim, base=config.rope_theta)
        self.cos, self.sin = context_parallel.update_rope_for_context_parallel(self.cos, self.sin)
        # set by context_parallel.apply_context_parallel at cp > 1: the input is the zig-zag shard of
        # the residual stream (RoPE rows: that shard's positions, _tables) whenever its length tiles
        self.cp_zigzag_residual = False
        # set by tensor_parallel.apply_tensor_parallel at tp > 1: the input is this rank's token-row
        # shard of the residual stream whenever the batch was sharded (the model's SPState)
        self.tp_sequence_parallel = False

    def _tables(self, device, zz_len=0):
        # tables follow the activations' device (the module may have been moved after init); the
        # zig-zag shard's rows depend on its local length zz_len (context_parallel.zigzag_rope_tables)
        if zz_len:
            cache = self.__dict__.setdefault("_zz_tables", {})
            key = (zz_len, device)
            if key not in cache:
                cos, sin = context_parallel.zigzag_rope_tables(*self._rope_args, S=zz_len)
                cache[key] = (cos.to(device=device, dtype=torch.bfloat16), sin.to(device=device, dtype=torch.bfloat16))
            return cache[key]
        cos, sin = self.cos, self.sin
        if cos.device != device or cos.dtype != torch.bfloat16:
            cos, sin = cos.to(device=device, dtype=torch.bfloat16), sin.to(device=device, dtype=torch.bfloat16)
            self.cos, self.sin = cos, sin
        return cos, sin

    def forward(self, x, attention_mask=None, position_ids=None):
        zz = self.cp_zigzag_residual and context_parallel.zigzag_enabled(x.shape[1], True)
        cos, sin = self._tables(x.device, x.shape[1] if zz else 0)
        n1, n2, at, mlp = self.input_layernorm, self.post_attention_layernorm, self.attention, self.mlp
        if _norm_mode(n1) != _norm_mode(n2) or _norm_eps(n1) != _norm_eps(n2):
            raise ValueError("DecoderLayer: both norms must be the same flavour")
        # a token-row shard of the residual stream (tensor_parallel/sequence_parallel.py)?  Then
        # sp = its layout's chunk count (the model's SPState, set by this forward's entry)
        st = getattr(self, "_pt_sp_state", None)
        sp = st.chunks if (self.tp_sequence_parallel and st is not None and st.local_len and
                           st.local_len == x.shape[1]) else 0
        return FN.DecoderLayerFunction.apply(
            x, n1.weight, n2.weight, *at.weights(), mlp.gate_proj.weight, mlp.up_proj.weight, mlp.down_proj.weight,
            cos, sin, _norm_eps(n1), _norm_mode(n1), at.num_local_heads, at.num_local_kv_heads, at.head_dim, zz, sp)


class Embedding(nn.Module):
    """model.py:211-225 on csrc/embedding.hip (lookup, and a backward that touches only the rows
    the micro-batch uses)."""

    def __init__(self, num_embeddings, embedding_dim, padding_idx=None):
        super().__init__()
        self.num_embeddings = num_embeddings
        self.embedding_dim = embedding_dim
        self.padding_idx = padding_idx
        self.weight = nn.Parameter(torch.empty(num_embeddings, embedding_dim))
        self.reset_parameters()

    def reset_parameters(self):
        torch.nn.init.normal_(self.weight, mean=0.0, std=1.0)

    def forward(self, x):
        return FN.embedding(x, self.weight, padding_idx=self.padding_idx)


class Llama(nn.Module):
    """model.py:227-272."""

    def __init__(self, config) -> None:
        super().__init__()
        assert config.hidden_size % config.num_attention_heads == 0
        assert config.num_attention_heads % config.num_key_value_heads == 0
        self.vocab_size = config.vocab_size
        self.hidden_size = config.hidden_size
        self.num_heads = config.num_attention_heads
        self.num_key_values = config.num_key_value_heads
        self.head_dim = self.hidden_size // self.num_heads
        self.max_position_embeddings = config.max_position_embeddings
        self.num_layers = config.num_hidden_layers
        self.model_config = config
        self.embedding = Embedding(self.vocab_size, self.hidden_size)
        self.decoder_layers = nn.ModuleList([DecoderLayer(config, layer_idx=i) for i in range(self.num_layers)])
        self.final_proj = Linear(self.hidden_size, self.vocab_size, bias=False)
        self.final_proj._pt_lm_head = True
        RMSNorm = TritonRMSNorm if _flash() else LlamaRMSNorm
        self.final_norm = RMSNorm(self.hidden_size, eps=config.rms_norm_eps)
        self.final_norm._pt_final_norm = True
        self.reset_parameters()

    def reset_parameters(self):
        self.embedding.reset_parameters()
        for layer in self.decoder_layers:
            layer.input_layernorm.reset_parameters()
            layer.attention.reset_parameters()
            layer.post_attention_layernorm.reset_parameters()
            layer.mlp.reset_parameters()
        self.final_norm.reset_parameters()
        self.final_proj.reset_parameters()

    def forward(self, input_ids, attention_mask=None, position_ids: torch.Tensor = None):
        x = self.embedding(input_ids)
        for layer in self.decoder_layers:
            x = layer(x)
        x = self.final_norm(x)
        return lm_head(self.final_proj, x)


def lm_head(final_proj, x):
    """model.py:270 `self.final_proj(x)` on the MFMA GEMM whatever module holds the weight: the
    build's Linear / ColumnParallelLinear call it themselves; a plain torch nn.Linear -- what
    init_model_with_materialized_weights swaps in (checkpoint.py:89-91) -- is run through
    functional.linear on its weight (+ bias) instead of torch's GEMM."""
    x = FN._plain(x)
    if type(final_proj) is nn.Linear:
        if final_proj.bias is None:
            y = FN.lm_head_linear(x, final_proj.weight)
        else:
            y = FN.linear(x, final_proj.weight) + final_proj.bias
    else:
        y = final_proj(x)
    return FN.as_logits(y)
