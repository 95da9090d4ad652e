"""Pipeline-parallel engine over the HIP decoder layers (picotron/pipeline_parallel/pipeline_parallel.py
of the reference: PipelineParallel 8-75, train_step_pipeline_afab 77-122, train_step_pipeline_1f1b
124-214) -- BASELINE config 4 (Llama-2-7B dp2 tp2 pp2 1f1b) runnable where the reference checkout
is not (the GPU box), with the same class, attribute and function surface, so the reference's
train.py drives either.

The two schedules are written as an action list per stage (`pipeline_schedule`: which micro-batch
runs forward / backward in which order, and which p2p transfers pair up) executed by one loop
(`_run_schedule`), instead of two hand-unrolled loops; the list is a pure function of (schedule,
pp size, pp rank, micro-batches) and is checked against the reference's ordering on CPU.

Semantics kept from the reference (so losses, gradients and the DP synchronisation match):
  * stage s holds layers [sum(n_0 .. n_{s-1}), +n_s), n_i = L / P (+1 for the first L % P stages);
    the first stage the embedding, the last final_norm + final_proj (nn.Identity elsewhere);
  * the last stage's loss is F.cross_entropy(logits.transpose(1, 2), targets) -- reduction 'mean',
    NOT divided by grad_acc as train.py:49 divides (pipeline_parallel.py:103,153); with HipLogits
    both the lm_head and this cross-entropy run on the HIP kernels (functional.HipLogits);
  * under DataParallelBucket, `require_backward_grad_sync` is True only for the stage's last
    backward of the step (pipeline_parallel.py:113-115,184-186,203-205);
  * the returned logging loss is the mean over micro-batches of the per-micro-batch loss.
Differences: the logging loss is summed on the device and read once per step (the reference calls
.item() per micro-batch: a host sync each); p2p is the stream-ordered pp_communications of this
package.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import process_group_manager as pgm
from .pp_communications import bidirectional_pipeline_communicate, pipeline_communicate


def stage_layers(num_layers, pp_size, pp_rank):
    """Layer indices of stage `pp_rank`: contiguous, the first num_layers % pp_size stages one more."""
    base, extra = divmod(num_layers, pp_size)
    start = pp_rank * base + min(pp_rank, extra)
    return list(range(start, start + base + (1 if pp_rank < extra else 0)))


class PipelineParallel(nn.Module):
    """One pipeline stage of `model` (pipeline_parallel.py:8-75): its slice of decoder_layers (a
    ModuleDict keyed by the global layer index), the embedding on the first stage and
    final_norm / final_proj on the last."""

    def __init__(self, model, config):
        super().__init__()
        m = pgm.process_group_manager
        self.layer_distribution = self.distribute_layers(config.num_hidden_layers)
        self.embedding = model.embedding if m.pp_is_first_stage else nn.Identity()
        self.decoder_layers = nn.ModuleDict({str(i): model.decoder_layers[i] for i in self.layer_distribution})
        self.final_norm = model.final_norm if m.pp_is_last_stage else nn.Identity()
        self.final_proj = model.final_proj if m.pp_is_last_stage else nn.Identity()
        self.reset_parameters()

    def reset_parameters(self):
        """pipeline_parallel.py:26-39: re-draw this stage's parameters in the reference's order."""
        m = pgm.process_group_manager
        if m.pp_is_first_stage:
            self.embedding.reset_parameters()
        for layer in self.decoder_layers.values():
            for sub in (layer.input_layernorm, layer.attention, layer.post_attention_layernorm, layer.mlp):
                sub.reset_parameters()
        if m.pp_is_last_stage:
            self.final_norm.reset_parameters()
            self.final_proj.reset_parameters()

    def distribute_layers(self, num_layers):
        m = pgm.process_group_manager
        return stage_layers(num_layers, m.pp_world_size, m.pp_rank)

    def forward(self, input_ids, position_ids, hidden_states):
        x = self.embedding(input_ids if hidden_states is None else hidden_states)
        for layer in self.decoder_layers.values():
            x = layer(x, position_ids=position_ids)
        return self.final_proj(self.final_norm(x))

    def backward(self, input_tensor, output_tensor, output_tensor_grad):
        """Backpropagate this stage's graph of one micro-batch from `output_tensor_grad` (the next
        stage's input gradient; on the last stage None: the loss itself, seeded with ones) and
        return the gradient of its received input (None on the first stage)."""
        if input_tensor is not None:
            input_tensor.retain_grad()
        grad = torch.ones_like(output_tensor) if output_tensor_grad is None else output_tensor_grad
        torch.autograd.backward(output_tensor, grad_tensors=grad)
        return None if input_tensor is None else input_tensor.grad


def pipeline_schedule(kind, pp_size, pp_rank, n_micro):
    """The stage's actions for one step: a list of (op, micro-batch) with op "F" / "B", plus for
    each action the p2p that brackets it -- as tuples (op, i, recv, send):
      recv: "fwd" (activation from the previous stage before F), "bwd" (gradient from the next
            stage before B), or None when the preceding action's paired transfer delivered it;
      send: "fwd" / "bwd" alone, "fwd+bwd" (send the activation and receive the next gradient in
            one batched exchange with the next stage), "bwd+fwd" (send the gradient and receive
            the next activation from the previous stage), or None.
    kind "afab": all forwards then all backwards (pipeline_parallel.py:77-122);
    kind "1f1b": warmup of min(P - rank - 1, n) forwards, then forward / backward pairs, then the
    remaining backwards (pipeline_parallel.py:124-214) -- the pairing of the steady state's
    transfers is what keeps neighbouring stages from waiting on each other's sends."""
    acts = []
    if kind == "afab":
        acts += [("F", i, "fwd", "fwd") for i in range(n_micro)]
        acts += [("B", i, "bwd", "bwd") for i in range(n_micro)]
        return acts
    if kind != "1f1b":
        raise ValueError(f"pipeline_schedule: unknown schedule {kind!r}")
    warm = min(pp_size - pp_rank - 1, n_micro)
    steady = n_micro - warm
    acts += [("F", i, "fwd", "fwd") for i in range(warm)]
    for k in range(steady):
        # F of micro-batch warm + k: its input came with the previous pair's exchange (first: recv)
        acts.append(("F", warm + k, "fwd" if k == 0 else None, "fwd+bwd"))
        acts.append(("B", k, None, "bwd" if k == steady - 1 else "bwd+fwd"))
    acts += [("B", steady + j, "bwd", "bwd") for j in range(warm)]
    return acts


def _run_schedule(kind, model, data_loader, tensor_shapes, device, dtype):
    m = pgm.process_group_manager
    n = data_loader.grad_acc_steps
    sync = m.cp_dp_world_size > 1
    acts = pipeline_schedule(kind, m.pp_world_size, m.pp_rank, n)
    last_b = max(k for k, a in enumerate(acts) if a[0] == "B")
    loss_sum = torch.zeros((), dtype=torch.float64, device=device)
    saved = {}             # micro-batch -> (input tensor, output tensor)
    carry = None           # what the previous action's paired exchange received
    for k, (op, i, recv, send) in enumerate(acts):
        if op == "F":
            x = pipeline_communicate("recv_forward", device, dtype, shapes=tensor_shapes) if recv else carry
            batch = next(data_loader)
            out = model.forward(input_ids=batch["input_ids"].to(device), position_ids=batch["position_ids"].to(device),
                                hidden_states=None if x is None else x.to(device))
            if m.pp_is_last_stage:
                out = F.cross_entropy(out.transpose(1, 2), batch["target_ids"].to(device), reduction="mean")
                loss_sum += out.detach().double()
            saved[i] = (x, out)
            if send == "fwd":
                pipeline_communicate("send_forward", device, dtype, tensor=out)
                carry = None
            else:   # "fwd+bwd": the gradient for the next action's backward comes back here
                carry = bidirectional_pipeline_communicate("send_fwd_recv_bwd", out, tensor_shapes, device, dtype)
        else:
            g = pipeline_communicate("recv_backward", device, dtype, shapes=tensor_shapes) if recv else carry
            if sync:
                model.require_backward_grad_sync = k == last_b
            x, out = saved.pop(i)
            dx = model.backward(x, out, g)
            if send == "bwd":
                pipeline_communicate("send_backward", device, dtype, tensor=dx)
                carry = None
            else:   # "bwd+fwd": the next forward's activation comes back here
                carry = bidirectional_pipeline_communicate("send_bwd_recv_fwd", dx, tensor_shapes, device, dtype)
    return (loss_sum / n).item() if m.pp_is_last_stage else 0.0


def train_step_pipeline_afab(model, data_loader, tensor_shapes, device, dtype):
    """All forwards, then all backwards (pipeline_parallel.py:77-122).  Returns the step's logging
    loss on the last stage (0.0 elsewhere, as the reference)."""
    return _run_schedule("afab", model, data_loader, tensor_shapes, device, dtype)


def train_step_pipeline_1f1b(model, data_loader, tensor_shapes, device, dtype):
    """One-forward-one-backward (pipeline_parallel.py:124-214)."""
    return _run_schedule("1f1b", model, data_loader, tensor_shapes, device, dtype)
