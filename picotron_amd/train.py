"""The training-step caller of the hot path: train.py:29-55 of the reference, plus offline stand-ins
for the pieces of train.py that need the network (SURVEY.md §7 hard part (e)).

* `train_step(model, data_loader, device)` -- train.py:29-55: grad-accumulation loop, DP sync only
  on the last micro-batch (:39-41), F.cross_entropy(...) / grad_acc (:46-49) -> the fused HIP
  cross-entropy, loss.backward().  One difference: the reference calls loss.item() after every
  micro-batch (:53), a host<->device synchronisation per micro-batch; here the loss is summed on the
  device and read once per step (same printed value).
* `SyntheticMicroBatchDataLoader` -- the MicroBatchDataLoader interface (data.py:12-136:
  grad_acc_steps, micro_batch_size, seq_length_per_gpu, global_batch_size, __next__ returning
  input_ids / target_ids / position_ids / hidden_states, CP chunking of data.py:102-116) over seeded
  random tokens already resident on the device.
* `SMOLLM_1_7B`, `LLAMA2_7B` -- the public HF configs, which are not on disk here.
* `flops_per_token` / `get_mfu` -- utils.py:42-48 with N counted once (the reference
  multiplies the replicated lm_head by tp).
"""
import types

import torch

from . import functional as FN
from . import kernels as K
from . import process_group_manager as pgm

SMOLLM_1_7B = dict(hidden_size=2048, intermediate_size=8192, num_attention_heads=32, num_key_value_heads=32,
                   vocab_size=49152, rms_norm_eps=1e-5, rope_theta=10000.0, num_hidden_layers=24)
LLAMA2_7B = dict(hidden_size=4096, intermediate_size=11008, num_attention_heads=32, num_key_value_heads=32,
                 vocab_size=32000, rms_norm_eps=1e-5, rope_theta=10000.0, num_hidden_layers=32)

MI355X_BF16_DENSE_PEAK = 2.5e15


def make_config(base, seq_length, **overrides):
    d = dict(base)
    d.update(overrides)
    d["max_position_embeddings"] = seq_length   # train.py:159
    return types.SimpleNamespace(**d)


class SyntheticMicroBatchDataLoader:
    """Seeded random tokens shaped like MicroBatchDataLoader's batches (data.py:102-136).
    fresh=False replays the same grad_acc micro-batches every step (a memorisation curve, what the
    loss-curve tests want); fresh=True draws a new step's worth of tokens after each pass, on the
    device (one launch per step), as the reference's loader streams new data (data.py:123-136) --
    the first pass is the same either way.  Every rank of one dp replica (tp / cp / pp) draws the
    same tokens: the generator is seeded by (seed, dp rank) only."""

    def __init__(self, micro_batch_size, seq_length, grad_acc_steps, vocab_size, device, seed=1234, fresh=False):
        m = pgm.current()
        self.micro_batch_size = micro_batch_size
        self.seq_length = seq_length
        self.grad_acc_steps = grad_acc_steps
        self.global_batch_size = micro_batch_size * grad_acc_steps * m.dp_world_size
        self.seq_length_per_gpu = seq_length // m.cp_world_size
        g = torch.Generator().manual_seed(seed)
        # [dp, ga, mbs, seq+1] for the whole job, sliced to this rank (DistributedSampler + CP chunk)
        tokens = torch.randint(0, vocab_size, (m.dp_world_size, grad_acc_steps, micro_batch_size, seq_length + 1),
                               generator=g)
        mine = tokens[m.dp_rank]
        lo = m.cp_rank * self.seq_length_per_gpu
        hi = lo + self.seq_length_per_gpu
        self._inputs = mine[:, :, :-1][:, :, lo:hi].contiguous().to(device)
        self._targets = mine[:, :, 1:][:, :, lo:hi].contiguous().to(device)
        self._pos = torch.arange(lo, hi, device=device).unsqueeze(0).expand(micro_batch_size, -1)
        self._i = 0
        self._fresh, self._vocab, self._span = fresh, vocab_size, (lo, hi)
        if fresh:
            self._gen = torch.Generator(device=device).manual_seed(seed * 1000003 + m.dp_rank)

    def __iter__(self):
        return self

    def __next__(self):
        i = self._i % self.grad_acc_steps
        if self._fresh and i == 0 and self._i > 0:   # a new step: new tokens
            lo, hi = self._span
            t = torch.randint(0, self._vocab, (self.grad_acc_steps, self.micro_batch_size, self.seq_length + 1),
                              generator=self._gen, device=self._inputs.device)
            self._inputs = t[:, :, :-1][:, :, lo:hi].contiguous()
            self._targets = t[:, :, 1:][:, :, lo:hi].contiguous()
        self._i += 1
        return {"input_ids": self._inputs[i], "target_ids": self._targets[i], "position_ids": self._pos,
                "hidden_states": None}


def train_step(model, data_loader, device, on_microbatch=None, read_loss=True):
    """train.py:29-55 with the fused HIP cross-entropy; returns the accumulated loss (float).
    on_microbatch(i): optional hook called before micro-batch i (bench.py samples its GEMM timing).
    read_loss=False: return the loss as a device scalar instead, so that the caller can enqueue the
    optimizer step before the host waits for the backward (`read_step_loss` reads it then): reading it
    here idles the GPU for the optimizer's host work (~1.5 ms at SmolLM-1.7B), and the AdamW launch that
    follows an idle gap runs at the idle clocks, 3.4 vs 2.8 ms (profiles/r05/notes_r05.md)."""
    acc_loss = torch.zeros((), dtype=torch.float32, device=device)
    # (bench.py --dp-bucket: a 1-rank DataParallelBucket syncs like N > 1 would)
    requires_grad_sync = pgm.current().cp_dp_world_size > 1 or getattr(model, "_force_grad_sync", False)
    for i in range(data_loader.grad_acc_steps):
        if on_microbatch is not None:
            on_microbatch(i)
        batch = next(data_loader)
        input_ids = batch["input_ids"].to(device)
        target_ids = batch["target_ids"].to(device)
        if requires_grad_sync:
            model.require_backward_grad_sync = (i == data_loader.grad_acc_steps - 1)
        outputs = model(input_ids=input_ids)
        batch_size, seq_len = input_ids.shape
        target_ids = target_ids.reshape(-1)
        outputs = outputs.view(seq_len * batch_size, -1)
        loss = FN.cross_entropy(outputs, target_ids, reduction="mean") / data_loader.grad_acc_steps
        loss.backward()
        acc_loss += loss.detach().float()
    return read_step_loss(acc_loss, device) if read_loss else acc_loss


def read_step_loss(acc_loss, device):
    """The step's loss as a float (one host <-> device synchronisation), then the device status check."""
    out = acc_loss.item()
    K.check_device_status(torch.device(device))   # the host has synchronised: surface device asserts
    return out


def count_params(model):
    """Parameters of the whole model, every tensor once: a tensor-parallel shard counts tp times
    (Column / VocabParallel weights and biases, RowParallel weights), a replicated tensor once.
    (utils.py:50-79 matches names instead, which counts the replicated dense lm_head of train.py tp
    times -- SURVEY.md §5; here the lm_head is whatever module holds it.)"""
    from .tensor_parallel.tensor_parallel import ColumnParallelLinear, RowParallelLinear, VocabParallelEmbedding
    tp = pgm.current().tp_world_size
    n = 0
    for mod in model.modules():
        for name, p in mod.named_parameters(recurse=False):
            sharded = isinstance(mod, (ColumnParallelLinear, VocabParallelEmbedding)) or (
                isinstance(mod, RowParallelLinear) and name == "weight")
            n += p.numel() * (tp if sharded else 1)
    return n


def flops_per_token(num_params, config):
    """utils.py:46: 6 N + 12 L H S."""
    return 6 * num_params + 12 * config.num_hidden_layers * config.hidden_size * config.max_position_embeddings


def get_mfu(tokens_per_second_per_gpu, num_params, config, peak=MI355X_BF16_DENSE_PEAK):
    return tokens_per_second_per_gpu * flops_per_token(num_params, config) / peak * 100
