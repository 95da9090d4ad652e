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
    follows an idle gap runs at the idle clocks, 3.4 vs 2.8 ms (profiles/r05/notes_r05.md).  Note that
    read_loss=False also postpones the device-status check (a bad cross-entropy target: NaN rows and
    gradients) to `read_step_loss`, i.e. after an optimizer step enqueued in between has already
    applied those gradients -- bench.py's ordering; a training loop that must not update weights
    from a flagged step reads the loss (read_loss=True) before its optimizer step."""
    acc_loss = torch.zeros((), dtype=torch.float32, device=device)
    # (bench.py --dp-bucket: a 1-rank DataParallelBucket syncs like N > 1 would)
    requires_grad_sync = pgm.current().cp_dp_world_size > 1 or getattr(model, "_force_grad_sync", False)
    ga = data_loader.grad_acc_steps
    pairing = wgrad_pairing_applies()
    try:
        for i in range(ga):
            if on_microbatch is not None:
                on_microbatch(i)
            batch = next(data_loader)
            input_ids = batch["input_ids"].to(device)
            target_ids = batch["target_ids"].to(device)
            if requires_grad_sync:
                model.require_backward_grad_sync = (i == ga - 1)
            outputs = model(input_ids=input_ids)
            batch_size, seq_len = input_ids.shape
            target_ids = target_ids.reshape(-1)
            outputs = outputs.view(seq_len * batch_size, -1)
            loss = FN.cross_entropy(outputs, target_ids, reduction="mean") / ga
            # micro-batches (2 j, 2 j + 1) share their weight-gradient launches (functional.WgradPairing):
            # the first defers, the second launches K = 2 T GEMMs; an odd last micro-batch on its own
            if pairing:
                FN.wgrad_pairing(pairing_phase(i, ga))
            loss.backward()
            acc_loss += loss.detach().float()
    finally:
        if pairing:
            FN.wgrad_pairing(None)
            FN.flush_wgrad_pairs()
    return read_step_loss(acc_loss, device) if read_loss else acc_loss


def pairing_phase(i, ga):
    """Micro-batch i of ga: 0 = defers its weight gradients, 1 = completes the pair (2 j, 2 j + 1),
    None = an odd last micro-batch on its own."""
    return 0 if i % 2 == 0 and i + 1 < ga else (1 if i % 2 == 1 else None)


def wgrad_pairing_applies():
    """Weight-gradient pairing (functional.WgradPairing) runs in train_step at tp = pp = 1 (the TP
    shards' split-K weight-gradient forms and the pipeline's interleaved micro-batches keep one
    launch per micro-batch); switch `wgrad_pair`."""
    from .switches import S as SW
    m = pgm.current()
    return SW.wgrad_pair != 0 and m.tp_world_size == 1 and m.pp_world_size == 1


def quiesce_collectives(device, poll_s=0.35):
    """Before a HIP-graph capture that contains RCCL collectives: wait for the device to drain, then
    for torch's NCCL watchdog thread (it polls its list of in-flight works about every 100 ms) to
    retire the works the eager collectives left in it, so that it queries no event of RCCL's stream
    while that stream is part of the capture (GraphedTrainStep's docstring).  One-time cost per
    capture."""
    import time
    torch.cuda.synchronize(device)
    if torch.distributed.is_initialized():
        time.sleep(poll_s)


class GraphedTrainStep:
    """train_step (train.py:29-55) with the micro-batch -- forward, F.cross_entropy / grad_acc on the
    fused HIP kernel, backward, the loss accumulation -- captured ONCE as a HIP graph and replayed for
    every later micro-batch.  For tensor parallelism: at the TP = 8 shard widths a micro-batch is
    ~425 short kernels plus its RCCL collectives, and launching them from Python + autograd + ctypes
    costs more host time than the GPU spends on them (bench.py --tp-proxy: 9.8 ms eager vs 6.5 ms
    replayed per SmolLM-1.7B micro-batch); a replay issues the same launches -- the collectives
    included, each on RCCL's stream with its fork / join edges as the eager layer issues them --
    from one call.

    Contract (what a replay can and cannot re-decide):
      * the micro-batch's input / target ids are copied into static device buffers before each
        replay; every micro-batch has the shape of the first;
      * the gradients are this object's: the captured weight-gradient epilogues accumulate into
        fixed .grad buffers, so each call re-attaches them to the parameters (an optimizer's
        zero_grad(set_to_none=True) in between is fine) and zeroes them in place before its first
        micro-batch (one multi-tensor launch);
      * one weight-gradient launch per micro-batch (train_step's pairing, a two-micro-batch pattern,
        is a tp = 1 optimisation and does not apply to a replayed micro-batch);
      * no data-parallel wrapper, no CP / PP (their per-micro-batch host decisions -- the bucket
        all-reduce on the last micro-batch, the ring's host-side schedule, the pipeline's p2p
        order -- would be frozen into the graph): `supported(model)` says whether it applies;
      * on RCCL, the capture starts only after torch's NCCL watchdog has retired every eager
        collective (`quiesce_collectives`): once the first captured collective joins RCCL's stream
        to the capture, HIP refuses a query of any event recorded on that stream ("operation not
        permitted on an event last recorded in a capturing stream") -- and the watchdog thread polls
        the end events of the works still in its list (seen intermittently on the one-rank tests
        before this wait).
    The first call runs its first `warmup` micro-batches eagerly on a side stream (they are real
    micro-batches: their gradients count), captures the next, replays it, and replays the rest;
    later calls only replay."""

    def __init__(self, model, data_loader, device, warmup=2):
        if not GraphedTrainStep.supported(model):
            raise ValueError("GraphedTrainStep: data-parallel wrappers, CP and PP are not captured")
        self.model, self.loader, self.device = model, data_loader, torch.device(device)
        self.warmup = max(1, warmup)
        self.graph = None
        self.params = [p for p in model.parameters() if p.requires_grad]
        self.grads = None
        self.acc = torch.zeros((), dtype=torch.float32, device=self.device)

    @staticmethod
    def supported(model):
        m = pgm.current()
        return not hasattr(model, "bucket_manager") and not getattr(model, "_force_grad_sync", False) and \
            m.cp_world_size == 1 and m.pp_world_size == 1 and m.cp_dp_world_size == 1

    def _micro_batch(self, input_ids, target_ids):
        outputs = self.model(input_ids=input_ids)
        batch_size, seq_len = input_ids.shape
        outputs = outputs.view(seq_len * batch_size, -1)
        loss = FN.cross_entropy(outputs, target_ids.reshape(-1), reduction="mean") / self.loader.grad_acc_steps
        loss.backward()
        self.acc += loss.detach().float()

    def _capture(self, batch):
        self.ids = batch["input_ids"].to(self.device).clone()
        self.tgt = batch["target_ids"].to(self.device).clone()
        # every parameter's gradient must exist (allocated eagerly, outside the graph's pool) so the
        # captured epilogues accumulate into buffers this object keeps
        missing = [p for p in self.params if p.grad is None]
        if missing:
            raise RuntimeError(f"GraphedTrainStep: {len(missing)} parameters got no gradient in the warm-up")
        self.grads = [p.grad for p in self.params]
        quiesce_collectives(self.device)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self._micro_batch(self.ids, self.tgt)

    def __call__(self, on_microbatch=None, read_loss=True):
        """One optimizer step's worth of micro-batches; returns the accumulated loss (float, or the
        device scalar with read_loss=False: see train_step)."""
        ga = self.loader.grad_acc_steps
        self.acc.zero_()
        if self.grads is not None:
            for p, g in zip(self.params, self.grads):
                if p.grad is not g:
                    p.grad = g
            torch._foreach_zero_(self.grads)
        for i in range(ga):
            if on_microbatch is not None:
                on_microbatch(i)
            batch = next(self.loader)
            if self.graph is None and i < self.warmup:
                side = torch.cuda.Stream(self.device)
                side.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(side):
                    self._micro_batch(batch["input_ids"].to(self.device), batch["target_ids"].to(self.device))
                torch.cuda.current_stream(self.device).wait_stream(side)
                continue
            if self.graph is None:
                self._capture(batch)
            else:
                self.ids.copy_(batch["input_ids"])
                self.tgt.copy_(batch["target_ids"])
            self.graph.replay()
        loss = self.acc.clone()
        return read_step_loss(loss, self.device) if read_loss else loss


def read_step_loss(acc_loss, device):
    """The step's loss as a float (one host <-> device synchronisation), then the device status check
    (HipKernelError on a bad cross-entropy target) -- called after an optimizer step that was enqueued
    first (train_step(read_loss=False)), the check comes after that update."""
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
