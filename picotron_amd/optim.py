"""AdamW for the training step (reference train.py:205-209: `torch.optim.AdamW(model.parameters(),
lr=learning_rate)`), with each tensor's update fused into one HIP pass (csrc/adamw.hip).

Same constructor, defaults, param_groups and state layout as torch.optim.AdamW (state['step'] a CPU
float tensor, state['exp_avg'] / state['exp_avg_sq'] in the parameter's dtype), so a checkpoint of
one loads into the other; the per-element math is torch's multi-tensor (foreach) Adam with
decoupled weight decay, op for op with the same roundings to the storage dtype.
"""
import torch

from . import kernels as K


class AdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, amsgrad=False,
                 maximize=False):
        if amsgrad or maximize:
            raise ValueError("picotron_amd.optim.AdamW: amsgrad / maximize are not used by picotron (train.py:209)")
        if not 0.0 <= lr or not 0.0 <= eps or not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"invalid AdamW hyper-parameters lr={lr} betas={betas} eps={eps}")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None):
        """torch.optim.AdamW.step (foreach, decoupled weight decay) on the HIP kernel: the bf16 tensors
        that share a step count go through ONE multi-tensor launch; anything else (f32, unaligned)
        per tensor."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            lr, (beta1, beta2), eps, wd = group["lr"], group["betas"], group["eps"], group["weight_decay"]
            batches = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("AdamW does not support sparse gradients")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                t = st["step"].item()
                item = (p, p.grad, st["exp_avg"], st["exp_avg_sq"])
                multi = p.dtype == torch.bfloat16 and all(x.is_contiguous() and x.data_ptr() % 16 == 0 for x in item) \
                    and p.grad.dtype == p.dtype
                batches.setdefault((t, multi), []).append(item)
            for (t, multi), items in batches.items():
                bc1 = 1 - beta1 ** t
                bc2 = 1 - beta2 ** t
                sc = dict(decay=1 - lr * wd, w1=1 - beta1, beta2=beta2, c2=1 - beta2, bc2_sqrt=bc2 ** 0.5, eps=eps,
                          step_size=(lr / bc1) * -1)
                if multi:
                    K.adamw_step_multi(items, **sc)
                else:
                    for p, g, m, v in items:
                        K.adamw_step(p, g, m, v, **sc)
        return loss
