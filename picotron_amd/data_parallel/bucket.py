"""Gradient buckets for the DP all-reduce (RCCL over xGMI).

Mirrors picotron/data_parallel/bucket.py (okoge-kaz/picotron @ 2025-03-02): Bucket (:6-57) and
BucketManager (:59-157) -- the same greedy assignment in parameters() order (a parameter that does
not fit opens a new bucket; one larger than the cap gets a bucket of its own), fp32 flat storage,
`param.main_grad` views, pre-division by the group size and one async all-reduce per bucket once
all of its parameters are ready.

MI355X notes: the fused wgrad GEMMs of functional.py accumulate straight into `main_grad` (fp32
epilogue), so no separate `main_grad += grad` pass runs for the projection weights.  Buckets are
allocated on the parameters' device; the all-reduce runs on RCCL's stream and is waited on from
torch's stream (no host synchronisation).
"""
from typing import List

import torch
import torch.distributed as dist


class Bucket:
    def __init__(self, params: List[torch.nn.Parameter], grad_data: torch.Tensor, process_group) -> None:
        self.params = set(params)
        self.params_with_grad_ready = set()
        self.grad_data = grad_data
        self.process_group = process_group
        self.process_group_size = dist.get_world_size(group=process_group)
        self.handle = None
        self.reset()

    def sync_gradient(self) -> None:
        assert self.handle is None
        self.grad_data /= self.process_group_size
        self.handle = dist.all_reduce(self.grad_data, group=self.process_group, async_op=True)

    def reset(self) -> None:
        self.handle = None
        self.params_with_grad_ready.clear()
        self.grad_data.zero_()

    def wait(self) -> None:
        assert self.handle is not None, "You should launch an allreduce operation before waiting for it to finish"
        self.handle.wait()

    def mark_param_as_ready(self, param: torch.nn.Parameter) -> None:
        assert param in self.params and param not in self.params_with_grad_ready
        self.params_with_grad_ready.add(param)
        if len(self.params_with_grad_ready) == len(self.params):
            self.sync_gradient()


class BucketManager:
    def __init__(self, params, process_group, bucket_size: int, grad_type: torch.dtype = torch.float32) -> None:
        self.params = list(params)
        self.device = self.params[0].device if self.params[0].is_cuda else torch.device("cpu")
        self.buckets = []
        self.process_group = process_group
        self.process_group_size = dist.get_world_size(group=process_group)
        self.params_to_bucket_location = {}
        self.bucket_size = bucket_size
        self.bucket_sizes = None
        self.grad_data_list = []
        self.grad_type = grad_type
        self._initialize_buckets()

    def _initialize_buckets(self) -> None:
        cur_size, cur_idx = 0, 0
        for param in self.params:
            if not param.requires_grad:
                continue
            n = param.numel()
            if cur_size == 0:
                self.params_to_bucket_location[param] = (0, n, cur_idx)
                cur_size = n
            elif cur_size + n > self.bucket_size:
                cur_idx += 1
                self.params_to_bucket_location[param] = (0, n, cur_idx)
                cur_size = n
            else:
                self.params_to_bucket_location[param] = (cur_size, cur_size + n, cur_idx)
                cur_size += n
        sizes = [0] * (cur_idx + 1)
        members = [[] for _ in range(cur_idx + 1)]
        for param, (_, end, idx) in self.params_to_bucket_location.items():
            sizes[idx] = max(sizes[idx], end)
            members[idx].append(param)
        self.bucket_sizes = sizes
        for i, s in enumerate(sizes):
            self.grad_data_list.append(torch.zeros(s, dtype=self.grad_type, device=self.device))
            self.buckets.append(Bucket(members[i], self.grad_data_list[i], self.process_group))
        for param in self.params[::-1]:
            if not param.requires_grad:
                continue
            start, end, idx = self.params_to_bucket_location[param]
            param.main_grad = self.grad_data_list[idx][start:end].view(param.shape)

    def reset(self) -> None:
        for bucket in self.buckets:
            bucket.reset()

    def wait(self) -> None:
        for bucket in self.buckets:
            bucket.wait()

    def mark_param_as_ready(self, param: torch.nn.Parameter) -> None:
        self.buckets[self.params_to_bucket_location[param][2]].mark_param_as_ready(param)
