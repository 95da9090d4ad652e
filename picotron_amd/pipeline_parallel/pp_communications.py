"""Pipeline-parallel p2p (picotron/pipeline_parallel/pp_communications.py:8-45), §8f row 4.

Same functions, arguments, return values, VERBOSE trace and module globals (STEP, VERBOSE) as the
reference's `pipeline_communicate` / `bidirectional_pipeline_communicate`, which the reference's
unchanged PipelineParallel engine (1F1B / AFAB, pipeline_parallel.py:77-214) calls through the
drop-in overlay.  One difference, with the semantics preserved: over RCCL the blanket
`torch.cuda.synchronize()` after every transfer (pp_comm.py:30,44) is dropped.  An RCCL p2p is
stream-ordered: ProcessGroupNCCL makes its communication stream wait for the current stream before
the send (the activations' producers have run) and `req.wait()` makes the current stream wait for
the transfer (every consumer of a received tensor runs after it), while the send buffer is kept
alive by the process group until the transfer completes.  So the host is never blocked and the
next micro-batch's kernels can be queued behind the transfer.  Over gloo (CPU tensors, or CUDA
tensors staged through the host in the multi-rank tests) the reference's synchronisation is kept.
"""
import os

import torch
import torch.distributed as dist

from .. import process_group_manager as pgm

STEP, VERBOSE = 0, os.environ.get("VERBOSE", "0") == "1"


def _host_sync():
    """The reference's torch.cuda.synchronize(), only where p2p is not stream-ordered."""
    if dist.get_backend() != "nccl" and torch.cuda.is_available():
        torch.cuda.synchronize()


def pipeline_communicate(operation, device, dtype, tensor=None, shapes=None):
    """pp_comm.py:8-32: one of recv_forward / send_forward / recv_backward / send_backward with the
    previous / next pipeline stage (global ranks from the process grid); None at the pipeline ends."""
    global STEP
    m = pgm.process_group_manager
    if operation == "recv_forward":
        if m.pp_is_first_stage:
            return None
        tensor = torch.empty(shapes, requires_grad=True, device=device, dtype=dtype)
        src = m.pp_prev_rank
    elif operation == "send_forward":
        if m.pp_is_last_stage:
            return None
        dest = m.pp_next_rank
    elif operation == "recv_backward":
        if m.pp_is_last_stage:
            return None
        tensor = torch.empty(shapes, requires_grad=True, device=device, dtype=dtype)
        src = m.pp_next_rank
    elif operation == "send_backward":
        if m.pp_is_first_stage:
            return None
        dest = m.pp_prev_rank
    else:
        raise ValueError(f"pipeline_communicate: unknown operation {operation!r}")
    is_send = operation.startswith("send")
    peer_rank = dest if is_send else src
    if is_send:
        _host_sync()   # gloo only: the tensor's producers have finished before it is read
    op = dist.P2POp(dist.isend if is_send else dist.irecv, tensor, peer_rank)
    if VERBOSE:
        print(f"{operation} | {'sending' if is_send else 'receiving'} {operation.split('_')[1]} {m.pp_rank} "
              f"{'→' if is_send else '←'} {peer_rank} | STEP:{STEP} | RANK:{m.pp_rank}", flush=True)
    for req in dist.batch_isend_irecv([op]):
        req.wait()
    _host_sync()
    if VERBOSE:
        STEP += 1
    return tensor if not is_send else None


def bidirectional_pipeline_communicate(operation, send_tensor, recv_shapes, device, dtype):
    """pp_comm.py:34-45: send_fwd_recv_bwd (with the next stage) / send_bwd_recv_fwd (with the
    previous one) as one batched isend + irecv; None at the pipeline end that has no peer."""
    global STEP
    m = pgm.process_group_manager
    is_fwd = operation == "send_fwd_recv_bwd"
    if (is_fwd and m.pp_is_last_stage) or (not is_fwd and m.pp_is_first_stage):
        return None
    peer_rank = m.pp_next_rank if is_fwd else m.pp_prev_rank
    recv_tensor = torch.empty(recv_shapes, requires_grad=True, device=device, dtype=dtype)
    _host_sync()
    reqs = dist.batch_isend_irecv([dist.P2POp(dist.isend, send_tensor, peer_rank),
                                   dist.P2POp(dist.irecv, recv_tensor, peer_rank)])
    if VERBOSE:
        print(f"{operation} | sending {'next' if is_fwd else 'prev'} {m.pp_rank} -> {peer_rank} | "
              f"receiving {'next' if is_fwd else 'prev'} {peer_rank} -> {m.pp_rank} | STEP {STEP=} | "
              f"RANK:{m.pp_rank}", flush=True)
    for req in reqs:
        req.wait()
    _host_sync()
    if VERBOSE:
        STEP += 1
    return recv_tensor
