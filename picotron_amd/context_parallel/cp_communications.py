"""Ring send/recv over the cp group (picotron/context_parallel/cp_communications.py:10-53).

Same interface as the reference's ContextCommunicate (send_recv / commit / wait, batched
isend/irecv to the next / from the previous cp rank).  One difference: `wait` does not call
torch.cuda.synchronize() (cp_comm.py:51).  Waiting on the RCCL work handle already orders torch's
current stream after the transfer, so the host is never blocked and the next block's attention
kernel can be queued while the transfer is in flight.  Over gloo (the multi-rank tests on one GPU),
p2p of CUDA tensors is not ordered with the compute stream, so there the reference's
synchronisation is kept: before the sends are posted and after the receives complete.
"""
import os

import torch
import torch.distributed as dist

from .. import process_group_manager as pgm

VERBOSE = os.environ.get("VERBOSE", "0") == "1"


class ContextCommunicate:
    def __init__(self, msg: str = ""):
        m = pgm.current()
        self._pending_operations = []
        self._active_requests = None
        self.msg = msg
        self.rank = m.cp_rank
        self.world_size = m.cp_world_size
        self.send_rank = m.cp_send_rank
        self.recv_rank = m.cp_recv_rank
        self.group = m.cp_group
        self._host_sync = dist.get_backend(self.group) != "nccl"   # gloo: not stream-ordered
        if VERBOSE:
            print(f"RingComm ({msg}) | initialized | RANK:{self.rank} | WORLD_SIZE:{self.world_size} | "
                  f"SEND_RANK:{self.send_rank} | RECV_RANK:{self.recv_rank}", flush=True)

    def send_recv(self, tensor_to_send, recv_tensor=None):
        result = recv_tensor if recv_tensor is not None else tensor_to_send.new_empty(tensor_to_send.shape)
        self._pending_operations.append(dist.P2POp(dist.isend, tensor_to_send, self.send_rank, group=self.group))
        self._pending_operations.append(dist.P2POp(dist.irecv, result, self.recv_rank, group=self.group))
        return result

    def commit(self):
        if self._active_requests is not None:
            raise RuntimeError("Commit called twice")
        if self._host_sync and torch.cuda.is_available():
            torch.cuda.synchronize()   # the send buffers' producers must have finished
        self._active_requests = dist.batch_isend_irecv(self._pending_operations)

    def wait(self):
        if self._active_requests is None:
            raise RuntimeError("Wait called before commit")
        for req in self._active_requests:
            req.wait()
        if self._host_sync and torch.cuda.is_available():
            torch.cuda.synchronize()   # cp_comm.py:51
        self._active_requests = None
        self._pending_operations = []


def _zz_home(h, C):
    """Zig-zag ring layout: global half-chunk h (of 2C) lives on cp rank h (first half, h < C) or
    2C - 1 - h (second half).  Returns (rank, slot)."""
    return (h, 0) if h < C else (2 * C - 1 - h, 1)


def zigzag_exchange(xs, dims, to_zigzag):
    """Re-lay sequence shards between the reference's contiguous split (cp rank r holds global
    half-chunks 2r and 2r + 1 of 2C, data.py:105-109 / update_rope_for_context_parallel) and the
    zig-zag split (rank r holds half-chunks r and 2C - 1 - r), so every rank does the same causal
    work in the ring.  xs: tensors whose dimension dims[i] is this rank's sequence (even length);
    returns new contiguous tensors in the other layout.  One batched isend/irecv over the cp group
    (RCCL: stream-ordered, no host synchronisation; gloo: the host synchronises around it, as
    ContextCommunicate does).  Messages between one pair of ranks are posted in slot order on both
    sides, so they match whatever the pairing."""
    m = pgm.current()
    C, r, ids, group = m.cp_world_size, m.cp_rank, m.cp_group_ids, m.cp_group
    halves = [[x.narrow(d, p * (x.shape[d] // 2), x.shape[d] // 2) for p in (0, 1)] for x, d in zip(xs, dims)]
    outs = [[None, None] for _ in xs]
    ops = []
    for p in (0, 1):    # my two source slots -> (rank, slot) in the other layout
        h = 2 * r + p if to_zigzag else (r if p == 0 else 2 * C - 1 - r)
        dst, dslot = _zz_home(h, C) if to_zigzag else (h // 2, h % 2)
        for i in range(len(xs)):
            if dst == r:
                outs[i][dslot] = halves[i][p]
            else:
                ops.append(dist.P2POp(dist.isend, halves[i][p].contiguous(), ids[dst], group=group))
    for s in (0, 1):    # my two destination slots <- (rank, slot) in this layout
        h = (r if s == 0 else 2 * C - 1 - r) if to_zigzag else 2 * r + s
        src = h // 2 if to_zigzag else _zz_home(h, C)[0]
        if src == r:
            continue
        for i in range(len(xs)):
            outs[i][s] = torch.empty_like(halves[i][s], memory_format=torch.contiguous_format)
            ops.append(dist.P2POp(dist.irecv, outs[i][s], ids[src], group=group))
    if ops:
        host_sync = dist.get_backend(group) != "nccl" and torch.cuda.is_available()
        if host_sync:
            torch.cuda.synchronize()
        for req in dist.batch_isend_irecv(ops):
            req.wait()
        if host_sync:
            torch.cuda.synchronize()
    return [torch.cat(o, dim=d) for o, d in zip(outs, dims)]
