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
