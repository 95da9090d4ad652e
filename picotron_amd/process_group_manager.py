"""The 4-D process grid (dp, pp, cp, tp) -- the topology the hot path's collectives run over.

Mirrors picotron/process_group_manager.py:5-67 of the reference (same grid order
`arange(world).view(dp, pp, cp, tp)`, TP innermost, same attribute names, module-global
`process_group_manager` set by `setup_process_group_manager`), so the TP/CP/DP code of this
package reads the same groups the reference's does.  One addition: without an initialised
torch.distributed job (a single-GPU bench or test) the manager describes a 1-rank grid with no
groups instead of failing.
"""
import os

import torch
import torch.distributed as dist

process_group_manager = None


class ProcessGroupManager:
    def __init__(self, tp_size, cp_size, pp_size, dp_size):
        distributed = dist.is_available() and dist.is_initialized()
        self.global_rank = dist.get_rank() if distributed else 0
        self.world_size = dist.get_world_size() if distributed else 1
        self.local_rank = int(os.environ.get("LOCAL_RANK", self.global_rank % self.world_size))
        assert self.world_size == tp_size * cp_size * pp_size * dp_size, (
            f"World size ({self.world_size}) != TP ({tp_size}) * CP ({cp_size}) * PP ({pp_size}) * DP ({dp_size})")
        self.grid = torch.arange(self.world_size).view(dp_size, pp_size, cp_size, tp_size)
        self.dp_rank, self.pp_rank, self.cp_rank, self.tp_rank = (self.grid == self.global_rank).nonzero().flatten().tolist()

        g = self.grid
        if distributed:
            def sub(ranks_lists):
                return dist.new_subgroups_by_enumeration(ranks_lists)[0]
            self.tp_group = sub([g[d, p, c, :].tolist() for d in range(dp_size) for p in range(pp_size) for c in range(cp_size)])
            self.cp_group = sub([g[d, p, :, t].tolist() for d in range(dp_size) for p in range(pp_size) for t in range(tp_size)])
            self.pp_group = sub([g[d, :, c, t].tolist() for d in range(dp_size) for c in range(cp_size) for t in range(tp_size)])
            self.dp_group = sub([g[:, p, c, t].tolist() for p in range(pp_size) for c in range(cp_size) for t in range(tp_size)])
            self.cp_dp_group = sub([g[:, p, :, t].flatten().tolist() for p in range(pp_size) for t in range(tp_size)])
            self.pp_dp_group = sub([g[:, :, c, t].flatten().tolist() for c in range(cp_size) for t in range(tp_size)])
            self.world_group = dist.group.WORLD
        else:
            self.tp_group = self.cp_group = self.pp_group = self.dp_group = None
            self.cp_dp_group = self.pp_dp_group = self.world_group = None

        dr, pr, cr, tr = self.dp_rank, self.pp_rank, self.cp_rank, self.tp_rank
        self.tp_group_ids = g[dr, pr, cr, :].tolist()
        self.cp_group_ids = g[dr, pr, :, tr].tolist()
        self.pp_group_ids = g[dr, :, cr, tr].tolist()
        self.dp_group_ids = g[:, pr, cr, tr].tolist()
        self.cp_dp_group_ids = g[:, pr, :, tr].flatten().tolist()

        self.tp_world_size = tp_size
        self.tp_first_rank, self.tp_last_rank = self.tp_group_ids[0], self.tp_group_ids[-1]

        self.cp_world_size = cp_size
        self.cp_first_rank, self.cp_last_rank = self.cp_group_ids[0], self.cp_group_ids[-1]
        self.cp_send_rank = self.cp_group_ids[(cr + 1) % cp_size]
        self.cp_recv_rank = self.cp_group_ids[(cr - 1) % cp_size]

        self.pp_world_size = pp_size
        self.pp_first_rank, self.pp_last_rank = self.pp_group_ids[0], self.pp_group_ids[-1]
        self.pp_is_first_stage = pr == 0
        self.pp_is_last_stage = pr == pp_size - 1
        self.pp_next_rank = None if pr == pp_size - 1 else int(g[dr, pr + 1, cr, tr].item())
        self.pp_prev_rank = None if pr == 0 else int(g[dr, pr - 1, cr, tr].item())

        self.dp_world_size = dp_size
        self.dp_first_rank, self.dp_last_rank = self.dp_group_ids[0], self.dp_group_ids[-1]
        self.cp_dp_world_size = cp_size * dp_size

    def __str__(self):
        return (f"TP({self.tp_world_size})-CP({self.cp_world_size})-PP({self.pp_world_size})-"
                f"DP({self.dp_world_size})-Rank({self.global_rank})")


def setup_process_group_manager(tp_size, cp_size, pp_size, dp_size):
    global process_group_manager
    process_group_manager = ProcessGroupManager(tp_size, cp_size, pp_size, dp_size)
    return process_group_manager


def current():
    """The active manager; a 1-rank grid if none was set up (single-GPU use)."""
    global process_group_manager
    if process_group_manager is None:
        setup_process_group_manager(1, 1, 1, 1)
    return process_group_manager
