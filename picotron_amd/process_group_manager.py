"""The 4-D process grid (dp, pp, cp, tp) -- the topology the hot path's collectives run over.

Same contract as picotron/process_group_manager.py:5-67 of the reference: ranks laid out as
`arange(world).view(dp, pp, cp, tp)` (TP innermost, so a TP group is a run of consecutive ranks --
on one 8-GPU node the TP all-reduce stays inside the xGMI mesh), the same attribute names
(`tp_group`, `cp_send_rank`, `pp_is_last_stage`, `cp_dp_world_size`, ...) and the module-global
`process_group_manager` set by `setup_process_group_manager`, so the reference's own callers
(utils.py, checkpoint.py, pipeline_parallel/) read it unchanged.

Built differently: every group family is "the ranks that vary along some grid axes while the others
stay fixed", computed by one permute + reshape of the grid (`_axis_groups`) instead of a nested
comprehension per family.  Addition: without an initialised torch.distributed job (a single-GPU
bench or test) the manager describes a 1-rank grid with no process groups instead of failing.
"""
import os

import torch
import torch.distributed as dist

process_group_manager = None

DP, PP, CP, TP = 0, 1, 2, 3   # grid axes


def _axis_groups(grid, axes):
    """All rank lists that run over `axes` (row-major in grid order) with the other axes fixed; the
    fixed axes are enumerated outermost-first, the order every rank creates the groups in."""
    fixed = [a for a in range(grid.dim()) if a not in axes]
    span = 1
    for a in axes:
        span *= grid.shape[a]
    return grid.permute(*fixed, *axes).reshape(-1, span).tolist()


def _mine(lists, rank):
    return next(ranks for ranks in lists if rank in ranks)


class ProcessGroupManager:
    def __init__(self, tp_size, cp_size, pp_size, dp_size):
        distributed = dist.is_available() and dist.is_initialized()
        self.global_rank = dist.get_rank() if distributed else 0
        self.world_size = dist.get_world_size() if distributed else 1
        self.local_rank = int(os.environ.get("LOCAL_RANK", self.global_rank % self.world_size))
        assert self.world_size == tp_size * cp_size * pp_size * dp_size, (
            f"World size ({self.world_size}) != TP ({tp_size}) * CP ({cp_size}) * PP ({pp_size}) * DP ({dp_size})")
        # on the CPU whatever device context the caller builds the model under (meta, cuda)
        self.grid = torch.arange(self.world_size, device="cpu").view(dp_size, pp_size, cp_size, tp_size)
        coord = (self.grid == self.global_rank).nonzero()[0].tolist()
        self.dp_rank, self.pp_rank, self.cp_rank, self.tp_rank = coord

        families = {"tp": (TP,), "cp": (CP,), "pp": (PP,), "dp": (DP,), "cp_dp": (DP, CP), "pp_dp": (DP, PP)}
        lists = {name: _axis_groups(self.grid, axes) for name, axes in families.items()}
        for name, ranks in lists.items():
            # new_subgroups_by_enumeration creates every group of the family on every rank (a
            # collective call) and returns the one this rank belongs to
            group = dist.new_subgroups_by_enumeration(ranks)[0] if distributed else None
            setattr(self, f"{name}_group", group)
            if name != "pp_dp":
                setattr(self, f"{name}_group_ids", _mine(ranks, self.global_rank))
        self.world_group = dist.group.WORLD if distributed else None

        self.tp_world_size, self.cp_world_size, self.pp_world_size, self.dp_world_size = (
            tp_size, cp_size, pp_size, dp_size)
        self.cp_dp_world_size = cp_size * dp_size
        for name in ("tp", "cp", "pp", "dp"):
            ids = getattr(self, f"{name}_group_ids")
            setattr(self, f"{name}_first_rank", ids[0])
            setattr(self, f"{name}_last_rank", ids[-1])

        # CP ring neighbours (rank r sends its K/V shard to r+1, receives from r-1)
        self.cp_send_rank = self.cp_group_ids[(self.cp_rank + 1) % cp_size]
        self.cp_recv_rank = self.cp_group_ids[(self.cp_rank - 1) % cp_size]
        # PP neighbours (global ranks; None at the ends)
        self.pp_is_first_stage = self.pp_rank == 0
        self.pp_is_last_stage = self.pp_rank == pp_size - 1
        self.pp_next_rank = None if self.pp_is_last_stage else self.pp_group_ids[self.pp_rank + 1]
        self.pp_prev_rank = None if self.pp_is_first_stage else self.pp_group_ids[self.pp_rank - 1]

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
