"""Multi-process gloo harness for the TP / CP / DP tests (world_size 2-4; CPU host logic, or all ranks on cuda:0)."""
import os
import socket
import sys
import traceback

import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, fn, args, errq, device, backend="gloo"):
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank) if device == "cpu" else "0", DEVICE=device)
    try:
        if backend == "nccl":   # RCCL: one rank per device (a one-rank group on the one-GPU box)
            import torch
            torch.cuda.set_device(rank)
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", rank))
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        fn(rank, world, *args)
        dist.barrier()
    except Exception:
        errq.put(f"rank {rank}:\n{traceback.format_exc()}")
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def run(fn, world, *args, device="cpu", backend="gloo"):
    """Run fn(rank, world, *args) on `world` gloo ranks (backend="nccl": RCCL, one rank per GPU);
    re-raise the first rank failure.
    device="cuda": every rank drives cuda:0 (the one-GPU box) and gloo moves the CUDA tensors of
    the collectives through host memory -- the HIP kernels under the TP / CP wrappers run for real,
    only the transport differs from RCCL."""
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, args, errq, device, backend)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    for p in procs:
        if p.is_alive():
            p.kill()
    if not errq.empty():
        raise AssertionError(errq.get())
    bad = [p.exitcode for p in procs if p.exitcode != 0]
    assert not bad, f"worker exit codes {bad}"
