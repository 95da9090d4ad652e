"""Probe: which torch.distributed gloo collectives accept CUDA tensors (2 ranks sharing cuda:0)."""
import os
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def run(rank, world):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29555")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    x = torch.full((4,), float(rank + 1), device="cuda")
    res = {}
    for name, fn in [
        ("all_reduce", lambda: dist.all_reduce(x.clone())),
        ("all_gather_into", lambda: dist.all_gather_into_tensor(torch.empty(8, device="cuda"), x)),
        ("all_gather", lambda: dist.all_gather([torch.empty(4, device="cuda") for _ in range(world)], x)),
        ("p2p", lambda: [r.wait() for r in dist.batch_isend_irecv([
            dist.P2POp(dist.isend, x, (rank + 1) % world), dist.P2POp(dist.irecv, torch.empty(4, device="cuda"), (rank - 1) % world)])]),
    ]:
        try:
            fn()
            torch.cuda.synchronize()
            res[name] = "ok"
        except Exception as e:  # noqa: BLE001
            res[name] = f"{type(e).__name__}: {str(e)[:120]}"
    print(rank, res, flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    mp.spawn(run, args=(2,), nprocs=2)
