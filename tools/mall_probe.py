"""Do the gfx950 TCC counters separate Infinity-Cache (MALL) hits from HBM reads?

Reads one 64 MiB buffer twice with the same kernel: the first read after 1 GiB of other traffic
(cold: the buffer cannot be in the 256 MiB Infinity Cache, nor in the 32 MiB of L2), the second
right after the first (warm: 64 MiB stays in the Infinity Cache, not in L2).  Run under
    rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --kernel-include-regex reduce ...
a counter that counts only HBM reads drops on the second read; one that counts every L2 miss does
not.  (tools/gpu.sh step `mall`.)"""
import torch


def main():
    dev = torch.device("cuda")
    x = torch.randn(16 << 20, device=dev)            # 64 MiB f32
    evict = torch.empty(256 << 20, device=dev)        # 1 GiB
    out = torch.empty((), device=dev)
    for _ in range(3):
        evict.fill_(1.0)                              # 1 GiB of writes: x leaves L2 and the Infinity Cache
        torch.sum(x, dim=0, out=out)                  # cold read
        torch.sum(x, dim=0, out=out)                  # warm read (Infinity Cache)
    torch.cuda.synchronize()
    print("mall probe done", out.item())


if __name__ == "__main__":
    main()
