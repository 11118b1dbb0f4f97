"""Is the 4-rank heap abort of the one-GPU gloo rehearsals in torch's gloo CUDA-tensor path itself?

No libdmx, no depthmapx_amd: W ranks share cuda:0 over gloo and run the collectives the un-staged
rehearsal ran on CUDA tensors (sharded.py before commit 5b56724): an all-gather of the blob sizes,
an all-gather of large ragged byte blobs padded to the largest, an all-reduce of int64 buffers, an
all-gather of float rows.  MODE=cuda uses CUDA tensors (gloo stages them internally), MODE=host
passes host tensors (what sharded._gather_host does now).

    torchrun --nproc-per-node 4 --master-addr 127.0.0.1 scripts/gloo_cuda_repro.py
"""
import os
import sys
import time

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    mode = os.environ.get("MODE", "cuda")
    iters = int(os.environ.get("ITERS", "20"))
    mb = int(os.environ.get("BLOB_MB", "150"))
    if mode == "cuda":
        torch.cuda.set_device(0)
    dev = torch.device("cuda", 0) if mode == "cuda" else torch.device("cpu")
    dist.init_process_group("gloo")
    g = torch.Generator().manual_seed(rank)
    t0 = time.time()
    for it in range(iters):
        n = (mb << 20) + rank * 4099 + it * 17            # ragged, rank-dependent sizes
        sz = torch.tensor([n], dtype=torch.int64, device=dev)
        sizes = [torch.zeros_like(sz) for _ in range(world)]
        dist.all_gather(sizes, sz)
        mx = max(int(s.item()) for s in sizes)
        mine = torch.zeros(mx, dtype=torch.uint8, device=dev)
        mine[:n] = rank + it
        parts = [torch.empty(mx, dtype=torch.uint8, device=dev) for _ in range(world)]
        dist.all_gather(parts, mine)
        for r in range(world):
            assert int(parts[r][0].item()) == (r + it) & 0xFF
        red = torch.randint(0, 1000, ((4 << 20) + it,), generator=g, dtype=torch.int64).to(dev)
        dist.all_reduce(red, op=dist.ReduceOp.SUM)
        rows = torch.full((65536 + rank, 7), float(rank), device=dev)
        per = 65536 + world
        pad = torch.zeros((per, 7), device=dev)
        pad[: rows.shape[0]] = rows
        outs = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(outs, pad)
        del parts, mine, red, outs
        if rank == 0:
            print("iter %d ok %.1f s" % (it, time.time() - t0), flush=True)
    dist.barrier()
    if rank == 0:
        print("REPRO_DONE mode=%s world=%d iters=%d" % (mode, world, iters), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
