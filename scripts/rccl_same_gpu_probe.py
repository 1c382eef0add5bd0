"""Probe: can two ranks share GPU 0 over RCCL ("nccl")?  (The box has one GPU; if RCCL accepts it,
the partitioned mode's device-to-device exchange can be rehearsed there.)  torchrun --nproc-per-node 2."""
import os

import torch
import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl")
x = torch.full((4,), float(rank + 1), device="cuda")
dist.all_reduce(x)
ops = [dist.P2POp(dist.isend, torch.full((3,), float(rank), device="cuda"), (rank + 1) % world),
       dist.P2POp(dist.irecv, y := torch.empty(3, device="cuda"), (rank - 1) % world)]
for r in dist.batch_isend_irecv(ops):
    r.wait()
torch.cuda.synchronize()
print(f"rank {rank}: all_reduce {x.tolist()} recv {y.tolist()}", flush=True)
dist.destroy_process_group()
