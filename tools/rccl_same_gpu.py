"""Probe: can RCCL (torch.distributed backend "nccl") run a communicator of
two ranks that share one GPU?  The one-GPU boxes this build is tested on
cannot otherwise run RCCL at world >= 2 (VERDICT r05 "What's missing" 2).
Run: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1
     --master-port 29533 tools/rccl_same_gpu.py"""
import os
import sys

import torch
import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
try:
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    x = torch.full((4,), float(rank + 1), device="cuda:0")
    out = [torch.empty_like(x) for _ in range(world)] if rank == 0 else None
    dist.gather(x, out, dst=0)
    torch.cuda.synchronize()
    if rank == 0:
        print("gather ok:", [t.tolist() for t in out], flush=True)
    dist.barrier()
    dist.destroy_process_group()
except Exception as e:  # noqa: BLE001 -- the probe reports what RCCL said
    print(f"rank {rank}: {type(e).__name__}: {str(e)[:400]}", flush=True)
    sys.exit(1)
