#!/usr/bin/env python3
"""Can two RCCL ranks share one GPU on this box? (a rehearsal path for the
N > 1 bench legs on a one-GPU box). Run under torch.distributed.run with 2
processes; every rank uses cuda:0."""
import os

import torch
import torch.distributed as dist

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
r, w = dist.get_rank(), dist.get_world_size()
t = torch.full((4,), float(r + 1), device=dev)
dist.all_reduce(t)
g = torch.empty(w * 4, device=dev)
dist.all_gather_into_tensor(g, torch.full((4,), float(r), device=dev))
print(f"rank {r}/{w}: all_reduce {t.tolist()} all_gather {g.tolist()}", flush=True)
dist.destroy_process_group()
