"""Probe: can two processes on ONE GPU form an RCCL (nccl backend) group?  Run with
python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P
tools/rccl_two_ranks_one_gpu.py"""
import os
from datetime import timedelta

import torch
import torch.distributed as dist

r = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0), timeout=timedelta(seconds=60))
t = torch.full((4,), float(r + 1), device="cuda:0")
dist.all_reduce(t)
torch.cuda.synchronize()
print(f"rank {r}: all_reduce -> {t.tolist()}", flush=True)
dist.destroy_process_group()
