"""RCCL probe (dev tool): two ranks on ONE GPU over the nccl (= RCCL) backend -- does RCCL accept it here?
Run: python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P tools/rccl_probe.py"""
import os
import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
t = torch.full((4,), float(rank + 1), device="cuda")
dist.all_reduce(t)
torch.cuda.synchronize()
print(f"rank {rank}: all_reduce -> {t.tolist()}", flush=True)
dist.destroy_process_group()
