"""Probe: can two ranks share one GPU over RCCL on this box (for testing the N>1 paths)?"""
import os, sys, torch, torch.distributed as dist
rank = int(os.environ["RANK"]); world = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
x = torch.full((4,), rank + 1, dtype=torch.int64, device="cuda:0")
out = [torch.zeros(4, dtype=torch.int64, device="cuda:0") for _ in range(world)]
dist.all_gather(out, x)
if rank == 0:
    y = torch.empty(1000, dtype=torch.uint8, device="cuda:0")
    dist.recv(y, 1)
    print("recv ok", int(y[0]), [int(o[0]) for o in out], flush=True)
else:
    dist.send(torch.full((1000,), 7, dtype=torch.uint8, device="cuda:0"), 0)
dist.barrier()
dist.destroy_process_group()
