#!/usr/bin/env python3
"""Probe: can two RCCL ranks share one GPU on this box?  (broadcast + all_to_all_single on cuda:0)"""
import datetime
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def body(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60),
                            device_id=torch.device("cuda", 0))
    t = torch.arange(8, dtype=torch.float64, device="cuda") * (rank + 1)
    dist.broadcast(t, src=0)
    x = torch.full((world * 2,), float(rank), device="cuda")
    y = torch.empty_like(x)
    dist.all_to_all_single(y, x)
    torch.cuda.synchronize()
    print(f"rank {rank}: bcast {t[:3].tolist()} a2a {y.tolist()}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    mp.start_processes(body, args=(world, 29700), nprocs=world, start_method="spawn")
    print("RCCL multi-rank-per-GPU: OK")
