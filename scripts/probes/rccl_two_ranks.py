"""Probe: can two processes on the box's ONE GPU form an RCCL (backend "nccl") group and run
an all-reduce?  Prints one JSON line per rank (or the error).  Run under a time limit:

    timeout -k 10 120 python scripts/probes/rccl_two_ranks.py
"""
import json
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def rank_main(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
        x = torch.full((1 << 20,), float(rank + 1), device="cuda:0")
        dist.all_reduce(x)
        torch.cuda.synchronize()
        print(json.dumps({"rank": rank, "ok": True, "value": float(x[0]), "expect": world * (world + 1) / 2}),
              flush=True)
        dist.destroy_process_group()
    except Exception as exc:  # noqa: BLE001
        print(json.dumps({"rank": rank, "ok": False, "error": str(exc)[:400]}), flush=True)
        sys.exit(1)


if __name__ == "__main__":
    world = 2
    mp.start_processes(rank_main, args=(world, _port()), nprocs=world, start_method="spawn")
