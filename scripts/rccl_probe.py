#!/usr/bin/env python3
"""Probe: can two RCCL ranks share the one GPU of a gpurun box?  Each rank of
`python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 scripts/rccl_probe.py`
binds cuda:0, initialises the "nccl" (RCCL) process group, and runs an all-reduce, a broadcast and
a batch_isend_irecv ring exchange; rank 0 prints one JSON line with what ran."""
import json
import os
import sys

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", int(os.environ.get("PROBE_DEVICE", "0")))
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    res = {"world": world, "backend": dist.get_backend()}
    x = torch.full((1 << 20,), float(rank + 1), device=dev)
    dist.all_reduce(x)
    res["all_reduce_ok"] = bool(torch.all(x == world * (world + 1) / 2).item())
    y = torch.arange(16, device=dev, dtype=torch.float64) * (rank + 1)
    dist.broadcast(y, src=0)
    res["broadcast_ok"] = bool(torch.equal(y, torch.arange(16, device=dev, dtype=torch.float64)))
    send = torch.full((4096,), float(rank), device=dev, dtype=torch.complex64)
    recv = torch.empty_like(send)
    ops = [dist.P2POp(dist.isend, send, (rank + 1) % world), dist.P2POp(dist.irecv, recv, (rank - 1) % world)]
    for r in dist.batch_isend_irecv(ops):
        r.wait()
    torch.cuda.synchronize()
    res["p2p_ok"] = bool(torch.all(recv == float((rank - 1) % world)).item())
    dist.barrier()
    if rank == 0:
        print(json.dumps(res), flush=True)
    dist.destroy_process_group()
    return 0 if all(v for k, v in res.items() if k.endswith("_ok")) else 1


if __name__ == "__main__":
    sys.exit(main())
