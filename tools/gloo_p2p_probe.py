#!/usr/bin/env python3
"""Rate of torch.distributed gloo point-to-point (batch_isend_irecv) at world 2,
the callback transport the N>1 rehearsals of bench.py use when only one GPU
is present (redset_amd/dist.py TorchTransport). Each rank sends `total` bytes
to the other in messages of `msg` bytes and receives as many, all posted as
one batch -- the shape of one sharded gather. Tensors on the CPU (--device
cpu) or on the GPU (--device cuda: what the rehearsal passes). Prints one
JSON line per (device, message size).

usage: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1
       --master-port 29577 tools/gloo_p2p_probe.py --device cpu
"""
import argparse
import json
import os
import time

import torch
import torch.distributed as dist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--total-mib", type=int, default=112)
    ap.add_argument("--msg-kib", type=int, nargs="*", default=[64, 1024, 8192, 57344])
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    peer = 1 - rank
    total = a.total_mib << 20
    for kib in a.msg_kib:
        msg = kib << 10
        n = max(1, total // msg)
        send = torch.randint(0, 256, (n * msg,), dtype=torch.uint8, device=a.device)
        recv = torch.empty(n * msg, dtype=torch.uint8, device=a.device)
        best = None
        for _ in range(a.reps):
            dist.barrier()
            t0 = time.perf_counter()
            ops = []
            for i in range(n):
                ops.append(dist.P2POp(dist.isend, send[i * msg:(i + 1) * msg], peer))
                ops.append(dist.P2POp(dist.irecv, recv[i * msg:(i + 1) * msg], peer))
            for req in dist.batch_isend_irecv(ops):
                req.wait()
            if a.device != "cpu":
                torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        if rank == 0:
            print(json.dumps({"device": a.device, "world": world, "messages_per_direction": n, "msg_bytes": msg,
                              "bytes_per_direction": n * msg, "seconds": round(best, 4),
                              "MBps_per_direction": round(n * msg / best / 1e6, 1)}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
