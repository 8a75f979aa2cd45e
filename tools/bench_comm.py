"""Latency of the one-shot IPC all-reduce (parallel/comm.py) vs message size.

    python tools/bench_comm.py [--world 2] [--iters 200]

Spawns ``--world`` ranks (gloo for the handle exchange; every rank on its own
device when there are enough, else all on device 0) and times back-to-back
calls with HIP events; rank 0 prints one JSON line per (dtype, bytes).  With
--rccl (one device per rank, nccl backend) the same sizes go through
``dist.all_reduce`` for comparison."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _bench(rank, world, iters, rccl):
    import torch.distributed as dist
    from fleetx_amd.parallel.comm import IpcAllReduce
    dev = rank if torch.cuda.device_count() >= world else 0
    torch.cuda.set_device(dev)
    ar = IpcAllReduce(None, max_bytes=256 * 1024)
    rows = []
    for nbytes in (4096, 16384, 65536, 262144):
        for dtype in (torch.float32, torch.bfloat16):
            n = nbytes // torch.tensor([], dtype=dtype).element_size()
            x = torch.randn(n, device="cuda").to(dtype)
            for _ in range(10):
                ar.all_reduce(x)
            torch.cuda.synchronize()
            dist.barrier()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(iters):
                ar.all_reduce(x)
            b.record()
            torch.cuda.synchronize()
            us = a.elapsed_time(b) * 1000.0 / iters
            row = {"op": "oneshot_allreduce", "world": world, "bytes": nbytes,
                   "dtype": str(dtype).replace("torch.", ""), "us_per_call": round(us, 2),
                   "shared_device": dev == 0 and world > 1 and torch.cuda.device_count() < world}
            rows.append(row)
    ar.check()
    dist.barrier()
    ar.close()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--iters", type=int, default=200)
    args = ap.parse_args()
    from tests import dist_utils
    res = dist_utils.run(_bench, args.world, args.iters, False, timeout=300)
    for row in res[0]:
        print(json.dumps(row))


if __name__ == "__main__":
    main()
