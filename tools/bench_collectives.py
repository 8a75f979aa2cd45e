"""RCCL collective bandwidth over the node's xGMI mesh.

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
        --master-addr 127.0.0.1 --master-port 29600 tools/bench_collectives.py

One rank per GPU, nccl (= RCCL) backend.  For every op in {all_reduce,
reduce_scatter, all_gather, all_to_all} and message size 1 MiB .. 1 GiB
(bf16; the size is the full per-rank buffer), times ``--iters`` back-to-back
calls with HIP events after warm-up, takes the MAX over ranks and prints one
JSON line per (op, size) from rank 0:

* ``algbw_GBps``  = bytes / time
* ``busbw_GBps``  = algbw x 2(n-1)/n (all-reduce) or (n-1)/n (the others) --
  the per-GPU link traffic a ring (or any bandwidth-optimal) algorithm moves,
  comparable across ops and with the link model
* ``links_equiv`` = busbw / the per-link xGMI rate (``--link-GBps``, 153 GB/s
  per direction): how many of a GPU's 7 point-to-point links the collective
  keeps busy.  A fully-connected 8-GPU node can in principle reach ~7.

The framework's large-message traffic is the data-parallel / ZeRO gradient
buckets (``Distributed.comm.dp_bucket_mb``, 256 MiB by default) and the ZeRO
parameter all-gather.  The communicator's CTA (channel) budget takes the same
keys as ``Distributed.comm.ctas`` (``parallel/topology.py``): ``--ctas dp``
benchmarks with the data-parallel group's default ``(min, max)``,
``--ctas 8,16`` with an explicit one, ``--ctas none`` with RCCL's own choice,
so the first 8-GPU run can A/B them; ``--rccl-env K=V,...`` exports extra RCCL
variables.  Numbers are only meaningful on a multi-GPU node (RCCL refuses two
ranks on one device).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

BUS_FACTOR = {
    "all_reduce": lambda n: 2.0 * (n - 1) / n,
    "reduce_scatter": lambda n: (n - 1) / n,
    "all_gather": lambda n: (n - 1) / n,
    "all_to_all": lambda n: (n - 1) / n,
}


def cta_budget(spec):
    """``--ctas`` -> ``(min, max)`` or None (same keys / value forms as
    ``Distributed.comm.ctas``)."""
    from fleetx_amd.parallel import topology as topo
    if spec in (None, "", "none"):
        return None
    if spec in topo.CTA_KEYS:
        return topo.parse_ctas("preset").get(topo.CTA_KEYS[spec])
    return topo.parse_ctas({"dp": spec})["data"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--min-mb", type=float, default=1)
    ap.add_argument("--max-mb", type=float, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--ops", default="all_reduce,reduce_scatter,all_gather,all_to_all")
    ap.add_argument("--link-GBps", type=float, default=153.0)
    ap.add_argument("--ctas", default="none",
                    help="CTA budget of the benchmarked communicator: a Distributed.comm.ctas "
                         "key (dp, mp, pp, sharding, data_world, check, embedding), 'min,max', "
                         "or 'none'")
    ap.add_argument("--rccl-env", default="", help="extra RCCL env, K=V[,K=V]")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from fleetx_amd.parallel import topology as topo

    for kv in (x for x in args.rccl_env.split(",") if x):
        k, v = kv.split("=", 1)
        os.environ.setdefault(k, v)
    budget = cta_budget(args.ctas)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    # the benchmarked communicator: the whole world with the chosen budget
    opts = topo.nccl_options(budget)
    grp = dist.new_group(ranks=list(range(dist.get_world_size())), pg_options=opts) \
        if opts is not None else None
    n = dist.get_world_size()
    rank = dist.get_rank()
    dt = torch.bfloat16
    esz = 2
    sizes = []
    mb = args.min_mb
    while mb <= args.max_mb:
        sizes.append(int(mb * 2 ** 20))
        mb *= 2
    for op in args.ops.split(","):
        for nbytes in sizes:
            numel = nbytes // esz // n * n
            x = torch.randn(numel, device="cuda").to(dt)
            if op == "all_reduce":
                fn = lambda: dist.all_reduce(x, group=grp)  # noqa: E731
            elif op == "reduce_scatter":
                out = torch.empty(numel // n, device="cuda", dtype=dt)
                fn = lambda: dist.reduce_scatter_tensor(out, x, group=grp)  # noqa: E731
            elif op == "all_gather":
                part = torch.randn(numel // n, device="cuda").to(dt)
                fn = lambda: dist.all_gather_into_tensor(x, part, group=grp)  # noqa: E731
            elif op == "all_to_all":
                out = torch.empty_like(x)
                fn = lambda: dist.all_to_all_single(out, x, group=grp)  # noqa: E731
            else:
                raise ValueError(op)
            for _ in range(args.warmup):
                fn()
            torch.cuda.synchronize()
            dist.barrier()
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.iters):
                fn()
            b.record()
            torch.cuda.synchronize()
            t = torch.tensor([a.elapsed_time(b) / 1000.0 / args.iters], device="cuda",
                             dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            sec = float(t.item())
            if rank == 0:
                alg = numel * esz / sec / 1e9
                bus = alg * BUS_FACTOR[op](n)
                print(json.dumps({"op": op, "world": n, "bytes": numel * esz, "dtype": "bf16",
                                  "us": round(sec * 1e6, 1), "algbw_GBps": round(alg, 1),
                                  "busbw_GBps": round(bus, 1),
                                  "links_equiv": round(bus / args.link_GBps, 2),
                                  "ctas": list(budget) if budget else None,
                                  "rccl_env": {k: v for k, v in os.environ.items()
                                               if k.startswith(("NCCL_", "RCCL_"))}}),
                      flush=True)
            del x
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
