"""Multi-process (gloo, CPU) harness for distributed tests."""
import os
import socket
import tempfile
import traceback

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, fn, args, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), FLEETX_LOG_RANK0_ONLY="1")
    torch.set_num_threads(1)
    hang = int(os.environ.get("FLEETX_TEST_HANG_DUMP", "0"))
    if hang > 0:  # debugging aid: dump every thread's stack if the rank hangs
        import faulthandler
        faulthandler.dump_traceback_later(hang, exit=True)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        res = fn(rank, world, *args)
        torch.save(res, os.path.join(outdir, "r%d.pt" % rank))
    except Exception:
        with open(os.path.join(outdir, "err%d.txt" % rank), "w") as f:
            f.write(traceback.format_exc())
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def run(fn, world, *args, timeout=600):
    """Run ``fn(rank, world, *args)`` on ``world`` gloo ranks; return results."""
    port = free_port()
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=_worker, args=(r, world, port, fn, args, d))
                 for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout)
        errs = []
        for r, p in enumerate(procs):
            if p.is_alive():
                p.kill()
                errs.append("rank %d timed out" % r)
            ef = os.path.join(d, "err%d.txt" % r)
            if os.path.exists(ef):
                errs.append(open(ef).read())
        if errs:
            raise RuntimeError("\n".join(errs))
        return [torch.load(os.path.join(d, "r%d.pt" % r), weights_only=False) for r in range(world)]
