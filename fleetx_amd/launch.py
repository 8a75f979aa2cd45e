"""Multi-process launcher: one process per GPU, per-rank logs, failure
detection, a hang watchdog and restart-from-the-latest-checkpoint.

    python -m fleetx_amd.launch --devices 0,1,2,3,4,5,6,7 [--log_dir log] \\
        [--max_restart 3] [--hang_timeout 1800] tools/train.py -c cfg.yaml -o k=v ...

Capability parity: ``python -m paddle.distributed.launch`` as used by every
multi-card recipe (``projects/gpt/*.sh``):
``--devices``/``--gpus``, ``--nnodes``/``--node_rank``/``--master``,
``--log_dir`` with one ``workerlog.N`` per rank, pod watching with
``--max_restart``, and a failure report that names the failing rank, its exit
code, its command and the tail of its log (``docs/deployment_faq.md:366-396``).

MI355X design:
* children get the torchrun env contract (``RANK``, ``LOCAL_RANK``,
  ``WORLD_SIZE``, ``LOCAL_WORLD_SIZE``, ``MASTER_ADDR/PORT``) that
  :func:`fleetx_amd.parallel.topology.init_distributed` reads; RCCL
  communicators are created inside the children by ``torch.distributed``.
  The Paddle variables (``PADDLE_TRAINER_ID``, ``PADDLE_RANK_IN_NODE``,
  ``FLAGS_selected_gpus``, ...) are exported too so reference-era scripts keep
  working;
* the launcher never touches the GPU itself (it only spawns and watches), so
  a faulting rank cannot take the watcher down;
* a restart re-runs the whole pod with ``-o Engine.save_load.ckpt_dir=auto``:
  the engine resumes from the newest ``epoch_*_step_*`` checkpoint, seeking
  the sampler by ``consumed_samples`` and restoring the dropout RNG streams
  (the reference launcher restarted but training re-read and discarded the
  consumed batches);
* ``--hang_timeout``: when no rank has written to its log for that long the
  pod is treated as hung (e.g. a stuck collective), killed and restarted.
"""
import argparse
import os
import signal
import socket
import subprocess
import sys
import time


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def parse_args(argv=None):
    ap = argparse.ArgumentParser(prog="python -m fleetx_amd.launch",
                                 description="one process per device, watched and restartable")
    ap.add_argument("--devices", "--gpus", dest="devices", default=None,
                    help="comma-separated local device ids, one process each")
    ap.add_argument("--nproc_per_node", type=int, default=None)
    ap.add_argument("--nnodes", type=int, default=1)
    ap.add_argument("--node_rank", type=int, default=0)
    ap.add_argument("--master", default=None, help="host:port of the rendezvous store")
    ap.add_argument("--log_dir", default="log")
    ap.add_argument("--max_restart", type=int, default=0)
    ap.add_argument("--hang_timeout", type=float, default=0.0,
                    help="seconds without log output from any rank before the pod is "
                         "declared hung (0 = off)")
    ap.add_argument("--resume", default="auto",
                    help="Engine.save_load.ckpt_dir passed to restarted pods ('' = scratch)")
    ap.add_argument("--poll", type=float, default=0.5)
    ap.add_argument("script")
    ap.add_argument("script_args", nargs=argparse.REMAINDER)
    return ap.parse_args(argv)


def _visible_device_count():
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([x for x in v.split(",") if x.strip()])
    # Count GPUs from the KFD topology in sysfs (nodes with SIMDs are GPUs):
    # the watcher process never loads the HIP runtime (it forks the ranks and
    # outlives them).
    root = "/sys/class/kfd/kfd/topology/nodes"
    n = 0
    try:
        for node in os.listdir(root):
            try:
                with open(os.path.join(root, node, "properties")) as f:
                    for line in f:
                        k, _, v = line.partition(" ")
                        if k == "simd_count" and int(v) > 0:
                            n += 1
                            break
            except (OSError, ValueError):
                continue
    except OSError:
        return 0
    return n


def device_list(args):
    if args.devices:
        return [d.strip() for d in args.devices.split(",") if d.strip()]
    n = args.nproc_per_node or _visible_device_count() or 1
    return [str(i) for i in range(n)]


def child_env(args, devices, local_rank, attempt, master_addr, master_port):
    n = len(devices)
    world = n * args.nnodes
    rank = args.node_rank * n + local_rank
    env = dict(os.environ)
    env.update({
        "RANK": str(rank), "LOCAL_RANK": str(local_rank), "WORLD_SIZE": str(world),
        "LOCAL_WORLD_SIZE": str(n), "GROUP_RANK": str(args.node_rank),
        "MASTER_ADDR": master_addr, "MASTER_PORT": str(master_port),
        "FLEETX_RESTART_COUNT": str(attempt),
        # Paddle launcher contract (docs/deployment_faq.md:370,589-601)
        "PADDLE_TRAINER_ID": str(rank), "PADDLE_TRAINERS_NUM": str(world),
        "PADDLE_RANK_IN_NODE": str(local_rank), "PADDLE_LOCAL_RANK": str(local_rank),
        "PADDLE_GLOBAL_RANK": str(rank), "PADDLE_GLOBAL_SIZE": str(world),
        "PADDLE_LOCAL_SIZE": str(n), "PADDLE_NNODES": str(args.nnodes),
        "PADDLE_MASTER": "%s:%d" % (master_addr, master_port),
        "PADDLE_CURRENT_ENDPOINT": "%s:%d" % (master_addr, master_port + 1 + rank),
        "FLAGS_selected_gpus": devices[local_rank],
    })
    if args.devices:
        env["HIP_VISIBLE_DEVICES"] = ",".join(devices)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    # one HIP hardware queue per peer-waiting stream for multi-rank jobs
    # (utils/streams.py): RCCL communicators must not share in-order queues
    if world > 1:
        from .utils.streams import ensure_hw_queues
        ensure_hw_queues(8, env=env)
    return env


class Pod:
    """The set of local rank processes of one launch attempt."""

    def __init__(self, args, devices, attempt, master_addr, master_port, extra_args):
        os.makedirs(args.log_dir, exist_ok=True)
        self.cmd = [sys.executable, "-u", args.script] + list(args.script_args) + list(extra_args)
        self.procs, self.logs, self.log_paths, self.ranks = [], [], [], []
        for lr in range(len(devices)):
            env = child_env(args, devices, lr, attempt, master_addr, master_port)
            path = os.path.join(args.log_dir, "workerlog.%s" % env["RANK"])
            f = open(path, "a")
            f.write("==== launch attempt %d: %s\n" % (attempt, " ".join(self.cmd)))
            f.flush()
            p = subprocess.Popen(self.cmd, env=env, stdout=f, stderr=subprocess.STDOUT,
                                 start_new_session=True)
            self.procs.append(p)
            self.logs.append(f)
            self.log_paths.append(path)
            self.ranks.append(int(env["RANK"]))

    def poll(self):
        """None while running; (ok, index, exit code) once decided."""
        codes = [p.poll() for p in self.procs]
        for i, c in enumerate(codes):
            if c is not None and c != 0:
                return False, i, c
        if all(c == 0 for c in codes):
            return True, None, 0
        return None

    def idle_seconds(self):
        now = time.time()
        ages = [now - os.path.getmtime(p) for p in self.log_paths]
        return min(ages), ages.index(max(ages))

    def terminate(self, grace=10.0):
        for p in self.procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        deadline = time.time() + grace
        for p in self.procs:
            try:
                p.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                p.wait()
        for f in self.logs:
            f.close()


def _tail(path, n=20):
    try:
        with open(path, "rb") as f:
            f.seek(0, 2)
            f.seek(max(0, f.tell() - 16384))
            return f.read().decode("utf-8", "replace").splitlines()[-n:]
    except OSError:
        return []


def report_failure(pod, idx, code, reason):
    lines = ["-" * 78,
             "Pod failed: %s -- rank %d, exit code %s" % (reason, pod.ranks[idx], code),
             "  command: %s" % " ".join(pod.cmd),
             "  log    : %s" % pod.log_paths[idx],
             "  last lines of the log:"]
    lines += ["    " + l for l in _tail(pod.log_paths[idx])]
    lines.append("-" * 78)
    print("\n".join(lines), flush=True)


def launch(args):
    devices = device_list(args)
    attempt = 0
    while True:
        if args.master:
            addr, port = args.master.rsplit(":", 1)
            port = int(port) + 2 * attempt  # a fresh store per attempt on every node
        else:
            addr, port = "127.0.0.1", _free_port()
        extra = ["-o", "Engine.save_load.ckpt_dir=%s" % args.resume] \
            if attempt > 0 and args.resume else []
        pod = Pod(args, devices, attempt, addr, port, extra)
        print("launch: attempt %d/%d, %d local ranks (world %d), logs in %s"
              % (attempt, args.max_restart, len(devices), len(devices) * args.nnodes,
                 args.log_dir), flush=True)
        status = None
        try:
            while status is None:
                time.sleep(args.poll)
                status = pod.poll()
                if status is None and args.hang_timeout > 0:
                    idle, stalest = pod.idle_seconds()
                    if idle > args.hang_timeout:
                        status = (False, stalest, "hang")
        except KeyboardInterrupt:
            pod.terminate()
            return 130
        ok, idx, code = status
        if ok:
            pod.terminate()
            print("launch: all %d ranks finished" % len(devices), flush=True)
            return 0
        report_failure(pod, idx, code,
                       "no log output for %.0f s (hang)" % args.hang_timeout if code == "hang"
                       else "a rank exited")
        pod.terminate()
        if attempt >= args.max_restart:
            return code if isinstance(code, int) and code > 0 else 1
        attempt += 1
        print("launch: restarting pod (%d/%d), resuming from %s"
              % (attempt, args.max_restart, args.resume or "scratch"), flush=True)


def main(argv=None):
    sys.exit(launch(parse_args(argv)))


if __name__ == "__main__":
    main()
