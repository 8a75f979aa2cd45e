"""Run a list of shell commands (one per line of a text file) over N workers:
batch download / unpack / preprocessing.

    python -m fleetx_amd.tools.multiprocess_tool --num_proc 10 \\
        --shell_cmd_list_filename batch_cmd.txt

Parity: reference ``ppfleetx/tools/multiprocess_tool.py`` (D13).  Commands are
handed out dynamically (a slow command does not stall a fixed partition as the
reference's static split did), every failure is reported with its exit code,
and the tool exits non-zero if any command failed.  Blank lines and ``#``
comments are skipped.
"""
import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import time
import warnings


def read_command(filename):
    with open(filename, "r") as f:
        return [l.strip() for l in f if l.strip() and not l.strip().startswith("#")]


def _run(cmd):
    return cmd, subprocess.run(cmd, shell=True).returncode


def parallel_process(cmd_list, nproc=20):
    """Returns the list of (command, exit code) that failed."""
    if nproc > (os.cpu_count() or 1):
        warnings.warn("the number of processes exceeds the number of CPU cores")
    failed = []
    # each command is its own process already: threads only wait on them
    with cf.ThreadPoolExecutor(max_workers=max(1, nproc)) as ex:
        for cmd, rc in ex.map(_run, cmd_list):
            if rc != 0:
                print("execute command: {} failed (exit code {})".format(cmd, rc), flush=True)
                failed.append((cmd, rc))
    return failed


def main(argv=None):
    ap = argparse.ArgumentParser(description="multi-process batch processing tool")
    ap.add_argument("--num_proc", type=int, default=20)
    ap.add_argument("--shell_cmd_list_filename", required=True,
                    help="a text file with one shell command per line")
    args = ap.parse_args(argv)
    t0 = time.time()
    failed = parallel_process(read_command(args.shell_cmd_list_filename), args.num_proc)
    print("Cost time: {:.2f}".format(time.time() - t0))
    return 1 if failed else 0


if __name__ == "__main__":
    sys.exit(main())
