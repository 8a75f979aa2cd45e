"""Profiler driven by the ``Profiler:`` YAML block (reference §5.1,
``eager_engine.py:197-219,679-738``).

Uses ``torch.profiler`` (Kineto + rocprofiler on ROCm) with the same keys:
``enable``, ``scheduler: [start, end)``, ``profiler_log``, ``record_shapes``,
``profile_memory``, ``detailed``.  Emits a Chrome trace per rank and prints an
op/kernel summary sorted by device time.  For HIP-kernel-level attribution
use ``rocprofv3 --kernel-trace --stats`` (see README "Profiling").
"""
import os

import torch

from .log import logger


class Profiler:
    def __init__(self, cfg):
        start, end = cfg.get("scheduler", [1, 5])
        self.log_dir = cfg.get("profiler_log", "profiler_log")
        self.detailed = cfg.get("detailed", False)
        acts = [torch.profiler.ProfilerActivity.CPU]
        if torch.cuda.is_available():
            acts.append(torch.profiler.ProfilerActivity.CUDA)
        rank = int(os.environ.get("RANK", "0"))
        os.makedirs(self.log_dir, exist_ok=True)

        def _ready(p):
            path = os.path.join(self.log_dir, "trace_rank{}_step{}.json".format(rank, p.step_num))
            p.export_chrome_trace(path)
            logger.info("profiler trace written to %s" % path)

        self.prof = torch.profiler.profile(
            activities=acts,
            schedule=torch.profiler.schedule(wait=max(0, start - 1), warmup=1,
                                             active=max(1, end - start), repeat=1),
            on_trace_ready=_ready,
            record_shapes=cfg.get("record_shapes", self.detailed),
            profile_memory=cfg.get("profile_memory", self.detailed),
            with_stack=False)

    def start(self):
        self.prof.start()

    def step(self):
        self.prof.step()

    def stop(self):
        self.prof.stop()
        try:
            key = "cuda_time_total" if torch.cuda.is_available() else "cpu_time_total"
            table = self.prof.key_averages().table(sort_by=key, row_limit=30)
            logger.info("\n" + table)
        except Exception as e:  # summary is best-effort
            logger.warning("profiler summary failed: %s" % e)
