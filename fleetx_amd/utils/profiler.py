"""Profiler driven by the ``Profiler:`` YAML block (reference §5.1,
``eager_engine.py:197-219,679-738``; views as in
``projects/gpt/docs/hybrid_profiler.md:93-181``).

Uses ``torch.profiler`` (Kineto + rocprofiler on ROCm) with the same keys:
``enable``, ``scheduler: [start, end)``, ``profiler_log``, ``record_shapes``,
``profile_memory``, ``detailed`` and ``summary.{overview, model, kernel, op,
dist, mem, memcpy}``.  Emits a Chrome trace per rank plus text views rebuilt
from the recorded events:

* Overview -- profiled span, device busy time (union of kernel intervals);
* Model    -- the engine's phases (Dataloader / Forward / Backward / GradSync /
  Optimization), CPU and device time, from :func:`phase` ranges;
* Kernel   -- device kernels grouped by name (our HIP kernels by symbol);
* Operator -- framework ops sorted by device time;
* Distributed -- RCCL kernel time vs compute kernel time and their overlap;
* Memory / Memcpy -- allocator usage per op, memcpy events.

:func:`phase` also emits roctx ranges (``FLEETX_ROCTX=1`` or ``roctx: True``)
so ``rocprofv3 --marker-trace`` attributes kernels to the same phases.
"""
import contextlib
import os

import torch

from .log import logger

_PHASES = {"profiling": False, "roctx": os.environ.get("FLEETX_ROCTX", "0") == "1",
           "marks": []}

PHASE_PREFIX = "FX::"
PHASES = ("Dataloader", "Forward", "Backward", "GradSync", "Optimization")


@contextlib.contextmanager
def phase(name):
    """Label a training-step phase for the profiler views / roctx."""
    on_prof, on_tx = _PHASES["profiling"], _PHASES["roctx"]
    if not (on_prof or on_tx):
        yield
        return
    if on_tx and torch.cuda.is_available():
        torch.cuda.nvtx.range_push(name)  # roctx on ROCm builds
    ev = None
    if on_prof and torch.cuda.is_available():
        # device-side span of the phase on the compute stream (autograd's
        # backward kernels are launched from another thread, so the
        # profiler's GPU annotations cannot attribute them)
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
    try:
        if on_prof:
            with torch.profiler.record_function(PHASE_PREFIX + name):
                yield
        else:
            yield
    finally:
        if ev is not None:
            ev[1].record()
            _PHASES["marks"].append((name, ev[0], ev[1]))
        if on_tx and torch.cuda.is_available():
            torch.cuda.nvtx.range_pop()


def _dev_time(e):
    for a in ("device_time_total", "cuda_time_total"):
        v = getattr(e, a, None)
        if v is not None:
            return float(v)
    return 0.0


def _self_dev_time(e):
    for a in ("self_device_time_total", "self_cuda_time_total"):
        v = getattr(e, a, None)
        if v is not None:
            return float(v)
    return 0.0


def _is_kernel(e):
    dt = getattr(e, "device_type", None)
    return dt is not None and dt == torch.autograd.DeviceType.CUDA and \
        not e.name.startswith(PHASE_PREFIX) and not e.name.startswith("ProfilerStep")


def _union(intervals):
    tot, cur_s, cur_e = 0.0, None, None
    for s, e in sorted(intervals):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def _merge(intervals):
    out = []
    for s, e in sorted(intervals):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def _overlap(a, b):
    """Length of the intersection of two interval sets."""
    a, b = _merge(a), _merge(b)
    i = j = 0
    tot = 0.0
    while i < len(a) and j < len(b):
        lo, hi = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if hi > lo:
            tot += hi - lo
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def _table(title, header, rows):
    cols = [header] + [[str(c) for c in r] for r in rows]
    w = [max(len(r[i]) for r in cols) for i in range(len(header))]
    line = "-" * (sum(w) + 3 * (len(w) - 1))
    out = ["", title, line, " | ".join(h.ljust(w[i]) for i, h in enumerate(header)), line]
    for r in cols[1:]:
        out.append(" | ".join(c.ljust(w[i]) if i == 0 else c.rjust(w[i]) for i, c in enumerate(r)))
    out.append(line)
    return "\n".join(out)


def _short(name):
    n = name.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    i = n.find("(")
    return n[:i] if i > 0 else n


def _is_comm(name):
    n = name.lower()
    return "nccl" in n or "rccl" in n or "allreduce" in n or "all_reduce" in n or \
        "reducescatter" in n or "allgather" in n


def summarize(events, views=None, steps=1, memory=False, top=25, device_phase_ms=None):
    """Text views over a ``torch.profiler`` event list (times in ms);
    ``device_phase_ms``: {phase: device-stream span} from :func:`phase` marks."""
    views = dict(views or {})
    want = {k: views.get(k, True) for k in ("overview", "model", "kernel", "op", "dist",
                                            "memcpy")}
    want["mem"] = views.get("mem", memory)
    steps = max(1, int(steps))
    kernels = [e for e in events if _is_kernel(e)]
    host = [e for e in events if not _is_kernel(e)]
    out = []
    span = 0.0
    if host:
        span = (max(e.time_range.end for e in host) - min(e.time_range.start for e in host)) / 1e3
    busy = _union([(e.time_range.start, e.time_range.end) for e in kernels]) / 1e3
    if want["overview"]:
        rows = [["profiled steps", steps], ["host span (ms)", "%.2f" % span],
                ["device busy (ms)", "%.2f" % busy],
                ["device utilisation", "%.1f%%" % (100.0 * busy / span if span else 0.0)],
                ["kernels launched", len(kernels)]]
        out.append(_table("Overview Summary", ["item", "value"], rows))
    if want["model"]:
        agg = {}
        for e in host:
            if e.name.startswith(PHASE_PREFIX):
                k = e.name[len(PHASE_PREFIX):]
                a = agg.setdefault(k, [0, 0.0, 0.0])
                a[0] += 1
                a[1] += e.cpu_time_total / 1e3
                a[2] += _dev_time(e) / 1e3
        for k, ms in (device_phase_ms or {}).items():
            agg.setdefault(k, [0, 0.0, 0.0])[2] = ms
        rows = []
        order = [p for p in PHASES if p in agg] + sorted(k for k in agg if k not in PHASES)
        for k in order:
            c, cpu, dev = agg[k]
            rows.append([k, c, "%.2f" % (cpu / steps), "%.2f" % (dev / steps)])
        out.append(_table("Model Summary (per step)", ["phase", "calls", "CPU ms", "device ms"],
                          rows))
    if want["kernel"]:
        agg = {}
        for e in kernels:
            a = agg.setdefault(_short(e.name), [0, 0.0])
            a[0] += 1
            a[1] += (e.time_range.end - e.time_range.start) / 1e3
        tot = sum(v[1] for v in agg.values()) or 1.0
        rows = [[n[:80], c, "%.3f" % (t / steps), "%.1f%%" % (100.0 * t / tot)]
                for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]]
        out.append(_table("Kernel Summary", ["kernel", "calls", "ms/step", "share"], rows))
    if want["op"]:
        agg = {}
        for e in host:
            if e.name.startswith(PHASE_PREFIX) or e.name.startswith("ProfilerStep"):
                continue
            a = agg.setdefault(e.name, [0, 0.0, 0.0])
            a[0] += 1
            a[1] += e.self_cpu_time_total / 1e3
            a[2] += _self_dev_time(e) / 1e3
        rows = [[n[:60], c, "%.3f" % (cpu / steps), "%.3f" % (dev / steps)]
                for n, (c, cpu, dev) in sorted(agg.items(),
                                               key=lambda kv: (-kv[1][2], -kv[1][1]))[:top]]
        out.append(_table("Operator Summary", ["op", "calls", "self CPU ms/step",
                                               "self device ms/step"], rows))
    if want["dist"]:
        comm = [(e.time_range.start, e.time_range.end) for e in kernels if _is_comm(e.name)]
        comp = [(e.time_range.start, e.time_range.end) for e in kernels if not _is_comm(e.name)]
        c, k = _union(comm) / 1e3, _union(comp) / 1e3
        ov = _overlap(comm, comp) / 1e3
        rows = [["communication", "%.3f" % (c / steps)], ["computation", "%.3f" % (k / steps)],
                ["overlap", "%.3f" % (ov / steps)],
                ["exposed communication", "%.3f" % ((c - ov) / steps)]]
        out.append(_table("Distributed Summary (ms/step)", ["item", "time"], rows))
    if want["memcpy"]:
        agg = {}
        for e in events:
            if "memcpy" in e.name.lower() or "copybuffer" in e.name.lower():
                a = agg.setdefault(e.name, [0, 0.0])
                a[0] += 1
                a[1] += (e.time_range.end - e.time_range.start) / 1e3
        rows = [[n[:60], c, "%.3f" % (t / steps)] for n, (c, t) in
                sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]]
        out.append(_table("Memcpy Summary", ["event", "calls", "ms/step"], rows))
    if want["mem"]:
        agg = {}
        for e in host:
            m = getattr(e, "self_device_memory_usage", None)
            if m is None:
                m = getattr(e, "self_cuda_memory_usage", 0)
            cm = getattr(e, "self_cpu_memory_usage", 0) or 0
            if not m and not cm:
                continue
            a = agg.setdefault(e.name, [0, 0, 0])
            a[0] += 1
            a[1] += m or 0
            a[2] += cm
        rows = [[n[:60], c, "%.1f" % (d / 2 ** 20), "%.1f" % (h / 2 ** 20)]
                for n, (c, d, h) in sorted(agg.items(), key=lambda kv: -abs(kv[1][1]))[:top]]
        out.append(_table("Memory Summary", ["op", "calls", "device MiB", "host MiB"], rows))
    return "\n".join(out)


class Profiler:
    def __init__(self, cfg):
        start, end = cfg.get("scheduler", [1, 5])
        self.start_step, self.end_step = int(start), int(end)
        self.log_dir = cfg.get("profiler_log", "profiler_log")
        self.detailed = cfg.get("detailed", False)
        self.views = dict(cfg.get("summary", {}) or {})
        self.memory = cfg.get("profile_memory", self.detailed)
        if cfg.get("roctx", False):
            _PHASES["roctx"] = True
        acts = [torch.profiler.ProfilerActivity.CPU]
        if torch.cuda.is_available():
            acts.append(torch.profiler.ProfilerActivity.CUDA)
        self.rank = int(os.environ.get("RANK", "0"))
        os.makedirs(self.log_dir, exist_ok=True)
        self.text = None

        def _ready(p):
            path = os.path.join(self.log_dir, "trace_rank{}_step{}.json".format(self.rank,
                                                                                p.step_num))
            p.export_chrome_trace(path)
            logger.info("profiler trace written to %s" % path)

        self.prof = torch.profiler.profile(
            activities=acts,
            schedule=torch.profiler.schedule(wait=max(0, self.start_step - 1), warmup=1,
                                             active=max(1, self.end_step - self.start_step),
                                             repeat=1),
            on_trace_ready=_ready,
            record_shapes=cfg.get("record_shapes", self.detailed),
            profile_memory=self.memory,
            with_stack=False)

    def start(self):
        self._step = 0
        self.prof.start()
        self._arm()

    def _arm(self):
        # phases are recorded only inside the active [start, end) window
        active = self.start_step <= self._step < self.end_step
        _PHASES["profiling"] = active
        if not active:
            return
        if self._step == self.start_step:
            _PHASES["marks"] = []

    def step(self):
        self.prof.step()
        self._step += 1
        self._arm()

    def _device_phase_ms(self):
        if not torch.cuda.is_available():
            return {}
        torch.cuda.synchronize()
        out = {}
        for name, a, b in _PHASES["marks"]:
            out[name] = out.get(name, 0.0) + a.elapsed_time(b)
        _PHASES["marks"] = []
        return out

    def stop(self):
        self.prof.stop()
        _PHASES["profiling"] = False
        try:
            self.text = summarize(self.prof.events(), self.views,
                                  steps=max(1, self.end_step - self.start_step),
                                  memory=self.memory, device_phase_ms=self._device_phase_ms())
            logger.info(self.text)
            with open(os.path.join(self.log_dir, "summary_rank%d.txt" % self.rank), "w") as f:
                f.write(self.text + "\n")
        except Exception as e:  # summary is best-effort
            logger.warning("profiler summary failed: %s" % e)
