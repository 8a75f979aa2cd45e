"""Summarise a rocprofv3 kernel trace (``*_kernel_trace.csv`` or
``*_kernel_stats.csv``, or the rocpd ``*_results.db`` that ROCm 7 writes by
default) into a short per-kernel table: total ms per step, calls, share -- with template noise stripped from the names.

    python tools/kernel_summary.py trace.csv [--steps N] [--top 30] [--md out.md]
        [--window adamw_flat:2:6]

``--window NAME:A:B`` (kernel traces only) keeps the kernels that start after
the A-th and up to the B-th completion of a kernel whose name contains NAME
-- e.g. the optimizer kernel closes every step, so this cuts warm-up and
start-up kernels out of a multi-step trace.
"""
import argparse
import collections
import csv
import re


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*$", "", n)                 # drop the argument list
    n = re.sub(r"^void\s+", "", n)
    if n.startswith("Cijk_") or n.startswith("Custom_Cijk"):
        mt = re.search(r"MT\d+x\d+x\d+", n)
        return "hipBLASLt GEMM %s %s" % (n.split("_")[1] if not n.startswith("Custom") else
                                         n.split("_")[2], mt.group(0) if mt else "")
    n = re.sub(r"<.*>", lambda m: "<" + m.group(0)[1:40] + ("..>" if len(m.group(0)) > 41 else ""), n)
    return n[:110]


def _window(rows, spec):
    name, a, b = spec.rsplit(":", 2)
    a, b = int(a), int(b)
    rows = sorted(rows, key=lambda r: float(r["Start_Timestamp"]))
    ends = sorted(float(r["End_Timestamp"]) for r in rows if name in r["Kernel_Name"])
    if len(ends) < b:
        raise SystemExit("only %d '%s' kernels in the trace" % (len(ends), name))
    lo = ends[a - 1] if a > 0 else float("-inf")
    hi = ends[b - 1]
    return [r for r in rows if lo < float(r["Start_Timestamp"]) <= hi]


def _rows_from_rocpd(path):
    """ROCm 7 rocprofv3 writes a rocpd SQLite database (``*_results.db``) by
    default; its ``kernels`` view has one row per dispatch."""
    import sqlite3
    con = sqlite3.connect(path)
    try:
        return [{"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e}
                for n, s, e in con.execute("select name, start, end from kernels order by start")]
    finally:
        con.close()


def load(path, window=None):
    if path.endswith(".db"):
        rows = _rows_from_rocpd(path)
    else:
        rows = list(csv.DictReader(open(path)))
    if window:
        rows = _window(rows, window)
    agg = collections.defaultdict(lambda: [0.0, 0])
    if rows and "TotalDurationNs" in rows[0]:
        for r in rows:
            a = agg[short(r["Name"])]
            a[0] += float(r["TotalDurationNs"])
            a[1] += int(r["Calls"])
    else:
        for r in rows:
            a = agg[short(r["Kernel_Name"])]
            a[0] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
            a[1] += 1
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=float, default=1.0, help="divide totals by this many steps")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--md", default=None)
    ap.add_argument("--window", default=None)
    a = ap.parse_args()
    agg = load(a.csv, a.window)
    total = sum(v[0] for v in agg.values())
    lines = ["| kernel | ms/step | calls/step | share |", "|---|---:|---:|---:|"]
    for k, (ns, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:a.top]:
        lines.append("| %s | %.2f | %.0f | %.1f%% |" % (k, ns / 1e6 / a.steps, c / a.steps,
                                                     100.0 * ns / total))
    lines.append("| **total GPU kernel time** | **%.2f** | | |" % (total / 1e6 / a.steps))
    text = "\n".join(lines)
    print(text)
    if a.md:
        with open(a.md, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
