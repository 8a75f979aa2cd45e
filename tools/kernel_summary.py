"""Summarise a rocprofv3 kernel trace (``*_kernel_trace.csv`` or
``*_kernel_stats.csv``) into a short per-kernel table: total ms per step,
calls, share -- with template noise stripped from the names.

    python tools/kernel_summary.py trace.csv [--steps N] [--top 30] [--md out.md]
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


def load(path):
    rows = list(csv.DictReader(open(path)))
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
    a = ap.parse_args()
    agg = load(a.csv)
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
