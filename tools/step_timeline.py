"""Where the wall time of one training step goes, from a rocprofv3 kernel
trace (``--kernel-trace --output-format csv``).

For a window of steady steps (same ``--window NAME:A:B`` syntax as
tools/kernel_summary.py) it reports, per step:

* wall span, GPU-busy time (union of kernel intervals) and idle gaps;
* time with two or more kernels in flight (stream overlap) and which kernel
  pairs overlap most (e.g. AdamW under the forward GEMMs);
* phase spans: forward (first kernel -> the cross-entropy statistics kernel),
  backward (cross-entropy backward -> last embedding backward) and the rest;
* register / LDS footprint per kernel (VGPR + AGPR decide whether a
  memory-bound kernel can share a CU with a GEMM).

    python tools/step_timeline.py trace.csv --window adamw_flat:132:330 --steps 3
"""
import argparse
import collections
import csv
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
from kernel_summary import short, _window  # noqa: E402


def union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--window", default=None)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    if a.window:
        rows = _window(rows, a.window)
    ev = [(float(r["Start_Timestamp"]), float(r["End_Timestamp"]), short(r["Kernel_Name"]), r)
          for r in rows]
    ev.sort()
    t0, t1 = ev[0][0], max(e for _, e, _, _ in ev)
    ns = a.steps
    wall = (t1 - t0) / ns / 1e6
    busy_iv = union([[s, e] for s, e, _, _ in ev])
    busy = sum(e - s for s, e in busy_iv) / ns / 1e6
    # overlap: sweep over start/end points
    pts = sorted([(s, 1, i) for i, (s, _, _, _) in enumerate(ev)] +
                 [(e, -1, i) for i, (_, e, _, _) in enumerate(ev)])
    live = set()
    last = pts[0][0]
    over = 0.0
    pair = collections.Counter()
    for t, d, i in pts:
        if len(live) >= 2:
            over += t - last
            names = sorted(set(ev[j][2] for j in live))
            if len(names) >= 2:
                pair[tuple(names[:2])] += t - last
        last = t
        if d > 0:
            live.add(i)
        else:
            live.discard(i)
    over /= ns * 1e6

    def span(first, last_name):
        st = [s for s, _, n, _ in ev if first in n]
        en = [e for _, e, n, _ in ev if last_name in n]
        return st, en

    lines = ["| quantity | ms/step |", "|---|---:|",
             "| wall span | %.2f |" % wall, "| GPU busy (union of kernels) | %.2f |" % busy,
             "| idle gaps | %.2f |" % (wall - busy),
             "| two or more kernels in flight | %.2f |" % over]
    ce_s = sorted(s for s, _, n, _ in ev if "ce_stats" in n)
    ce_b = sorted(s for s, _, n, _ in ev if "ce_bwd" in n)
    if len(ce_s) == ns and len(ce_b) == ns:
        # forward: previous step's last embedding backward (or the window
        # start) -> this step's CE statistics kernel
        emb = sorted(e for _, e, n, _ in ev if "embedding_bwd" in n)
        last_emb = [max(e for e in emb if ce_b[k] < e and (k + 1 >= ns or e < ce_s[k + 1]))
                    for k in range(ns)]
        fw = [ce_s[0] - t0] + [ce_s[k] - last_emb[k - 1] for k in range(1, ns)]
        bw = [last_emb[k] - ce_b[k] for k in range(ns)]
        lines.append("| forward (step start -> CE stats) | %.2f |" % (sum(fw) / ns / 1e6))
        lines.append("| backward (CE bwd -> last embedding bwd) | %.2f |" % (sum(bw) / ns / 1e6))
    lines += ["", "| overlapping pair | ms/step |", "|---|---:|"]
    for (x, y), v in pair.most_common(a.top):
        lines.append("| %s + %s | %.2f |" % (x[:60], y[:60], v / ns / 1e6))
    regs = {}
    for _, _, n, r in ev:
        if n not in regs:
            regs[n] = (r.get("VGPR_Count", "?"), r.get("Accum_VGPR_Count", "?"),
                       r.get("LDS_Block_Size", r.get("Lds_Size", "?")),
                       r.get("Workgroup_Size", "?"))
    tot = collections.Counter()
    for s, e, n, _ in ev:
        tot[n] += e - s
    lines += ["", "| kernel | ms/step | VGPR | AGPR | LDS B | WG |", "|---|---:|---:|---:|---:|---:|"]
    for n, v in tot.most_common(a.top):
        g = regs[n]
        lines.append("| %s | %.2f | %s | %s | %s | %s |" % (n[:70], v / ns / 1e6, *g))
    text = "\n".join(lines)
    print(text)
    if a.md:
        open(a.md, "w").write(text + "\n")


if __name__ == "__main__":
    main()
