"""Summarise a rocprofv3 ``--pmc`` run (the rocpd SQLite database ROCm 7 writes)
per kernel: mean duration, each counter summed over the dispatch (mean over
dispatches), and derived ratios.

    python tools/pmc_summary.py gpurun_out/pmc/pmc_results.db [--filter gemm] [--md]

Derived (when the counters are present):
* clock_GHz  = GRBM_GUI_ACTIVE / 8 XCDs / duration  (MI355X_MICROARCH.md, DVFS)
* wait_any / wait_inst / active = fractions of SQ_WAVE_CYCLES
* lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (if collected)
"""
import argparse
import collections
import sqlite3


def load(path, flt):
    con = sqlite3.connect(path)
    q = ("select dispatch_id, kernel_name, counter_name, value, start, end from counters_collection")
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for did, kn, cn, v, s, e in con.execute(q):
        if flt and flt not in kn:
            continue
        per[(did, kn)][cn] += v
        meta[(did, kn)] = (e - s)
    by_kernel = collections.defaultdict(list)
    for (did, kn), ctr in per.items():
        by_kernel[kn].append((meta[(did, kn)], ctr))
    return by_kernel


def short(name, n=90):
    name = name.replace("(anonymous namespace)::", "")
    return name if len(name) <= n else name[:n] + ".."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--filter", default="")
    ap.add_argument("--md", action="store_true")
    a = ap.parse_args()
    rows = []
    for kn, lst in load(a.db, a.filter).items():
        n = len(lst)
        dur = sum(d for d, _ in lst) / n
        keys = sorted({k for _, c in lst for k in c})
        avg = {k: sum(c.get(k, 0.0) for _, c in lst) / n for k in keys}
        der = {}
        if "GRBM_GUI_ACTIVE" in avg and dur > 0:
            der["clock_GHz"] = avg["GRBM_GUI_ACTIVE"] / 8 / dur
        wc = avg.get("SQ_WAVE_CYCLES")
        if wc:
            for k, nm in (("SQ_WAIT_ANY", "wait_any"), ("SQ_WAIT_INST_ANY", "wait_inst"),
                          ("SQ_ACTIVE_INST_ANY", "active"), ("SQ_WAIT_INST_LDS", "wait_lds")):
                if k in avg:
                    der[nm] = avg[k] / wc
        if "SQ_LDS_BANK_CONFLICT" in avg and avg.get("SQ_LDS_IDX_ACTIVE"):
            der["lds_conflict"] = avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_LDS_IDX_ACTIVE"]
        rows.append((kn, n, dur, avg, der))
    rows.sort(key=lambda r: -r[2] * r[1])
    for kn, n, dur, avg, der in rows:
        if a.md:
            print("| {} | {} | {:.1f} us | {} | {} |".format(
                short(kn), n, dur / 1e3, ", ".join("%s=%.4g" % kv for kv in avg.items()),
                ", ".join("%s=%.3f" % kv for kv in der.items())))
        else:
            print("{}  x{}  {:.1f} us".format(short(kn), n, dur / 1e3))
            for k, v in avg.items():
                print("    {:28s} {:.6g}".format(k, v))
            for k, v in der.items():
                print("    {:28s} {:.3f}".format(k, v))


if __name__ == "__main__":
    main()
