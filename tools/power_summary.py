"""Summarise `amd-smi metric -p -c --json` samples (concatenated JSON
documents, one per sample): socket power and the mean / min / max gfx clock
over the XCDs.  Used by scripts/gpu_r6_al.sh (power and clocks during a step).

    python tools/power_summary.py [--min-power W] samples.jsonl [more.jsonl ...]

``--min-power`` keeps only samples at or above W (drops start-up / idle).
"""
import json
import statistics
import sys


def docs(path):
    txt = open(path).read()
    dec, i, out = json.JSONDecoder(), 0, []
    while i < len(txt):
        while i < len(txt) and txt[i].isspace():
            i += 1
        if i >= len(txt):
            break
        o, i = dec.raw_decode(txt, i)
        out.append(o)
    return out


def main():
    args = sys.argv[1:]
    floor = 0
    if args and args[0] == "--min-power":
        floor, args = float(args[1]), args[2:]
    for path in args:
        pw, clk = [], []
        for d in docs(path):
            g = d["gpu_data"][0] if isinstance(d, dict) and "gpu_data" in d else d[0]
            if g["power"]["socket_power"]["value"] < floor:
                continue
            pw.append(g["power"]["socket_power"]["value"])
            c = [v["clk"]["value"] for k, v in g["clock"].items()
                 if k.startswith("gfx_") and isinstance(v, dict) and isinstance(v["clk"]["value"], (int, float))]
            if c:
                clk.append(statistics.mean(c))
        print("%s: %d samples, socket power mean %.0f W (min %d, max %d), gfx clock mean %.0f MHz "
              "(min %.0f, max %.0f)" % (path, len(pw), statistics.mean(pw), min(pw), max(pw),
                                        statistics.mean(clk), min(clk), max(clk)))


if __name__ == "__main__":
    main()
