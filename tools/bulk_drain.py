#!/usr/bin/env python3
"""Bulk / drain split of each render in a `make prof` megaprof log (tools/gpu_steps.sh megaprof=...).

Each render prints a "[mega prof] count=..." summary, the wave end percentiles and one
"[mega tb]" line per 5-ms bucket (waves alive, traversal iterations, lanes busy, ...).  For the
parity renders (count=0):

  bulk   from the start to the first bucket in which fewer waves are alive than at the peak
         (every wave still holds work: the chip's lanes are full);
  drain  from there to the last wave's end (waves leave one by one; their lanes idle).

The hand-off frame has two launches (the plain kernel, then the runahead kernel over the
parked pixels): the wave times are on one clock, so the drain includes the second launch.
Times are those of the diagnostics build (its per-iteration clock reads make it slower); the
fractions are what carry over to the production build.

  python3 tools/bulk_drain.py profiles/r06_megaprof.txt [--labels w1,w2,w4,w8]
"""
import argparse
import re

SUM = re.compile(r"\[mega prof\] count=(\d) waves=(\d+)")
END = re.compile(r"\[mega prof\] wave end ms: p10=([\d.]+) .* max=([\d.]+)")
TB = re.compile(r"\[mega tb\] t=\s*(\d+)-\s*(\d+) ms waves=(\d+) iters/wave=(\d+) trav_lanes=([\d.]+) busy_lanes=([\d.]+)")


def sections(path):
    cur = None
    for line in open(path):
        m = SUM.search(line)
        if m:
            cur = {"count": int(m.group(1)), "waves": int(m.group(2)), "tb": []}
            yield cur
            continue
        if cur is None:
            continue
        m = END.search(line)
        if m:
            cur["p10"], cur["max"] = float(m.group(1)), float(m.group(2))
            continue
        m = TB.search(line)
        if m:
            cur["tb"].append((int(m.group(1)), int(m.group(3)), float(m.group(6))))


def split(sec):
    tb = sec["tb"]
    peak = max(w for _, w, _ in tb)
    first = next((t for t, w, _ in tb if w < peak - 1 and t > 0), tb[-1][0])
    drain = sec["max"] - first
    return {"waves": sec["waves"], "peak_alive": peak, "bulk_ms": first, "drain_ms": round(drain, 1),
            "total_ms": sec["max"], "drain_frac": round(drain / sec["max"], 3), "p10_end": sec["p10"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("log")
    ap.add_argument("--labels", default="", help="names of the parity renders, in log order")
    a = ap.parse_args()
    labels = [x for x in a.labels.split(",") if x]
    secs = list(sections(a.log))
    rows = [split(s) for s in secs if s["count"] == 0 and s["tb"]]
    print("| render | waves (peak alive) | bulk ms | drain ms | total ms | drain share | p10 wave end |")
    print("|---|---|---|---|---|---|---|")
    for i, r in enumerate(rows):
        name = labels[i] if i < len(labels) else str(i)
        print(f"| {name} | {r['waves']} ({r['peak_alive']}) | {r['bulk_ms']} | {r['drain_ms']} | {r['total_ms']} | "
              f"{r['drain_frac']:.3f} | {r['p10_end']} |")


if __name__ == "__main__":
    main()
