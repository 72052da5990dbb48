#!/usr/bin/env python3
"""Summary of tools/fetch_calib.sh: per load shape, FETCH_SIZE bytes per launch against the
bytes the shape asks for and the 128-B lines it touches (every line by one access only, on a
2 GiB buffer: each is a miss to memory).

    python tools/fetch_calib_summary.py run.json fetch.csv tcc.csv out.csv

Columns: fetch_bytes (FETCH_SIZE KiB x 1024, mean per dispatch), fetch_per_line, and
`hbm_per_fetch` = lines x 128 / fetch_bytes: the factor that turns counted FETCH_SIZE bytes of
that shape into the bytes of the 128-B lines filled (the guide's streaming case reads 2).
bench.py weights the shapes' factors by the render kernel's algorithmic byte shares."""
import csv
import json
import sys


def pmc(path):
    d = {}
    for row in csv.DictReader(open(path)):
        d[(row["Kernel"].split("(")[0].replace("void ", ""), row["Counter"])] = float(row["MeanPerDispatch"])
    return d


def main():
    allrows = json.load(open(sys.argv[1]))
    run = [r for r in allrows if r["rep"] == 1 and "requested_bytes" in r]
    f, t = pmc(sys.argv[2]), pmc(sys.argv[3])
    with open(sys.argv[4], "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["kernel", "requested_bytes", "lines_128b", "ms", "fetch_bytes", "fetch_per_line", "fetch_per_requested",
                    "hbm_per_fetch", "tcc_ea_rdreq", "tcc_ea_rdreq_32b", "tcc_hit", "tcc_miss"])
        for r in run:
            k = r["kernel"]
            fb = f.get((k, "FETCH_SIZE"), 0.0) * 1024.0
            w.writerow([k, int(r["requested_bytes"]), int(r["lines_128b"]), r["ms"], int(fb),
                        round(fb / r["lines_128b"], 3) if fb else None,
                        round(fb / r["requested_bytes"], 4) if fb else None,
                        round(r["lines_128b"] * 128.0 / fb, 4) if fb else None,
                        t.get((k, "TCC_EA0_RDREQ_sum")), t.get((k, "TCC_EA0_RDREQ_32B_sum")),
                        t.get((k, "TCC_HIT_sum")), t.get((k, "TCC_MISS_sum"))])
    # the L2-resident gather rates (no FETCH_SIZE case): the fastest of the repetitions
    best = {}
    for r in allrows:
        if "wave_load_insts" in r and (r["kernel"] not in best or r["ms"] < best[r["kernel"]]["ms"]):
            best[r["kernel"]] = r
    with open(sys.argv[4].replace(".csv", "_gather.csv"), "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["kernel", "wave_load_insts", "lines_per_inst", "ms", "insts_per_cu_cycle", "line_accesses_per_cu_cycle",
                    "bytes_per_cu_cycle"])
        for k, r in best.items():
            w.writerow([k, int(r["wave_load_insts"]), int(r["lines_per_inst"]), r["ms"], r["insts_per_cu_cycle"],
                        r["line_accesses_per_cu_cycle"], r["bytes_per_cu_cycle"]])


if __name__ == "__main__":
    main()
