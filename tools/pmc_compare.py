#!/usr/bin/env python3
"""Per-kernel counter summary from tools/pmc_cmd.sh (or pmc_shard.sh / profile.sh) CSVs.

    python tools/pmc_compare.py DIR_OR_PREFIX [kernel-substring ...]

For every kernel whose name contains one of the substrings (default: rt_mega_kernel):
duration, VALU / SALU instructions, lane utilisation (SQ_THREAD_CYCLES_VALU / (ACTIVE_INST_VALU x 64)),
wait share, VALU instructions per SIMD-cycle, HBM-side bytes (2 x FETCH_SIZE + WRITE_SIZE)."""
import csv
import glob
import os
import sys


def load(d):
    files = {}
    for p in ["sq1", "sq2", "sq3", "fetch", "write", "tcc"]:
        for cand in [os.path.join(d, p + ".csv"), d + f"_{p}_1080p256.csv"]:
            if os.path.exists(cand):
                files[p] = cand
    vals = {}
    for p, f in files.items():
        for r in csv.reader(open(f)):
            if len(r) < 6 or r[0] == "Kernel":
                continue
            vals.setdefault(r[0], {})[r[1]] = (float(r[4]), float(r[5]) * 1e-9, int(r[2]))
    return vals


def main():
    d = sys.argv[1]
    keys = sys.argv[2:] or ["rt_mega_kernel"]
    for k, v in load(d).items():
        if not any(s in k for s in keys):
            continue
        g = lambda c: v.get(c, (None, None, None))[0]
        dur = next((x[1] for x in v.values() if x[1]), None)
        out = {"kernel": k[:60], "dispatches": next(iter(v.values()))[2], "ms": round(dur * 1e3, 2) if dur else None}
        if g("SQ_INSTS_VALU"):
            out["valu_G"] = round(g("SQ_INSTS_VALU") / 1e9, 2)
            out["salu_G"] = round(g("SQ_INSTS_SALU") / 1e9, 2)
            out["vmem_rd_G"] = round(g("SQ_INSTS_VMEM_RD") / 1e9, 3)
            out["vmem_wr_G"] = round(g("SQ_INSTS_VMEM_WR") / 1e9, 3)
            out["lds_G"] = round(g("SQ_INSTS_LDS") / 1e9, 3)
        if g("SQ_THREAD_CYCLES_VALU"):
            out["lane_util"] = round(g("SQ_THREAD_CYCLES_VALU") / (g("SQ_ACTIVE_INST_VALU") * 64), 4)
            out["wait_frac"] = round(g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES"), 4)
            if g("GRBM_GUI_ACTIVE") and dur and g("SQ_INSTS_VALU"):
                clk = g("GRBM_GUI_ACTIVE") / 8 / dur
                out["valu_per_simd_cycle"] = round(g("SQ_INSTS_VALU") / (1024 * dur * clk), 4)
        if g("FETCH_SIZE") is not None and g("WRITE_SIZE") is not None:
            out["hbm_TB"] = round((2 * g("FETCH_SIZE") + g("WRITE_SIZE")) * 1024 / 1e12, 3)
            out["write_TB"] = round(g("WRITE_SIZE") * 1024 / 1e12, 3)
        print(out)


if __name__ == "__main__":
    main()
