"""Summarise a tools/gpu_pmc.sh output directory (gpurun_out/pmc/<TAG>) and optionally a
rocprofv3 --stats database into one JSON for profiles/: per kernel, the median of every
counter over its dispatches, plus derived figures (HBM bytes with the gfx950 FETCH_SIZE x2
correction, LDS bank-conflict share, VALU issue share, wait share).

usage: pmc_table.py OUT.json PMC_DIR [STATS_DB] [--note TEXT]
"""
import collections
import csv
import glob
import json
import os
import sqlite3
import statistics
import sys


def pmc(dirpath):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(dirpath, "*", "*_counter_collection.csv")):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                per[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {}
    for k, cs in per.items():
        m = {c: statistics.median(v) for c, v in cs.items()}
        d = {"dispatches": max(len(v) for v in cs.values()), "median": m}
        if "FETCH_SIZE" in m:
            d["hbm_read_bytes_corrected"] = 2.0 * 1024.0 * m["FETCH_SIZE"]  # gfx950: half of wide reads
        if "WRITE_SIZE" in m:
            d["hbm_write_bytes"] = 1024.0 * m["WRITE_SIZE"]
        if m.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_bank_conflict_share"] = m.get("SQ_LDS_BANK_CONFLICT", 0.0) / m["SQ_LDS_IDX_ACTIVE"]
        if m.get("GRBM_GUI_ACTIVE"):
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs: per-XCD cycles = /8; 256 CUs x 4 SIMDs
            cyc = m["GRBM_GUI_ACTIVE"] / 8.0
            d["gpu_cycles"] = cyc
            if "SQ_INSTS_VALU" in m:
                d["valu_issue_share"] = 4.0 * m["SQ_INSTS_VALU"] / (1024.0 * cyc)
        if m.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in m:
            d["wait_any_per_wave_cycle"] = m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]
        if m.get("SQ_WAVE_CYCLES") and m.get("GRBM_GUI_ACTIVE"):
            # measured occupancy: SQ_WAVE_CYCLES (quad-cycles, summed over every wave of the
            # dispatch) x 4 = wave-cycles; over the dispatch's busy cycles per XCD (GRBM_GUI_ACTIVE / 8)
            # and the 256 CUs x 4 SIMDs -> mean resident waves per SIMD over the kernel's lifetime
            # (ramp-up and tail included, so below the launch's steady-state residency)
            d["mean_waves_per_simd"] = 4.0 * m["SQ_WAVE_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8.0 * 1024.0)
            d["occupancy_basis"] = "4 * SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE / 8 * 256 CUs * 4 SIMDs)"
        out[k] = d
    return out


def stats(db):
    c = sqlite3.connect(db)
    return [{"kernel": r[0], "calls": r[1], "total_us": round(r[2], 1), "avg_us": round(r[3], 2), "pct": round(r[4], 2)}
            for r in c.execute("select * from top_kernels")]


def main():
    args = sys.argv[1:]
    note = ""
    if "--note" in args:
        i = args.index("--note")
        note = args[i + 1]
        del args[i:i + 2]
    out, d = args[0], args[1]
    res = {"note": note, "pmc": pmc(d)}
    if len(args) > 2:
        res["kernel_stats"] = stats(args[2])
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
