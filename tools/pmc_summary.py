"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes for one kernel into the JSON that
bench.py reads as roofline.traffic (profiles/rNN_<name>_pmc.json).

usage: pmc_summary.py OUT.json KERNEL_REGEX POINTS_PER_LAUNCH FETCH.csv WRITE.csv [note]
Only dispatches whose corrected FETCH_SIZE is within 2x of the algorithmic bytes are kept (a run
may also launch the kernel on other sizes, e.g. a verification pass).
FETCH_SIZE is doubled (MI355X_MICROARCH.md: gfx950 reports half of wide streaming reads)."""
import csv
import json
import re
import statistics
import sys


def per_launch(path, counter, rx, keep=None):
    vals, name = [], None
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter and re.search(rx, row["Kernel_Name"]):
                if keep is not None and row["Dispatch_Id"] not in keep:
                    continue
                vals.append(float(row["Counter_Value"]))
                name = row["Kernel_Name"]
    return name, vals


def sized_dispatches(path, rx, algo_bytes):
    keep = set()
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == "FETCH_SIZE" and re.search(rx, row["Kernel_Name"]):
                b = 2048.0 * float(row["Counter_Value"])
                if 0.5 * algo_bytes <= b <= 2.0 * algo_bytes:
                    keep.add(row["Dispatch_Id"])
    return keep


def main():
    out, rx, pts, fetch, write = sys.argv[1:6]
    note = sys.argv[6] if len(sys.argv) > 6 else ""
    res = {}
    keep = sized_dispatches(fetch, rx, 16.0 * int(pts))
    for counter, path in (("FETCH_SIZE", fetch), ("WRITE_SIZE", write)):
        name, v = per_launch(path, counter, rx, keep if counter == "FETCH_SIZE" else None)
        if not v:
            raise SystemExit(f"no {counter} rows for /{rx}/ in {path}")
        med = statistics.median(v)
        res[counter] = {"kernel": name, "dispatches": len(v), "median_KB": med, "min_KB": min(v), "max_KB": max(v)}
        if counter == "FETCH_SIZE":
            res[counter]["corrected_bytes_per_launch"] = 2.0 * 1024.0 * med
    res["points_per_launch"] = int(pts)
    res["algorithmic_bytes_per_launch"] = 16 * int(pts)
    res["traffic_bytes_per_launch"] = res["FETCH_SIZE"]["corrected_bytes_per_launch"] + 1024.0 * res["WRITE_SIZE"]["median_KB"]
    res["note"] = note
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
