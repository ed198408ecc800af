"""Launch interval of a kernel from a rocprofv3 --kernel-trace CSV: with two launches in flight
(kNN pipeline depth 3) a launch's own duration overlaps its neighbour's, so the kernel's
sustained rate is set by the interval between consecutive launch ends, not by the duration.
usage: python tools/trace_interval.py <kernel_trace.csv> <kernel-name-substring> [skip]"""
import csv
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if name in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    rows = rows[skip:]
    if len(rows) < 3:
        raise SystemExit("too few launches")
    # longest run of back-to-back launches (gaps < 50 us): the steady-state timed region
    runs, cur = [], [rows[0]]
    for a, b in zip(rows, rows[1:]):
        if b[0] - max(e for _, e in cur) < 50_000:
            cur.append(b)
        else:
            runs.append(cur)
            cur = [b]
    runs.append(cur)
    run = max(runs, key=len)
    ends = sorted(e for _, e in run)
    durs = [e - s for s, e in run]
    interval = (ends[-1] - ends[0]) / (len(ends) - 1)
    overlap = sum(durs) / (ends[-1] - run[0][0])
    print(f"{name}: {len(run)} back-to-back launches, mean duration {sum(durs) / len(durs) / 1e3:.2f} us, "
          f"mean end-to-end interval {interval / 1e3:.2f} us, mean launches in flight {overlap:.2f}")


if __name__ == "__main__":
    main()
