"""Kernel durations and start-to-start gaps from a rocprofv3 kernel-trace CSV.

    python tools/kgap.py <kernel_trace.csv> [name-substring]

Prints, per kernel name (or only the one matching the substring): launches, mean /
median duration, and the median interval from one launch's start to the next one's
(back-to-back launches of the same stream: interval - duration = the dispatch gap).
"""
import csv
import statistics
import sys


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("KernelName") or ""
            if sub and sub not in name:
                continue
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    by = {}
    for i, (s, e, n) in enumerate(rows):
        by.setdefault(n, []).append((s, e))
    for n, v in sorted(by.items(), key=lambda kv: -len(kv[1])):
        d = [e - s for s, e in v]
        iv = [v[i + 1][0] - v[i][0] for i in range(len(v) - 1)]
        print("%-90s n=%6d dur mean %8.2f us med %8.2f us | start-to-start med %8.2f us" % (
            n[:90], len(v), statistics.mean(d) / 1e3, statistics.median(d) / 1e3,
            (statistics.median(iv) / 1e3) if iv else float("nan")))


if __name__ == "__main__":
    main()
