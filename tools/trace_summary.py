#!/usr/bin/env python3
"""Per-dispatch durations of the dominant kernel in a rocprofv3 kernel trace
(run_kernel_trace.csv): the mean over every dispatch (what run_kernel_stats.csv reports) and over
the last TIMED dispatches only (the bench's timed steps: the warm-up dispatches before them run
while the clocks ramp -- C4's first launches of a short run take up to 13 % longer).

  python tools/trace_summary.py TRACE_CSV KERNEL_PREFIX TIMED [BENCH_JSON]  -> one JSON line
"""
import csv
import json
import sys


def main():
    path, prefix, timed = sys.argv[1], sys.argv[2], int(sys.argv[3])
    rows = [r for r in csv.DictReader(open(path)) if r["Kernel_Name"].startswith(prefix)]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    last = us[-timed:] if timed > 0 else us
    out = {"kernel": rows[0]["Kernel_Name"][:120] if rows else None, "dispatches": len(us),
           "mean_us_all": round(sum(us) / max(len(us), 1), 2),
           "mean_us_timed": round(sum(last) / max(len(last), 1), 2), "timed_dispatches": len(last),
           "min_us": round(min(us), 2) if us else None, "max_us": round(max(us), 2) if us else None}
    if len(sys.argv) > 4:
        line = [l for l in open(sys.argv[4]).read().splitlines() if l.startswith("{")][-1]
        out["traced_run_ms_per_step"] = json.loads(line)["ms_per_step"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
