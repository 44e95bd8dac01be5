#!/usr/bin/env python3
"""Average a rocprofv3 --pmc counter over the dispatches of one kernel (csv output).

  python tools/parse_pmc.py <counter_collection.csv> [kernel-substring]
Prints per-dispatch mean/median of every counter for the matching kernel.  gfx950 note
(MI355X_MICROARCH.md §HBM): FETCH_SIZE reports ~1/2 of the bytes of a wide coalesced stream;
values are in KB (FETCH_SIZE/WRITE_SIZE are defined in kilobytes by rocprofv3).
"""
import csv
import json
import statistics
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "picp_round_kernel"
    vals = defaultdict(list)
    with open(path) as fh:
        for row in csv.DictReader(fh):
            name = row.get("Kernel_Name", "")
            if sub not in name:
                continue
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {}
    for k, v in vals.items():
        out[k] = {"dispatches": len(v), "mean": statistics.fmean(v), "median": statistics.median(v),
                  "min": min(v), "max": max(v)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
