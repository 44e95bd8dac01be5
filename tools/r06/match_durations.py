#!/usr/bin/env python3
"""The last 12 matcher dispatches of a kernel trace (tools/r06/match_8e.py: 4 map prefixes x 3
repetitions): mean duration per prefix of the MFMA kernel and the merge."""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1]))
        if "picp_match_mfma" in r["Kernel_Name"] or "picp_match_merge" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
mf = [r for r in rows if "mfma" in r["Kernel_Name"]][-12:]
mg = [r for r in rows if "merge" in r["Kernel_Name"]][-12:]
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tag = sys.argv[2] if len(sys.argv) > 2 else ""
for k, frac in enumerate((0.25, 0.5, 0.8, 1.0)):
    a = [dur(r) for r in mf[3 * k:3 * k + 3]]
    b = [dur(r) for r in mg[3 * k:3 * k + 3]]
    print("%s map x%.2f: mfma %.1f us (grid %s, VGPR %s), merge %.1f us" % (
        tag, frac, sum(a) / len(a), mf[3 * k]["Grid_Size_X"], mf[3 * k]["VGPR_Count"], sum(b) / max(len(b), 1)))
