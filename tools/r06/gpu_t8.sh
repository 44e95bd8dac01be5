#!/bin/bash
# Round 6, call 8: the 8e world match in isolation (tools/r06/match_8e.py): candidate counters
# (stamps library) and the kernel trace of 4-problem launches against map prefixes.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t8}
mkdir -p $OUT
# (stamps counters: profiles/r06/t8/stamps.log)

timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 -u tools/r06/match_8e.py > $OUT/trace.log 2>&1 || { echo "trace run failed"; tail $OUT/trace.log; exit 1; }
f=$(find $OUT/prof -name '*kernel_trace.csv' | head -1)
python - "$f" <<'PY' | tee $OUT/match_durations.txt
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "picp_match_mfma" in r["Kernel_Name"] or "merge" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the VO run's launches come first; the script's own 4-problem launches are the last ones
for r in rows[-40:]:
    print(r["Kernel_Name"][:60], r["Grid_Size"], r["Workgroup_Size"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, "us")
PY
