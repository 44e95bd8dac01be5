#!/bin/bash
# Round 6, call 20: the bucketed world match simulated (tools/r06/match_bucket_sim.py) under the
# kernel tracer: sign cells of 2 / 3 / 4 components, groups of 128 / 64 queries.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t20}
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/r06/match_8e.py --save $OUT/maps.npz > $OUT/save.log 2>&1 || { echo "save failed"; tail $OUT/save.log; exit 1; }
: > $OUT/sim.txt
for cfg in "2 128" "3 128" "4 128" "4 64" "5 64"; do
  n=$(echo $cfg | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof_$n -o run --output-format csv -- python3 -u tools/r06/match_bucket_sim.py $OUT/maps.npz $cfg > $OUT/sim_$n.log 2>&1 || { echo "sim $cfg failed"; tail $OUT/sim_$n.log; exit 1; }
  grep -v "^W2026\|rocprofv3\|^$" $OUT/sim_$n.log | grep -v "HSA\|simple_timer\|tool.cpp" | tee -a $OUT/sim.txt
  python3 - $(find $OUT/prof_$n -name '*kernel_trace.csv' | head -1) <<'PY' | tee -a $OUT/sim.txt
import csv, sys
rows = sorted([r for r in csv.DictReader(open(sys.argv[1])) if "picp_match_mfma" in r["Kernel_Name"] or "merge" in r["Kernel_Name"]], key=lambda r: int(r["Start_Timestamp"]))
d = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
mf = [r for r in rows if "mfma" in r["Kernel_Name"]]
mg = [r for r in rows if "merge" in r["Kernel_Name"]]
# launches: ref, 3 brute, 3 bucketed (each: mfma + merge when split)
print("  brute  mfma %s us" % [round(d(r), 1) for r in mf[1:4]], "grid", mf[1]["Grid_Size_X"])
print("  bucket mfma %s us" % [round(d(r), 1) for r in mf[4:7]], "grid", mf[4]["Grid_Size_X"])
print("  merges %s us" % [round(d(r), 1) for r in mg[-6:]])
PY
done
rm -f $OUT/maps.npz
