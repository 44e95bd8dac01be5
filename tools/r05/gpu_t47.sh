#!/bin/bash
# Round 5, call 47: where the folded matcher's tile loop waits -- diagnostic timing builds (wrong
# results by design): no tile loads in the loop (MM_DIAG_NOFETCH, stale tiles), no candidate
# extraction (MM_DIAG_NOCAND), both; 1,024 x 2,000 x 2,000 accept-only, rocprofv3 kernel stats.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t47}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
for v in libpicp_amd libpicp_amd_nofetch libpicp_amd_nocand libpicp_amd_nofnc; do
  PICP_LIB=$L/$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/$v -o run --output-format csv -- python3 tools/match_ab.py 1024 2000 2000 "PICP_MATCH_ACCEPT_ONLY=1" > $OUT/$v.log 2>&1 || { echo "mab $v failed"; tail $OUT/$v.log; exit 1; }
  python3 - <<PY
import csv
for r in csv.DictReader(open("$OUT/$v/run_kernel_stats.csv")):
    if "mfma" in r["Name"]: print("$v", r["Calls"], "avg_us %.1f" % (float(r["AverageNs"]) / 1e3))
PY
done
