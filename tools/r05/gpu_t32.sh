#!/bin/bash
# Round 5, call 32: the accept-only matcher's launch time against the reference count (1,024
# problems x 2,000 queries x 1,000 / 2,000 / 4,000 / 8,000 references): the per-tile slope and
# the per-block intercept.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t32}
mkdir -p $OUT
for nr in 1000 2000 4000 8000; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/nr_$nr -o run --output-format csv -- python3 tools/match_ab.py 1024 2000 $nr "PICP_MATCH_ACCEPT_ONLY=1" > $OUT/nr_$nr.log 2>&1 || { echo "nr $nr failed"; tail $OUT/nr_$nr.log; exit 1; }
  python3 - <<PY
import csv
for r in csv.DictReader(open("$OUT/nr_$nr/run_kernel_stats.csv")):
    if "mfma" in r["Name"]: print("nr=$nr", r["Name"][:50], r["Calls"], "avg_us %.1f" % (float(r["AverageNs"]) / 1e3))
PY
done
