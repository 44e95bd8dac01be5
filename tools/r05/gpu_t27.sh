#!/bin/bash
# Round 5, call 27: where the folded matcher's time goes now (1,024 x 2,000 x 2,000 accept-only,
# timing builds with wrong results): shipped vs no candidate extraction (-DMM_DIAG_NOCAND) vs no
# tile fetch and no tile barrier (-DMM_DIAG_NOFETCH: tile 0's data for every tile); rocprofv3
# kernel stats, 2 reps.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t27}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
for rep in 1 2; do for v in libpicp_amd libpicp_amd_nocand libpicp_amd_nofetch; do
  PICP_LIB=$L/$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/mab_${v}_$rep -o run --output-format csv -- python3 tools/match_ab.py 1024 2000 2000 "PICP_MATCH_ACCEPT_ONLY=1" > $OUT/mab_${v}_$rep.log 2>&1 || { echo "mab $v failed"; tail $OUT/mab_${v}_$rep.log; exit 1; }
  python3 - <<PY
import csv
for r in csv.DictReader(open("$OUT/mab_${v}_$rep/run_kernel_stats.csv")):
    if "mfma" in r["Name"]: print("$v rep $rep", r["Calls"], "avg_us %.1f" % (float(r["AverageNs"]) / 1e3))
PY
done; done
