#!/bin/bash
# Round 5, call 13: the matcher's vote max as a balanced tree (depth 3) against the chain of eight
# dependent max3 (-DMM_MAX_TREE=0, lib/libpicp_amd_nomt.so): matcher tests on the candidate, the
# 1,024 x 2,000 x 2,000 accept-only launch under rocprofv3, C5 interleaved.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t13}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
OUT=$OUT/ab TESTS="tests/test_gpu_match.py" WLS="c5" LIBS="libpicp_amd_nomt libpicp_amd" REPS=3 bash tools/gpu_ab.sh || exit 1
for rep in 1 2; do for v in libpicp_amd_nomt libpicp_amd; do
  PICP_LIB=$L/$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/mab_${v}_$rep -o run --output-format csv -- python3 tools/match_ab.py 1024 2000 2000 "PICP_MATCH_ACCEPT_ONLY=1" > $OUT/mab_${v}_$rep.log 2>&1 || { echo "mab $v failed"; tail $OUT/mab_${v}_$rep.log; exit 1; }
  python3 - <<PY
import csv
for r in csv.DictReader(open("$OUT/mab_${v}_$rep/run_kernel_stats.csv")):
    if "mfma" in r["Name"]: print("$v rep $rep", r["Calls"], "avg_us %.1f" % (float(r["AverageNs"]) / 1e3))
PY
done; done
