#!/bin/bash
# Round 5, call 30: the accept-only matcher's key-ordered window (picp_launch_match_order):
# matcher GPU tests, then 1,024 x 2,000 x 2,000 accept-only with the window on / off (rocprofv3
# kernel stats), and C5 against HEAD (the VO sequence does not order yet: a no-change check).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t30}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
for ord in 1 0; do
  PICP_MATCH_ORDER=$ord timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/mab_$ord -o run --output-format csv -- python3 tools/match_ab.py 1024 2000 2000 "PICP_MATCH_ACCEPT_ONLY=1" > $OUT/mab_$ord.log 2>&1 || { echo "mab $ord failed"; tail $OUT/mab_$ord.log; exit 1; }
  python3 - <<PY
import csv
for r in csv.DictReader(open("$OUT/mab_$ord/run_kernel_stats.csv")):
    if "match" in r["Name"]: print("order=$ord", r["Name"][:60], r["Calls"], "avg_us %.1f" % (float(r["AverageNs"]) / 1e3))
PY
done
