#!/bin/bash
# Round 5, call 31: matcher blocks of eight waves (-DMM_WAVES=8, lib/libpicp_amd_w8.so: two blocks
# per CU sharing each reference tile among 512 queries) against four, with and without the
# key-ordered window: 1,024 x 2,000 x 2,000 accept-only kernel stats; then C5 interleaved.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t31}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
PICP_LIB=$L/libpicp_amd_w8.so timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_w8.log 2>&1
rc=$?; echo "pytest w8 rc=$rc"; tail -2 $OUT/pytest_w8.log; [ $rc -eq 0 ] || exit 1
for v in libpicp_amd libpicp_amd_w8; do for ord in 1 0; do
  PICP_LIB=$L/$v.so PICP_MATCH_ORDER=$ord timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/mab_${v}_$ord -o run --output-format csv -- python3 tools/match_ab.py 1024 2000 2000 "PICP_MATCH_ACCEPT_ONLY=1" > $OUT/mab_${v}_$ord.log 2>&1 || { echo "mab $v $ord failed"; tail $OUT/mab_${v}_$ord.log; exit 1; }
  python3 - <<PY
import csv
for r in csv.DictReader(open("$OUT/mab_${v}_$ord/run_kernel_stats.csv")):
    if "mfma" in r["Name"]: print("$v order=$ord", r["Calls"], "avg_us %.1f" % (float(r["AverageNs"]) / 1e3))
PY
done; done
OUT=$OUT/ab TESTS= WLS="c5" LIBS="libpicp_amd libpicp_amd_w8" REPS=2 bash tools/gpu_ab.sh || exit 1
