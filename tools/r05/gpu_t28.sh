#!/bin/bash
# Round 5, call 28: the folded matcher fetching its reference tiles two ahead (MM_PF2) against one
# ahead (-DMM_PF2=0, lib/libpicp_amd_pf1.so): matcher + VO tests on the candidate, the 1,024 x
# 2,000 x 2,000 accept-only launch (rocprofv3, both duplicate settings), C5 interleaved, 3 reps.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t28}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
OUT=$OUT/ab TESTS="tests/test_gpu_match.py tests/test_gpu_vo.py tests/test_gpu_vo_long.py" WLS="c5" LIBS="libpicp_amd_pf1 libpicp_amd" REPS=3 bash tools/gpu_ab.sh || exit 1
for v in libpicp_amd_pf1 libpicp_amd; do for dup in 0 0.5; do
  MATCH_DUP=$dup PICP_LIB=$L/$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/mab_${v}_$dup -o run --output-format csv -- python3 tools/match_ab.py 1024 2000 2000 "PICP_MATCH_ACCEPT_ONLY=1" > $OUT/mab_${v}_$dup.log 2>&1 || { echo "mab $v failed"; tail $OUT/mab_${v}_$dup.log; exit 1; }
  python3 - <<PY
import csv
for r in csv.DictReader(open("$OUT/mab_${v}_$dup/run_kernel_stats.csv")):
    if "mfma" in r["Name"]: print("$v dup=$dup", r["Calls"], "avg_us %.1f" % (float(r["AverageNs"]) / 1e3))
PY
done; done
OUT=$OUT/ab8e TESTS= WLS="c5" ARGS="--seg-len 1250 --steps 2 --warmup 1 --samples 1" LIBS="libpicp_amd_pf1 libpicp_amd" REPS=2 bash tools/gpu_ab.sh || exit 1
