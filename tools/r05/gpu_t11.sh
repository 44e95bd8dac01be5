#!/bin/bash
# Round 5, call 11: the whole GPU suite + smoke on the candidate (the matcher's candidate entries
# as one 16-bit block mask per lane instead of a per-candidate loop), then the C5 A/B against HEAD
# (lib/libpicp_amd_head.so), interleaved, and the matcher's kernel time on 1,024 x 2,000 x 2,000.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t11}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -o "step [0-9]*: map.*" $OUT/pytest_gpu.log | cut -c1-260; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit 1
OUT=$OUT/ab TESTS= WLS="c5" LIBS="libpicp_amd_head libpicp_amd" REPS=3 bash tools/gpu_ab.sh || exit 1
OUT=$OUT/ab8e TESTS= WLS="c5" ARGS="--seg-len 1250 --steps 2 --warmup 1 --samples 1" LIBS="libpicp_amd_head libpicp_amd" REPS=2 bash tools/gpu_ab.sh || exit 1
for v in libpicp_amd_head libpicp_amd; do for dup in 0 0.5; do
  MATCH_DUP=$dup PICP_LIB=$L/$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/mab_${v}_$dup -o run --output-format csv -- python3 tools/match_ab.py 1024 2000 2000 "PICP_MATCH_ACCEPT_ONLY=1" > $OUT/mab_${v}_$dup.log 2>&1 || { echo "mab $v failed"; tail $OUT/mab_${v}_$dup.log; exit 1; }
  python3 - <<PY
import csv
for r in csv.DictReader(open("$OUT/mab_${v}_$dup/run_kernel_stats.csv")):
    if "match" in r["Name"]: print("$v dup=$dup", r["Name"][:60], r["Calls"], "avg_us %.1f" % (float(r["AverageNs"]) / 1e3))
PY
done; done
# the split exchange's L2 path (PICP_XG_L2) at the 128-frame per-rank shape: A/B against -DPICP_XG_L2=0
OUT=$OUT/ab_xg TESTS= WLS="c4" ARGS="--problems 128" LIBS="libpicp_amd_xg0 libpicp_amd" REPS=3 bash tools/gpu_ab.sh || exit 1
