#!/bin/bash
# Round 5, call 5: the GPU suite with the matcher's reference-range split and the round-3 dpp /
# contraction forms restored; C2/C3 A/B against the round-3 library; the C5 shapes (default, 8e,
# N = 8 per-rank) timed once each.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t5}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_vo_long.py tests/test_gpu_match.py} -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" $OUT/pytest_gpu.log | tail -8; grep -E "^step " $OUT/pytest_gpu.log | head; [ $rc -le 1 ] || exit 1
OUT=$OUT/ab TESTS= WLS="c2 c3" LIBS="libpicp_amd_r03 libpicp_amd" REPS=3 bash tools/gpu_ab.sh || exit 1
for W in c5 c5_8e c5_n8; do
  case $W in
    c5) A="--workload c5 --steps 5 --warmup 2" ;;
    c5_8e) A="--workload c5 --seg-len 1250 --steps 2 --warmup 1" ;;
    c5_n8) A="--workload c5 --frames 1281 --steps 10 --warmup 2" ;;
  esac
  timeout -k 10 300 python3 bench.py $A --no-cpu --skip-extras --samples 3 --detail $OUT/detail_$W.json > $OUT/bench_$W.log 2>&1 || { echo "bench $W failed"; tail $OUT/bench_$W.log; exit 1; }
  tail -1 $OUT/bench_$W.log | cut -c1-400
done
