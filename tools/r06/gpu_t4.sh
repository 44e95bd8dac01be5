#!/bin/bash
# Round 6, call 4: the merge kernel's loads batched (16 ranges in flight instead of one at a time;
# lib/libpicp_amd_merge0.so = the one-at-a-time loop) at the split shapes, interleaved, 3 reps; the
# matcher GPU tests with the batched merge; the persistent kernel's error-word check against round
# 5's kernel (lib/libpicp_amd_perr0.so) on C2/C3.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t4}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_vo_long.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_match.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest_match.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
run() {  # tag workload-args env...
  local tag=$1; local A=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --no-cpu --skip-extras --detail - $A > $OUT/run.log 2>&1 || { echo "bench $tag failed"; tail $OUT/run.log; return 1; }
  python -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('$tag', '$A', d['value'], d.get('chain_step_us'), d['ms_per_step'])" | tee -a $OUT/ab.log
}
: > $OUT/ab.log
for A in "--workload c5 --seg-len 1250 --steps 2 --warmup 1 --samples 1" "--workload c5 --frames 1281"; do for rep in 1 2 3; do
  run merge0 "$A" PICP_LIB=$L/libpicp_amd_merge0.so || exit 1
  run merge16 "$A" PICP_LIB=$L/libpicp_amd.so || exit 1
done; done
for A in "--workload c2" "--workload c3"; do for rep in 1 2 3; do
  run perr0 "$A" PICP_LIB=$L/libpicp_amd_perr0.so || exit 1
  run perr "$A" PICP_LIB=$L/libpicp_amd.so || exit 1
done; done
