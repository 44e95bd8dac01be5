#!/bin/bash
# Round 6, call 38: VERDICT r05 item 4 -- the solvers wait on a per-problem arrival counter (one
# line, bumped by every block after its publish) before the granule sweep.  lib/libpicp_amd_arrival.so
# = -DPICP_ARRIVAL; the shipped library carries the counter space but does not touch it.  Parity
# tests with both libraries, then C2/C3 interleaved, 4 reps, and one FETCH_SIZE pass on C3 each.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t38}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_head.log 2>&1
rc=$?; echo "pytest head rc=$rc"; tail -2 $OUT/pytest_head.log; [ $rc -eq 0 ] || exit 1
PICP_LIB=$L/libpicp_amd_arrival.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_arrival.log 2>&1
rc=$?; echo "pytest arrival rc=$rc"; tail -2 $OUT/pytest_arrival.log; [ $rc -eq 0 ] || exit 1
run() {  # tag workload-args env...
  local tag=$1; local A=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --no-cpu --skip-extras --detail - $A > $OUT/run.log 2>&1 || { echo "bench $tag failed"; tail $OUT/run.log; return 1; }
  python -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('$tag', '$A', d['value'], d['ms_per_step'])" | tee -a $OUT/ab.log
}
: > $OUT/ab.log
for A in "--workload c2" "--workload c3"; do for rep in 1 2 3 4; do
  run head "$A" PICP_LIB=$L/libpicp_amd.so || exit 1
  run arrival "$A" PICP_LIB=$L/libpicp_amd_arrival.so || exit 1
done; done
A="--no-cpu --skip-extras --steps 5 --warmup 1 --samples 1 --workload c3"
for v in head arrival; do
  lib=$L/libpicp_amd.so; [ $v = arrival ] && lib=$L/libpicp_amd_arrival.so
  PICP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch_$v -o run --output-format csv -- python3 bench.py $A > $OUT/fetch_$v.log 2>&1 || { echo "pmc $v failed"; tail $OUT/fetch_$v.log; exit 1; }
  python3 tools/parse_pmc.py $OUT/fetch_$v/run_counter_collection.csv picp_persistent > $OUT/c3_fetch_$v.json
  python3 -c "import json; d=json.load(open('$OUT/c3_fetch_$v.json')); print('c3 FETCH_SIZE $v', d['FETCH_SIZE'])"
done
