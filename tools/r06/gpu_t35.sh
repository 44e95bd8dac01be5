#!/bin/bash
# Round 6, call 35: the next tile's fetch issued at the previous step's end, before the barrier
# (-DMM_EARLY=1, lib/libpicp_amd_early.so), against HEAD: matcher tests with it, the isolated 8e
# world match, the three C5 shapes interleaved.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t35}
mkdir -p $OUT
PICP_LIB=02-visualodometry_amd/lib/libpicp_amd_early.so timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_vo_long.py -x -q -m gpu -k match --timeout 300 --timeout-method thread > $OUT/pytest_early.log 2>&1 || { echo "early tests failed"; grep -E "FAIL|Error|error" $OUT/pytest_early.log | tail -30; exit 1; }
tail -1 $OUT/pytest_early.log
timeout -k 10 300 python3 -u tools/r06/match_8e.py --save $OUT/maps.npz > $OUT/save.log 2>&1 || { echo "save failed"; tail $OUT/save.log; exit 1; }
: > $OUT/iso.txt
for v in base early; do
  L=02-visualodometry_amd/lib/libpicp_amd.so; [ $v != base ] && L=02-visualodometry_amd/lib/libpicp_amd_$v.so
  PICP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/prof_$v -o run --output-format csv -- python3 -u tools/r06/match_8e.py --load $OUT/maps.npz > $OUT/iso_$v.log 2>&1 || { echo "iso $v failed"; tail $OUT/iso_$v.log; exit 1; }
  python3 tools/r06/match_durations.py $(find $OUT/prof_$v -name '*kernel_trace.csv' | head -1) $v | tee -a $OUT/iso.txt
done
rm -f $OUT/maps.npz
: > $OUT/ab.log
for rep in 1 2 3; do for A in "--seg-len 1250 --steps 2 --warmup 1 --samples 3" "--frames 1281" ""; do for v in base early; do
  L=02-visualodometry_amd/lib/libpicp_amd.so; [ $v != base ] && L=02-visualodometry_amd/lib/libpicp_amd_$v.so
  PICP_LIB=$L timeout -k 10 300 python bench.py --workload c5 --no-cpu --skip-extras --detail - $A > $OUT/run.log 2>&1 || { echo "bench $v failed"; tail $OUT/run.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5 [$A]', '$v', d['value'], d.get('chain_step_us'))" | tee -a $OUT/ab.log
done; done; done
