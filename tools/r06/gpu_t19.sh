#!/bin/bash
# Round 6, call 19: B operands straight from memory per wave (PICP_MATCH_DIRECT=1; no LDS tile, no
# block barrier per tile), groups of 4 (default build) or 2 (lib/libpicp_amd_dg2.so) column blocks
# ahead: the matcher tests bit-exact with it, the isolated 8e world match, the three C5 shapes.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t19}
mkdir -p $OUT
PICP_MATCH_DIRECT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_vo_long.py -x -q -m gpu -k "match" --timeout 300 --timeout-method thread > $OUT/pytest_direct.log 2>&1 || { echo "direct tests failed"; grep -E "FAIL|Error|error" $OUT/pytest_direct.log | tail -30; exit 1; }
tail -1 $OUT/pytest_direct.log
timeout -k 10 300 python3 -u tools/r06/match_8e.py --save $OUT/maps.npz > $OUT/save.log 2>&1 || { echo "save failed"; tail $OUT/save.log; exit 1; }
: > $OUT/iso.txt
for v in base direct:base direct:dg2; do
  lib=${v#*:}; [ $v = base ] && lib=base
  d=0; [ ${v%%:*} = direct ] && d=1
  L=02-visualodometry_amd/lib/libpicp_amd.so; [ $lib != base ] && L=02-visualodometry_amd/lib/libpicp_amd_$lib.so
  n=$(echo $v | tr ':' '_')
  PICP_MATCH_DIRECT=$d PICP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/prof_$n -o run --output-format csv -- python3 -u tools/r06/match_8e.py --load $OUT/maps.npz > $OUT/iso_$n.log 2>&1 || { echo "iso $v failed"; tail $OUT/iso_$n.log; exit 1; }
  python3 tools/r06/match_durations.py $(find $OUT/prof_$n -name '*kernel_trace.csv' | head -1) $v | tee -a $OUT/iso.txt
done
rm -f $OUT/maps.npz
: > $OUT/ab.log
for rep in 1 2; do for A in "--seg-len 1250 --steps 2 --warmup 1 --samples 3" "--frames 1281" ""; do for v in base direct:base direct:dg2; do
  lib=${v#*:}; [ $v = base ] && lib=base
  d=0; [ ${v%%:*} = direct ] && d=1
  L=02-visualodometry_amd/lib/libpicp_amd.so; [ $lib != base ] && L=02-visualodometry_amd/lib/libpicp_amd_$lib.so
  PICP_MATCH_DIRECT=$d PICP_LIB=$L timeout -k 10 300 python bench.py --workload c5 --no-cpu --skip-extras --detail - $A > $OUT/run.log 2>&1 || { echo "bench $v failed"; tail $OUT/run.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5 [$A]', '$v', d['value'], d.get('chain_step_us'))" | tee -a $OUT/ab.log
done; done; done
