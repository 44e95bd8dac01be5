#!/bin/bash
# Round 6, call 10: where the 8e world match's time goes.  The maps of segments 0-3 saved once, then
# the isolated 4-problem launches (tools/r06/match_8e.py --load) under the kernel tracer for the
# shipped library and the A/B builds: two-deep tile prefetch (pf2), software-pipelined MFMAs
# (pipe, pipepf2), one vote per row-block pair (pair) and the diagnostic build without the wave vote (novote).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t10}
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/r06/match_8e.py --save $OUT/maps.npz > $OUT/save.log 2>&1 || { echo "save failed"; tail $OUT/save.log; exit 1; }
: > $OUT/iso.txt
for v in base pf2 pipe pipepf2 pair novote; do
  L=02-visualodometry_amd/lib/libpicp_amd.so; [ $v != base ] && L=02-visualodometry_amd/lib/libpicp_amd_$v.so
  PICP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/prof_$v -o run --output-format csv -- python3 -u tools/r06/match_8e.py --load $OUT/maps.npz > $OUT/iso_$v.log 2>&1 || { echo "iso $v failed"; tail $OUT/iso_$v.log; exit 1; }
  python3 tools/r06/match_durations.py $(find $OUT/prof_$v -name '*kernel_trace.csv' | head -1) $v | tee -a $OUT/iso.txt
done
rm -f $OUT/maps.npz
PICP_LIB=02-visualodometry_amd/lib/libpicp_amd_pipe.so timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_pipe.log 2>&1 || { echo "pipe tests failed"; tail -30 $OUT/pytest_pipe.log; exit 1; }
tail -1 $OUT/pytest_pipe.log
: > $OUT/ab.log
for rep in 1 2; do for A in "--seg-len 1250 --steps 2 --warmup 1 --samples 3" "--frames 1281" ""; do for v in base pipe pair; do
  L=02-visualodometry_amd/lib/libpicp_amd.so; [ $v != base ] && L=02-visualodometry_amd/lib/libpicp_amd_$v.so
  PICP_LIB=$L timeout -k 10 300 python bench.py --workload c5 --no-cpu --skip-extras --detail - $A > $OUT/run.log 2>&1 || { echo "bench $v failed"; tail $OUT/run.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5 [$A]', '$v', d['value'], d.get('chain_step_us'))" | tee -a $OUT/ab.log
done; done; done
