#!/bin/bash
# Round 6, call 12: the isolated 8e world match (tools/r06/match_8e.py --load) for the balanced
# max tree (tree, treepipe) and for forced range splits / row blocks of the shipped library; then
# the VO A/B of tree and treepipe at the three C5 shapes.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t12}
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/r06/match_8e.py --save $OUT/maps.npz > $OUT/save.log 2>&1 || { echo "save failed"; tail $OUT/save.log; exit 1; }
: > $OUT/iso.txt
for v in base tree treepipe base:KS=24 base:KS=28 base:KS=32 base:KS=8 base:RB=1 base:KS=28:RB=1; do
  lib=${v%%:*}; envs=""; [ "$lib" != "$v" ] && envs=$(echo ${v#*:} | sed 's/KS=/PICP_MATCH_KSPLIT=/; s/RB=/PICP_MATCH_RB=/; s/:/ /g')
  L=02-visualodometry_amd/lib/libpicp_amd.so; [ $lib != base ] && L=02-visualodometry_amd/lib/libpicp_amd_$lib.so
  n=$(echo $v | tr ':=' '__')
  env $envs PICP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/prof_$n -o run --output-format csv -- python3 -u tools/r06/match_8e.py --load $OUT/maps.npz > $OUT/iso_$n.log 2>&1 || { echo "iso $v failed"; tail $OUT/iso_$n.log; exit 1; }
  python3 tools/r06/match_durations.py $(find $OUT/prof_$n -name '*kernel_trace.csv' | head -1) $v | tee -a $OUT/iso.txt
done
rm -f $OUT/maps.npz
: > $OUT/ab.log
for rep in 1 2; do for A in "--seg-len 1250 --steps 2 --warmup 1 --samples 3" "--frames 1281" ""; do for v in base tree treepipe; do
  L=02-visualodometry_amd/lib/libpicp_amd.so; [ $v != base ] && L=02-visualodometry_amd/lib/libpicp_amd_$v.so
  PICP_LIB=$L timeout -k 10 300 python bench.py --workload c5 --no-cpu --skip-extras --detail - $A > $OUT/run.log 2>&1 || { echo "bench $v failed"; tail $OUT/run.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5 [$A]', '$v', d['value'], d.get('chain_step_us'))" | tee -a $OUT/ab.log
done; done; done
