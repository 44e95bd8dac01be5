#!/bin/bash
# Round 4: does the LITE form run?  SQ passes (VALU instructions) on C4 for the default build, the
# build that takes LITE without its checks (-DPICP_LITE_FORCE, a diagnostic switch since removed),
# and -DPICP_LITE=0.
export TMPDIR=/tmp
O=gpurun_out/lite3; mkdir -p $O
L=$PWD/02-visualodometry_amd/lib
for v in new:libpicp_amd.so force:libpicp_amd_liteforce.so nolite:libpicp_amd_nolite.so; do
  t=${v%%:*}; lib=${v#*:}
  export PICP_LIB=$L/$lib
  for W in "c4" "c3"; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $O/sq_${t}_$W -o run --output-format csv -- python3 bench.py --workload $W --no-cpu --skip-extras --steps 5 --warmup 1 --samples 1 > $O/sq_${t}_$W.log 2>&1 || { echo "pmc $t failed"; tail $O/sq_${t}_$W.log; exit 1; }
  K=picp_block; [ $W = c3 ] && K=picp_persistent
  python3 tools/parse_pmc.py $O/sq_${t}_$W/run_counter_collection.csv $K > $O/${W}_sq_$t.json
  python3 -c "import json; d=json.load(open('$O/${W}_sq_$t.json')); print('$t', '$W', {k: v['mean'] for k, v in d.items()})"
  done
  unset PICP_LIB
done
