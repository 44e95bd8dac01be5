#!/bin/bash
# SQ counters (one --pmc pass, 7 SQ + 1 GRBM) of one workload's dominant kernel for each build in
# LIBS: WL=c4 K=picp_block LIBS="libpicp_amd_c1 libpicp_amd"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc_sq}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
for v in ${LIBS:-libpicp_amd}; do
  PICP_LIB=$L/$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $OUT/${v}_${WL:-c4} -o run --output-format csv -- python3 bench.py --workload ${WL:-c4} --no-cpu --skip-extras --steps 5 --warmup 1 > $OUT/${v}.log 2>&1 || { echo "pmc $v failed"; tail -5 $OUT/${v}.log; exit 1; }
  python3 tools/parse_pmc.py $OUT/${v}_${WL:-c4}/run_counter_collection.csv ${K:-picp_block} > $OUT/${v}_${WL:-c4}.json
  echo "== $v"; python3 -c "import json; d=json.load(open('$OUT/${v}_${WL:-c4}.json')); print({k:round(v['mean']) for k,v in d.items()})"
done
