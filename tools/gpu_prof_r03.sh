#!/bin/bash
# Round-3 profiles of the bench configs: rocprofv3 kernel-trace/stats per workload, then the HBM
# traffic counters FETCH_SIZE and WRITE_SIZE in SEPARATE --pmc passes (MI355X_MICROARCH.md).
# Every step time-limited; stop at the first failure.  OUT=${OUT:-gpurun_out/r03/prof}
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r03/prof}
mkdir -p $OUT
for W in ${WLS:-c2 c4 c3 c5}; do
  ARGS="--no-cpu --skip-extras --steps 10 --warmup 2 --samples 1 --workload $W"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${W}_trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/${W}_trace.log 2>&1 || { echo "trace $W failed"; tail $OUT/${W}_trace.log; exit 1; }
  cp $OUT/${W}_trace/run_kernel_stats.csv $OUT/kernel_stats_$W.csv
  python3 -c "import json; d=json.loads([l for l in open('$OUT/${W}_trace.log').read().splitlines() if l.startswith('{')][-1]); print('$W', d['value'], d['unit'], d['ms_per_step'])"
done
for P in ${PMCS:-c2:c2_persistent:picp_persistent c4:c4x1024_block:picp_block c3:c3_persistent:picp_persistent c2n16m:stream16m:picp_round_kernel}; do
  W=${P%%:*}; R=${P#*:}; NAME=${R%%:*}; K=${R#*:}
  EXTRA=""; [ "$W" = c2n16m ] && { W=c2; EXTRA="--n 16000000 --rounds 50"; }
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/${NAME}_$C -o run --output-format csv -- python3 bench.py --no-cpu --skip-extras --steps 5 --warmup 1 --samples 1 --workload $W $EXTRA > $OUT/${NAME}_$C.log 2>&1 || { echo "pmc $NAME $C failed"; tail $OUT/${NAME}_$C.log; exit 1; }
    python3 tools/parse_pmc.py $OUT/${NAME}_$C/run_counter_collection.csv $K > $OUT/${NAME}_pmc_$C.json
    python3 -c "import json; d=json.load(open('$OUT/${NAME}_pmc_$C.json')); print('$NAME', '$C', d['$C']['mean'], d['$C']['dispatches'])"
  done
done
