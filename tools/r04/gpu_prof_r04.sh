#!/bin/bash
# Round-4 profiles at HEAD: rocprofv3 kernel-trace/stats per bench workload (C2, C3, C4 at 1024 and
# at the 128-frame per-rank shape, C5, the 16M streaming frame), then the HBM traffic counters
# FETCH_SIZE and WRITE_SIZE in SEPARATE --pmc passes (MI355X_MICROARCH.md), and one SQ pass
# (VALU instructions, waves, busy cycles) for the VALU-bound kernels.  Each trace also gets a
# trace_summary_<workload>.json: the dominant kernel's mean over every dispatch and over the timed
# ones (tools/trace_summary.py).  Every step time-limited;
# stop at the first failure.  OUT=${OUT:-gpurun_out/r04/prof}
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04/prof}
mkdir -p $OUT
args() {  # workload tag -> bench arguments
  case $1 in
    c2n16m) echo "--workload c2 --n 16000000 --rounds 50" ;;
    c4x128) echo "--workload c4 --problems 128" ;;
    *) echo "--workload $1" ;;
  esac
}
for W in ${WLS:-c2 c3 c4 c4x128 c5 c2n16m}; do
  # warm-up long enough for the clocks to settle (C4's first launches run up to 13 % longer)
  A="--no-cpu --skip-extras --steps 10 --warmup ${TRACE_WARMUP:-10} --samples 1 $(args $W)"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${W}_trace -o run --output-format csv -- python3 bench.py $A > $OUT/${W}_trace.log 2>&1 || { echo "trace $W failed"; tail $OUT/${W}_trace.log; exit 1; }
  cp $OUT/${W}_trace/run_kernel_stats.csv $OUT/kernel_stats_$W.csv
  case $W in c5) KP="_Z22picp_match" ;; c2n16m) KP="void picp_round" ;; *) KP="void picp_" ;; esac
  T=10; [ $W = c5 ] && T=0
  python3 tools/trace_summary.py $OUT/${W}_trace/run_kernel_trace.csv "$KP" $T $OUT/${W}_trace.log > $OUT/trace_summary_$W.json
  python3 -c "import json; d=json.loads([l for l in open('$OUT/${W}_trace.log').read().splitlines() if l.startswith('{')][-1]); print('$W', d['value'], d['unit'], d['ms_per_step'])"
done
for P in ${PMCS:-c2:c2_persistent:picp_persistent c3:c3_persistent:picp_persistent c4:c4x1024_block:picp_block c4x128:c4x128:picp_ c2n16m:stream16m:picp_round_kernel}; do
  W=${P%%:*}; R=${P#*:}; NAME=${R%%:*}; K=${R#*:}
  A="--no-cpu --skip-extras --steps 5 --warmup 1 --samples 1 $(args $W)"
  for C in FETCH_SIZE WRITE_SIZE SQ; do
    CTRS=$C; [ $C = SQ ] && CTRS="SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
    [ $C = SQ ] && [ $W = c2 -o $W = c2n16m ] && continue
    timeout -s KILL 120 rocprofv3 --pmc $CTRS -d $OUT/${NAME}_$C -o run --output-format csv -- python3 bench.py $A > $OUT/${NAME}_$C.log 2>&1 || { echo "pmc $NAME $C failed"; tail $OUT/${NAME}_$C.log; exit 1; }
    python3 tools/parse_pmc.py $OUT/${NAME}_$C/run_counter_collection.csv $K > $OUT/${NAME}_pmc_$C.json
    python3 -c "import json; d=json.load(open('$OUT/${NAME}_pmc_$C.json')); print('$NAME', '$C', {k: v['mean'] for k, v in d.items()})"
  done
done
