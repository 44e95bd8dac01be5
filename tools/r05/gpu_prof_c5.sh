#!/bin/bash
# Round 5: kernel breakdown of the C5 shapes (VERDICT r04 "What's missing" 3 / next 6): the default
# 250-segment partition, SURVEY §8e's 8 x 1,250-step partition (8e) and the N = 8 per-rank shape
# (rank 0's 32 of the 250 segments: frames 0 .. 1,280).  rocprofv3 --kernel-trace --stats each,
# then tools/vo_timeline.py over the trace: per stream (each step chain, the frame->next side
# stream) the busy time by kernel, and the device's concurrency.  Every step time-limited.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/prof_c5}
mkdir -p $OUT
for W in ${WLS:-c5 c5_8e c5_n8}; do
  case $W in
    c5) A="--workload c5 --steps 3 --warmup 2" ;;
    c5_8e) A="--workload c5 --seg-len 1250 --steps 1 --warmup 1" ;;
    c5_n8) A="--workload c5 --frames 1281 --steps 5 --warmup 2" ;;
  esac
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/${W}_trace -o run --output-format csv -- python3 bench.py $A --no-cpu --skip-extras --samples 1 --detail - > $OUT/${W}_trace.log 2>&1 || { echo "trace $W failed"; tail $OUT/${W}_trace.log; exit 1; }
  cp $OUT/${W}_trace/run_kernel_stats.csv $OUT/kernel_stats_$W.csv
  python3 tools/vo_timeline.py $OUT/${W}_trace/run_kernel_trace.csv ${LAST_MS:-} > $OUT/timeline_$W.txt
  python3 -c "import json; d=json.loads([l for l in open('$OUT/${W}_trace.log').read().splitlines() if l.startswith('{')][-1]); print('$W', d['value'], d['unit'], d['ms_per_step'], d.get('chain_step_us'))"
  head -8 $OUT/timeline_$W.txt
  rm -f $OUT/${W}_trace/run_kernel_trace.csv
done
