#!/bin/bash
# Round 6, call 3: the reverted library (the separate merge kernel, the round-5 append) at the three
# C5 shapes; then A/B at those shapes: the side stream's frame->next matches on a CU-masked queue
# (PICP_VO_SIDE_CU_SKIP = 8, 4, 2: every k-th CU left to the step chains); then the world match's
# knobs at the latency-bound shapes: the reference-range split (PICP_MATCH_KSPLIT, default ~4
# blocks per CU) and the row blocks per wave (PICP_MATCH_RB).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t3}
mkdir -p $OUT
run() {  # tag env...   (bench args in $ARGS)
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --workload c5 --no-cpu --skip-extras --detail - $ARGS > $OUT/run.log 2>&1 || { echo "bench $tag failed"; tail $OUT/run.log; return 1; }
  python -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('$tag', '$ARGS', d['value'], d.get('chain_step_us'), d.get('ate_m'), d.get('rounds_sync'))" | tee -a $OUT/ab.log
}
: > $OUT/ab.log
for ARGS in "" "--seg-len 1250 --steps 2 --warmup 1 --samples 1" "--frames 1281"; do for rep in 1 2; do
  run default X=1 || exit 1
  for k in 8 4 2; do run sidecu$k PICP_VO_SIDE_CU_SKIP=$k || exit 1; done
done; done
for ARGS in "--seg-len 1250 --steps 2 --warmup 1 --samples 1" "--frames 1281"; do
  for k in 4 8 24 32; do run ksplit$k PICP_MATCH_KSPLIT=$k || exit 1; done
  for rb in 1 2; do run rb$rb PICP_MATCH_RB=$rb || exit 1; done
  run noxcd PICP_MATCH_XCD=0 || exit 1
  run nophase PICP_VO_PHASE=0 || exit 1
  run default X=1 || exit 1
done
