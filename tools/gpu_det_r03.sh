#!/bin/bash
# Round-3 determinism probe on one box: the VO schedule check and the concurrency check on the
# shipped library, then the per-round block-kernel records (diagnostic build) beside a VO sequence.
export TMPDIR=/tmp
OUT=gpurun_out/r03/${TAG:-det}
mkdir -p $OUT
timeout -k 10 240 python -u tools/vo_chains_check.py 2001 "PICP_VO_CHAINS=1,PICP_VO_OVERLAP=0" "PICP_VO_OVERLAP=1" "PICP_VO_CHAINS=2" > $OUT/vo_chains.log 2>&1 || { echo "vo_chains failed"; tail $OUT/vo_chains.log; exit 1; }
grep setting $OUT/vo_chains.log
timeout -k 10 300 python -u tools/concurrency_check.py > $OUT/conc.log 2>&1 || { echo "conc failed"; tail $OUT/conc.log; exit 1; }
grep -v beside: $OUT/conc.log
timeout -k 10 300 python -u tools/bdiag_check.py ${BDIAG_REPS:-12} > $OUT/bdiag.log 2>&1 || { echo "bdiag failed"; tail $OUT/bdiag.log; exit 1; }
tail -30 $OUT/bdiag.log
