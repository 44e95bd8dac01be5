#!/bin/bash
# Round 4: which packed-FP32 instructions of permlane_stress victim 9 carry the lane 48-63
# disagreement beside the MFMA aggressor (tools/ubench/pk_bisect.py).
export TMPDIR=/tmp
O=gpurun_out/pkb; mkdir -p $O
timeout -k 10 1050 python -u tools/ubench/pk_bisect.py $O/work ${ITERS:-1000} > $O/bisect.log 2>&1
rc=$?; tail -40 $O/bisect.log; exit $rc
