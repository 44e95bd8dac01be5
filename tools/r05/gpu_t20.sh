#!/bin/bash
# Round 5, call 20: phase stamps (diagnostic stamp build) of the eight-solver persistent kernel (C2,
# C3) and of the split-4 block kernel at 128 frames with the aligned exchange.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t20}
mkdir -p $OUT
timeout -k 10 200 python tools/pstamps.py --n 100000 > $OUT/pstamps_c2.log 2>&1 || { tail $OUT/pstamps_c2.log; exit 1; }
cat $OUT/pstamps_c2.log
timeout -k 10 200 python tools/pstamps.py --n 1000000 --outlier 0.3 > $OUT/pstamps_c3.log 2>&1 || { tail $OUT/pstamps_c3.log; exit 1; }
cat $OUT/pstamps_c3.log
PICP_BLOCK_SPLIT=4 timeout -k 10 200 python tools/bstamps.py --problems 128 --n 10000 > $OUT/bstamps_c4x128.log 2>&1 || { tail $OUT/bstamps_c4x128.log; exit 1; }
cat $OUT/bstamps_c4x128.log
