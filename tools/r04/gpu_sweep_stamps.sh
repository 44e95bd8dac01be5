#!/bin/bash
# Round 4: the persistent kernel's phases with the leader's sweep passes (diagnostic stamp build):
# C2 (100k) and C3 (1M, 30 % outliers).
export TMPDIR=/tmp
O=gpurun_out/swst; mkdir -p $O
timeout -k 10 200 python tools/pstamps.py --n 100000 > $O/pstamps_c2.log 2>&1 || { tail $O/pstamps_c2.log; exit 1; }
cat $O/pstamps_c2.log
timeout -k 10 200 python tools/pstamps.py --n 1000000 --outlier 0.3 > $O/pstamps_c3.log 2>&1 || { tail $O/pstamps_c3.log; exit 1; }
cat $O/pstamps_c3.log
